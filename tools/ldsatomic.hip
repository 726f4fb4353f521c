// LDS counting-rate probe (gfx950): how fast can a CU count 10-bit digits?
//   A: ds_add_u32 (no return) per element into one 1024-bin histogram
//   B: ds_add_rtn_u32 per element into per-wave 16-bit packed counters (the
//      stable scatter's rank)
//   C: wave match (10 ballots) -> rank inside the step; the first lane of
//      every digit class does a plain read-modify-write of the wave's private
//      16-bit counter (no atomics: the active addresses are distinct)
// Digits come from a per-lane xorshift in registers (no memory traffic).
//   hipcc -O3 --offload-arch=gfx950 tools/ldsatomic.hip -o build_lab/ldsatomic
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int THREADS = 512, W = THREADS / 64, NB = 1024;

__device__ __forceinline__ uint32_t xs(uint32_t& s) {
    s ^= s << 13; s ^= s >> 17; s ^= s << 5; return s;
}

__device__ __forceinline__ uint64_t match10(uint32_t d) {
    uint64_t peers = ~0ull;
#pragma unroll
    for (int b = 0; b < 10; b++) {
        const bool bit = (d >> b) & 1u;
        const uint64_t m = __ballot(bit);
        peers &= bit ? m : ~m;
    }
    return peers;
}

template <int MODE>
__global__ void __launch_bounds__(THREADS) k_probe(int iters, uint32_t* sink) {
    __shared__ uint32_t h[W * NB];
    for (int i = threadIdx.x; i < W * NB; i += THREADS) h[i] = 0;
    __syncthreads();
    uint32_t s = 0x9e3779b9u * (blockIdx.x * THREADS + threadIdx.x + 1);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t acc = 0;
    uint16_t* c16 = reinterpret_cast<uint16_t*>(h) + wid * NB;
    const uint64_t lt = (1ull << lane) - 1;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const uint32_t d = xs(s) & (NB - 1);
            if (MODE == 0) {
                atomicAdd(&h[d], 1u);
            } else if (MODE == 1) {
                const uint32_t sh = (d & 1u) * 16u;
                const uint32_t old = atomicAdd(&h[wid * (NB / 2) + (d >> 1)], 1u << sh);
                acc += (old >> sh) & 0xffffu;
            } else {
                const uint64_t p = match10(d);
                const uint32_t r = __popcll(p & lt);
                const uint32_t old = c16[d];
                if (r == 0) c16[d] = (uint16_t)(old + __popcll(p));
                acc += old + r;
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) sink[blockIdx.x] = acc + h[lane];
}

template <int MODE>
static int run(const char* name, int iters, uint32_t* sink) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    const int grid = 256;
    hipLaunchKernelGGL(k_probe<MODE>, dim3(grid), dim3(THREADS), 0, 0, iters, sink);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(k_probe<MODE>, dim3(grid), dim3(THREADS), 0, 0, iters, sink);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms; CHECK(hipEventElapsedTime(&ms, a, b));
    const double el = (double)grid * THREADS * iters * 16;
    printf("%-28s %8.3f ms  %.3g elements/s  %.3f elements/clk/CU (2.4 GHz, 256 CUs)\n", name, ms,
           el / (ms * 1e-3), el / (ms * 1e-3) / 2.4e9 / 256);
    return 0;
}

int main() {
    uint32_t* sink;
    CHECK(hipMalloc(&sink, 4096 * 4));
    const int iters = 64;  // 2^27 elements in all: one bench_partitioning pass
    if (run<0>("A ds_add 1024 bins", iters, sink)) return 1;
    if (run<1>("B ds_add_rtn per-wave u16", iters, sink)) return 1;
    if (run<2>("C match + leader RMW u16", iters, sink)) return 1;
    if (run<0>("A ds_add 1024 bins", iters, sink)) return 1;
    return 0;
}
