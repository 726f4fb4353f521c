// scatterlab.hip -- lab probe (not part of the library): can ONE scatter pass
// reach LDS-sized buckets?  A two-pass sort of 2^27 8-byte elements needs a
// level-1 fan-out of ~8192 (16K-element buckets = 128 KB, one workgroup's
// LDS); the library's write-combining scatter keeps a 64-byte carry per
// partition in LDS, which caps it at ~1024 partitions.  This probe times the
// alternative with no carry at all: exact per-workgroup offsets from a
// histogram pass, then every element stored straight to its place (8-byte
// stores, 64 lanes -> up to 64 lines), the L2 left to merge the partial lines.
//
//   hipcc -O3 --offload-arch=gfx950 tools/scatterlab.hip -o build_lab/scatterlab
//   build_lab/scatterlab [log2 n = 27]
//
// For B = 8 .. 13 bins bits and 256 / 1024 workgroups it prints the scatter
// kernel's time and rate (2 x 8 bytes per element) for
//   direct   : contiguous chunk per workgroup, rank by LDS atomic, plain store
//   direct-nt: the same with non-temporal stores
//   inter    : tiles interleaved over the workgroups (tile t -> wg t % G), so
//              all workgroups advance through the input together
//   staged   : the tile counting-sorted by bin in LDS first, then stored in
//              bin order (neighbouring lanes write neighbouring addresses
//              where a bin has several elements in the tile)
// and checks the output is a permutation grouped by bin.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

constexpr int THREADS = 512;
constexpr int ITEMS = 16;
constexpr int TILE = THREADS * ITEMS;

__device__ __forceinline__ uint32_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return (uint32_t)x;
}

__global__ void k_gen(uint64_t* a, uint64_t n, int lg) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
        const uint32_t key = mix(i * 0x9E3779B97F4A7C15ull) & ((1u << lg) - 1);
        a[i] = ((uint64_t)key << 32) | (uint32_t)i;
    }
}

__device__ __forceinline__ uint32_t bin_of(uint64_t v, int lg, int B) {
    return (uint32_t)(v >> 32) >> (lg - B);
}

// tile t of workgroup g: contiguous chunk (INTER = 0) or interleaved tiles
template <bool INTER>
__device__ __forceinline__ uint64_t tile_base(uint32_t k, uint64_t chunk_tiles) {
    return INTER ? ((uint64_t)k * gridDim.x + blockIdx.x) * TILE
                 : ((uint64_t)blockIdx.x * chunk_tiles + k) * TILE;
}

template <bool INTER>
__global__ void __launch_bounds__(THREADS) k_hist(const uint64_t* a, uint64_t n, int lg, int B,
                                                  uint64_t chunk_tiles, uint32_t* hist) {
    extern __shared__ uint32_t h[];
    const uint32_t nb = 1u << B;
    for (uint32_t i = threadIdx.x; i < nb; i += THREADS) h[i] = 0;
    __syncthreads();
    for (uint32_t k = 0; k < chunk_tiles; k++) {
        const uint64_t base = tile_base<INTER>(k, chunk_tiles);
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint64_t i = base + j * THREADS + threadIdx.x;
            if (i < n) atomicAdd(&h[bin_of(a[i], lg, B)], 1u);
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nb; i += THREADS) hist[(size_t)i * gridDim.x + blockIdx.x] = h[i];
}

template <bool INTER, bool NT>
__global__ void __launch_bounds__(THREADS) k_scatter(const uint64_t* a, uint64_t n, int lg, int B,
                                                     uint64_t chunk_tiles, const uint32_t* off,
                                                     uint64_t* out) {
    extern __shared__ uint32_t cur[];
    const uint32_t nb = 1u << B;
    for (uint32_t i = threadIdx.x; i < nb; i += THREADS) cur[i] = off[(size_t)i * gridDim.x + blockIdx.x];
    __syncthreads();
    for (uint32_t k = 0; k < chunk_tiles; k++) {
        const uint64_t base = tile_base<INTER>(k, chunk_tiles);
        uint64_t v[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint64_t i = base + j * THREADS + threadIdx.x;
            v[j] = i < n ? __builtin_nontemporal_load(a + i) : ~0ull;
        }
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            if (v[j] == ~0ull) continue;
            const uint32_t p = atomicAdd(&cur[bin_of(v[j], lg, B)], 1u);
            if (NT) __builtin_nontemporal_store(v[j], out + p);
            else out[p] = v[j];
        }
    }
}

// staged: counting sort of the tile by bin in LDS, then stores in bin order
__global__ void __launch_bounds__(THREADS) k_scatter_staged(const uint64_t* a, uint64_t n, int lg,
                                                            int B, uint64_t chunk_tiles,
                                                            const uint32_t* off, uint64_t* out) {
    extern __shared__ uint32_t sm[];
    const uint32_t nb = 1u << B;
    uint32_t* cur = sm;             // nb: global cursor of the bin
    uint32_t* cnt = sm + nb;        // nb: tile count -> tile start
    uint64_t* stage = (uint64_t*)(sm + 2 * nb);  // TILE
    uint32_t* sbin = (uint32_t*)(stage + TILE);  // TILE: bin of each staged element
    __shared__ uint32_t wsum[THREADS / 64];
    for (uint32_t i = threadIdx.x; i < nb; i += THREADS) cur[i] = off[(size_t)i * gridDim.x + blockIdx.x];
    for (uint32_t k = 0; k < chunk_tiles; k++) {
        const uint64_t base = tile_base<false>(k, chunk_tiles);
        for (uint32_t i = threadIdx.x; i < nb; i += THREADS) cnt[i] = 0;
        __syncthreads();
        uint64_t v[ITEMS];
        uint32_t r[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint64_t i = base + j * THREADS + threadIdx.x;
            v[j] = i < n ? __builtin_nontemporal_load(a + i) : ~0ull;
            r[j] = v[j] == ~0ull ? 0 : atomicAdd(&cnt[bin_of(v[j], lg, B)], 1u);
        }
        __syncthreads();
        // exclusive scan of cnt (nb / THREADS bins per thread)
        const uint32_t per = nb / THREADS > 0 ? nb / THREADS : 1;
        uint32_t s = 0;
        if (threadIdx.x * per < nb)
            for (uint32_t q = 0; q < per; q++) s += cnt[threadIdx.x * per + q];
        uint32_t x = s;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if ((threadIdx.x & 63) >= (uint32_t)o) x += y;
        }
        if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = x;
        __syncthreads();
        uint32_t pre = x - s;
        for (uint32_t w = 0; w < (threadIdx.x >> 6); w++) pre += wsum[w];
        __syncthreads();
        if (threadIdx.x * per < nb)
            for (uint32_t q = 0; q < per; q++) {
                const uint32_t c = cnt[threadIdx.x * per + q];
                cnt[threadIdx.x * per + q] = pre;
                pre += c;
            }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            if (v[j] == ~0ull) continue;
            const uint32_t b = bin_of(v[j], lg, B);
            const uint32_t p = cnt[b] + r[j];
            stage[p] = v[j];
            sbin[p] = b;
        }
        __syncthreads();
        const uint32_t len = (uint32_t)min((uint64_t)TILE, n - base);
        for (uint32_t p = threadIdx.x; p < len; p += THREADS) {
            const uint32_t b = sbin[p];
            out[cur[b] + (p - cnt[b])] = stage[p];
        }
        __syncthreads();
        // advance the cursors by the tile's counts
        for (uint32_t b = threadIdx.x; b < nb; b += THREADS) {
            const uint32_t next = b + 1 < nb ? cnt[b + 1] : len;
            cur[b] += next - cnt[b];
        }
        __syncthreads();
    }
}

int main(int argc, char** argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 27;
    const uint64_t n = 1ull << lg;
    uint64_t *a, *o;
    uint32_t *hist, *off;
    CK(hipMalloc(&a, n * 8));
    CK(hipMalloc(&o, n * 8));
    const int GMAX = 1024, BMAX = 13;
    CK(hipMalloc(&hist, (size_t)GMAX << BMAX << 2));
    CK(hipMalloc(&off, (size_t)GMAX << BMAX << 2));
    hipLaunchKernelGGL(k_gen, dim3(4096), dim3(256), 0, 0, a, n, lg);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<uint32_t> h((size_t)GMAX << BMAX);
    std::vector<uint64_t> hout(n);
    const char* names[4] = {"direct", "direct-nt", "inter", "staged"};
    for (int B : {8, 10, 11, 12, 13}) {
        for (int G : {256, 1024}) {
            const uint64_t tiles = (n + TILE - 1) / TILE;
            const uint64_t ct = (tiles + G - 1) / G;
            const uint32_t nb = 1u << B;
            for (int mode = 0; mode < 4; mode++) {
                const bool inter = mode == 2;
                const size_t lds_h = (size_t)nb * 4;
                const size_t lds_st = (size_t)2 * nb * 4 + (size_t)TILE * 12;
                if (mode == 3 && lds_st + 64 > 160 * 1024) continue;
                if (inter)
                    hipLaunchKernelGGL(k_hist<true>, dim3(G), dim3(THREADS), lds_h, 0, a, n, lg, B, ct, hist);
                else
                    hipLaunchKernelGGL(k_hist<false>, dim3(G), dim3(THREADS), lds_h, 0, a, n, lg, B, ct, hist);
                CK(hipMemcpy(h.data(), hist, (size_t)G * nb * 4, hipMemcpyDeviceToHost));
                uint32_t s = 0;
                for (size_t i = 0; i < (size_t)G * nb; i++) {
                    const uint32_t c = h[i];
                    h[i] = s;
                    s += c;
                }
                CK(hipMemcpy(off, h.data(), (size_t)G * nb * 4, hipMemcpyHostToDevice));
                float best = 1e9;
                for (int rep = 0; rep < 4; rep++) {
                    CK(hipEventRecord(e0, 0));
                    if (mode == 0)
                        hipLaunchKernelGGL((k_scatter<false, false>), dim3(G), dim3(THREADS), lds_h, 0, a, n, lg, B, ct, off, o);
                    else if (mode == 1)
                        hipLaunchKernelGGL((k_scatter<false, true>), dim3(G), dim3(THREADS), lds_h, 0, a, n, lg, B, ct, off, o);
                    else if (mode == 2)
                        hipLaunchKernelGGL((k_scatter<true, false>), dim3(G), dim3(THREADS), lds_h, 0, a, n, lg, B, ct, off, o);
                    else
                        hipLaunchKernelGGL(k_scatter_staged, dim3(G), dim3(THREADS), lds_st, 0, a, n, lg, B, ct, off, o);
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    best = std::min(best, ms);
                }
                // check: a permutation of the input, grouped by bin
                CK(hipMemcpy(hout.data(), o, n * 8, hipMemcpyDeviceToHost));
                bool ok = true;
                uint64_t x = 0;
                for (uint64_t i = 0; i < n; i++) {
                    x ^= hout[i] * 0x9E3779B97F4A7C15ull + (hout[i] >> 17);
                    if (i && (uint32_t)(hout[i] >> 32) >> (lg - B) < (uint32_t)(hout[i - 1] >> 32) >> (lg - B)) ok = false;
                }
                static uint64_t want = 0;
                if (!want) want = x;
                ok = ok && x == want;
                printf("B=%2d G=%4d %-10s %.4f ms  %.2f TB/s  %s\n", B, G, names[mode], best,
                       2.0 * n * 8 / (best * 1e-3) / 1e12, ok ? "ok" : "WRONG");
                fflush(stdout);
            }
        }
    }
    return 0;
}
