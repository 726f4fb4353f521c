// ldsorder.hip -- does ds_add_rtn_u32 return lane-ordered values when several
// lanes of one wave instruction hit the same LDS address?  Counts violations
// against the ballot-matched expectation.  Development probe, not product.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void __launch_bounds__(1024) k_order(uint32_t K, uint32_t iters, unsigned long long* bad,
                                                unsigned long long* total) {
    __shared__ uint32_t ctr[16][1024];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int i = lane; i < 1024; i += 64) ctr[wid][i] = 0;
    __syncthreads();
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    unsigned long long nb = 0, nt = 0;
    uint32_t h = blockIdx.x * 7919u + threadIdx.x * 104729u;
    for (uint32_t it = 0; it < iters; it++) {
        h = h * 1664525u + 1013904223u;
        const uint32_t d = (h >> 8) % K;
        uint64_t peers = ~0ull;
        for (int b = 0; b < 10; b++) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bal = __ballot(bit);
            peers &= bit ? bal : ~bal;
        }
        const uint32_t snap = ctr[wid][d];
        __builtin_amdgcn_wave_barrier();
        const uint32_t old = atomicAdd(&ctr[wid][d], 1u);
        __builtin_amdgcn_wave_barrier();
        const uint32_t want = snap + (uint32_t)__popcll(peers & lt);
        nb += old != want;
        nt += __popcll(peers) > 1;
    }
    atomicAdd(bad, nb);
    atomicAdd(total, nt);
}

int main() {
    unsigned long long *bad, *tot;
    hipMalloc(&bad, 8);
    hipMalloc(&tot, 8);
    const uint32_t Ks[] = {1, 2, 3, 4, 16, 64, 256, 1024};
    for (uint32_t K : Ks) {
        hipMemset(bad, 0, 8);
        hipMemset(tot, 0, 8);
        hipLaunchKernelGGL(k_order, dim3(2048), dim3(1024), 0, 0, K, 2000u, bad, tot);
        unsigned long long hb, ht;
        hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
        hipMemcpy(&ht, tot, 8, hipMemcpyDeviceToHost);
        printf("K %4u: %llu out-of-lane-order returns, %llu lane-updates with a peer\n", K, hb, ht);
    }
    return 0;
}
