// planelab.hip -- lab probe (not part of the library): what do 48-bit
// elements stored as two planes (uint32 lo + uint16 hi) buy over 64-bit words
// in the tile pass's access shape?  Each workgroup reads one 8192-element tile
// and writes it back (a copy through registers, as k_tilepass does around its
// LDS grouping), 2^27 elements:
//   w64      : 16 items of 8-byte words per thread (k_tilepass today)
//   p48      : 16 items, lo 4-byte + hi 2-byte loads/stores per item
//   p48pair  : 8 pairs per thread, lo 8-byte + hi 4-byte accesses (2 items)
//   hipcc -O3 --offload-arch=gfx950 tools/planelab.hip -o build_lab/planelab
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

constexpr int T = 512, I = 16, TILE = T * I;

__global__ void __launch_bounds__(T) k_w64(const uint64_t* a, uint64_t* b) {
    const uint64_t off = (uint64_t)blockIdx.x * TILE;
    uint64_t v[I];
#pragma unroll
    for (int j = 0; j < I; j++) v[j] = a[off + j * T + threadIdx.x];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < I; j++) __builtin_nontemporal_store(v[j] ^ 1, b + off + j * T + threadIdx.x);
}

__global__ void __launch_bounds__(T) k_p48(const uint32_t* alo, const uint16_t* ahi, uint32_t* blo,
                                           uint16_t* bhi) {
    const uint64_t off = (uint64_t)blockIdx.x * TILE;
    uint64_t v[I];
#pragma unroll
    for (int j = 0; j < I; j++) {
        const uint64_t i = off + j * T + threadIdx.x;
        v[j] = (uint64_t)alo[i] | ((uint64_t)ahi[i] << 32);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < I; j++) {
        const uint64_t i = off + j * T + threadIdx.x;
        __builtin_nontemporal_store((uint32_t)(v[j] ^ 1), blo + i);
        __builtin_nontemporal_store((uint16_t)(v[j] >> 32), bhi + i);
    }
}

__global__ void __launch_bounds__(T) k_p48pair(const uint32_t* alo, const uint16_t* ahi,
                                               uint32_t* blo, uint16_t* bhi) {
    const uint64_t off = (uint64_t)blockIdx.x * TILE;
    uint64_t v[I];
    typedef uint32_t U2 __attribute__((ext_vector_type(2)));
    typedef uint16_t H2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int p = 0; p < I / 2; p++) {
        const uint64_t i = off + 2 * ((uint64_t)p * T + threadIdx.x);
        const U2 lo = *reinterpret_cast<const U2*>(alo + i);
        const H2 hi = *reinterpret_cast<const H2*>(ahi + i);
        v[2 * p] = (uint64_t)lo.x | ((uint64_t)hi.x << 32);
        v[2 * p + 1] = (uint64_t)lo.y | ((uint64_t)hi.y << 32);
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < I / 2; p++) {
        const uint64_t i = off + 2 * ((uint64_t)p * T + threadIdx.x);
        U2 lo = {(uint32_t)(v[2 * p] ^ 1), (uint32_t)(v[2 * p + 1] ^ 1)};
        H2 hi = {(uint16_t)(v[2 * p] >> 32), (uint16_t)(v[2 * p + 1] >> 32)};
        __builtin_nontemporal_store(lo, reinterpret_cast<U2*>(blo + i));
        __builtin_nontemporal_store(hi, reinterpret_cast<H2*>(bhi + i));
    }
}

int main() {
    const uint64_t n = 1ull << 27;
    const uint32_t g = n / TILE;
    uint64_t *a, *b;
    CK(hipMalloc(&a, n * 8));
    CK(hipMalloc(&b, n * 8));
    CK(hipMemset(a, 1, n * 8));
    uint32_t* alo = (uint32_t*)a;
    uint16_t* ahi = (uint16_t*)(alo + n);
    uint32_t* blo = (uint32_t*)b;
    uint16_t* bhi = (uint16_t*)(blo + n);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* nm[3] = {"w64", "p48", "p48pair"};
    for (int rep = 0; rep < 3; rep++)
        for (int m = 0; m < 3; m++) {
            float best = 1e9;
            for (int k = 0; k < 5; k++) {
                CK(hipEventRecord(e0, 0));
                if (m == 0) hipLaunchKernelGGL(k_w64, dim3(g), dim3(T), 0, 0, a, b);
                if (m == 1) hipLaunchKernelGGL(k_p48, dim3(g), dim3(T), 0, 0, alo, ahi, blo, bhi);
                if (m == 2) hipLaunchKernelGGL(k_p48pair, dim3(g), dim3(T), 0, 0, alo, ahi, blo, bhi);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
            }
            const double bytes = 2.0 * n * (m == 0 ? 8 : 6);
            printf("rep %d %-8s %.4f ms  %.2f TB/s (its bytes)  %.2f TB/s (as 8-byte words)\n", rep,
                   nm[m], best, bytes / (best * 1e-3) / 1e12, 2.0 * n * 8 / (best * 1e-3) / 1e12);
            fflush(stdout);
        }
    return 0;
}
