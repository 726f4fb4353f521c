// bwprobe.hip -- HBM bandwidth ceilings on this MI355X for the access shapes
// the join kernels use (16 B per lane): copy, read-only, write-only, with and
// without non-temporal hints, and chunked copies (each workgroup a contiguous
// chunk, like the partition kernels).  Diagnostic tool, not part of the library.
//   hipcc -O3 --offload-arch=gfx950 tools/bwprobe.hip -o build/bwprobe
#include <hip/hip_runtime.h>
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

typedef unsigned int V __attribute__((ext_vector_type(4)));

template <int UNROLL, bool NT>
__global__ void __launch_bounds__(256) k_copy(const V* __restrict__ a, V* __restrict__ b, size_t n) {
    size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
        V v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; u++) v[u] = NT ? __builtin_nontemporal_load(&a[i + u * stride]) : a[i + u * stride];
#pragma unroll
        for (int u = 0; u < UNROLL; u++) {
            if (NT) __builtin_nontemporal_store(v[u], &b[i + u * stride]);
            else b[i + u * stride] = v[u];
        }
    }
    for (; i < n; i += stride) b[i] = a[i];
}

// each workgroup copies one contiguous chunk, tile by tile (partition shape)
template <int ITEMS>
__global__ void __launch_bounds__(512) k_copy_chunk(const V* __restrict__ a, V* __restrict__ b, size_t n, size_t chunk) {
    size_t beg = (size_t)blockIdx.x * chunk, end = beg + chunk;
    if (end > n) end = n;
    for (size_t base = beg; base < end; base += 512 * ITEMS) {
        V v[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            size_t i = base + j * 512 + threadIdx.x;
            if (i < end) v[j] = a[i];
        }
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            size_t i = base + j * 512 + threadIdx.x;
            if (i < end) b[i] = v[j];
        }
    }
}

template <int UNROLL>
__global__ void __launch_bounds__(256) k_read(const V* __restrict__ a, size_t n, unsigned* out) {
    size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned acc = 0;
    for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
        V v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; u++) v[u] = a[i + u * stride];
#pragma unroll
        for (int u = 0; u < UNROLL; u++) acc ^= v[u].x ^ v[u].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void __launch_bounds__(256) k_write(V* __restrict__ b, size_t n) {
    size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        b[i] = V{(unsigned)i, 1u, 2u, 3u};
}

template <class F>
static float timeit(F f, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++) f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main(int argc, char** argv) {
    size_t bytes = argc > 1 ? strtoull(argv[1], 0, 10) : (size_t)2048000000;
    size_t n = bytes / sizeof(V);
    V *a, *b;
    unsigned* o;
    CK(hipMalloc(&a, n * sizeof(V)));
    CK(hipMalloc(&b, n * sizeof(V)));
    CK(hipMalloc(&o, 64));
    CK(hipMemset(a, 1, n * sizeof(V)));
    CK(hipMemset(b, 2, n * sizeof(V)));
    const int reps = 10;
    double gb = (double)n * sizeof(V) / 1e9;
    for (int g : {1024, 2048, 4096, 8192}) {
        float t = timeit([&] { hipLaunchKernelGGL((k_copy<4, false>), dim3(g), dim3(256), 0, 0, a, b, n); }, reps);
        printf("{\"probe\": \"copy_u4\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", g, t, 2 * gb * 1e3 / t);
        t = timeit([&] { hipLaunchKernelGGL((k_copy<4, true>), dim3(g), dim3(256), 0, 0, a, b, n); }, reps);
        printf("{\"probe\": \"copy_u4_nt\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", g, t, 2 * gb * 1e3 / t);
        t = timeit([&] { hipLaunchKernelGGL((k_read<8>), dim3(g), dim3(256), 0, 0, a, n, o); }, reps);
        printf("{\"probe\": \"read_u8\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", g, t, gb * 1e3 / t);
        t = timeit([&] { hipLaunchKernelGGL(k_write, dim3(g), dim3(256), 0, 0, b, n); }, reps);
        printf("{\"probe\": \"write\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", g, t, gb * 1e3 / t);
    }
    for (int wg : {512, 1024, 2048, 4096}) {
        size_t chunk = (n + wg - 1) / wg;
        chunk = (chunk + 8191) / 8192 * 8192;
        int g = (int)((n + chunk - 1) / chunk);
        float t = timeit([&] { hipLaunchKernelGGL((k_copy_chunk<16>), dim3(g), dim3(512), 0, 0, a, b, n, chunk); }, reps);
        printf("{\"probe\": \"copy_chunk16\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", g, t, 2 * gb * 1e3 / t);
    }
    float t = timeit([&] { CK(hipMemcpyAsync(b, a, n * sizeof(V), hipMemcpyDeviceToDevice, 0)); }, reps);
    printf("{\"probe\": \"hipMemcpyD2D\", \"ms\": %.4f, \"GBps\": %.1f}\n", t, 2 * gb * 1e3 / t);
    return 0;
}
