// datagen.hip -- deterministic synthetic relations generated in HBM.
//
// The reference generates R and S on the host (src/datagen/generator.c:254-350:
// keys 1..N, payload 5+i, then a Knuth shuffle seeded from time(NULL);
// genzipf.c:97-159: Zipf via an alphabet permutation and a CDF lookup table).
// For 128M..1024M-tuple relations that is seconds-to-minutes of host work plus
// a PCIe copy, and the time seed makes runs irreproducible.  Here the shuffle
// is a keyed bijection (4-round Feistel network + cycle walking) evaluated per
// index, so any shard [first, first+n) of a relation is produced
// independently on its own GPU and the primary-key property holds exactly
// (every key 1..total appears once).  Zipf samples use rejection-inversion
// (Hörmann & Derflinger), which draws exactly from the Zipf(theta) law on
// 1..maxid without an 8 GB CDF table; hot ranks are spread over the key
// domain by the same kind of bijection the reference's alphabet provides.
#include <math.h>

#include "smj_common.hpp"
#include "smj_internal.hpp"

namespace smj {

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct Perm {
    uint64_t total;
    uint32_t half;  // bits per Feistel half
    uint64_t key[4];
    __host__ __device__ uint64_t feistel(uint64_t x) const {
        const uint64_t m = (1ull << half) - 1;
        uint64_t l = x >> half, r = x & m;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            uint64_t f = mix64(r ^ key[i]) & m;
            uint64_t nl = r;
            r = l ^ f;
            l = nl;
        }
        return (l << half) | r;
    }
    __host__ __device__ uint64_t operator()(uint64_t x) const {
        uint64_t y = feistel(x);
        while (y >= total) y = feistel(y);  // cycle walking
        return y;
    }
};

static Perm make_perm(uint64_t total, uint64_t seed) {
    Perm p;
    p.total = total ? total : 1;
    uint32_t bits = 2;
    while (bits < 64 && (1ull << bits) < p.total) bits++;
    if (bits & 1) bits++;
    p.half = bits / 2;
    for (int i = 0; i < 4; i++) p.key[i] = mix64(seed * 4 + i + 0x5151);
    return p;
}

__global__ void k_gen_perm(Tup* __restrict__ out, uint64_t n, uint64_t first,
                           Perm perm, uint64_t maxid, int payload_mode) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += stride) {
        const uint64_t g = first + i;
        const int64_t key = (int64_t)(perm(g) % maxid) + 1;
        const int64_t pay = payload_mode ? (int64_t)(5 + g) : 0;
#ifdef KEY_8B
        Tup t;
        t.key = key;
        t.payload = pay;
#else
        Tup t = ((uint64_t)(uint32_t)(int32_t)key << 32) |
                (uint64_t)(uint32_t)(int32_t)pay;
#endif
        out[i] = t;
    }
}

// ---- Zipf by rejection-inversion --------------------------------------
struct ZipfParams {
    double s, hX1, hN, sStar;
    uint64_t N;
};

__host__ __device__ inline double zh1(double x) {  // log1p(x)/x
    return fabs(x) > 1e-8 ? log1p(x) / x : 1.0 - x * (0.5 - x * (1.0 / 3.0 - 0.25 * x));
}
__host__ __device__ inline double zh2(double x) {  // expm1(x)/x
    return fabs(x) > 1e-8 ? expm1(x) / x : 1.0 + x * 0.5 * (1.0 + x * (1.0 / 3.0) * (1.0 + 0.25 * x));
}
__host__ __device__ inline double zH(double s, double x) {
    const double lx = log(x);
    return zh2((1.0 - s) * lx) * lx;
}
__host__ __device__ inline double zhh(double s, double x) { return exp(-s * log(x)); }
__host__ __device__ inline double zHinv(double s, double x) {
    double t = x * (1.0 - s);
    if (t < -1.0) t = -1.0;
    return exp(zh1(t) * x);
}

static ZipfParams make_zipf(uint64_t N, double s) {
    ZipfParams z;
    z.s = s;
    z.N = N;
    z.hX1 = zH(s, 1.5) - 1.0;
    z.hN = zH(s, (double)N + 0.5);
    z.sStar = 2.0 - zHinv(s, zH(s, 2.5) - zhh(s, 2.0));
    return z;
}

__device__ inline double u01(uint64_t a, uint64_t b) {
    return (double)(mix64(a ^ mix64(b)) >> 11) * (1.0 / 9007199254740992.0);
}

__global__ void k_gen_zipf(Tup* __restrict__ out, uint64_t n, uint64_t first,
                           ZipfParams z, Perm alpha, uint64_t seed) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += stride) {
        const uint64_t g = first + i;
        uint64_t k = 1;
        for (uint32_t att = 0; att < 1000; att++) {
            const double u = z.hN + u01(seed * 0x100000001B3ull + att, g) * (z.hX1 - z.hN);
            const double x = zHinv(z.s, u);
            double kd = floor(x + 0.5);
            if (kd < 1.0) kd = 1.0;
            if (kd > (double)z.N) kd = (double)z.N;
            k = (uint64_t)kd;
            if (kd - x <= z.sStar || u >= zH(z.s, kd + 0.5) - zhh(z.s, kd)) break;
        }
        // rank k (1 = most frequent) -> key through the alphabet permutation
        const int64_t key = (int64_t)alpha(k - 1) + 1;
#ifdef KEY_8B
        Tup t;
        t.key = key;
        t.payload = 0;
#else
        Tup t = ((uint64_t)(uint32_t)(int32_t)key << 32);
#endif
        out[i] = t;
    }
}

static uint32_t grid_for(uint64_t n) {
    uint64_t b = (n + 255) / 256;
    return (uint32_t)(b < 8192 ? (b ? b : 1) : 8192);
}

void gen_pk(Tup* out, uint64_t n, uint64_t first, uint64_t total,
            uint64_t seed, hipStream_t st) {
    if (n == 0) return;
    Perm p = make_perm(total, seed);
    hipLaunchKernelGGL(k_gen_perm, dim3(grid_for(n)), dim3(256), 0, st, out, n,
                       first, p, total ? total : 1, 1);
    SMJ_CHECK(hipGetLastError());
}

void gen_fk(Tup* out, uint64_t n, uint64_t first, uint64_t total,
            uint64_t maxid, uint64_t seed, hipStream_t st) {
    if (n == 0) return;
    Perm p = make_perm(total, seed);
    hipLaunchKernelGGL(k_gen_perm, dim3(grid_for(n)), dim3(256), 0, st, out, n,
                       first, p, maxid ? maxid : 1, 1);
    SMJ_CHECK(hipGetLastError());
}

void gen_zipf(Workspace* ws, Tup* out, uint64_t n, uint64_t first,
              uint64_t maxid, double theta, uint64_t seed, hipStream_t st) {
    (void)ws;
    if (n == 0) return;
    ZipfParams z = make_zipf(maxid ? maxid : 1, theta);
    Perm alpha = make_perm(maxid ? maxid : 1, seed ^ 0xA1FA);
    hipLaunchKernelGGL(k_gen_zipf, dim3(grid_for(n)), dim3(256), 0, st, out, n,
                       first, z, alpha, seed);
    SMJ_CHECK(hipGetLastError());
}

// keys 1..total permuted, payload 0 (create_relation_pk leaves it unset)
void gen_pk_nopayload(Tup* out, uint64_t n, uint64_t first, uint64_t total,
                      uint64_t seed, hipStream_t st) {
    if (n == 0) return;
    Perm p = make_perm(total, seed);
    hipLaunchKernelGGL(k_gen_perm, dim3(grid_for(n)), dim3(256), 0, st, out, n,
                       first, p, total ? total : 1, 0);
    SMJ_CHECK(hipGetLastError());
}

}  // namespace smj
