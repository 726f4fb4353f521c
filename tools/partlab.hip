// partlab.hip -- experiments for the stable reference-API partitioner
// (partition_relation_optimized, BASELINE config 3: 2^27 tuples, 10 bits).
// Standalone: hipcc -O3 --offload-arch=gfx950 [-DKEY_8B] tools/partlab.hip
// Every variant is checked against a host stable partition; times are HIP
// events over the reps.  Development tool, not part of the library.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>
#include <vector>

#include "../avx-sort-merge-joins_amd/csrc/smj_common.hpp"
#include "../avx-sort-merge-joins_amd/csrc/smj_internal.hpp"

using namespace smj;

static uint32_t host_digit(const Tup& t, uint32_t mask, uint32_t shift) {
    return (uint32_t)(((uint64_t)(tup_key(t) - 1) & (uint64_t)mask) >> shift);
}

// ------------------------------------------------------------------ histogram
template <int THREADS, int ITEMS>
__global__ void __launch_bounds__(THREADS)
k_hist_l(const Tup* __restrict__ in, uint64_t n, uint64_t chunk, RefDigit dig,
         uint32_t nbins, uint32_t* __restrict__ counts, uint32_t nwg) {
    extern __shared__ uint32_t lh[];
    for (uint32_t d = threadIdx.x; d < nbins; d += THREADS) lh[d] = 0;
    __syncthreads();
    const uint64_t beg = (uint64_t)blockIdx.x * chunk;
    const uint64_t end = min(beg + chunk, n);
    constexpr int TILE = THREADS * ITEMS;
    for (uint64_t base = beg; base < end; base += TILE) {
        Tup v[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint64_t i = base + (uint64_t)j * THREADS + threadIdx.x;
            v[j] = in[i < end ? i : end - 1];
        }
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint64_t i = base + (uint64_t)j * THREADS + threadIdx.x;
            if (i < end) atomicAdd(&lh[dig(v[j])], 1u);
        }
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < nbins; d += THREADS)
        counts[(uint64_t)d * nwg + blockIdx.x] = lh[d];
}

__global__ void __launch_bounds__(256)
k_scanrow_l(uint32_t* __restrict__ counts, uint32_t nwg, uint64_t* __restrict__ totals) {
    __shared__ uint32_t scratch[8];
    uint32_t* row = counts + (uint64_t)blockIdx.x * nwg;
    const uint32_t per = (nwg + 255) / 256;
    const uint32_t b = threadIdx.x * per;
    uint32_t loc = 0;
    for (uint32_t k = 0; k < per; k++)
        if (b + k < nwg) loc += row[b + k];
    uint32_t tot;
    uint32_t ex = block_exclusive_scan(loc, scratch, &tot);
    for (uint32_t k = 0; k < per; k++) {
        if (b + k < nwg) {
            uint32_t c = row[b + k];
            row[b + k] = ex;
            ex += c;
        }
    }
    if (threadIdx.x == 0) totals[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(256)
k_scandig_l(const uint64_t* __restrict__ totals, uint32_t nbins, uint64_t* __restrict__ starts) {
    __shared__ uint64_t sh[256];
    const uint32_t per = (nbins + 255) / 256;
    const uint32_t b = threadIdx.x * per;
    uint64_t loc = 0;
    for (uint32_t k = 0; k < per; k++)
        if (b + k < nbins) loc += align_tuples(totals[b + k]);
    sh[threadIdx.x] = loc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t run = 0;
        for (int t = 0; t < 256; t++) {
            uint64_t x = sh[t];
            sh[t] = run;
            run += x;
        }
    }
    __syncthreads();
    uint64_t ex = sh[threadIdx.x];
    for (uint32_t k = 0; k < per; k++) {
        uint32_t d = b + k;
        if (d < nbins) {
            starts[d] = ex;
            ex += align_tuples(totals[d]);
        }
    }
}

// ------------------------------------------------------------- stable scatter
// RANK 0: ballot matching over the digit bits (one ballot per bit).
// RANK 1: per-wave LDS table of 64-bit lane masks indexed by the low
//         HB bits of the digit (atomic OR, read back, cleared), the other
//         digit bits matched by ballots.
// The tile is staged in LDS in digit order and written with consecutive
// lanes on consecutive addresses of one partition (no carry).
template <int THREADS, int ITEMS, int RANK, int HB>
struct SsGeom {
    static constexpr int W = THREADS / 64;
    static constexpr int TILE = THREADS * ITEMS;
    // stage | wcnt u16 [B][W] | run u64 [B] | tstart u32 [B] | table u64 [W][2^HB] | scr
    static size_t lds(uint32_t B) {
        return (size_t)TILE * sizeof(Tup) + (size_t)B * W * 2 + (size_t)B * 8 + (size_t)B * 4 +
               (RANK == 1 ? (size_t)W * (1u << HB) * 8 : 0) + 128;
    }
};

template <int THREADS, int ITEMS, int RANK, int HB>
__global__ void __launch_bounds__(THREADS)
k_sscatter(const Tup* __restrict__ in, uint64_t n, uint64_t chunk, RefDigit dig,
           uint32_t nbins, uint32_t dbits, const uint32_t* __restrict__ counts, uint32_t nwg,
           const uint64_t* __restrict__ starts, Tup* __restrict__ out) {
    typedef SsGeom<THREADS, ITEMS, RANK, HB> G;
    constexpr int W = G::W;
    constexpr int TILE = G::TILE;
    extern __shared__ __attribute__((aligned(16))) unsigned char lraw[];
    Tup* stage = reinterpret_cast<Tup*>(lraw);
    uint16_t* wcnt = reinterpret_cast<uint16_t*>(stage + TILE);
    uint64_t* run = reinterpret_cast<uint64_t*>(wcnt + (size_t)nbins * W);
    uint32_t* tstart = reinterpret_cast<uint32_t*>(run + nbins);
    uint64_t* table = reinterpret_cast<uint64_t*>(tstart + nbins);
    uint32_t* scr = reinterpret_cast<uint32_t*>(table + (RANK == 1 ? W * (1u << HB) : 0));

    const int lane = lane_id();
    const int wid = threadIdx.x >> 6;
    const uint64_t lt = lanemask_lt();
    uint64_t* mytab = table + (size_t)wid * (1u << HB);
    for (uint32_t d = threadIdx.x; d < nbins; d += THREADS) {
        run[d] = starts[d] + counts[(uint64_t)d * nwg + blockIdx.x];
#pragma unroll
        for (int w = 0; w < W; w++) wcnt[d * W + w] = 0;
    }
    if (RANK == 1)
        for (uint32_t q = lane; q < (1u << HB); q += 64) mytab[q] = 0;
    const uint64_t beg = (uint64_t)blockIdx.x * chunk;
    const uint64_t end = min(beg + chunk, n);
    const uint32_t wbase = wid * 64 * ITEMS;
    constexpr int DPT = 4;  // digits per thread (nbins <= DPT * THREADS)
    Tup v[ITEMS], nv[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        const uint64_t i = beg + wbase + j * 64 + lane;
        if (i < end) v[j] = in[i];
    }
    __syncthreads();
    for (uint64_t base = beg; base < end; base += TILE) {
        const uint32_t tcount = (uint32_t)min((uint64_t)TILE, end - base);
        uint32_t dg[ITEMS], rk[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint32_t li = wbase + j * 64 + lane;
            const bool valid = li < tcount;
            dg[j] = valid ? dig(v[j]) : 0xffffffffu;
            const uint32_t d = valid ? dg[j] : 0;
            uint64_t peers;
            if (RANK == 0) {
                peers = __ballot(valid);
                for (uint32_t b = 0; b < dbits; b++) {
                    const bool bit = (d >> b) & 1u;
                    const uint64_t bal = __ballot(bit);
                    peers &= bit ? bal : ~bal;
                }
            } else {
                const uint32_t slot = d & ((1u << HB) - 1);
                if (valid) atomicOr((unsigned long long*)&mytab[slot], 1ull << lane);
                peers = valid ? mytab[slot] : 0ull;
                for (uint32_t b = HB; b < dbits; b++) {
                    const bool bit = (d >> b) & 1u;
                    const uint64_t bal = __ballot(bit);
                    peers &= bit ? bal : ~bal;
                }
                if (valid) mytab[slot] = 0ull;
            }
            uint32_t before = 0;
            if (valid) before = wcnt[d * W + wid];
            const uint32_t r = (uint32_t)__popcll(peers & lt);
            if (valid && r == 0) wcnt[d * W + wid] = (uint16_t)(before + __popcll(peers));
            rk[j] = before + r;
        }
        __syncthreads();
        // per digit: count over waves, tile exclusive scan, per-wave prefixes
        uint32_t c[DPT];
        uint32_t loc = 0;
#pragma unroll
        for (int k = 0; k < DPT; k++) {
            const uint32_t d = threadIdx.x * DPT + k;
            c[k] = 0;
            if (d < nbins) {
#pragma unroll
                for (int w = 0; w < W; w++) c[k] += wcnt[d * W + w];
            }
            loc += c[k];
        }
        uint32_t tot;
        uint32_t ex = block_exclusive_scan(loc, scr, &tot);
#pragma unroll
        for (int k = 0; k < DPT; k++) {
            const uint32_t d = threadIdx.x * DPT + k;
            if (d < nbins) {
                tstart[d] = ex;
                uint32_t o = ex;
#pragma unroll
                for (int w = 0; w < W; w++) {
                    const uint32_t x = wcnt[d * W + w];
                    wcnt[d * W + w] = (uint16_t)o;
                    o += x;
                }
                ex += c[k];
            }
        }
        // prefetch the next tile
        const uint64_t nb = base + TILE;
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint64_t i = nb + wbase + j * 64 + lane;
            if (i < end) nv[j] = in[i];
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < ITEMS; j++)
            if (dg[j] != 0xffffffffu) stage[wcnt[dg[j] * W + wid] + rk[j]] = v[j];
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < tcount; i += THREADS) {
            const Tup t = stage[i];
            const uint32_t d = dig(t);
            st_stream(out + run[d] + (i - tstart[d]), t);
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < DPT; k++) {
            const uint32_t d = threadIdx.x * DPT + k;
            if (d < nbins) {
                run[d] += c[k];
#pragma unroll
                for (int w = 0; w < W; w++) wcnt[d * W + w] = 0;
            }
        }
#pragma unroll
        for (int j = 0; j < ITEMS; j++) v[j] = nv[j];
        __syncthreads();
    }
}

// plain copy for the bandwidth reference
__global__ void k_copy(const Tup* __restrict__ in, Tup* __restrict__ out, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        st_stream(out + i, in[i]);
}

// ------------------------------------------------------------------- harness
struct Ctx {
    uint64_t n;
    uint32_t bits, shift, nbins;
    Tup* din;
    Tup* dout;
    std::vector<Tup> hin, want;
    std::vector<uint64_t> woff, wcnt;
    size_t cap;
};

static void check(Ctx& c, const char* name) {
    std::vector<Tup> got(c.cap);
    SMJ_CHECK(hipMemcpy(got.data(), c.dout, c.cap * sizeof(Tup), hipMemcpyDeviceToHost));
    uint64_t bad = 0;
    for (uint32_t d = 0; d < c.nbins; d++)
        for (uint64_t k = 0; k < c.wcnt[d]; k++) {
            const uint64_t p = c.woff[d] + k;
            if (!tup_eq(got[p], c.want[p])) {
                if (bad < 3) fprintf(stderr, "  %s mismatch digit %u elem %llu\n", name, d,
                                     (unsigned long long)k);
                bad++;
            }
        }
    printf("  check %s: %s (%llu bad)\n", name, bad ? "FAIL" : "ok", (unsigned long long)bad);
}

template <int HT, int HI, int THREADS, int ITEMS, int RANK, int HB>
static void run_variant(Ctx& c, uint32_t wg_per_cu, int reps, const char* label) {
    typedef SsGeom<THREADS, ITEMS, RANK, HB> G;
    const uint64_t TILE = G::TILE;
    uint64_t ntiles = (c.n + TILE - 1) / TILE;
    uint32_t nwg = (uint32_t)std::min<uint64_t>(ntiles, 256ull * wg_per_cu);
    const uint64_t tpw = (ntiles + nwg - 1) / nwg;
    const uint64_t chunk = tpw * TILE;
    nwg = (uint32_t)((ntiles + tpw - 1) / tpw);
    uint32_t* counts;
    uint64_t *totals, *starts;
    SMJ_CHECK(hipMalloc(&counts, (size_t)c.nbins * nwg * 4));
    SMJ_CHECK(hipMalloc(&totals, c.nbins * 8));
    SMJ_CHECK(hipMalloc(&starts, c.nbins * 8));
    const size_t lds = G::lds(c.nbins);
    if (lds > 160 * 1024) {
        printf("%s: LDS %zu too big\n", label, lds);
        return;
    }
    SMJ_CHECK(hipFuncSetAttribute((const void*)k_sscatter<THREADS, ITEMS, RANK, HB>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    const uint32_t mask = (uint32_t)(((1ull << c.bits) - 1) << c.shift);
    RefDigit dig{mask, c.shift};
    hipEvent_t e[4];
    for (auto& x : e) SMJ_CHECK(hipEventCreate(&x));
    float th = 0, ts = 0, tc = 0;
    SMJ_CHECK(hipMemset(c.dout, 0, c.cap * sizeof(Tup)));
    for (int r = -1; r < reps; r++) {
        SMJ_CHECK(hipEventRecord(e[0]));
        hipLaunchKernelGGL((k_hist_l<HT, HI>), dim3(nwg), dim3(HT), c.nbins * 4, 0, c.din, c.n,
                           chunk, dig, c.nbins, counts, nwg);
        SMJ_CHECK(hipEventRecord(e[1]));
        hipLaunchKernelGGL(k_scanrow_l, dim3(c.nbins), dim3(256), 0, 0, counts, nwg, totals);
        hipLaunchKernelGGL(k_scandig_l, dim3(1), dim3(256), 0, 0, totals, c.nbins, starts);
        SMJ_CHECK(hipEventRecord(e[2]));
        hipLaunchKernelGGL((k_sscatter<THREADS, ITEMS, RANK, HB>), dim3(nwg), dim3(THREADS), lds,
                           0, c.din, c.n, chunk, dig, c.nbins, c.bits, counts, nwg, starts,
                           c.dout);
        SMJ_CHECK(hipEventRecord(e[3]));
        SMJ_CHECK(hipEventSynchronize(e[3]));
        SMJ_CHECK(hipGetLastError());
        if (r >= 0) {
            float a, b, d;
            SMJ_CHECK(hipEventElapsedTime(&a, e[0], e[1]));
            SMJ_CHECK(hipEventElapsedTime(&b, e[1], e[2]));
            SMJ_CHECK(hipEventElapsedTime(&d, e[2], e[3]));
            th += a;
            tc += b;
            ts += d;
        }
    }
    const double alg = 2.0 * c.n * sizeof(Tup);
    const double tot = (th + tc + ts) / reps;
    printf("%-40s nwg %4u lds %6zu  hist %.3f scan %.3f scatter %.3f total %.3f ms  frac %.3f\n",
           label, nwg, lds, th / reps, tc / reps, ts / reps, tot, alg / (tot * 1e-3) / 8e12);
    check(c, label);
    SMJ_CHECK(hipFree(counts));
    SMJ_CHECK(hipFree(totals));
    SMJ_CHECK(hipFree(starts));
}

int main(int argc, char** argv) {
    Ctx c;
    c.n = argc > 1 ? strtoull(argv[1], 0, 10) : (1ull << 27);
    c.bits = argc > 2 ? atoi(argv[2]) : 10;
    c.shift = argc > 3 ? atoi(argv[3]) : 0;
    const std::string only = argc > 4 ? argv[4] : "";
    c.nbins = 1u << c.bits;
    c.cap = c.n + c.nbins * 64 / sizeof(Tup);
    c.hin.resize(c.n);
    const uint64_t M = 1ull << 40;
    for (uint64_t i = 0; i < c.n; i++) {
        const uint64_t k = (i * 0x9E3779B97F4A7C15ull >> 13) % c.n + 1;  // keys ~uniform
#ifdef KEY_8B
        c.hin[i].payload = (int64_t)i;
        c.hin[i].key = (int64_t)k;
#else
        c.hin[i] = ((uint64_t)(uint32_t)k << 32) | (uint32_t)i;
#endif
    }
    (void)M;
    // host stable partition
    const uint32_t mask = (uint32_t)(((1ull << c.bits) - 1) << c.shift);
    c.wcnt.assign(c.nbins, 0);
    for (auto& t : c.hin) c.wcnt[host_digit(t, mask, c.shift)]++;
    c.woff.resize(c.nbins);
    uint64_t o = 0;
    std::vector<uint64_t> dst(c.nbins);
    for (uint32_t d = 0; d < c.nbins; d++) {
        c.woff[d] = dst[d] = o;
        o += align_tuples(c.wcnt[d]);
    }
    c.want.assign(c.cap, Tup());
    for (auto& t : c.hin) c.want[dst[host_digit(t, mask, c.shift)]++] = t;
    SMJ_CHECK(hipMalloc(&c.din, c.n * sizeof(Tup)));
    SMJ_CHECK(hipMalloc(&c.dout, c.cap * sizeof(Tup)));
    SMJ_CHECK(hipMemcpy(c.din, c.hin.data(), c.n * sizeof(Tup), hipMemcpyHostToDevice));
    {
        hipEvent_t a, b;
        SMJ_CHECK(hipEventCreate(&a));
        SMJ_CHECK(hipEventCreate(&b));
        float t = 0;
        for (int r = -1; r < 10; r++) {
            SMJ_CHECK(hipEventRecord(a));
            hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, 0, c.din, c.dout, c.n);
            SMJ_CHECK(hipEventRecord(b));
            SMJ_CHECK(hipEventSynchronize(b));
            float x;
            SMJ_CHECK(hipEventElapsedTime(&x, a, b));
            if (r >= 0) t += x;
        }
        printf("copy %.3f ms (%.0f GB/s of read+write)\n", t / 10,
               2.0 * c.n * sizeof(Tup) / (t / 10 * 1e-3) / 1e9);
    }
    const int reps = 10;
#define V(HT, HI, T, I, R, HB, W, name)                                  \
    if (only.empty() || only == name) run_variant<HT, HI, T, I, R, HB>(c, W, reps, name);
    V(512, 16, 512, 8, 0, 8, 1, "ballot 512x8 1/CU");
    V(512, 16, 512, 8, 0, 8, 2, "ballot 512x8 2/CU");
    V(512, 16, 512, 16, 0, 8, 1, "ballot 512x16 1/CU");
    V(512, 16, 1024, 8, 0, 8, 1, "ballot 1024x8 1/CU");
    V(512, 16, 512, 8, 1, 8, 2, "table8 512x8 2/CU");
    V(512, 16, 512, 8, 1, 6, 2, "table6 512x8 2/CU");
    V(512, 16, 1024, 8, 1, 6, 1, "table6 1024x8 1/CU");
    V(256, 16, 256, 8, 0, 8, 4, "ballot 256x8 4/CU");
    V(256, 16, 256, 16, 0, 8, 2, "ballot 256x16 2/CU");
    return 0;
}
