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

template <int THREADS, int ITEMS, int RANK, int HB, int ST>
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
        if (i < end) v[j] = ST == 2 ? ld_nt(in + i) : in[i];
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
            if (i < end) nv[j] = ST == 2 ? ld_nt(in + i) : in[i];
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < ITEMS; j++)
            if (dg[j] != 0xffffffffu) stage[wcnt[dg[j] * W + wid] + rk[j]] = v[j];
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < tcount; i += THREADS) {
            const Tup t = stage[i];
            const uint32_t d = dig(t);
            if (ST == 0) st_stream(out + run[d] + (i - tstart[d]), t);
            else if (ST == 3) out[base + i] = t;               // ablation: linear write
            else if (ST == 4) { if (tup_key(t) == -7) out[0] = t; }  // ablation: no write
            else out[run[d] + (i - tstart[d])] = t;
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

// Version 2: the per-digit phase is vectorised and spread over all threads
// (wcnt[d][0..W) is 16 or 32 bytes, read and written with 16-byte LDS ops),
// the write phase reads one precomputed delta[d] = run[d] - tstart[d] per
// element, and the counters are zeroed during the write phase.
template <int THREADS, int ITEMS>
struct Ss2Geom {
    static constexpr int W = THREADS / 64;
    static constexpr int TILE = THREADS * ITEMS;
    // stage | wcnt u16 [W][B] | run u32 [B] | delta i32 [B] | table u64 [W][64] | scr
    static size_t lds(uint32_t B, int rank) {
        return (size_t)TILE * sizeof(Tup) + (size_t)B * W * 2 + (size_t)B * 8 +
               (rank == 1 ? (size_t)W * 64 * 8 : 0) + 128;
    }
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int THREADS, int ITEMS, int RANK, int ST>
__global__ void __launch_bounds__(THREADS)
k_sscat2(const Tup* __restrict__ in, uint64_t n, uint64_t chunk, RefDigit dig,
         uint32_t nbins, uint32_t dbits, const uint32_t* __restrict__ counts, uint32_t nwg,
         const uint64_t* __restrict__ starts, Tup* __restrict__ out) {
    typedef Ss2Geom<THREADS, ITEMS> G;
    constexpr int W = G::W;
    constexpr int TILE = G::TILE;
    constexpr int HB = 6;
    constexpr int NV = W / 8;  // 16-byte vectors of counters per digit
    extern __shared__ __attribute__((aligned(16))) unsigned char lraw[];
    Tup* stage = reinterpret_cast<Tup*>(lraw);
    uint16_t* wcnt = reinterpret_cast<uint16_t*>(stage + TILE);
    uint32_t* run = reinterpret_cast<uint32_t*>(wcnt + (size_t)nbins * W);
    int32_t* delta = reinterpret_cast<int32_t*>(run + nbins);
    uint64_t* table = reinterpret_cast<uint64_t*>(delta + nbins);
    uint32_t* scr = reinterpret_cast<uint32_t*>(table + (RANK == 1 ? W * 64 : 0));

    const int lane = lane_id();
    const int wid = threadIdx.x >> 6;
    const uint64_t lt = lanemask_lt();
    uint64_t* mytab = table + (size_t)wid * 64;
    u32x4* wv = reinterpret_cast<u32x4*>(wcnt);
    const u32x4 zero4 = {0u, 0u, 0u, 0u};
    uint32_t* w32 = reinterpret_cast<uint32_t*>(wcnt);
    const uint32_t hb = nbins / 2;  // digit pairs
    for (uint32_t d = threadIdx.x; d < nbins; d += THREADS)
        run[d] = (uint32_t)(starts[d] + counts[(uint64_t)d * nwg + blockIdx.x]);
    for (uint32_t q = threadIdx.x; q < W * hb; q += THREADS) w32[q] = 0;
    if (RANK == 1) mytab[lane] = 0;
    const uint64_t beg = (uint64_t)blockIdx.x * chunk;
    const uint64_t end = min(beg + chunk, n);
    const uint32_t wbase = wid * 64 * ITEMS;
    constexpr int DPT = 2;  // digits per thread (nbins <= DPT * THREADS)
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
            if (RANK == 3) {
                // LDS atomics return lane-ordered values for lanes of one
                // instruction that hit the same word (tools/ldsorder.hip), so
                // the returned count is the stable rank; two digits share a
                // word (16-bit halves)
                const uint32_t sh = (d & 1u) * 16u;
                uint32_t old = 0;
                if (valid) old = atomicAdd(&w32[wid * hb + (d >> 1)], 1u << sh);
                rk[j] = (old >> sh) & 0xffffu;
                continue;
            }
            uint64_t peers;
            if (RANK == 0) {
                peers = __ballot(valid);
                for (uint32_t b = 0; b < dbits; b++) {
                    const bool bit = (d >> b) & 1u;
                    const uint64_t bal = __ballot(bit);
                    peers &= bit ? bal : ~bal;
                }
            } else {
                const uint32_t slot = d & 63u;
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
            if (valid) before = wcnt[wid * nbins + d];
            const uint32_t r = (uint32_t)__popcll(peers & lt);
            if (valid && r == 0) wcnt[wid * nbins + d] = (uint16_t)(before + __popcll(peers));
            rk[j] = before + r;
        }
        __syncthreads();
        // ---- per digit pair (2t, 2t+1): counters -> tile offsets, delta, run
        const uint32_t t2 = threadIdx.x;
        uint32_t cw[W];
        uint32_t c0 = 0, c1 = 0;
        if (t2 < hb) {
#pragma unroll
            for (int w = 0; w < W; w++) {
                cw[w] = w32[w * hb + t2];
                c0 += cw[w] & 0xffffu;
                c1 += cw[w] >> 16;
            }
        }
        uint32_t tot;
        const uint32_t ex = block_exclusive_scan(c0 + c1, scr, &tot);
        if (t2 < hb) {
            uint32_t o0 = ex, o1 = ex + c0;
#pragma unroll
            for (int w = 0; w < W; w++) {
                const uint32_t x = cw[w];
                w32[w * hb + t2] = o0 | (o1 << 16);
                o0 += x & 0xffffu;
                o1 += x >> 16;
            }
            const uint32_t d = 2 * t2;
            const uint32_t r0 = run[d], r1 = run[d + 1];
            delta[d] = (int32_t)(r0 - ex);
            delta[d + 1] = (int32_t)(r1 - (ex + c0));
            run[d] = r0 + c0;
            run[d + 1] = r1 + c1;
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
            if (dg[j] != 0xffffffffu) stage[wcnt[wid * nbins + dg[j]] + rk[j]] = v[j];
        __syncthreads();
        if (t2 < hb) {
#pragma unroll
            for (int w = 0; w < W; w++) w32[w * hb + t2] = 0;
        }
        for (uint32_t i = threadIdx.x; i < tcount; i += THREADS) {
            const Tup t = stage[i];
            const uint32_t d = dig(t);
            Tup* p = out + (uint32_t)(delta[d] + (int32_t)i);
            if (ST == 4) { if (tup_key(t) == -7) out[0] = t; }
            else if (ST == 3) out[base + i] = t;
            else *p = t;
        }
#pragma unroll
        for (int j = 0; j < ITEMS; j++) v[j] = nv[j];
        __syncthreads();
    }
}

template <int W>
__device__ __forceinline__ uint32_t scan_1bar(uint32_t v, uint32_t* scr, uint32_t* total) {
    const int lane = lane_id();
    const int wid = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) scr[wid] = x;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < W; w++) {
        const uint32_t t = scr[w];
        before += w < wid ? t : 0u;
        all += t;
    }
    *total = all;
    return before + x - v;
}

// Version 3: atomic (lane-ordered) ranks + write combining.  Each digit's
// output stream of this workgroup is cut at aligned SEGB-byte boundaries: the
// tail that does not fill a segment stays in an LDS carry and goes out with
// the next tile, so every store but the region's first and last segment is a
// whole aligned segment written by SEG consecutive lanes.
template <int THREADS, int ITEMS, int SEGB>
struct Ss3Geom {
    static constexpr int W = THREADS / 64;
    static constexpr int TILE = THREADS * ITEMS;
    static constexpr int SEG = SEGB / (int)sizeof(Tup);
    static constexpr int CW = SEG - 1;
    static constexpr int MAXSEG = TILE / SEG + 2 * 1024;
    // stage | carry [B][CW] | counters u32 [W][B/2] | info u32x4 [B] | segown u16 [MAXSEG] | scr
    static size_t lds(uint32_t B) {
        return (size_t)TILE * sizeof(Tup) + (size_t)B * CW * sizeof(Tup) + (size_t)W * B * 2 +
               (size_t)B * 16 + (size_t)(TILE / SEG + 2 * B) * 2 + 128;
    }
};

template <int THREADS, int ITEMS, int SEGB>
__global__ void __launch_bounds__(THREADS)
k_sscat3(const Tup* __restrict__ in, uint64_t n, uint64_t chunk, RefDigit dig,
         uint32_t nbins, const uint32_t* __restrict__ counts, uint32_t nwg,
         const uint64_t* __restrict__ starts, Tup* __restrict__ out) {
    typedef Ss3Geom<THREADS, ITEMS, SEGB> G;
    constexpr int W = G::W;
    constexpr int TILE = G::TILE;
    constexpr uint32_t SEG = G::SEG;
    constexpr uint32_t CW = G::CW;
    extern __shared__ __attribute__((aligned(16))) unsigned char lraw[];
    Tup* stage = reinterpret_cast<Tup*>(lraw);
    Tup* carry = stage + TILE;
    uint32_t* w32 = reinterpret_cast<uint32_t*>(carry + (size_t)nbins * CW);
    const uint32_t hb = nbins / 2;
    u32x4* info = reinterpret_cast<u32x4*>(w32 + (size_t)W * hb);
    uint16_t* segown = reinterpret_cast<uint16_t*>(info + nbins);
    uint32_t* scr = reinterpret_cast<uint32_t*>(
        (reinterpret_cast<uintptr_t>(segown + (TILE / SEG + 2 * nbins)) + 15) & ~uintptr_t(15));

    const int lane = lane_id();
    const int wid = threadIdx.x >> 6;
    const uint32_t t2 = threadIdx.x;
    const bool owner = t2 < hb;
    // per-digit state of the owner thread (digits 2*t2, 2*t2 + 1)
    uint32_t pos[2] = {0, 0}, kc[2] = {0, 0};
    if (owner) {
        for (int h = 0; h < 2; h++)
            pos[h] = (uint32_t)(starts[2 * t2 + h] + counts[(uint64_t)(2 * t2 + h) * nwg + blockIdx.x]);
    }
    for (uint32_t q = threadIdx.x; q < W * hb; q += THREADS) w32[q] = 0;
    const uint64_t beg = (uint64_t)blockIdx.x * chunk;
    const uint64_t end = min(beg + chunk, n);
    const uint32_t wbase = wid * 64 * ITEMS;
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
            const uint32_t sh = (d & 1u) * 16u;
            uint32_t old = 0;
            if (valid) old = atomicAdd(&w32[wid * hb + (d >> 1)], 1u << sh);
            rk[j] = (old >> sh) & 0xffffu;
        }
        __syncthreads();
        // ---- owner: counts, emission sizes, one packed scan
        uint32_t cw[W];
        uint32_t c[2] = {0, 0}, E[2] = {0, 0}, ns[2] = {0, 0};
        if (owner) {
#pragma unroll
            for (int w = 0; w < W; w++) {
                cw[w] = w32[w * hb + t2];
                c[0] += cw[w] & 0xffffu;
                c[1] += cw[w] >> 16;
            }
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const uint32_t T = kc[h] + c[h];
                const uint32_t m = (pos[h] + T) % SEG;
                E[h] = m <= T ? T - m : 0u;
                ns[h] = E[h] ? (pos[h] + E[h]) / SEG - pos[h] / SEG : 0u;
            }
        }
        uint32_t tot;
        const uint32_t ex = block_exclusive_scan((c[0] + c[1]) | ((ns[0] + ns[1]) << 16), scr, &tot);
        const uint32_t nsegT = tot >> 16;
        uint32_t ts[2];
        if (owner) {
            ts[0] = ex & 0xffffu;
            ts[1] = ts[0] + c[0];
            const uint32_t sp0 = ex >> 16, sp1 = sp0 + ns[0];
            uint32_t o0 = ts[0], o1 = ts[1];
#pragma unroll
            for (int w = 0; w < W; w++) {
                const uint32_t x = cw[w];
                w32[w * hb + t2] = o0 | (o1 << 16);
                o0 += x & 0xffffu;
                o1 += x >> 16;
            }
            const uint32_t sp[2] = {sp0, sp1};
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const uint32_t d = 2 * t2 + h;
                u32x4 I;
                I[0] = pos[h];
                I[1] = E[h];
                I[2] = ts[h];
                I[3] = sp[h] | (kc[h] << 16);
                info[d] = I;
                for (uint32_t k = 0; k < ns[h]; k++) segown[sp[h] + k] = (uint16_t)d;
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
            if (dg[j] != 0xffffffffu) {
                const uint32_t d = dg[j];
                const uint32_t wo = (w32[wid * hb + (d >> 1)] >> ((d & 1u) * 16u)) & 0xffffu;
                stage[wo + rk[j]] = v[j];
            }
        __syncthreads();
        // ---- whole segments: SEG consecutive lanes per aligned segment
        if (owner) {
#pragma unroll
            for (int w = 0; w < W; w++) w32[w * hb + t2] = 0;
        }
        for (uint32_t q = threadIdx.x; q < nsegT * SEG; q += THREADS) {
            const uint32_t sg = q / SEG;
            const uint32_t d = segown[sg];
            const u32x4 I = info[d];
            const uint32_t p = I[0];
            const uint32_t addr = (p / SEG + (sg - (I[3] & 0xffffu))) * SEG + q % SEG;
            if (addr >= p && addr < p + I[1]) {
                const uint32_t e = addr - p;
                const uint32_t k = I[3] >> 16;
                out[addr] = e < k ? carry[d * CW + e] : stage[I[2] + e - k];
            }
        }
        __syncthreads();
        // ---- owner: leftovers become the carry
        if (owner) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const uint32_t d = 2 * t2 + h;
                const uint32_t T = kc[h] + c[h];
                for (uint32_t e = E[h]; e < T; e++)
                    carry[d * CW + (e - E[h])] =
                        e < kc[h] ? carry[d * CW + e] : stage[ts[h] + e - kc[h]];
                pos[h] += E[h];
                kc[h] = T - E[h];
            }
        }
#pragma unroll
        for (int j = 0; j < ITEMS; j++) v[j] = nv[j];
    }
    // ---- the region's last partial segment
    if (owner) {
        for (int h = 0; h < 2; h++) {
            const uint32_t d = 2 * t2 + h;
            for (uint32_t e = 0; e < kc[h]; e++) out[pos[h] + e] = carry[d * CW + e];
        }
    }
}

template <int THREADS, int ITEMS, int SEGB>
__global__ void __launch_bounds__(THREADS)
k_sscat5(const Tup* __restrict__ in, uint64_t n, uint64_t chunk, RefDigit dig,
         uint32_t nbins, const uint32_t* __restrict__ counts, uint32_t nwg,
         const uint64_t* __restrict__ starts, Tup* __restrict__ out) {
    typedef Ss3Geom<THREADS, ITEMS, SEGB> G;
    constexpr int W = G::W;
    constexpr int TILE = G::TILE;
    constexpr uint32_t SEG = G::SEG;
    constexpr uint32_t CW = G::CW;
    extern __shared__ __attribute__((aligned(16))) unsigned char lraw[];
    Tup* stage = reinterpret_cast<Tup*>(lraw);
    Tup* carry = stage + TILE;
    uint32_t* w32 = reinterpret_cast<uint32_t*>(carry + (size_t)nbins * CW);
    const uint32_t hb = nbins / 2;
    u32x4* info = reinterpret_cast<u32x4*>(w32 + (size_t)W * hb);
    uint16_t* segown = reinterpret_cast<uint16_t*>(info + nbins);
    uint32_t* scr = reinterpret_cast<uint32_t*>(
        (reinterpret_cast<uintptr_t>(segown + (TILE / SEG + 2 * nbins)) + 15) & ~uintptr_t(15));

    const int lane = lane_id();
    const int wid = threadIdx.x >> 6;
    const uint32_t t2 = threadIdx.x;
    const bool owner = t2 < hb;
    // per-digit state of the owner thread (digits 2*t2, 2*t2 + 1)
    uint32_t pos[2] = {0, 0}, kc[2] = {0, 0};
    if (owner) {
        for (int h = 0; h < 2; h++)
            pos[h] = (uint32_t)(starts[2 * t2 + h] + counts[(uint64_t)(2 * t2 + h) * nwg + blockIdx.x]);
    }
    for (uint32_t q = threadIdx.x; q < W * hb; q += THREADS) w32[q] = 0;
    const uint64_t beg = (uint64_t)blockIdx.x * chunk;
    const uint64_t end = min(beg + chunk, n);
    const uint32_t wbase = wid * 64 * ITEMS;
    Tup v[ITEMS], nv[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        const uint64_t i = beg + wbase + j * 64 + lane;
        if (i < end) v[j] = in[i];
    }
    __syncthreads();
    uint32_t par = 0;
    for (uint64_t base = beg; base < end; base += TILE) {
        const uint32_t tcount = (uint32_t)min((uint64_t)TILE, end - base);
        uint32_t dg[ITEMS], rk[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint32_t li = wbase + j * 64 + lane;
            const bool valid = li < tcount;
            dg[j] = valid ? dig(v[j]) : 0xffffffffu;
            const uint32_t d = valid ? dg[j] : 0;
            const uint32_t sh = (d & 1u) * 16u;
            uint32_t old = 0;
            if (valid) old = atomicAdd(&w32[wid * hb + (d >> 1)], 1u << sh);
            rk[j] = (old >> sh) & 0xffffu;
        }
        __syncthreads();
        // ---- owner: counts, emission sizes, one packed scan
        uint32_t cw[W];
        uint32_t c[2] = {0, 0}, E[2] = {0, 0}, ns[2] = {0, 0};
        if (owner) {
#pragma unroll
            for (int w = 0; w < W; w++) {
                cw[w] = w32[w * hb + t2];
                c[0] += cw[w] & 0xffffu;
                c[1] += cw[w] >> 16;
            }
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const uint32_t T = kc[h] + c[h];
                const uint32_t m = (pos[h] + T) % SEG;
                E[h] = m <= T ? T - m : 0u;
                ns[h] = E[h] ? (pos[h] + E[h]) / SEG - pos[h] / SEG : 0u;
            }
        }
        uint32_t tot;
        const uint32_t ex = scan_1bar<W>((c[0] + c[1]) | ((ns[0] + ns[1]) << 16), scr + par * W, &tot);
        const uint32_t nsegT = tot >> 16;
        uint32_t ts[2];
        if (owner) {
            ts[0] = ex & 0xffffu;
            ts[1] = ts[0] + c[0];
            const uint32_t sp0 = ex >> 16, sp1 = sp0 + ns[0];
            uint32_t o0 = ts[0], o1 = ts[1];
#pragma unroll
            for (int w = 0; w < W; w++) {
                const uint32_t x = cw[w];
                w32[w * hb + t2] = o0 | (o1 << 16);
                o0 += x & 0xffffu;
                o1 += x >> 16;
            }
            const uint32_t sp[2] = {sp0, sp1};
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const uint32_t d = 2 * t2 + h;
                u32x4 I;
                I[0] = pos[h];
                I[1] = E[h] | ((kc[h] + c[h]) << 16);
                I[2] = ts[h];
                I[3] = sp[h] | (kc[h] << 16);
                info[d] = I;
                for (uint32_t k = 0; k < ns[h]; k++) segown[sp[h] + k] = (uint16_t)d;
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
            if (dg[j] != 0xffffffffu) {
                const uint32_t d = dg[j];
                const uint32_t wo = (w32[wid * hb + (d >> 1)] >> ((d & 1u) * 16u)) & 0xffffu;
                stage[wo + rk[j]] = v[j];
            }
        __syncthreads();
        // ---- whole segments: SEG consecutive lanes per aligned segment
        if (owner) {
#pragma unroll
            for (int w = 0; w < W; w++) w32[w * hb + t2] = 0;
        }
        for (uint32_t q = threadIdx.x; q < nsegT * SEG; q += THREADS) {
            const uint32_t sg = q / SEG;
            const uint32_t d = segown[sg];
            const u32x4 I = info[d];
            const uint32_t p = I[0];
            const uint32_t addr = (p / SEG + (sg - (I[3] & 0xffffu))) * SEG + q % SEG;
            if (addr >= p && addr < p + (I[1] & 0xffffu)) {
                const uint32_t e = addr - p;
                const uint32_t k = I[3] >> 16;
                out[addr] = e < k ? carry[d * CW + e] : stage[I[2] + e - k];
            }
        }
        __syncthreads();
        // ---- leftovers become the carry: one (digit, slot) per item, all
        // threads (E > 0: every leftover comes from the stage; E == 0: the old
        // carry stays in place and the tile's run is appended)
        for (uint32_t q = threadIdx.x; q < nbins * CW; q += THREADS) {
            const uint32_t d = q / CW, j = q - d * CW;
            const u32x4 I = info[d];
            const uint32_t Ed = I[1] & 0xffffu, Td = I[1] >> 16, kd = I[3] >> 16;
            if (j < Td - Ed && !(Ed == 0 && j < kd)) carry[q] = stage[I[2] + Ed + j - kd];
        }
        if (owner) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                pos[h] += E[h];
                kc[h] = kc[h] + c[h] - E[h];
            }
        }
        par ^= 1u;
#pragma unroll
        for (int j = 0; j < ITEMS; j++) v[j] = nv[j];
    }
    // ---- the region's last partial segment
    if (owner) {
        for (int h = 0; h < 2; h++) {
            const uint32_t d = 2 * t2 + h;
            for (uint32_t e = 0; e < kc[h]; e++) out[pos[h] + e] = carry[d * CW + e];
        }
    }
}

// Version 4: one digit per thread (1024 threads, nbins <= 1024), lane-ordered
// atomic ranks into double-buffered 16-bit counters, a one-barrier scan, and
// write combining whose carry lives in the digit owner's REGISTERS: the owner
// stores its carried tuples at the head of the digit's next whole segment
// while the lanes store the rest of that segment from the stage (both in the
// same phase, so the two halves meet in L2).  Four barriers per tile.
template <int THREADS, int ITEMS, int SEGB>
struct Ss4Geom {
    static constexpr int W = THREADS / 64;
    static constexpr int TILE = THREADS * ITEMS;
    static constexpr int SEG = SEGB / (int)sizeof(Tup);
    // stage | cnt u16 [2][W][B] | info u32x2 [B] | segown u16 [TILE/SEG + B] | scr u32 [2][W]
    static size_t lds(uint32_t B) {
        return (size_t)TILE * sizeof(Tup) + (size_t)2 * W * B * 2 + (size_t)B * 8 +
               (((size_t)(TILE / SEG + B) * 2 + 15) / 16) * 16 + 2 * W * 4 + 64;
    }
};

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));


template <int THREADS, int ITEMS, int SEGB>
__global__ void __launch_bounds__(THREADS)
k_sscat4(const Tup* __restrict__ in, uint64_t n, uint64_t chunk, RefDigit dig,
         uint32_t nbins, const uint32_t* __restrict__ counts, uint32_t nwg,
         const uint64_t* __restrict__ starts, Tup* __restrict__ out) {
    typedef Ss4Geom<THREADS, ITEMS, SEGB> G;
    constexpr int W = G::W;
    constexpr int TILE = G::TILE;
    constexpr uint32_t SEG = G::SEG;
    constexpr int CW = (int)SEG - 1;
    extern __shared__ __attribute__((aligned(16))) unsigned char lraw[];
    Tup* stage = reinterpret_cast<Tup*>(lraw);
    uint16_t* cnt = reinterpret_cast<uint16_t*>(stage + TILE);
    u32x2* info = reinterpret_cast<u32x2*>(cnt + (size_t)2 * W * nbins);
    uint16_t* segown = reinterpret_cast<uint16_t*>(info + nbins);
    uint32_t* scr = reinterpret_cast<uint32_t*>(
        (reinterpret_cast<uintptr_t>(segown + (TILE / SEG + nbins)) + 15) & ~uintptr_t(15));
    const uint32_t hb = nbins / 2;
    const int lane = lane_id();
    const int wid = threadIdx.x >> 6;
    const uint32_t d0 = threadIdx.x;
    const bool own = d0 < nbins;
    uint32_t pos = own ? (uint32_t)(starts[d0] + counts[(uint64_t)d0 * nwg + blockIdx.x]) : 0u;
    uint32_t kc = 0;
    Tup cr[CW > 0 ? CW : 1];
    {
        uint32_t* c32 = reinterpret_cast<uint32_t*>(cnt);
        for (uint32_t q = threadIdx.x; q < (uint32_t)W * nbins; q += THREADS) c32[q] = 0;
    }
    const uint64_t beg = (uint64_t)blockIdx.x * chunk;
    const uint64_t end = min(beg + chunk, n);
    const uint32_t wbase = wid * 64 * ITEMS;
    Tup v[ITEMS], nv[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        const uint64_t i = beg + wbase + j * 64 + lane;
        if (i < end) v[j] = in[i];
    }
    __syncthreads();
    uint32_t par = 0;
    for (uint64_t base = beg; base < end; base += TILE) {
        const uint32_t tcount = (uint32_t)min((uint64_t)TILE, end - base);
        uint16_t* cb = cnt + (size_t)par * W * nbins;
        uint32_t* c32 = reinterpret_cast<uint32_t*>(cb);
        uint32_t dg[ITEMS], rk[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint32_t li = wbase + j * 64 + lane;
            const bool valid = li < tcount;
            dg[j] = valid ? dig(v[j]) : 0xffffffffu;
            const uint32_t d = valid ? dg[j] : 0;
            const uint32_t sh = (d & 1u) * 16u;
            uint32_t old = 0;
            if (valid) old = atomicAdd(&c32[wid * hb + (d >> 1)], 1u << sh);
            rk[j] = (old >> sh) & 0xffffu;
        }
        __syncthreads();
        // ---- owner of digit d0: counts, emission size, packed scan
        uint32_t x[W];
        uint32_t c = 0;
        if (own) {
#pragma unroll
            for (int w = 0; w < W; w++) {
                x[w] = cb[w * nbins + d0];
                c += x[w];
            }
        }
        const uint32_t T = kc + c;
        const uint32_t m = (pos + T) & (SEG - 1);
        const uint32_t E = m <= T ? T - m : 0u;
        const uint32_t ns = E ? (pos + E) / SEG - pos / SEG : 0u;
        uint32_t tot;
        const uint32_t ex = scan_1bar<W>(own ? (c | (ns << 16)) : 0u, scr + par * W, &tot);
        const uint32_t nsegT = tot >> 16;
        const uint32_t ts = ex & 0xffffu, sp = ex >> 16;
        if (own) {
            uint32_t o = ts;
#pragma unroll
            for (int w = 0; w < W; w++) {
                cb[w * nbins + d0] = (uint16_t)o;
                o += x[w];
            }
            u32x2 I;
            I[0] = pos;
            I[1] = ts | (sp << 14) | (kc << 26);
            info[d0] = I;
            for (uint32_t k = 0; k < ns; k++) segown[sp + k] = (uint16_t)d0;
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
            if (dg[j] != 0xffffffffu) stage[cb[wid * nbins + dg[j]] + rk[j]] = v[j];
        __syncthreads();
        // ---- whole segments from the stage (their carried head: the owner)
        for (uint32_t q = threadIdx.x; q < nsegT * SEG; q += THREADS) {
            const uint32_t sg = q / SEG;
            const uint32_t d = segown[sg];
            const u32x2 I = info[d];
            const uint32_t p = I[0];
            const uint32_t spd = (I[1] >> 14) & 0xfffu, kcd = I[1] >> 26, tsd = I[1] & 0x3fffu;
            const uint32_t addr = (p / SEG + (sg - spd)) * SEG + (q & (SEG - 1));
            if (addr >= p) {
                const uint32_t e = addr - p;
                if (e >= kcd) out[addr] = stage[tsd + e - kcd];
            }
        }
        if (own) {
            if (E) {
#pragma unroll
                for (int j = 0; j < CW; j++)
                    if ((uint32_t)j < kc) out[pos + j] = cr[j];
            }
            // leftovers -> carry registers (E > 0: all from the stage)
            const uint32_t left = T - E;
#pragma unroll
            for (int j = 0; j < CW; j++) {
                if (E == 0 && (uint32_t)j < kc) continue;
                if ((uint32_t)j < left) cr[j] = stage[ts + E + j - kc];
            }
            pos += E;
            kc = left;
#pragma unroll
            for (int w = 0; w < W; w++) cb[w * nbins + d0] = 0;
        }
#pragma unroll
        for (int j = 0; j < ITEMS; j++) v[j] = nv[j];
        par ^= 1u;
    }
    if (own) {
#pragma unroll
        for (int j = 0; j < CW; j++)
            if ((uint32_t)j < kc) out[pos + j] = cr[j];
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

template <int HT, int HI, int THREADS, int ITEMS, int RANK, int HB, int ST = 0>
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
    SMJ_CHECK(hipFuncSetAttribute((const void*)k_sscatter<THREADS, ITEMS, RANK, HB, ST>,
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
        hipLaunchKernelGGL((k_sscatter<THREADS, ITEMS, RANK, HB, ST>), dim3(nwg), dim3(THREADS), lds,
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


template <int HT, int HI, int THREADS, int ITEMS, int RANK, int ST>
static void run_v2(Ctx& c, int reps, const char* label, uint32_t wpc = 1) {
    typedef Ss2Geom<THREADS, ITEMS> G;
    const uint64_t TILE = G::TILE;
    uint64_t ntiles = (c.n + TILE - 1) / TILE;
    uint32_t nwg = (uint32_t)std::min<uint64_t>(ntiles, 256ull * wpc);
    const uint64_t tpw = (ntiles + nwg - 1) / nwg;
    const uint64_t chunk = tpw * TILE;
    nwg = (uint32_t)((ntiles + tpw - 1) / tpw);
    uint32_t* counts;
    uint64_t *totals, *starts;
    SMJ_CHECK(hipMalloc(&counts, (size_t)c.nbins * nwg * 4));
    SMJ_CHECK(hipMalloc(&totals, c.nbins * 8));
    SMJ_CHECK(hipMalloc(&starts, c.nbins * 8));
    const size_t lds = G::lds(c.nbins, RANK);
    if (lds > 160 * 1024 || c.nbins > 2u * THREADS || (c.nbins & 1)) {
        printf("%s: LDS %zu too big\n", label, lds);
        return;
    }
    SMJ_CHECK(hipFuncSetAttribute((const void*)k_sscat2<THREADS, ITEMS, RANK, ST>,
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
        hipLaunchKernelGGL((k_sscat2<THREADS, ITEMS, RANK, ST>), dim3(nwg), dim3(THREADS), lds,
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
    if (ST < 3) check(c, label);
    SMJ_CHECK(hipFree(counts));
    SMJ_CHECK(hipFree(totals));
    SMJ_CHECK(hipFree(starts));
}

template <int HT, int HI, int THREADS, int ITEMS, int SEGB>
static void run_v3(Ctx& c, int reps, const char* label, uint32_t wpc = 1) {
    typedef Ss3Geom<THREADS, ITEMS, SEGB> G;
    const uint64_t TILE = G::TILE;
    uint64_t ntiles = (c.n + TILE - 1) / TILE;
    uint32_t nwg = (uint32_t)std::min<uint64_t>(ntiles, 256ull * wpc);
    const uint64_t tpw = (ntiles + nwg - 1) / nwg;
    const uint64_t chunk = tpw * TILE;
    nwg = (uint32_t)((ntiles + tpw - 1) / tpw);
    uint32_t* counts;
    uint64_t *totals, *starts;
    SMJ_CHECK(hipMalloc(&counts, (size_t)c.nbins * nwg * 4));
    SMJ_CHECK(hipMalloc(&totals, c.nbins * 8));
    SMJ_CHECK(hipMalloc(&starts, c.nbins * 8));
    const size_t lds = G::lds(c.nbins);
    if (lds > 160 * 1024 || c.nbins > 2u * THREADS || (c.nbins & 1)) {
        printf("%s: LDS %zu too big\n", label, lds);
        return;
    }
    SMJ_CHECK(hipFuncSetAttribute((const void*)k_sscat3<THREADS, ITEMS, SEGB>,
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
        hipLaunchKernelGGL((k_sscat3<THREADS, ITEMS, SEGB>), dim3(nwg), dim3(THREADS), lds,
                           0, c.din, c.n, chunk, dig, c.nbins, counts, nwg, starts, c.dout);
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
template <int HT, int HI, int THREADS, int ITEMS, int SEGB>
static void run_v4(Ctx& c, int reps, const char* label, uint32_t wpc = 1) {
    typedef Ss4Geom<THREADS, ITEMS, SEGB> G;
    const uint64_t TILE = G::TILE;
    uint64_t ntiles = (c.n + TILE - 1) / TILE;
    uint32_t nwg = (uint32_t)std::min<uint64_t>(ntiles, 256ull * wpc);
    const uint64_t tpw = (ntiles + nwg - 1) / nwg;
    const uint64_t chunk = tpw * TILE;
    nwg = (uint32_t)((ntiles + tpw - 1) / tpw);
    uint32_t* counts;
    uint64_t *totals, *starts;
    SMJ_CHECK(hipMalloc(&counts, (size_t)c.nbins * nwg * 4));
    SMJ_CHECK(hipMalloc(&totals, c.nbins * 8));
    SMJ_CHECK(hipMalloc(&starts, c.nbins * 8));
    const size_t lds = G::lds(c.nbins);
    if (lds > 160 * 1024 || c.nbins > (uint32_t)THREADS || (c.nbins & 1)) {
        printf("%s: LDS %zu too big\n", label, lds);
        return;
    }
    SMJ_CHECK(hipFuncSetAttribute((const void*)k_sscat4<THREADS, ITEMS, SEGB>,
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
        hipLaunchKernelGGL((k_sscat4<THREADS, ITEMS, SEGB>), dim3(nwg), dim3(THREADS), lds,
                           0, c.din, c.n, chunk, dig, c.nbins, counts, nwg, starts, c.dout);
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
template <int HT, int HI, int THREADS, int ITEMS, int SEGB>
static void run_v5(Ctx& c, int reps, const char* label, uint32_t wpc = 1) {
    typedef Ss3Geom<THREADS, ITEMS, SEGB> G;
    const uint64_t TILE = G::TILE;
    uint64_t ntiles = (c.n + TILE - 1) / TILE;
    uint32_t nwg = (uint32_t)std::min<uint64_t>(ntiles, 256ull * wpc);
    const uint64_t tpw = (ntiles + nwg - 1) / nwg;
    const uint64_t chunk = tpw * TILE;
    nwg = (uint32_t)((ntiles + tpw - 1) / tpw);
    uint32_t* counts;
    uint64_t *totals, *starts;
    SMJ_CHECK(hipMalloc(&counts, (size_t)c.nbins * nwg * 4));
    SMJ_CHECK(hipMalloc(&totals, c.nbins * 8));
    SMJ_CHECK(hipMalloc(&starts, c.nbins * 8));
    const size_t lds = G::lds(c.nbins);
    if (lds > 160 * 1024 || c.nbins > 2u * THREADS || (c.nbins & 1)) {
        printf("%s: LDS %zu too big\n", label, lds);
        return;
    }
    SMJ_CHECK(hipFuncSetAttribute((const void*)k_sscat5<THREADS, ITEMS, SEGB>,
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
        hipLaunchKernelGGL((k_sscat5<THREADS, ITEMS, SEGB>), dim3(nwg), dim3(THREADS), lds,
                           0, c.din, c.n, chunk, dig, c.nbins, counts, nwg, starts, c.dout);
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
#define V(HT, HI, T, I, R, HB, ST, W, name)                              \
    if (only.empty() || only == name) run_variant<HT, HI, T, I, R, HB, ST>(c, W, reps, name);
#define V3(T, I, SB, WPC, name)                              \
    if (only.empty() || only == name) run_v3<512, 16, T, I, SB>(c, reps, name, WPC);
#define V4(T, I, SB, WPC, name)                              \
    if (only.empty() || only == name) run_v4<512, 16, T, I, SB>(c, reps, name, WPC);
#define V5(T, I, SB, WPC, name)                              \
    if (only.empty() || only == name) run_v5<512, 16, T, I, SB>(c, reps, name, WPC);
    V3(512, 16, 64, 1, "v3 512x16 seg64");
    V5(512, 16, 64, 1, "v5 512x16 seg64");
    V5(512, 8, 64, 1, "v5 512x8 seg64");
    V5(512, 12, 64, 1, "v5 512x12 seg64");
    V5(512, 8, 32, 1, "v5 512x8 seg32");
    return 0;
}
