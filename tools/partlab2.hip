// partlab2.hip -- block-interleaved stable partition experiments
// (partition_relation_optimized, BASELINE config 3: 2^27 tuples, 10 bits).
//
// The chunked design (one contiguous chunk of 2^27/256 tuples per workgroup)
// keeps 256 x 1024 output streams open, each advancing 64 B per tile: DRAM
// sees scattered 64-byte writes.  Here the input is cut into blocks of K
// tiles; workgroup b takes block xmap(b), so the 32 workgroups of one XCD run
// on consecutive blocks at the same time and, per digit, write one contiguous
// window.  The histogram pass counts per block; a row scan per digit gives
// every block its offset; the scatter ranks a tile with lane-ordered LDS
// atomics, stages it in digit order with the digit of every staged slot, and
// writes it straight out (no carry).
//
// Standalone: hipcc -O3 --offload-arch=gfx950 [-DKEY_8B] tools/partlab2.hip
// Development tool, not part of the library.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../avx-sort-merge-joins_amd/csrc/smj_common.hpp"
#include "../avx-sort-merge-joins_amd/csrc/smj_internal.hpp"

using namespace smj;

static uint32_t host_digit(const Tup& t, uint32_t mask, uint32_t shift) {
    return (uint32_t)(((uint64_t)(tup_key(t) - 1) & (uint64_t)mask) >> shift);
}

// XCD-aware block order: block b runs on XCD b % 8; XCD x takes the blocks
// [x * per, (x + 1) * per) in order
__device__ __forceinline__ uint32_t xmap(uint32_t b, uint32_t nblk_pad) {
    const uint32_t per = nblk_pad >> 3;
    return (b & 7u) * per + (b >> 3);
}

template <int THREADS, int ITEMS, bool XM>
__global__ void __launch_bounds__(THREADS)
k_h6(const Tup* __restrict__ in, uint64_t n, uint64_t blk, RefDigit dig, uint32_t nbins,
     uint32_t* __restrict__ counts, uint32_t ntb) {
    extern __shared__ uint32_t lh[];
    const uint32_t tb = XM ? xmap(blockIdx.x, gridDim.x) : blockIdx.x;
    if (tb >= ntb) return;
    for (uint32_t d = threadIdx.x; d < nbins; d += THREADS) lh[d] = 0;
    __syncthreads();
    const uint64_t beg = (uint64_t)tb * blk;
    const uint64_t end = min(beg + blk, n);
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
        counts[(uint64_t)d * ntb + tb] = lh[d];
}

__global__ void __launch_bounds__(256)
k_scanrow6(uint32_t* __restrict__ counts, uint32_t nwg, uint64_t* __restrict__ totals) {
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
k_scandig6(const uint64_t* __restrict__ totals, uint32_t nbins, uint64_t* __restrict__ starts) {
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

template <int THREADS, int ITEMS>
struct S6Geom {
    static constexpr int W = THREADS / 64;
    static constexpr int TILE = THREADS * ITEMS;
    // stage Tup[TILE] | dgt u16[TILE] | w32 u32[W][B/2] | base u32[B] | wtot u32[W]
    static size_t lds(uint32_t B) {
        return (size_t)TILE * sizeof(Tup) + (size_t)TILE * 2 + (size_t)W * B * 2 + (size_t)B * 4 +
               64;
    }
};

__device__ __forceinline__ void wave_lds_sync6() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// NT: 0 plain stores, 1 non-temporal
template <int THREADS, int ITEMS, bool XM, int NT>
__global__ void __launch_bounds__(THREADS)
k_s6(const Tup* __restrict__ in, uint64_t n, uint64_t blk, RefDigit dig, uint32_t nbins,
     const uint32_t* __restrict__ boff, uint32_t ntb, const uint64_t* __restrict__ starts,
     Tup* __restrict__ out) {
    typedef S6Geom<THREADS, ITEMS> G;
    constexpr int W = G::W;
    constexpr int TILE = G::TILE;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    Tup* stage = reinterpret_cast<Tup*>(lds_raw);
    uint16_t* dgt = reinterpret_cast<uint16_t*>(stage + TILE);
    uint32_t* w32 = reinterpret_cast<uint32_t*>(dgt + TILE);
    const uint32_t hb = nbins / 2;
    uint32_t* base = w32 + W * hb;
    uint32_t* wtot = base + nbins;
    const uint32_t tb = XM ? xmap(blockIdx.x, gridDim.x) : blockIdx.x;
    if (tb >= ntb) return;
    const int lane = lane_id();
    const int wid = threadIdx.x >> 6;
    const uint32_t t2 = threadIdx.x;
    const bool owner = t2 < hb;
    uint32_t run[2] = {0, 0};
    if (owner) {
#pragma unroll
        for (int h = 0; h < 2; h++)
            run[h] = (uint32_t)starts[2 * t2 + h] + boff[(uint64_t)(2 * t2 + h) * ntb + tb];
    }
    for (uint32_t q = threadIdx.x; q < W * hb; q += THREADS) w32[q] = 0;
    const uint64_t beg = (uint64_t)tb * blk;
    const uint64_t end = min(beg + blk, n);
    const uint32_t wbase = wid * 64 * ITEMS;
    Tup v[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        const uint64_t i = beg + wbase + j * 64 + lane;
        if (i < end) v[j] = in[i];
    }
    __syncthreads();
    for (uint64_t tbase = beg; tbase < end; tbase += TILE) {
        const uint32_t tcount = (uint32_t)min((uint64_t)TILE, end - tbase);
        uint32_t dg[ITEMS], rk[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const bool valid = wbase + j * 64 + lane < tcount;
            const uint32_t d = valid ? dig(v[j]) : 0u;
            const uint32_t sh = (d & 1u) * 16u;
            uint32_t old = 0;
            if (valid) old = atomicAdd(&w32[wid * hb + (d >> 1)], 1u << sh);
            rk[j] = (old >> sh) & 0xffffu;
            dg[j] = valid ? d : 0xffffffffu;
        }
        __syncthreads();
        uint32_t c0 = 0, c1 = 0;
        uint32_t cw[W];
        if (owner) {
#pragma unroll
            for (int w = 0; w < W; w++) {
                cw[w] = w32[w * hb + t2];
                c0 += cw[w] & 0xffffu;
                c1 += cw[w] >> 16;
            }
        }
        // block scan of c0 + c1: wave scan, wave totals through LDS (1 barrier)
        const uint32_t loc = c0 + c1;
        uint32_t x = loc;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wtot[wid] = x;
        __syncthreads();
        uint32_t ex = x - loc;
#pragma unroll
        for (int w = 0; w < W; w++)
            if (w < wid) ex += wtot[w];
        if (owner) {
            uint32_t o0 = ex, o1 = ex + c0;
            base[2 * t2] = run[0] - o0;
            base[2 * t2 + 1] = run[1] - o1;
            run[0] += c0;
            run[1] += c1;
#pragma unroll
            for (int w = 0; w < W; w++) {
                w32[w * hb + t2] = o0 | (o1 << 16);
                o0 += cw[w] & 0xffffu;
                o1 += cw[w] >> 16;
            }
        }
        Tup nv[ITEMS];
        const uint64_t nb = tbase + TILE;
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
                const uint32_t p = wo + rk[j];
                stage[p] = v[j];
                dgt[p] = (uint16_t)d;
            }
        wave_lds_sync6();
        for (uint32_t q = lane; q < hb; q += 64) w32[wid * hb + q] = 0;
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < tcount; i += THREADS) {
            const uint32_t d = dgt[i];
            Tup* p = out + (uint32_t)(base[d] + i);
            if (NT)
                st_stream(p, stage[i]);
            else
                *p = stage[i];
        }
#pragma unroll
        for (int j = 0; j < ITEMS; j++) v[j] = nv[j];
    }
}

// copy of the library's k_scatter_swa (partition.hip) with wait-count fixes:
// FIX 1 waits for the first tile before the loop, 2 makes the prefetch
// unconditional (clamped), 4 waits for the prefetch before the segment stores
template <int THREADS, int ITEMS>
struct SwaGeom {
    static constexpr int W = THREADS / 64;
    static constexpr int TILE = THREADS * ITEMS;
    static constexpr uint32_t SEG = 64 / sizeof(Tup);
    static constexpr uint32_t CW = SEG - 1;
    // stage Tup[TILE] | carry Tup[B][CW] | counters u32[W][B/2] | info u32x4[B] |
    // segown u16[TILE/SEG + 2B] | scan scratch
    static __host__ __device__ constexpr size_t lds_bytes(uint32_t B) {
        return (size_t)TILE * sizeof(Tup) + (size_t)B * CW * sizeof(Tup) + (size_t)W * B * 2 +
               (size_t)B * 16 + ((size_t)(TILE / SEG + 2 * B) * 2 + 15) / 16 * 16 + 128;
    }
};

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

template <int THREADS, int ITEMS, class Digit, int FIX>
__global__ void __launch_bounds__(THREADS)
k_swa_lab(const Tup* __restrict__ in, uint64_t n, uint64_t chunk, Digit dig_arg,
              uint32_t nbins, const uint32_t* __restrict__ counts, uint32_t nwg,
              const uint64_t* __restrict__ starts, Tup* __restrict__ out) {
    typedef SwaGeom<THREADS, ITEMS> G;
    constexpr int W = G::W;
    constexpr int TILE = G::TILE;
    constexpr uint32_t SEG = G::SEG;
    constexpr uint32_t CW = G::CW;
    const auto dig = dig_arg.load();
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    Tup* stage = reinterpret_cast<Tup*>(lds_raw);
    Tup* carry = stage + TILE;
    uint32_t* w32 = reinterpret_cast<uint32_t*>(carry + (size_t)nbins * CW);
    const uint32_t hb = nbins / 2;
    u32x4_t* info = reinterpret_cast<u32x4_t*>(w32 + (size_t)W * hb);
    uint16_t* segown = reinterpret_cast<uint16_t*>(info + nbins);
    // plain pointer arithmetic (no integer casts): the scan scratch stays an
    // LDS pointer, not a flat one that every vmcnt wait would have to cover
    uint32_t* scr = reinterpret_cast<uint32_t*>(segown + ((TILE / SEG + 2 * nbins + 7) & ~7u));

    const int lane = lane_id();
    const int wid = threadIdx.x >> 6;
    const uint32_t t2 = threadIdx.x;
    const bool owner = t2 < hb;
    // the owner's state of digits 2 t2 and 2 t2 + 1: output cursor, carry size
    uint32_t pos[2] = {0, 0}, kc[2] = {0, 0};
    if (owner) {
#pragma unroll
        for (int h = 0; h < 2; h++)
            pos[h] = (uint32_t)(starts[2 * t2 + h] +
                                counts[(uint64_t)(2 * t2 + h) * nwg + blockIdx.x]);
    }
    for (uint32_t q = threadIdx.x; q < W * hb; q += THREADS) w32[q] = 0;
    const uint64_t beg = (uint64_t)blockIdx.x * chunk;
    const uint64_t end = min(beg + chunk, n);
    const uint32_t wbase = wid * 64 * ITEMS;
    Tup v[ITEMS], nv[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        const uint64_t i = beg + wbase + j * 64 + lane;
        if (FIX & 2) v[j] = in[i < end ? i : end - 1];
        else if (i < end) v[j] = in[i];
    }
    if (FIX & 1) __builtin_amdgcn_s_waitcnt(0x0f70);
    __syncthreads();
    for (uint64_t base = beg; base < end; base += TILE) {
        const uint32_t tcount = (uint32_t)min((uint64_t)TILE, end - base);
        // ---- ranks (lane-ordered atomics, see the header)
        uint32_t dg[ITEMS], rk[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const bool valid = wbase + j * 64 + lane < tcount;
            dg[j] = valid ? dig(v[j]) : 0xffffffffu;
            const uint32_t d = valid ? dg[j] : 0;
            const uint32_t sh = (d & 1u) * 16u;
            uint32_t old = 0;
            if (valid) old = atomicAdd(&w32[wid * hb + (d >> 1)], 1u << sh);
            rk[j] = (old >> sh) & 0xffffu;
        }
        __syncthreads();
        // ---- owner: tile counts, emission sizes (up to the last segment
        // boundary of carry + tile), stage offsets and segment numbers in one
        // packed scan (both sums stay below 2^16)
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
        const uint32_t ex =
            block_exclusive_scan((c[0] + c[1]) | ((ns[0] + ns[1]) << 16), scr, &tot);
        const uint32_t nsegT = tot >> 16;
        uint32_t ts[2] = {0, 0};
        if (owner) {
            ts[0] = ex & 0xffffu;
            ts[1] = ts[0] + c[0];
            const uint32_t sp[2] = {ex >> 16, (ex >> 16) + ns[0]};
            uint32_t o0 = ts[0], o1 = ts[1];
#pragma unroll
            for (int w = 0; w < W; w++) {
                const uint32_t x = cw[w];
                w32[w * hb + t2] = o0 | (o1 << 16);
                o0 += x & 0xffffu;
                o1 += x >> 16;
            }
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const uint32_t d = 2 * t2 + h;
                u32x4_t I;
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
            if (FIX & 2) nv[j] = in[i < end ? i : end - 1];
            else if (i < end) nv[j] = in[i];
        }
        __syncthreads();
        // ---- stage the tile in digit order
#pragma unroll
        for (int j = 0; j < ITEMS; j++)
            if (dg[j] != 0xffffffffu) {
                const uint32_t d = dg[j];
                const uint32_t wo = (w32[wid * hb + (d >> 1)] >> ((d & 1u) * 16u)) & 0xffffu;
                stage[wo + rk[j]] = v[j];
            }
        __syncthreads();
        // ---- whole aligned segments, SEG consecutive lanes each; element e
        // of a digit's emission is its carry (e < kc) or its staged run
        if (owner) {
#pragma unroll
            for (int w = 0; w < W; w++) w32[w * hb + t2] = 0;
        }
        if (FIX & 4) __builtin_amdgcn_s_waitcnt(0x0f70);
        for (uint32_t q = threadIdx.x; q < nsegT * SEG; q += THREADS) {
            const uint32_t sg = q / SEG;
            const uint32_t d = segown[sg];
            const u32x4_t I = info[d];
            const uint32_t p = I[0];
            const uint32_t addr = (p / SEG + (sg - (I[3] & 0xffffu))) * SEG + q % SEG;
            if (addr >= p && addr < p + I[1]) {
                const uint32_t e = addr - p;
                const uint32_t k = I[3] >> 16;
                const Tup x = e < k ? carry[d * CW + e] : stage[I[2] + e - k];
                if (!(FIX & 8) || addr == 0xffffffffu) out[addr] = x;  // 8: no stores
            }
        }
        __syncthreads();
        // ---- owner: the leftovers (< SEG) become the carry
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
    // ---- the partial last segment of every region
    if (owner) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const uint32_t d = 2 * t2 + h;
            for (uint32_t e = 0; e < kc[h]; e++) out[pos[h] + e] = carry[d * CW + e];
        }
    }
}

// k_swb: k_swa_lab restructured for LDS latency -- every LDS phase issues
// its reads as a batch before using them (no per-item branches on full
// tiles, invalid items go to a dump slot), the segment-store loop handles 4
// stores per thread per trip, the carry is read into registers before it is
// rewritten.  FIX 8: no global stores (measurement only).
template <int THREADS, int ITEMS>
struct SwbGeom {
    static constexpr int W = THREADS / 64;
    static constexpr int TILE = THREADS * ITEMS;
    static constexpr uint32_t SEG = 64 / sizeof(Tup);
    static constexpr uint32_t CW = SEG - 1;
    // stage Tup[TILE + SEG] (dump slot) | carry Tup[B][CW] | counters u32[W][B/2] |
    // info u32x4[B] | segown u16[TILE/SEG + 2B] | scan scratch
    static __host__ __device__ constexpr size_t lds_bytes(uint32_t B) {
        return (size_t)(TILE + SEG) * sizeof(Tup) + (size_t)B * CW * sizeof(Tup) +
               (size_t)W * B * 2 + (size_t)B * 16 +
               ((size_t)(TILE / SEG + 2 * B) * 2 + 15) / 16 * 16 + 128;
    }
};

template <bool FULL, int THREADS, int ITEMS, class DigitL>
__device__ __forceinline__ void swb_rank(const Tup (&v)[ITEMS], uint32_t (&dg)[ITEMS],
                                         uint32_t (&rk)[ITEMS], uint32_t* w32, uint32_t hb,
                                         uint32_t wbase, uint32_t tcount, const DigitL& dig) {
    const int lane = lane_id();
    const int wid = threadIdx.x >> 6;
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        const bool valid = FULL || wbase + j * 64 + lane < tcount;
        const uint32_t d = dig(v[j]);
        const uint32_t sh = (d & 1u) * 16u;
        const uint32_t old = atomicAdd(&w32[wid * hb + (d >> 1)], valid ? 1u << sh : 0u);
        rk[j] = (old >> sh) & 0xffffu;
        dg[j] = valid ? d : 0xffffffffu;
    }
}

template <int THREADS, int ITEMS, class Digit, int FIX>
__global__ void __launch_bounds__(THREADS)
k_swb(const Tup* __restrict__ in, uint64_t n, uint64_t chunk, Digit dig_arg,
      uint32_t nbins, const uint32_t* __restrict__ counts, uint32_t nwg,
      const uint64_t* __restrict__ starts, Tup* __restrict__ out, uint32_t hsub) {
    typedef SwbGeom<THREADS, ITEMS> G;
    constexpr int W = G::W;
    constexpr int TILE = G::TILE;
    constexpr uint32_t SEG = G::SEG;
    constexpr uint32_t CW = G::CW;
    constexpr int U = 4;  // segment stores per thread per trip
    const auto dig = dig_arg.load();
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    Tup* stage = reinterpret_cast<Tup*>(lds_raw);
    Tup* carry = stage + TILE + SEG;
    uint32_t* w32 = reinterpret_cast<uint32_t*>(carry + (size_t)nbins * CW);
    const uint32_t hb = nbins / 2;
    u32x4_t* info = reinterpret_cast<u32x4_t*>(w32 + (size_t)W * hb);
    uint16_t* segown = reinterpret_cast<uint16_t*>(info + nbins);
    uint32_t* scr = reinterpret_cast<uint32_t*>(segown + ((TILE / SEG + 2 * nbins + 7) & ~7u));

    const int lane = lane_id();
    const int wid = threadIdx.x >> 6;
    const uint32_t t2 = threadIdx.x;
    const bool owner = t2 < hb;
    uint32_t pos[2] = {0, 0}, kc[2] = {0, 0};
    if (owner) {
#pragma unroll
        for (int h = 0; h < 2; h++)
            pos[h] = (uint32_t)(starts[2 * t2 + h] +
                                counts[(uint64_t)(2 * t2 + h) * nwg * hsub + blockIdx.x * hsub]);
    }
    for (uint32_t q = threadIdx.x; q < W * hb; q += THREADS) w32[q] = 0;
    const uint64_t beg = (uint64_t)blockIdx.x * chunk;
    const uint64_t end = min(beg + chunk, n);
    const uint32_t wbase = wid * 64 * ITEMS;
    Tup v[ITEMS], nv[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        const uint64_t i = beg + wbase + j * 64 + lane;
        v[j] = in[i < end ? i : end - 1];
    }
    __builtin_amdgcn_s_waitcnt(0x0f70);
    __syncthreads();
    for (uint64_t base = beg; base < end; base += TILE) {
        const uint32_t tcount = (uint32_t)min((uint64_t)TILE, end - base);
        uint32_t dg[ITEMS], rk[ITEMS];
        if (tcount == TILE)
            swb_rank<true, THREADS, ITEMS>(v, dg, rk, w32, hb, wbase, tcount, dig);
        else
            swb_rank<false, THREADS, ITEMS>(v, dg, rk, w32, hb, wbase, tcount, dig);
        __syncthreads();
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
        uint32_t tot, ex;
        if (FIX & 16) {
            // wave scan, wave totals through LDS: one barrier (scr is not
            // touched again before the next tile's barriers)
            const uint32_t loc = (c[0] + c[1]) | ((ns[0] + ns[1]) << 16);
            uint32_t x = loc;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(x, o, 64);
                if (lane >= o) x += y;
            }
            if (lane == 63) scr[wid] = x;
            __syncthreads();
            ex = x - loc;
            tot = 0;
#pragma unroll
            for (int w = 0; w < W; w++) {
                const uint32_t t = scr[w];
                if (w < wid) ex += t;
                tot += t;
            }
        } else {
            ex = block_exclusive_scan((c[0] + c[1]) | ((ns[0] + ns[1]) << 16), scr, &tot);
        }
        const uint32_t nsegT = tot >> 16;
        uint32_t ts[2] = {0, 0};
        if (owner) {
            ts[0] = ex & 0xffffu;
            ts[1] = ts[0] + c[0];
            const uint32_t sp[2] = {ex >> 16, (ex >> 16) + ns[0]};
            uint32_t o0 = ts[0], o1 = ts[1];
#pragma unroll
            for (int w = 0; w < W; w++) {
                const uint32_t x = cw[w];
                w32[w * hb + t2] = o0 | (o1 << 16);
                o0 += x & 0xffffu;
                o1 += x >> 16;
            }
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const uint32_t d = 2 * t2 + h;
                u32x4_t I;
                I[0] = pos[h];
                I[1] = E[h];
                I[2] = ts[h];
                I[3] = sp[h] | (kc[h] << 16);
                info[d] = I;
                for (uint32_t k = 0; k < ns[h]; k++) segown[sp[h] + k] = (uint16_t)d;
            }
        }
        const uint64_t nb = base + TILE;
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint64_t i = nb + wbase + j * 64 + lane;
            nv[j] = in[i < end ? i : end - 1];
        }
        __syncthreads();
        // ---- stage: all counter reads first, then all stores (dump slot for
        // invalid items)
        {
            uint32_t wo[ITEMS];
#pragma unroll
            for (int j = 0; j < ITEMS; j++) {
                const uint32_t d = dg[j] == 0xffffffffu ? 0u : dg[j];
                wo[j] = w32[wid * hb + (d >> 1)];
            }
#pragma unroll
            for (int j = 0; j < ITEMS; j++) {
                const uint32_t d = dg[j];
                const uint32_t p = d == 0xffffffffu
                                       ? (uint32_t)TILE
                                       : ((wo[j] >> ((d & 1u) * 16u)) & 0xffffu) + rk[j];
                stage[p] = v[j];
            }
        }
        __syncthreads();
        if (owner) {
#pragma unroll
            for (int w = 0; w < W; w++) w32[w * hb + t2] = 0;
        }
        // ---- whole aligned segments, U per thread per trip: the segment
        // owners, then the infos, then the data, then the stores
        const uint32_t nq = nsegT * SEG;
        for (uint32_t q0 = threadIdx.x; q0 < nq; q0 += U * THREADS) {
            uint32_t dd[U], addr[U];
            bool ok[U];
            Tup x[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t q = min(q0 + u * THREADS, nq - 1);
                dd[u] = segown[q / SEG];
            }
            u32x4_t I[U];
#pragma unroll
            for (int u = 0; u < U; u++) I[u] = info[dd[u]];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t q = q0 + u * THREADS;
                const uint32_t qc = min(q, nq - 1);
                const uint32_t sg = qc / SEG;
                const uint32_t p = I[u][0];
                addr[u] = (p / SEG + (sg - (I[u][3] & 0xffffu))) * SEG + qc % SEG;
                ok[u] = q < nq && addr[u] >= p && addr[u] < p + I[u][1];
                const uint32_t e = ok[u] ? addr[u] - p : 0u;
                const uint32_t k = I[u][3] >> 16;
                x[u] = e < k ? carry[dd[u] * CW + e] : stage[I[u][2] + e - k];
            }
#pragma unroll
            for (int u = 0; u < U; u++)
                if (ok[u] && (!(FIX & 8) || addr[u] == 0xffffffffu)) out[addr[u]] = x[u];
        }
        __syncthreads();
        // ---- owner: the leftovers (< SEG) become the carry: read, then write
        if (owner) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const uint32_t d = 2 * t2 + h;
                const uint32_t T = kc[h] + c[h];
                const uint32_t left = T - E[h];
                Tup tmp[CW];
#pragma unroll
                for (uint32_t e = 0; e < CW; e++) {
                    const uint32_t idx = E[h] + e;
                    tmp[e] = idx < kc[h] ? carry[d * CW + idx]
                                         : stage[e < left ? ts[h] + idx - kc[h] : 0u];
                }
#pragma unroll
                for (uint32_t e = 0; e < CW; e++)
                    if (e < left) carry[d * CW + e] = tmp[e];
                pos[h] += E[h];
                kc[h] = left;
            }
        }
#pragma unroll
        for (int j = 0; j < ITEMS; j++) v[j] = nv[j];
    }
    if (owner) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const uint32_t d = 2 * t2 + h;
            for (uint32_t e = 0; e < kc[h]; e++) out[pos[h] + e] = carry[d * CW + e];
        }
    }
}

// plain copy for the bandwidth reference
__global__ void k_copy(const Tup* __restrict__ in, Tup* __restrict__ out, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        st_stream(out + i, in[i]);
}

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
                if (bad < 3)
                    fprintf(stderr, "  %s mismatch digit %u elem %llu\n", name, d,
                            (unsigned long long)k);
                bad++;
            }
        }
    printf("  check %s: %s (%llu bad)\n", name, bad ? "FAIL" : "ok", (unsigned long long)bad);
}

template <int THREADS, int ITEMS, int K, bool XM, int NT>
static void run_v6(Ctx& c, int reps, const char* label) {
    typedef S6Geom<THREADS, ITEMS> G;
    const uint64_t blk = (uint64_t)K * G::TILE;
    const uint32_t ntb = (uint32_t)((c.n + blk - 1) / blk);
    const uint32_t grid = XM ? (ntb + 7) / 8 * 8 : ntb;
    const size_t lds = G::lds(c.nbins);
    if (lds > 160 * 1024 || c.nbins > 2u * THREADS || (c.nbins & 1)) {
        printf("%s: LDS %zu too big\n", label, lds);
        return;
    }
    uint32_t* counts;
    uint64_t *totals, *starts;
    SMJ_CHECK(hipMalloc(&counts, (size_t)c.nbins * ntb * 4));
    SMJ_CHECK(hipMalloc(&totals, c.nbins * 8));
    SMJ_CHECK(hipMalloc(&starts, c.nbins * 8));
    SMJ_CHECK(hipFuncSetAttribute((const void*)k_s6<THREADS, ITEMS, XM, NT>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    const uint32_t mask = (uint32_t)(((1ull << c.bits) - 1) << c.shift);
    RefDigit dig{mask, c.shift};
    hipEvent_t e[4];
    for (auto& x : e) SMJ_CHECK(hipEventCreate(&x));
    float th = 0, ts = 0, tc = 0;
    SMJ_CHECK(hipMemset(c.dout, 0, c.cap * sizeof(Tup)));
    for (int r = -1; r < reps; r++) {
        SMJ_CHECK(hipEventRecord(e[0]));
        hipLaunchKernelGGL((k_h6<512, 16, XM>), dim3(grid), dim3(512), c.nbins * 4, 0, c.din, c.n,
                           blk, dig, c.nbins, counts, ntb);
        SMJ_CHECK(hipEventRecord(e[1]));
        hipLaunchKernelGGL(k_scanrow6, dim3(c.nbins), dim3(256), 0, 0, counts, ntb, totals);
        hipLaunchKernelGGL(k_scandig6, dim3(1), dim3(256), 0, 0, totals, c.nbins, starts);
        SMJ_CHECK(hipEventRecord(e[2]));
        hipLaunchKernelGGL((k_s6<THREADS, ITEMS, XM, NT>), dim3(grid), dim3(THREADS), lds, 0,
                           c.din, c.n, blk, dig, c.nbins, counts, ntb, starts, c.dout);
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
    printf("%-40s ntb %5u lds %6zu  hist %.3f scan %.3f scatter %.3f total %.3f ms  frac %.3f\n",
           label, ntb, lds, th / reps, tc / reps, ts / reps, tot, alg / (tot * 1e-3) / 8e12);
    check(c, label);
    SMJ_CHECK(hipFree(counts));
    SMJ_CHECK(hipFree(totals));
    SMJ_CHECK(hipFree(starts));
}

template <int THREADS, int ITEMS, int FIX, bool B = false, int HS = 1, int WPC = 1,
          int HT = 512, int HI = 16>
static void run_swa(Ctx& c, int reps, const char* label) {
    typedef SwaGeom<THREADS, ITEMS> G;
    typedef SwbGeom<THREADS, ITEMS> GB;
    uint64_t ntiles = (c.n + G::TILE - 1) / G::TILE;
    uint32_t nwg = (uint32_t)std::min<uint64_t>(ntiles, 256 * WPC);
    const uint64_t tpw = (ntiles + nwg - 1) / nwg;
    const uint64_t chunk = tpw * G::TILE;
    nwg = (uint32_t)((ntiles + tpw - 1) / tpw);
    const size_t lds = B ? GB::lds_bytes(c.nbins) : G::lds_bytes(c.nbins);
    if (lds > 160 * 1024) {
        printf("%s: LDS %zu too big\n", label, lds);
        return;
    }
    uint32_t* counts;
    uint64_t *totals, *starts;
    SMJ_CHECK(hipMalloc(&counts, (size_t)c.nbins * nwg * HS * 4));
    SMJ_CHECK(hipMalloc(&totals, c.nbins * 8));
    SMJ_CHECK(hipMalloc(&starts, c.nbins * 8));
    SMJ_CHECK(hipFuncSetAttribute((const void*)k_swa_lab<THREADS, ITEMS, RefDigit, FIX>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    SMJ_CHECK(hipFuncSetAttribute((const void*)k_swb<THREADS, ITEMS, RefDigit, FIX>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    const uint32_t mask = (uint32_t)(((1ull << c.bits) - 1) << c.shift);
    RefDigit dig{mask, c.shift};
    hipEvent_t e[4];
    for (auto& x : e) SMJ_CHECK(hipEventCreate(&x));
    float th = 0, ts = 0, tc = 0;
    SMJ_CHECK(hipMemset(c.dout, 0, c.cap * sizeof(Tup)));
    for (int r = -1; r < reps; r++) {
        SMJ_CHECK(hipEventRecord(e[0]));
        hipLaunchKernelGGL((k_h6<HT, HI, false>), dim3(nwg * HS), dim3(HT), c.nbins * 4, 0, c.din,
                           c.n, chunk / HS, dig, c.nbins, counts, nwg * HS);
        SMJ_CHECK(hipEventRecord(e[1]));
        hipLaunchKernelGGL(k_scanrow6, dim3(c.nbins), dim3(256), 0, 0, counts, nwg * HS, totals);
        hipLaunchKernelGGL(k_scandig6, dim3(1), dim3(256), 0, 0, totals, c.nbins, starts);
        SMJ_CHECK(hipEventRecord(e[2]));
        if (B)
            hipLaunchKernelGGL((k_swb<THREADS, ITEMS, RefDigit, FIX>), dim3(nwg), dim3(THREADS), lds, 0,
                               c.din, c.n, chunk, dig, c.nbins, counts, nwg, starts, c.dout, (uint32_t)HS);
        else
            hipLaunchKernelGGL((k_swa_lab<THREADS, ITEMS, RefDigit, FIX>), dim3(nwg), dim3(THREADS), lds, 0,
                               c.din, c.n, chunk, dig, c.nbins, counts, nwg, starts, c.dout);
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
    printf("%-40s nwg %5u lds %6zu  hist %.3f scan %.3f scatter %.3f total %.3f ms  frac %.3f\n",
           label, nwg, lds, th / reps, tc / reps, ts / reps, tot, alg / (tot * 1e-3) / 8e12);
    check(c, label);
    SMJ_CHECK(hipFree(counts));
    SMJ_CHECK(hipFree(totals));
    SMJ_CHECK(hipFree(starts));
}

int main(
int argc, char** argv) {
    Ctx c;
    c.n = argc > 1 ? strtoull(argv[1], 0, 10) : (1ull << 27);
    c.bits = argc > 2 ? atoi(argv[2]) : 10;
    c.shift = argc > 3 ? atoi(argv[3]) : 0;
    const std::string only = argc > 4 ? argv[4] : "";
    c.nbins = 1u << c.bits;
    c.cap = c.n + c.nbins * 64 / sizeof(Tup);
    c.hin.resize(c.n);
    for (uint64_t i = 0; i < c.n; i++) {
        const uint64_t k = (i * 0x9E3779B97F4A7C15ull >> 13) % c.n + 1;  // keys ~uniform
#ifdef KEY_8B
        c.hin[i].payload = (int64_t)i;
        c.hin[i].key = (int64_t)k;
#else
        c.hin[i] = ((uint64_t)(uint32_t)k << 32) | (uint32_t)i;
#endif
    }
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
#define V6(T, I, K, XM, NT, name) \
    if (only.empty() || only == name) run_v6<T, I, K, XM, NT>(c, reps, name);
#define SWA(T, I, F, name) \
    if (only.empty() || only == name) run_swa<T, I, F>(c, reps, name);
#define SWB(T, I, F, name) \
    if (only.empty() || only == name) run_swa<T, I, F, true>(c, reps, name);
#define SWAW(T, I, F, W, name) \
    if (only.empty() || only == name) run_swa<T, I, F, false, 1, W>(c, reps, name);
#define SWAH(HT, HI, name) \
    if (only.empty() || only == name) run_swa<512, 16, 1, false, 1, 1, HT, HI>(c, reps, name);
#define SWBH(T, I, F, H, name) \
    if (only.empty() || only == name) run_swa<T, I, F, true, H>(c, reps, name);
#ifdef KEY_8B
    SWA(512, 8, 1, "swa 512x8 fix1");
    SWB(512, 8, 1, "swb 512x8");
    SWB(512, 8, 17, "swb 512x8 scan1");
    SWBH(512, 8, 17, 4, "swb 512x8 scan1 h4");
    SWB(1024, 3, 17, "swb 1024x3 scan1");
#else
    SWA(512, 16, 1, "swa 512x16 fix1");
    SWAH(1024, 16, "hist 1024x16");
    SWAH(1024, 8, "hist 1024x8");
    SWAH(1024, 32, "hist 1024x32");
    SWAH(512, 32, "hist 512x32");
    SWAW(512, 8, 1, 1, "swa 512x8 1/cu");
    SWAW(512, 8, 1, 2, "swa 512x8 2/cu");
    SWAW(256, 16, 1, 1, "swa 256x16 1/cu");
    SWAW(256, 16, 1, 2, "swa 256x16 2/cu");
    SWAW(256, 8, 1, 3, "swa 256x8 3/cu");
    SWB(512, 16, 1, "swb 512x16");
    SWB(512, 16, 17, "swb 512x16 scan1");
    SWB(1024, 6, 1, "swb 1024x6");
    SWB(1024, 6, 17, "swb 1024x6 scan1");
    SWBH(1024, 6, 17, 4, "swb 1024x6 scan1 h4");
    SWBH(1024, 6, 17, 8, "swb 1024x6 scan1 h8");
#endif
    return 0;
}
