// partition.hip -- stable radix partitioning on MI355X (gfx950).
//
// Device form of partition_relation / partition_relation_optimized
// (reference src/partition/partition.c:93-219, 301-354).  The reference does
// a histogram pass, then a single-threaded scatter through 64-byte software
// write-combining buffers flushed with non-temporal stores.  Here:
//
//   k_hist    : one pass over the input; every workgroup counts its chunk in an
//               LDS histogram and writes counts[digit][wg] (digit-major).
//   k_scanrow : per digit, exclusive scan over workgroups (stable order).
//   k_scandig : one workgroup; partition starts = exclusive scan over digits of
//               the (optionally 64-byte padded, ALIGN_NUMTUPLES) totals.
//   k_scatter : every workgroup re-reads its chunk tile by tile.  Each wave
//               ranks its 64-item steps with ballot matching (__ballot over the
//               digit bits -> peers mask -> popcount of lower lanes), which
//               keeps input order inside a digit (stable == radix_cluster).
//               The tile is then staged in LDS sorted by digit and written out
//               so that consecutive lanes write consecutive addresses of one
//               partition: the LDS tile plays the role of the reference's
//               cache-line write-combining buffers, and the bigger the tile
//               the longer each partition's contiguous run per store.
//
// Digits wider than 12 bits are done as two stable LSD passes plus a
// padding copy (stable_partition below).
#include <stdlib.h>
#include <string.h>

#include "smj_common.hpp"
#include "smj_internal.hpp"

namespace smj {

// ---------------------------------------------------------------------------
template <int THREADS, int ITEMS, class Digit>
__global__ void __launch_bounds__(THREADS)
k_hist(const Tup* __restrict__ in, uint64_t n, uint64_t chunk, Digit dig_arg,
       uint32_t nbins, uint32_t* __restrict__ counts, uint32_t nwg) {
    const auto dig = dig_arg.load();
    constexpr int TILE = THREADS * ITEMS;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_hist[];
    for (uint32_t d = threadIdx.x; d < nbins; d += THREADS) lds_hist[d] = 0;
    __syncthreads();
    const uint64_t beg = (uint64_t)blockIdx.x * chunk;
    uint64_t end = beg + chunk;
    if (end > n) end = n;
    for (uint64_t base = beg; base < end; base += TILE) {
        Tup v[ITEMS];
        // unconditional (clamped) loads: all in flight at once
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint64_t i = base + (uint64_t)j * THREADS + threadIdx.x;
            v[j] = in[i < end ? i : end - 1];
        }
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            uint64_t i = base + (uint64_t)j * THREADS + threadIdx.x;
            if (i < end) atomicAdd(&lds_hist[dig(v[j])], 1u);
        }
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < nbins; d += THREADS)
        counts[(uint64_t)d * nwg + blockIdx.x] = lds_hist[d];
}

// per digit: exclusive scan of counts[d][0..nwg) in place, total -> totals[d]
__global__ void __launch_bounds__(256)
k_scanrow(uint32_t* __restrict__ counts, uint32_t nwg,
          uint64_t* __restrict__ totals) {
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

// one workgroup: starts[d] = sum_{d'<d} (padded ? align(tot) : tot)
__global__ void __launch_bounds__(256)
k_scandig(const uint64_t* __restrict__ totals, uint32_t nbins, int padded,
          uint64_t* __restrict__ starts, int64_t* __restrict__ hist_out,
          int64_t* __restrict__ off_out) {
    __shared__ uint64_t sh[256];
    const uint32_t per = (nbins + 255) / 256;
    const uint32_t b = threadIdx.x * per;
    uint64_t loc = 0;
    for (uint32_t k = 0; k < per; k++) {
        if (b + k < nbins) {
            uint64_t t = totals[b + k];
            loc += padded ? align_tuples(t) : t;
        }
    }
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
            uint64_t t = totals[d];
            starts[d] = ex;
            if (hist_out) hist_out[d] = (int64_t)t;
            if (off_out) off_out[d] = (int64_t)ex;
            ex += padded ? align_tuples(t) : t;
        }
    }
}

// ---------------------------------------------------------------------------
// stable scatter.  Dynamic LDS layout (16-byte aligned pieces):
//   stage  : TILE Tups
//   run    : nbins uint64  (this workgroup's next output slot per digit)
//   tstart : nbins uint32  (tile-exclusive start of every digit)
//   wcnt   : WAVES * nbins uint16 (per-wave counts -> per-wave offsets)
//   scr    : 16 uint32
template <int THREADS, int ITEMS>
constexpr size_t scatter_lds(uint32_t nbins) {
    return (size_t)THREADS * ITEMS * sizeof(Tup) + (size_t)nbins * 8 +
           (size_t)nbins * 4 + (size_t)(THREADS / 64) * nbins * 2 + 64;
}

template <int THREADS, int ITEMS, class Digit>
__global__ void __launch_bounds__(THREADS)
k_scatter(const Tup* __restrict__ in, uint64_t n, uint64_t chunk, Digit dig_arg,
          uint32_t nbins, uint32_t dbits, const uint32_t* __restrict__ counts,
          uint32_t nwg, const uint64_t* __restrict__ starts,
          Tup* __restrict__ out) {
    const auto dig = dig_arg.load();
    constexpr int TILE = THREADS * ITEMS;
    constexpr int WAVES = THREADS / 64;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    Tup* stage = reinterpret_cast<Tup*>(lds_raw);
    uint64_t* run = reinterpret_cast<uint64_t*>(lds_raw + TILE * sizeof(Tup));
    uint32_t* tstart = reinterpret_cast<uint32_t*>(run + nbins);
    uint16_t* wcnt = reinterpret_cast<uint16_t*>(tstart + nbins);
    uint32_t* scr = reinterpret_cast<uint32_t*>(wcnt + ((WAVES * nbins + 7) & ~7u));

    const int lane = lane_id();
    const int wid = threadIdx.x >> 6;
    const uint64_t lt = lanemask_lt();

    for (uint32_t d = threadIdx.x; d < nbins; d += THREADS) {
        run[d] = starts[d] + counts[(uint64_t)d * nwg + blockIdx.x];
#pragma unroll
        for (int w = 0; w < WAVES; w++) wcnt[w * nbins + d] = 0;
    }
    __syncthreads();

    const uint64_t beg = (uint64_t)blockIdx.x * chunk;
    uint64_t end = beg + chunk;
    if (end > n) end = n;
    // digits handled by this thread in the per-tile scans (contiguous range)
    const uint32_t dper = (nbins + THREADS - 1) / THREADS;
    const uint32_t d0 = threadIdx.x * dper;

    for (uint64_t base = beg; base < end; base += TILE) {
        const uint32_t tcount =
            (uint32_t)((end - base) < (uint64_t)TILE ? (end - base) : TILE);
        // wave `wid` owns items [wid*64*ITEMS, (wid+1)*64*ITEMS) of the tile
        Tup v[ITEMS];
        uint32_t dg[ITEMS];
        uint32_t rk[ITEMS];
        const uint32_t wbase = wid * 64 * ITEMS;
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            uint32_t li = wbase + j * 64 + lane;
            if (li < tcount) v[j] = in[base + li];
        }
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            uint32_t li = wbase + j * 64 + lane;
            dg[j] = li < tcount ? dig(v[j]) : 0xffffffffu;
        }
        uint16_t* mycnt = wcnt + wid * nbins;
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const bool valid = dg[j] != 0xffffffffu;
            uint64_t peers = __ballot(valid);
            const uint32_t d = valid ? dg[j] : 0;
            for (uint32_t b = 0; b < dbits; b++) {
                const bool bit = (d >> b) & 1u;
                const uint64_t bal = __ballot(bit);
                peers &= bit ? bal : ~bal;
            }
            uint32_t before = 0;
            if (valid) before = mycnt[d];
            const uint32_t r = (uint32_t)__popcll(peers & lt);
            const uint32_t c = (uint32_t)__popcll(peers);
            // lowest lane of the peer group publishes the new count
            if (valid && r == 0) mycnt[d] = (uint16_t)(before + c);
            rk[j] = before + r;
        }
        __syncthreads();
        // per digit: total over waves, tile exclusive scan, per-wave offsets
        uint32_t loc = 0;
        for (uint32_t k = 0; k < dper; k++) {
            uint32_t d = d0 + k;
            if (d < nbins) {
#pragma unroll
                for (int w = 0; w < WAVES; w++) loc += wcnt[w * nbins + d];
            }
        }
        uint32_t tot;
        uint32_t ex = block_exclusive_scan(loc, scr, &tot);
        for (uint32_t k = 0; k < dper; k++) {
            uint32_t d = d0 + k;
            if (d < nbins) {
                tstart[d] = ex;
#pragma unroll
                for (int w = 0; w < WAVES; w++) {
                    uint32_t c = wcnt[w * nbins + d];
                    wcnt[w * nbins + d] = (uint16_t)ex;
                    ex += c;
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            if (dg[j] != 0xffffffffu) stage[mycnt[dg[j]] + rk[j]] = v[j];
        }
        __syncthreads();
#pragma unroll 4
        for (uint32_t i = threadIdx.x; i < tcount; i += THREADS) {
            Tup t = stage[i];
            uint32_t d = dig(t);
            out[run[d] + (i - tstart[d])] = t;
        }
        __syncthreads();
        for (uint32_t k = 0; k < dper; k++) {
            uint32_t d = d0 + k;
            if (d < nbins) {
                uint32_t nxt = (d + 1 < nbins) ? tstart[d + 1] : tcount;
                run[d] += nxt - tstart[d];
#pragma unroll
                for (int w = 0; w < WAVES; w++) wcnt[w * nbins + d] = 0;
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Stable scatter with write combining (partition_relation[_optimized]): the
// ranks of k_scatter (ballot matching, per-wave counters: input order kept
// inside every digit), the tile's runs prepended with each partition's carry
// (the tail of this workgroup's output that does not yet end on a 64-byte
// boundary), and SEG consecutive lanes write one aligned 64-byte segment --
// the reference's cache-line write-combining buffers
// (src/partition/partition.c:38-46, 191-206) with whole-segment stores.  The
// next tile is loaded while the current one is ranked and written.
template <int THREADS, int ITEMS>
struct SwcGeom {
    static constexpr uint32_t SEG = 64 / sizeof(Tup);
    static constexpr uint32_t TILE = THREADS * ITEMS;
    static constexpr uint32_t WAVES = THREADS / 64;
    static __host__ __device__ constexpr uint32_t max_segs(uint32_t nbins) {
        return (TILE + nbins * (SEG - 1)) / SEG + 2 * nbins;
    }
    // stage Tup[TILE] | carry Tup[nbins * (SEG-1)] | run u64[nbins] |
    // tstart, kc, segpre, emit u32[nbins] | wcnt u16[WAVES * nbins] |
    // segown u16[max_segs] | scan scratch
    static __host__ __device__ constexpr size_t lds_bytes(uint32_t nbins) {
        return (size_t)TILE * sizeof(Tup) + (size_t)nbins * (SEG - 1) * sizeof(Tup) +
               (size_t)nbins * (8 + 4 * 4) + (size_t)WAVES * nbins * 2 +
               ((size_t)max_segs(nbins) * 2 + 15) / 16 * 16 + 64;
    }
};

template <int THREADS, int ITEMS, class Digit>
__global__ void __launch_bounds__(THREADS)
k_scatter_swc(const Tup* __restrict__ in, uint64_t n, uint64_t chunk, Digit dig_arg,
              uint32_t nbins, uint32_t dbits, const uint32_t* __restrict__ counts,
              uint32_t nwg, const uint64_t* __restrict__ starts, Tup* __restrict__ out) {
    typedef SwcGeom<THREADS, ITEMS> Geo;
    constexpr uint32_t SEG = Geo::SEG;
    constexpr uint32_t CW = SEG - 1;  // carry slots per partition
    constexpr int TILE = (int)Geo::TILE;
    constexpr int WAVES = (int)Geo::WAVES;
    const auto dig = dig_arg.load();
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    Tup* stage = reinterpret_cast<Tup*>(lds_raw);
    Tup* carry = stage + TILE;
    uint64_t* run = reinterpret_cast<uint64_t*>(carry + (size_t)nbins * CW);
    uint32_t* tstart = reinterpret_cast<uint32_t*>(run + nbins);
    uint32_t* kc = tstart + nbins;
    uint32_t* segpre = kc + nbins;
    uint32_t* emit = segpre + nbins;
    uint16_t* wcnt = reinterpret_cast<uint16_t*>(emit + nbins);
    uint16_t* segown = wcnt + (size_t)WAVES * nbins;
    uint32_t* scr = reinterpret_cast<uint32_t*>(
        reinterpret_cast<unsigned char*>(segown) + ((size_t)Geo::max_segs(nbins) * 2 + 15) / 16 * 16);

    const int lane = lane_id();
    const int wid = threadIdx.x >> 6;
    const uint64_t lt = lanemask_lt();
    for (uint32_t d = threadIdx.x; d < nbins; d += THREADS) {
        run[d] = starts[d] + counts[(uint64_t)d * nwg + blockIdx.x];
        kc[d] = 0;
#pragma unroll
        for (int w = 0; w < WAVES; w++) wcnt[w * nbins + d] = 0;
    }
    const uint64_t beg = (uint64_t)blockIdx.x * chunk;
    uint64_t end = beg + chunk;
    if (end > n) end = n;
    const uint32_t dper = (nbins + THREADS - 1) / THREADS;
    const uint32_t d0 = threadIdx.x * dper;
    // wave `wid` owns items [wid*64*ITEMS, (wid+1)*64*ITEMS) of a tile
    const uint32_t wbase = wid * 64 * ITEMS;
    Tup v[ITEMS], nv[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        const uint64_t i = beg + wbase + j * 64 + lane;
        if (i < end) v[j] = in[i];
    }
    __syncthreads();
    for (uint64_t base = beg; base < end; base += TILE) {
        const uint32_t tcount =
            (uint32_t)((end - base) < (uint64_t)TILE ? (end - base) : TILE);
        __builtin_amdgcn_s_waitcnt(0x0f70);  // this tile's loads have landed
        uint32_t dg[ITEMS], rk[ITEMS];
        uint16_t* mycnt = wcnt + wid * nbins;
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint32_t li = wbase + j * 64 + lane;
            dg[j] = li < tcount ? dig(v[j]) : 0xffffffffu;
            const bool valid = dg[j] != 0xffffffffu;
            uint64_t peers = __ballot(valid);
            const uint32_t d = valid ? dg[j] : 0;
            for (uint32_t b = 0; b < dbits; b++) {
                const bool bit = (d >> b) & 1u;
                const uint64_t bal = __ballot(bit);
                peers &= bit ? bal : ~bal;
            }
            uint32_t before = 0;
            if (valid) before = mycnt[d];
            const uint32_t r = (uint32_t)__popcll(peers & lt);
            if (valid && r == 0) mycnt[d] = (uint16_t)(before + __popcll(peers));
            rk[j] = before + r;
        }
        __syncthreads();
        // ---- per digit: tile count, stage start, per-wave offsets, and the
        // emission: everything up to the last 64-byte boundary (E of the
        // T = carry + tile elements) as whole aligned segments
        uint32_t c[4], E[4], ns[4];  // dper <= 4 (nbins <= 4 * THREADS)
        uint32_t loc = 0;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const uint32_t d = d0 + k;
            c[k] = E[k] = ns[k] = 0;
            if (k < dper && d < nbins) {
#pragma unroll
                for (int w = 0; w < WAVES; w++) c[k] += wcnt[w * nbins + d];
                const uint64_t p = run[d];
                const uint32_t T = kc[d] + c[k];
                const uint32_t m = (uint32_t)((p + T) % SEG);
                E[k] = m <= T ? T - m : 0u;
                ns[k] = E[k] ? (uint32_t)((p + E[k] - (p - p % SEG)) / SEG) : 0u;
                loc += c[k] | (ns[k] << 16);
            }
        }
        uint32_t tot;
        uint32_t ex = block_exclusive_scan(loc, scr, &tot);
        const uint32_t nsegT = tot >> 16;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const uint32_t d = d0 + k;
            if (k < dper && d < nbins) {
                tstart[d] = ex & 0xffffu;
                segpre[d] = ex >> 16;
                emit[d] = E[k];
                uint32_t o = ex & 0xffffu;
#pragma unroll
                for (int w = 0; w < WAVES; w++) {
                    const uint32_t cw = wcnt[w * nbins + d];
                    wcnt[w * nbins + d] = (uint16_t)o;
                    o += cw;
                }
                for (uint32_t q = 0; q < ns[k]; q++) segown[(ex >> 16) + q] = (uint16_t)d;
                ex += c[k] | (ns[k] << 16);
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
            if (dg[j] != 0xffffffffu) stage[mycnt[dg[j]] + rk[j]] = v[j];
        __syncthreads();
        // ---- whole segments: SEG consecutive lanes per aligned 64-byte block
        for (uint32_t q = threadIdx.x; q < nsegT * SEG; q += THREADS) {
            const uint32_t sg = q / SEG;
            const uint32_t d = segown[sg];
            const uint64_t p = run[d];
            const uint64_t addr = p - p % SEG + (uint64_t)(sg - segpre[d]) * SEG + q % SEG;
            if (addr >= p && addr < p + emit[d]) {
                const uint32_t e = (uint32_t)(addr - p);
                const uint32_t k = kc[d];
                out[addr] = e < k ? carry[d * CW + e] : stage[tstart[d] + e - k];
            }
        }
        __syncthreads();
        // ---- leftovers (< SEG) become the carry; counters for the next tile
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const uint32_t d = d0 + k;
            if (k < dper && d < nbins) {
                const uint32_t kk = kc[d];
                const uint32_t T = kk + c[k];
                for (uint32_t e = E[k]; e < T; e++)
                    carry[d * CW + (e - E[k])] =
                        e < kk ? carry[d * CW + e] : stage[tstart[d] + e - kk];
                run[d] += E[k];
                kc[d] = T - E[k];
#pragma unroll
                for (int w = 0; w < WAVES; w++) wcnt[w * nbins + d] = 0;
            }
        }
#pragma unroll
        for (int j = 0; j < ITEMS; j++) v[j] = nv[j];
        __syncthreads();
    }
    // ---- the partial last segments of this workgroup's regions
    for (uint32_t q = threadIdx.x; q < nbins * CW; q += THREADS) {
        const uint32_t d = q / CW, j = q % CW;
        if (j < kc[d]) out[run[d] + j] = carry[q];
    }
}

// ---------------------------------------------------------------------------
// Stable scatter with write combining and ATOMIC ranks (partition_relation
// [_optimized] for 1..10 radix bits; src/partition/partition.c:152-219).
//
// Ranks: a wave ranks its items step by step (item j of every lane = input
// elements wbase + 64 j + lane, in input order) with one LDS atomic add per
// element on a per-wave 16-bit digit counter (two digits per 32-bit word).
// When several lanes of one ds_add_rtn instruction hit the same word, gfx950
// returns their old values in lane order (tools/ldsorder.hip: 0 violations in
// ~1.6e10 colliding lane updates; tests/test_gpu_parity.py re-checks it
// through smj_selfcheck_lds_order), so the returned count is the element's
// stable rank inside the wave -- one LDS op per element instead of one ballot
// per digit bit.  Per-wave counts -> tile offsets by the owner of each digit
// pair (thread t owns digits 2t, 2t+1) and one packed scan.
//
// Writes: each digit's output region of this workgroup is emitted in whole
// aligned 64-byte segments, SEG consecutive lanes per segment; the tail of a
// tile that does not fill a segment stays in an LDS carry and leads the
// digit's next segment (the reference's cache-line write-combining buffers,
// src/partition/partition.c:38-46).  Only the region's first and last segment
// are partial.
//
// MI355X, 2^27 tuples, 10 bits (tools/partlab.hip): 8 B 0.73 ms, 16 B 1.14 ms
// for the first form of this scatter, against 1.46 / 1.51 ms for
// k_scatter_swc (ballot ranks) and 0.84 ms for the same atomic ranks without
// the carry (34 % extra write bytes, 41 % partial write requests).
#ifndef SMJ_SWP_SEG
#define SMJ_SWP_SEG 64  // bytes a segment of the stable scatter
#endif
template <int THREADS, int ITEMS>
struct SwaGeom {
    static constexpr int W = THREADS / 64;
    static constexpr int TILE = THREADS * ITEMS;
    static constexpr uint32_t SEG = SMJ_SWP_SEG / sizeof(Tup);
    static constexpr uint32_t CW = SEG - 1;
    // stage Tup[TILE] | carry Tup[B][CW] | counters u32[W][B/2] | info u32x4[B] |
    // segown u16[TILE/SEG + 2B] | scan scratch
    static __host__ __device__ constexpr size_t lds_bytes(uint32_t B) {
        return (size_t)TILE * sizeof(Tup) + (size_t)B * CW * sizeof(Tup) + (size_t)W * B * 2 +
               (size_t)B * 16 + ((size_t)(TILE / SEG + 2 * B) * 2 + 15) / 16 * 16 + 128;
    }
};

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

// s_waitcnt immediate for vmcnt(N), expcnt and lgkmcnt left free (gfx9 layout:
// vmcnt[3:0] + vmcnt[5:4] at bits 15:14)
constexpr int vmcnt_imm(int n) { return (n & 15) | ((n >> 4) << 14) | 0x0f70; }

// k_scatter_swp: the next-but-one tile's loads are in flight: three register
// tiles rotate (the loop is unrolled by three so that no tile is copied
// between registers -- a copy would wait for its loads), and the wait before a
// tile's segment stores is vmcnt(ITEMS): everything but the loads issued in
// this tile (the next-but-one) has landed, i.e. the next tile and the previous
// tile's stores.  The loads thus fly under a whole tile of LDS work instead of
// the stage phase alone.  Loads are non-temporal (NT; the input is read
// once), 8-byte tuples leave in 16-byte pair stores.
template <int THREADS, int ITEMS, class DigitL, bool NT>
struct SwpTile {
    // info[d][3] = segment start (12 bits) | carry size (3) | emission + carry (17)
    static_assert(SwaGeom<THREADS, ITEMS>::TILE / SwaGeom<THREADS, ITEMS>::SEG + 2 * 1024 <= 4096,
                  "segment numbers fit 12 bits");
    static_assert(SwaGeom<THREADS, ITEMS>::CW <= 7, "carry size fits 3 bits");
    static_assert(SwaGeom<THREADS, ITEMS>::TILE + 8 < (1 << 17), "T fits 17 bits");
    typedef SwaGeom<THREADS, ITEMS> G;
    static constexpr int W = G::W;
    static constexpr int TILE = G::TILE;
    static constexpr uint32_t SEG = G::SEG;
    static constexpr uint32_t CW = G::CW;
    const Tup* __restrict__ in;
    Tup* __restrict__ out;
    DigitL dig;
    Tup* stage;
    Tup* carry;
    uint32_t* w32;
    u32x4_t* info;
    uint16_t* segown;
    uint32_t* scr;
    uint32_t hb, t2, wbase;
    int lane, wid;
    bool owner;
    bool pairs;  // 8-byte tuples, 16-byte aligned output: pair stores
    uint64_t end;
    uint32_t pos[2], kc[2];

    // exclusive scan over the workgroup (v < 2^32 in total): wave scan by
    // shuffles, wave totals through LDS, one barrier (the scratch is next
    // written a tile later, after several barriers)
    __device__ __forceinline__ uint32_t scan(uint32_t v, uint32_t* total) const {
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

    __device__ __forceinline__ void load(Tup (&v)[ITEMS], uint64_t base) const {
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint64_t i = base + wbase + j * 64 + lane;
            const uint64_t c = i < end ? i : end - 1;  // unconditional: a fixed count in flight
            v[j] = NT ? ld_nt(in + c) : in[c];
        }
    }

    __device__ __forceinline__ void tile(const Tup (&v)[ITEMS], Tup (&pre)[ITEMS],
                                         uint64_t base) {
        const uint32_t tcount = (uint32_t)min((uint64_t)TILE, end - base);
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
        const uint32_t ex = scan((c[0] + c[1]) | ((ns[0] + ns[1]) << 16), &tot);
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
                I[3] = sp[h] | (kc[h] << 12) | ((kc[h] + c[h]) << 15);
                info[d] = I;
                for (uint32_t k = 0; k < ns[h]; k++) segown[sp[h] + k] = (uint16_t)d;
            }
        }
        // the next-but-one tile (its registers held the previous tile)
        load(pre, base + 2 * (uint64_t)TILE);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < ITEMS; j++)
            if (dg[j] != 0xffffffffu) {
                const uint32_t d = dg[j];
                const uint32_t wo = (w32[wid * hb + (d >> 1)] >> ((d & 1u) * 16u)) & 0xffffu;
                stage[wo + rk[j]] = v[j];
            }
        __syncthreads();
        if (owner) {
#pragma unroll
            for (int w = 0; w < W; w++) w32[w * hb + t2] = 0;
        }
        // the next tile and the previous tile's stores have landed; the
        // next-but-one tile's ITEMS loads stay in flight
        __builtin_amdgcn_s_waitcnt(vmcnt_imm(ITEMS));
#ifndef KEY_8B
        // 8-byte tuples: a lane writes two adjacent tuples of a segment with
        // one 16-byte store (SEG / 2 lanes per segment); a pair cut by its
        // region's first or last partial segment stores its one tuple alone
        if (NT && pairs) {
            typedef unsigned long long V2 __attribute__((ext_vector_type(2)));
            constexpr uint32_t PS = SEG / 2;
            for (uint32_t q = threadIdx.x; q < nsegT * PS; q += THREADS) {
                const uint32_t sg = q / PS;
                const uint32_t d = segown[sg];
                const u32x4_t I = info[d];
                const uint32_t p = I[0];
                const uint32_t a0 = (p / SEG + (sg - (I[3] & 0xfffu))) * SEG + 2 * (q % PS);
                const uint32_t k = (I[3] >> 12) & 7u;
                const bool v0 = a0 >= p && a0 < p + I[1];
                const bool v1 = a0 + 1 >= p && a0 + 1 < p + I[1];
                const uint32_t e0 = a0 - p, e1 = a0 + 1 - p;
                const Tup x0 = e0 < k ? carry[d * CW + e0] : stage[v0 ? I[2] + e0 - k : 0u];
                const Tup x1 = e1 < k ? carry[d * CW + e1] : stage[v1 ? I[2] + e1 - k : 0u];
                if (v0 && v1) {
                    V2 y;
                    y.x = x0;
                    y.y = x1;
                    __builtin_nontemporal_store(y, reinterpret_cast<V2*>(out + a0));
                } else if (v0) {
                    st_stream(out + a0, x0);
                } else if (v1) {
                    st_stream(out + a0 + 1, x1);
                }
            }
        } else
#endif
        for (uint32_t q = threadIdx.x; q < nsegT * SEG; q += THREADS) {
            const uint32_t sg = q / SEG;
            const uint32_t d = segown[sg];
            const u32x4_t I = info[d];
            const uint32_t p = I[0];
            const uint32_t addr = (p / SEG + (sg - (I[3] & 0xfffu))) * SEG + q % SEG;
            if (addr >= p && addr < p + I[1]) {
                const uint32_t e = addr - p;
                const uint32_t k = (I[3] >> 12) & 7u;
                const Tup x = e < k ? carry[d * CW + e] : stage[I[2] + e - k];
                if (NT)
                    st_stream(out + addr, x);
                else
                    out[addr] = x;
            }
        }
        __syncthreads();
        // ---- the owner's leftovers (< SEG) become the carry.  An emission
        // (E > 0) ends on a segment boundary past the old carry (E > kc), so
        // the new carry comes from the stage alone; without one the old carry
        // stays in place and the tile's elements follow it.  All stage reads
        // are issued before the carry writes (no read-after-write chain).
        if (owner) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const uint32_t d = 2 * t2 + h;
                const uint32_t T = kc[h] + c[h];
                Tup x[CW];
#pragma unroll
                for (uint32_t j = 0; j < CW; j++) {
                    const uint32_t e = E[h] + j;
                    x[j] = stage[e >= kc[h] && e < T ? ts[h] + e - kc[h] : 0u];
                }
#pragma unroll
                for (uint32_t j = 0; j < CW; j++) {
                    const uint32_t e = E[h] + j;
                    if (e >= kc[h] && e < T) carry[d * CW + j] = x[j];
                }
                pos[h] += E[h];
                kc[h] = T - E[h];
            }
        }
    }
};

template <int THREADS, int ITEMS, class Digit, bool NT>
__global__ void __launch_bounds__(THREADS)
k_scatter_swp(const Tup* __restrict__ in, uint64_t n, uint64_t chunk, Digit dig_arg,
              uint32_t nbins, const uint32_t* __restrict__ counts, uint32_t nwg,
              const uint64_t* __restrict__ starts, Tup* __restrict__ out, int pairs_ok) {
    typedef SwpTile<THREADS, ITEMS, decltype(dig_arg.load()), NT> P;
    constexpr int W = P::W;
    constexpr int TILE = P::TILE;
    constexpr uint32_t SEG = P::SEG;
    constexpr uint32_t CW = P::CW;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    P s;
    s.in = in;
    s.out = out;
    s.dig = dig_arg.load();
    s.stage = reinterpret_cast<Tup*>(lds_raw);
    s.carry = s.stage + TILE;
    s.w32 = reinterpret_cast<uint32_t*>(s.carry + (size_t)nbins * CW);
    s.hb = nbins / 2;
    s.info = reinterpret_cast<u32x4_t*>(s.w32 + (size_t)W * s.hb);
    s.segown = reinterpret_cast<uint16_t*>(s.info + nbins);
    s.scr = reinterpret_cast<uint32_t*>(s.segown + ((TILE / SEG + 2 * nbins + 7) & ~7u));
    s.lane = lane_id();
    s.wid = threadIdx.x >> 6;
    s.t2 = threadIdx.x;
    s.owner = s.t2 < s.hb;
    s.pairs = sizeof(Tup) == 8 && pairs_ok && ((uintptr_t)out & 15) == 0;
    s.pos[0] = s.pos[1] = s.kc[0] = s.kc[1] = 0;
    if (s.owner) {
#pragma unroll
        for (int h = 0; h < 2; h++)
            s.pos[h] = (uint32_t)(starts[2 * s.t2 + h] +
                                  counts[(uint64_t)(2 * s.t2 + h) * nwg + blockIdx.x]);
    }
    for (uint32_t q = threadIdx.x; q < W * s.hb; q += THREADS) s.w32[q] = 0;
    const uint64_t beg = (uint64_t)blockIdx.x * chunk;
    s.end = min(beg + chunk, n);
    s.wbase = s.wid * 64 * ITEMS;
    Tup a[ITEMS], b[ITEMS], c[ITEMS];
    s.load(a, beg);
    s.load(b, beg + TILE);
    __builtin_amdgcn_s_waitcnt(vmcnt_imm(ITEMS));  // the first tile
    __syncthreads();
    for (uint64_t base = beg;;) {
        s.tile(a, c, base);
        if ((base += TILE) >= s.end) break;
        s.tile(b, a, base);
        if ((base += TILE) >= s.end) break;
        s.tile(c, b, base);
        if ((base += TILE) >= s.end) break;
    }
    // the partial last segment of every region (carry slots are written by
    // every thread of the last tile's carry phase)
    __syncthreads();
    if (s.owner) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const uint32_t d = 2 * s.t2 + h;
            for (uint32_t e = 0; e < s.kc[h]; e++) out[s.pos[h] + e] = s.carry[d * CW + e];
        }
    }
}


// Histogram of the stable write-combining partition: counts[d][wg] of each
// workgroup's chunk (the scatter's chunking), two register tiles alternating
// (the next tile's loads fly while this one is counted).  Loads are
// unconditional (clamped to the chunk) so that every load of a tile is in
// flight at once.
template <int THREADS, int ITEMS, class Digit, bool NT>
__global__ void __launch_bounds__(THREADS)
k_hist_p(const Tup* __restrict__ in, uint64_t n, uint64_t chunk, Digit dig_arg,
         uint32_t nbins, uint32_t* __restrict__ counts, uint32_t nwg) {
    const auto dig = dig_arg.load();
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_hp[];
    for (uint32_t d = threadIdx.x; d < nbins; d += THREADS) lds_hp[d] = 0;
    __syncthreads();
    const uint64_t beg = (uint64_t)blockIdx.x * chunk;
    const uint64_t end = min(beg + chunk, n);
    constexpr int TILE = THREADS * ITEMS;
    Tup a[ITEMS], b[ITEMS];
    auto load = [&](Tup (&v)[ITEMS], uint64_t base) {
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint64_t i = base + (uint64_t)j * THREADS + threadIdx.x;
            const uint64_t c = i < end ? i : end - 1;
            v[j] = NT ? ld_nt(in + c) : in[c];
        }
    };
    auto count = [&](const Tup (&v)[ITEMS], uint64_t base) {
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint64_t i = base + (uint64_t)j * THREADS + threadIdx.x;
            if (i < end) atomicAdd(&lds_hp[dig(v[j])], 1u);
        }
    };
    if (beg < end) load(a, beg);
    for (uint64_t base = beg; base < end;) {
        load(b, base + TILE);
        count(a, base);
        if ((base += TILE) >= end) break;
        load(a, base + TILE);
        count(b, base);
        base += TILE;
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < nbins; d += THREADS)
        counts[(uint64_t)d * nwg + blockIdx.x] = lds_hp[d];
}

// 8-byte tuples: k_hist_p with 16-byte loads (two tuples per lane and load,
// non-temporal), for a 16-byte aligned input and even chunks; the odd last
// tuple of the input is counted by thread 0 of the last workgroup.
typedef unsigned long long HvVec __attribute__((ext_vector_type(2)));
template <int THREADS, int VITEMS, class Digit>
__global__ void __launch_bounds__(THREADS)
k_hist_v(const Tup* __restrict__ in, uint64_t n, uint64_t chunk, Digit dig_arg,
         uint32_t nbins, uint32_t* __restrict__ counts, uint32_t nwg) {
    static_assert(sizeof(Tup) == 8, "8-byte tuples");
    const auto dig = dig_arg.load();
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_hv[];
    for (uint32_t d = threadIdx.x; d < nbins; d += THREADS) lds_hv[d] = 0;
    __syncthreads();
    const uint64_t beg = (uint64_t)blockIdx.x * chunk;
    const uint64_t end = min(beg + chunk, n);
    const HvVec* __restrict__ vin = reinterpret_cast<const HvVec*>(in);
    const uint64_t vb = beg / 2, ve = end / 2;  // whole pairs of the chunk
    constexpr int TILE = THREADS * VITEMS;
    HvVec a[VITEMS], b[VITEMS];
    auto load = [&](HvVec (&v)[VITEMS], uint64_t base) {
#pragma unroll
        for (int j = 0; j < VITEMS; j++) {
            const uint64_t i = base + (uint64_t)j * THREADS + threadIdx.x;
            v[j] = __builtin_nontemporal_load(vin + (i < ve ? i : ve - 1));
        }
    };
    auto count = [&](const HvVec (&v)[VITEMS], uint64_t base) {
#pragma unroll
        for (int j = 0; j < VITEMS; j++) {
            const uint64_t i = base + (uint64_t)j * THREADS + threadIdx.x;
            if (i < ve) {
                atomicAdd(&lds_hv[dig((Tup)v[j].x)], 1u);
                atomicAdd(&lds_hv[dig((Tup)v[j].y)], 1u);
            }
        }
    };
    if (vb < ve) load(a, vb);
    for (uint64_t base = vb; base < ve;) {
        load(b, base + TILE);
        count(a, base);
        if ((base += TILE) >= ve) break;
        load(a, base + TILE);
        count(b, base);
        base += TILE;
    }
    if (threadIdx.x == 0 && (end & 1) && end > beg) atomicAdd(&lds_hv[dig(in[end - 1])], 1u);
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < nbins; d += THREADS)
        counts[(uint64_t)d * nwg + blockIdx.x] = lds_hv[d];
}

// Unstable scatter for the join's level-1 partition (the join re-sorts every
// bucket completely, so the order inside a partition is free).  Ranks come
// from LDS atomics on tile-level digit counters -- two ds_add per tuple instead
// of a ballot per digit bit -- and the next tile's tuples are loaded while the
// current tile is ranked, staged and written.
// LDS: stage TILE Tups | run nbins u64 | tstart nbins u32 | tfill nbins u32
template <int THREADS, int ITEMS>
constexpr size_t scatter_u_lds(uint32_t nbins) {
    return (size_t)THREADS * ITEMS * sizeof(Tup) + (size_t)nbins * 16 + 64;
}

template <int THREADS, int ITEMS, class Digit, class Pack = PackNone>
__global__ void __launch_bounds__(THREADS)
k_scatter_u(const Tup* __restrict__ in, uint64_t n, uint64_t chunk, Digit dig_arg,
            uint32_t nbins, const uint32_t* __restrict__ counts, uint32_t nwg,
            const uint64_t* __restrict__ starts, typename Pack::OutT* __restrict__ out,
            Pack pk = Pack(), unsigned int* __restrict__ bad_flag = nullptr) {
    const auto dig = dig_arg.load();
    uint32_t bad = 0;
    constexpr int TILE = THREADS * ITEMS;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    Tup* stage = reinterpret_cast<Tup*>(lds_raw);
    uint64_t* run = reinterpret_cast<uint64_t*>(lds_raw + TILE * sizeof(Tup));
    uint32_t* tstart = reinterpret_cast<uint32_t*>(run + nbins);
    uint32_t* tfill = tstart + nbins;
    uint32_t* scr = tfill + nbins;

    for (uint32_t d = threadIdx.x; d < nbins; d += THREADS) {
        run[d] = starts[d] + counts[(uint64_t)d * nwg + blockIdx.x];
        tfill[d] = 0;
    }
    const uint64_t beg = (uint64_t)blockIdx.x * chunk;
    uint64_t end = beg + chunk;
    if (end > n) end = n;
    const uint32_t dper = (nbins + THREADS - 1) / THREADS;
    const uint32_t d0 = threadIdx.x * dper;

    Tup v[ITEMS], nv[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        const uint64_t i = beg + (uint64_t)j * THREADS + threadIdx.x;
        if (i < end) v[j] = in[i];
    }
    __syncthreads();
    for (uint64_t base = beg; base < end; base += TILE) {
        const uint32_t tcount =
            (uint32_t)((end - base) < (uint64_t)TILE ? (end - base) : TILE);
        // prefetch the next tile
        const uint64_t nb = base + TILE;
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint64_t i = nb + (uint64_t)j * THREADS + threadIdx.x;
            if (i < end) nv[j] = in[i];
        }
        uint32_t dg[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint32_t li = j * THREADS + threadIdx.x;
            dg[j] = li < tcount ? dig(v[j]) : 0xffffffffu;
            if (dg[j] != 0xffffffffu) atomicAdd(&tfill[dg[j]], 1u);
        }
        __syncthreads();
        uint32_t loc = 0;
        for (uint32_t k = 0; k < dper; k++)
            if (d0 + k < nbins) loc += tfill[d0 + k];
        uint32_t tot;
        uint32_t ex = block_exclusive_scan(loc, scr, &tot);
        for (uint32_t k = 0; k < dper; k++) {
            const uint32_t d = d0 + k;
            if (d < nbins) {
                const uint32_t c = tfill[d];
                tstart[d] = ex;
                tfill[d] = ex;
                ex += c;
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            if (dg[j] != 0xffffffffu) stage[atomicAdd(&tfill[dg[j]], 1u)] = v[j];
        }
        __syncthreads();
#pragma unroll 4
        for (uint32_t i = threadIdx.x; i < tcount; i += THREADS) {
            const Tup t = stage[i];
            const uint32_t d = dig(t);
            out[run[d] + (i - tstart[d])] = pk(t, bad);
        }
        __syncthreads();
        for (uint32_t k = 0; k < dper; k++) {
            const uint32_t d = d0 + k;
            if (d < nbins) {
                run[d] += tfill[d] - tstart[d];
                tfill[d] = 0;
            }
        }
#pragma unroll
        for (int j = 0; j < ITEMS; j++) v[j] = nv[j];
        __syncthreads();
    }
    if (bad_flag && bad) atomicOr(bad_flag, bad);
}

// Write-combining scatter for the join's level-1 partition (order inside a
// partition is free).  The reference flushes 64-byte software write-combining
// buffers per partition (src/partition/partition.c:38-46, 191-206); here each
// workgroup keeps, per partition, the tail of its output that does not yet
// fill a 64-byte segment in an LDS carry buffer and prepends it to the next
// tile's run, so apart from the first and last segment of a workgroup's
// region every store completes a whole aligned segment.  Ranks come from LDS
// atomics; the next tile is loaded while the current one is ranked, staged
// and written.
// LDS: stage TILE | carry nbins*SEG Tups | pos nbins u64 | tstart, tfill, kc
//      nbins u32 each | scan scratch
template <int THREADS, int ITEMS>
constexpr size_t scatter_wc_lds(uint32_t nbins) {
    return (size_t)THREADS * ITEMS * sizeof(Tup) + (size_t)nbins * 64 +
           (size_t)nbins * (8 + 4 + 4 + 4) + 64;
}

template <int THREADS, int ITEMS, class Digit>
__global__ void __launch_bounds__(THREADS)
k_scatter_wc(const Tup* __restrict__ in, uint64_t n, uint64_t chunk, Digit dig_arg,
             uint32_t nbins, const uint32_t* __restrict__ counts, uint32_t nwg,
             const uint64_t* __restrict__ starts, Tup* __restrict__ out) {
    const auto dig = dig_arg.load();
    constexpr int TILE = THREADS * ITEMS;
    constexpr uint32_t SEG = 64 / sizeof(Tup);  // tuples per 64-byte segment
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    Tup* stage = reinterpret_cast<Tup*>(lds_raw);
    Tup* carry = stage + TILE;
    uint64_t* pos = reinterpret_cast<uint64_t*>(carry + (size_t)nbins * SEG);
    uint32_t* tstart = reinterpret_cast<uint32_t*>(pos + nbins);
    uint32_t* tfill = tstart + nbins;
    uint32_t* kc = tfill + nbins;
    uint32_t* scr = kc + nbins;

    for (uint32_t d = threadIdx.x; d < nbins; d += THREADS) {
        pos[d] = starts[d] + counts[(uint64_t)d * nwg + blockIdx.x];
        tfill[d] = 0;
        kc[d] = 0;
    }
    const uint64_t beg = (uint64_t)blockIdx.x * chunk;
    uint64_t end = beg + chunk;
    if (end > n) end = n;
    const uint32_t dper = (nbins + THREADS - 1) / THREADS;
    const uint32_t d0 = threadIdx.x * dper;

    Tup v[ITEMS], nv[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        const uint64_t i = beg + (uint64_t)j * THREADS + threadIdx.x;
        if (i < end) v[j] = in[i];
    }
    __syncthreads();
    for (uint64_t base = beg; base < end; base += TILE) {
        const uint32_t tcount =
            (uint32_t)((end - base) < (uint64_t)TILE ? (end - base) : TILE);
        // prefetch the next tile
        const uint64_t nb = base + TILE;
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint64_t i = nb + (uint64_t)j * THREADS + threadIdx.x;
            if (i < end) nv[j] = in[i];
        }
        // ---- rank: tile counts per partition
        uint32_t dg[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint32_t li = j * THREADS + threadIdx.x;
            dg[j] = li < tcount ? dig(v[j]) : 0xffffffffu;
            if (dg[j] != 0xffffffffu) atomicAdd(&tfill[dg[j]], 1u);
        }
        __syncthreads();
        uint32_t loc = 0;
        for (uint32_t k = 0; k < dper; k++)
            if (d0 + k < nbins) loc += tfill[d0 + k];
        uint32_t tot;
        uint32_t ex = block_exclusive_scan(loc, scr, &tot);
        for (uint32_t k = 0; k < dper; k++) {
            const uint32_t d = d0 + k;
            if (d < nbins) {
                const uint32_t c = tfill[d];
                tstart[d] = ex;
                tfill[d] = ex;
                ex += c;
            }
        }
        __syncthreads();
        // ---- stage the tile grouped by partition
#pragma unroll
        for (int j = 0; j < ITEMS; j++)
            if (dg[j] != 0xffffffffu) stage[atomicAdd(&tfill[dg[j]], 1u)] = v[j];
        __syncthreads();
        // ---- per partition: emit E of the T = carry + tile elements so that
        // the region cursor lands on a segment boundary (tfill := E)
        for (uint32_t k = 0; k < dper; k++) {
            const uint32_t d = d0 + k;
            if (d < nbins) {
                const uint32_t T = kc[d] + (tfill[d] - tstart[d]);
                const uint32_t m = (uint32_t)((pos[d] + T) % SEG);
                tfill[d] = m <= T ? T - m : 0u;
            }
        }
        __syncthreads();
        // ---- emit: old carry first (a carry never moves: it is either
        // emitted whole or kept when nothing is emitted), then the tile
        for (uint32_t q = threadIdx.x; q < nbins * SEG; q += THREADS) {
            const uint32_t d = q / SEG, j = q % SEG;
            if (j < kc[d] && j < tfill[d]) out[pos[d] + j] = carry[q];
        }
        Tup keep[ITEMS];
        uint32_t kslot[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint32_t i = j * THREADS + threadIdx.x;
            kslot[j] = 0xffffffffu;
            if (i < tcount) {
                const Tup t = stage[i];
                const uint32_t d = dig(t);
                const uint32_t vv = kc[d] + (i - tstart[d]);
                const uint32_t E = tfill[d];
                if (vv < E) {
                    out[pos[d] + vv] = t;
                } else {
                    keep[j] = t;
                    kslot[j] = d * SEG + (vv - E);
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < ITEMS; j++)
            if (kslot[j] != 0xffffffffu) carry[kslot[j]] = keep[j];
        __syncthreads();
        for (uint32_t k = 0; k < dper; k++) {
            const uint32_t d = d0 + k;
            if (d < nbins) {
                const uint32_t cnt = ((d + 1 < nbins) ? tstart[d + 1] : tcount) - tstart[d];
                const uint32_t E = tfill[d];
                const uint32_t T = kc[d] + cnt;
                pos[d] += E;
                kc[d] = T - E;
                tfill[d] = 0;
            }
        }
#pragma unroll
        for (int j = 0; j < ITEMS; j++) v[j] = nv[j];
        __syncthreads();
    }
    // ---- flush the carries (partial last segments of this region)
    for (uint32_t q = threadIdx.x; q < nbins * SEG; q += THREADS) {
        const uint32_t d = q / SEG, j = q % SEG;
        if (j < kc[d]) out[pos[d] + j] = carry[q];
    }
}

// ---------------------------------------------------------------------------
// Sampled partitioning (join level 1): no histogram pass.  A strided 1/stride
// sample estimates every partition's size; each partition gets a region of
// 9/8 of the estimate plus slack, and workgroups reserve whole 64-byte
// segments in it with one atomic per (tile, partition) while write-combining
// exactly like k_scatter_wc.  Partitions come out contiguous from their
// region start (unstable order), followed by unused slack.  A region that
// would overflow raises a flag and the caller repeats the exact
// (histogram) partition.
// the relations of one sampled partition launch (blockIdx.y = relation)
struct SampleRel {
    const Tup* in[2];
    uint64_t n[2];
    unsigned int* hist[2];  // nbins counters each, zeroed by the caller
};

template <class Digit>
__global__ void __launch_bounds__(256)
k_sample_hist(SampleRel S, uint32_t stride, Digit dig_arg, uint32_t nbins) {
    const auto dig = dig_arg.load();
    const Tup* __restrict__ in = S.in[blockIdx.y];
    const uint64_t n = S.n[blockIdx.y];
    unsigned int* __restrict__ hist = S.hist[blockIdx.y];
    extern __shared__ unsigned int sh_hist[];
    for (uint32_t d = threadIdx.x; d < nbins; d += 256) sh_hist[d] = 0;
    __syncthreads();
    // sample points every 4 * stride tuples, 4 consecutive tuples each (one
    // 64-byte read for 16-byte tuples): 1/stride of the input
    const uint64_t pstride = 4ull * stride;
    const uint64_t step = (uint64_t)gridDim.x * 256 * pstride;
    // clamped, unconditional loads (a conditional load waits alone)
    for (uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * pstride; i < n; i += step) {
        Tup t[4];
#pragma unroll
        for (int k = 0; k < 4; k++) t[k] = in[i + k < n ? i + k : n - 1];
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (i + k < n) atomicAdd(&sh_hist[dig(t[k])], 1u);
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < nbins; d += 256)
        if (sh_hist[d]) atomicAdd(&hist[d], sh_hist[d]);
}

// one workgroup: region capacities from the sample, their starts, cursors.
// Every partition's region is cut into kShards shards (one per group of
// workgroups, blockIdx % kShards), so that the reservation atomics of a
// partition are spread over kShards cursors (kShards: smj_internal.hpp).

// Write unit of the sampled scatter: a partition's run of a tile is written
// in whole segments of this many bytes (of the first plane), the rest waits in
// the partition's LDS carry for the next tile.  Round 4, with the 48-bit
// layout (tools/r04_sclab.sh, two interleaved rounds on one box,
// profiles/r04_lab/sclab_b.txt, sclab_c.txt): 64 -> 16 bytes took the 16-byte
// join 3.34 / 3.30 -> 3.14 / 3.15 ms, the 8-byte join 2.77 / 2.76 -> 2.68 /
// 2.68, the 8-byte sort 1.50 / 1.53 -> 1.45 / 1.48 (k_scatter -0.06 to -0.1
// ms): the runs are as long either way (one per partition and tile), the
// carries and their per-tile copies shrink.  8 bytes: the scatter no faster,
// the 16-byte join's group pass 0.1 ms slower; 32 between 64 and 16.
#ifndef SMJ_SC_SEG
#define SMJ_SC_SEG 16
#endif
constexpr uint32_t kSegBytes = SMJ_SC_SEG;
constexpr uint32_t kRegionAlign = 128;  // bytes; a multiple of kSegBytes
static_assert(kRegionAlign % kSegBytes == 0, "regions hold whole segments");

// per-relation region tables of one sampled partition launch
struct RegionRel {
    const unsigned int* sample[2];
    uint64_t* base[2];
    uint64_t* seg_start[2];
    unsigned long long* cursor[2];
    uint64_t* cap_end[2];
    int64_t* hist_out[2];
    int64_t* seg_cnt[2];
};

__global__ void __launch_bounds__(256)
k_regions(RegionRel R, uint32_t nbins, uint32_t stride, uint64_t slack, uint32_t elem_bytes) {
    const int r = blockIdx.x;
    const unsigned int* __restrict__ sample = R.sample[r];
    uint64_t* __restrict__ base = R.base[r];
    uint64_t* __restrict__ seg_start = R.seg_start[r];
    unsigned long long* __restrict__ cursor = R.cursor[r];
    uint64_t* __restrict__ cap_end = R.cap_end[r];
    __shared__ uint64_t sh[256];
    // shard capacities are whole 128-byte lines (a multiple of the scatter's
    // segment), so every region starts on a line of its own: the tiles the
    // bucket pass cuts from different regions never share a cache line
    const uint64_t ALIGN = kRegionAlign / elem_bytes;
    const uint32_t per = (nbins + 255) / 256;
    const uint32_t b = threadIdx.x * per;
    // capacity of one shard of partition d
    auto cap = [&](uint32_t d) {
        const uint64_t est = (uint64_t)sample[d] * stride / kShards;
        return (est + est / 8 + slack + ALIGN - 1) / ALIGN * ALIGN;
    };
    uint64_t loc = 0;
    for (uint32_t k = 0; k < per; k++)
        if (b + k < nbins) loc += kShards * cap(b + k);
    sh[threadIdx.x] = loc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t run = 0;
        for (int t = 0; t < 256; t++) {
            const uint64_t x = sh[t];
            sh[t] = run;
            run += x;
        }
    }
    __syncthreads();
    uint64_t ex = sh[threadIdx.x];
    for (uint32_t k = 0; k < per; k++) {
        const uint32_t d = b + k;
        if (d < nbins) {
            base[d] = ex;
            const uint64_t c = cap(d);
            for (uint32_t q = 0; q < kShards; q++) {
                seg_start[d * kShards + q] = ex;
                cursor[d * kShards + q] = ex;
                ex += c;
                cap_end[d * kShards + q] = ex;
            }
        }
    }
}

// partition and shard sizes from the cursors; flag = 1 when a shard overflowed
// (blockIdx.x = relation)
__global__ void __launch_bounds__(256)
k_regions_done(RegionRel R, uint32_t nbins, unsigned int* __restrict__ flag) {
    const int r = blockIdx.x;
    const uint64_t* __restrict__ seg_start = R.seg_start[r];
    const unsigned long long* __restrict__ cursor = R.cursor[r];
    const uint64_t* __restrict__ cap_end = R.cap_end[r];
    for (uint32_t d = threadIdx.x; d < nbins; d += 256) {
        int64_t tot = 0;
        for (uint32_t q = 0; q < kShards; q++) {
            const uint32_t i = d * kShards + q;
            // clamped: after an overflow the (discarded) result must still
            // describe memory inside the region
            const uint64_t e = cursor[i] < cap_end[i] ? cursor[i] : cap_end[i];
            const int64_t c = (int64_t)(e - seg_start[i]);
            R.seg_cnt[r][i] = c;
            tot += c;
            if (cursor[i] > cap_end[i]) atomicOr(flag, 1u);
        }
        R.hist_out[r][d] = tot;
    }
}

// Exact shard regions (round 6): the exchange's range partition across ranks
// takes the sampled scatter (k_scatter_res) with its regions sized from an
// exact count of every (partition, shard) instead of a sample, laid out back
// to back with no slack.  A shard is the scatter workgroup's blockIdx %
// kShards, so the count follows the scatter's chunking (scatter_chunk).  The
// partitions come out contiguous and exactly sized, as from the exact
// partition (histogram + unstable scatter, plan_partition_packed), and no
// region slack travels with the rows.
template <int THREADS, int ITEMS, class Digit>
__global__ void __launch_bounds__(THREADS)
k_shard_hist(const Tup* __restrict__ in, uint64_t n, uint64_t chunk, uint32_t split,
             Digit dig_arg, uint32_t nbins, unsigned int* __restrict__ counts) {
    const auto dig = dig_arg.load();
    extern __shared__ unsigned int lh[];
    for (uint32_t d = threadIdx.x; d < nbins; d += THREADS) lh[d] = 0;
    __syncthreads();
    // scatter chunk c is counted by `split` workgroups
    const uint32_t c = blockIdx.x / split, s = blockIdx.x % split;
    const uint64_t sub = (chunk + split - 1) / split;
    const uint64_t beg = (uint64_t)c * chunk + (uint64_t)s * sub;
    const uint64_t end = min(min(beg + sub, (uint64_t)(c + 1) * chunk), n);
    constexpr int TILE = THREADS * ITEMS;
    for (uint64_t base = beg; base < end; base += TILE) {
        Tup v[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint64_t i = base + (uint64_t)j * THREADS + threadIdx.x;
            v[j] = ld_stream(in + (i < end ? i : end - 1));  // clamped: all in flight
        }
#pragma unroll
        for (int j = 0; j < ITEMS; j++)
            if (base + (uint64_t)j * THREADS + threadIdx.x < end) atomicAdd(&lh[dig(v[j])], 1u);
    }
    __syncthreads();
    const uint32_t q = c % kShards;
    for (uint32_t d = threadIdx.x; d < nbins; d += THREADS)
        if (lh[d]) atomicAdd(&counts[(size_t)d * kShards + q], lh[d]);
}

// the regions of k_shard_hist's counts (R.sample: nbins * kShards each),
// partition-major, shard-minor, back to back (blockIdx.x = relation)
__global__ void __launch_bounds__(1024)
k_regions_exact(RegionRel R, uint32_t nbins) {
    const int r = blockIdx.x;
    const unsigned int* __restrict__ cnt = R.sample[r];
    __shared__ uint32_t scr[1024 / 64 + 1];
    const uint32_t per = (nbins + 1023) / 1024;
    const uint32_t b = threadIdx.x * per;
    uint32_t loc = 0;
    for (uint32_t k = 0; k < per; k++)
        if (b + k < nbins)
            for (uint32_t q = 0; q < kShards; q++) loc += cnt[(size_t)(b + k) * kShards + q];
    uint32_t tot;
    uint64_t e = block_exclusive_scan(loc, scr, &tot);
    for (uint32_t k = 0; k < per; k++) {
        const uint32_t d = b + k;
        if (d >= nbins) break;
        R.base[r][d] = e;
        for (uint32_t q = 0; q < kShards; q++) {
            const size_t i = (size_t)d * kShards + q;
            R.seg_start[r][i] = e;
            R.cursor[r][i] = e;
            e += cnt[i];
            R.cap_end[r][i] = e;
        }
    }
}

// lanes of the scatter write whole 64-byte segments: the complete segments
// of a tile are numbered, segown[s] = the partition of segment s
// (SB: bytes an element takes in the output's first plane: the segment is
// kSegBytes of that plane; one plane for every layout but LayP48)
template <int THREADS, int ITEMS, class OutT, uint32_t SB = sizeof(OutT)>
struct ScatterGeom {
    static constexpr uint32_t SEG = kSegBytes >= SB ? kSegBytes / SB : 1;  // elements per segment
    static constexpr uint32_t TILE = THREADS * ITEMS;
    static __host__ __device__ constexpr uint32_t max_segs(uint32_t nbins) {
        return (TILE + nbins * (SEG - 1)) / SEG;
    }
    // stage OutT[TILE] | carry OutT[nbins * SEG] | pos u64[nbins] |
    // tstart, tfill, kc, segpre u32[nbins] | segown u16[max_segs] | scan scratch
    static __host__ __device__ constexpr size_t lds_bytes(uint32_t nbins) {
        return (size_t)TILE * sizeof(OutT) + (size_t)nbins * SEG * sizeof(OutT) +
               (size_t)nbins * (8 + 4 * 4) + ((size_t)max_segs(nbins) * 2 + 15) / 16 * 16 +
               (THREADS / 64 + 1) * 4;
    }
};

// whether a Pack stores whole 16-byte segments with one store (store4)
template <class P, class = void>
struct requires_quads : std::false_type {};
template <class P>
struct requires_quads<P, std::void_t<decltype(P::kQuads)>> : std::true_type {};
template <class Pack>
constexpr bool pack_quads() {
    if constexpr (requires_quads<Pack>::value) return Pack::kQuads;
    else return false;
}

// VEC (8-byte tuples, ITEMS even): item pair (2p, 2p+1) of a thread is one
// 16-byte load of two adjacent tuples -- the order inside a partition is free
// here, so the pairing needs no transpose
template <int THREADS, int ITEMS, class Digit, class Pack, bool VEC>
__global__ void __launch_bounds__(THREADS)
k_scatter_res(const Tup* __restrict__ in, uint64_t n, uint64_t chunk, Digit dig_arg,
              uint32_t nbins, unsigned long long* __restrict__ cursor_all,
              const uint64_t* __restrict__ cap_end_all,
              void* __restrict__ out, uint64_t ostride, Pack pk,
              unsigned int* __restrict__ bad_flag) {
    typedef typename Pack::OutT OutT;
    typedef ScatterGeom<THREADS, ITEMS, OutT, Pack::kStoreBytes> Geo;
    constexpr uint32_t SEG = Geo::SEG;
    constexpr int TILE = (int)Geo::TILE;
    uint32_t bad = 0;
    const auto dig = dig_arg.load();
    // this workgroup's shard of every partition: cursor[d * kShards + shard]
    const uint32_t shard = blockIdx.x % kShards;
    unsigned long long* cursor = cursor_all + shard;
    const uint64_t* cap_end = cap_end_all + shard;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    OutT* stage = reinterpret_cast<OutT*>(lds_raw);
    OutT* carry = stage + TILE;
    uint64_t* pos = reinterpret_cast<uint64_t*>(carry + (size_t)nbins * SEG);
    uint32_t* tstart = reinterpret_cast<uint32_t*>(pos + nbins);
    uint32_t* tfill = tstart + nbins;
    uint32_t* kc = tfill + nbins;
    uint32_t* segpre = kc + nbins;
    uint16_t* segown = reinterpret_cast<uint16_t*>(segpre + nbins);
    uint32_t* scr = reinterpret_cast<uint32_t*>(
        reinterpret_cast<unsigned char*>(segown) + ((size_t)Geo::max_segs(nbins) * 2 + 15) / 16 * 16);

    for (uint32_t d = threadIdx.x; d < nbins; d += THREADS) {
        tfill[d] = 0;
        kc[d] = 0;
    }
    const uint64_t beg = (uint64_t)blockIdx.x * chunk;
    uint64_t end = beg + chunk;
    if (end > n) end = n;
    // one partition per thread (the host launches nbins <= THREADS): the
    // per-partition state lives in registers, no dynamic indexing
    const uint32_t d0 = threadIdx.x;
    const bool own = d0 < nbins;
    const uint64_t my_cap = own ? cap_end[(size_t)d0 * kShards] : 0;
    uint32_t my_kc = 0;

    static_assert(!VEC || (sizeof(Tup) == 8 && ITEMS % 2 == 0), "VEC: 8-byte tuples, ITEMS even");
    // tile position of item j (VEC: pairs of adjacent tuples per thread)
    auto item_pos = [](int j) -> uint32_t {
        return VEC ? 2u * ((uint32_t)(j / 2) * THREADS + threadIdx.x) + (uint32_t)(j & 1)
                   : (uint32_t)j * THREADS + threadIdx.x;
    };
    // clamped loads of the tile at b0 (VEC: n and the chunks are even)
    auto load_tile = [&](Tup (&x)[ITEMS], uint64_t b0) {
#ifndef KEY_8B
        typedef unsigned long long V2 __attribute__((ext_vector_type(2)));
        if constexpr (VEC) {
            const V2* __restrict__ vin = reinterpret_cast<const V2*>(in);
            const uint64_t vl = end / 2 - 1;
#pragma unroll
            for (int p = 0; p < ITEMS / 2; p++) {
                const uint64_t vi = b0 / 2 + (uint64_t)p * THREADS + threadIdx.x;
#if SMJ_NT_LOADS
                const V2 y = __builtin_nontemporal_load(vin + (vi < vl ? vi : vl));
#else
                const V2 y = vin[vi < vl ? vi : vl];
#endif
                x[2 * p] = (Tup)y.x;
                x[2 * p + 1] = (Tup)y.y;
            }
        } else
#endif
        {
#pragma unroll
            for (int j = 0; j < ITEMS; j++) {
                const uint64_t i = b0 + (uint64_t)j * THREADS + threadIdx.x;
                x[j] = ld_stream(in + (i < end ? i : end - 1));
            }
        }
    };
    Tup v[ITEMS], nv[ITEMS];
    if (beg < end) load_tile(v, beg);
    __syncthreads();
    for (uint64_t base = beg; base < end; base += TILE) {
        const uint32_t tcount =
            (uint32_t)((end - base) < (uint64_t)TILE ? (end - base) : TILE);
        const uint64_t nb = base + TILE;
        // this tile's loads (the previous prefetch) have landed: an explicit
        // vmcnt(0) on every path, so the compiler's own bookkeeping does not
        // re-wait (for the next prefetch) at each conditional use below
        __builtin_amdgcn_s_waitcnt(0x0f70);
        // ---- rank: tile counts per partition
        uint32_t dg[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint32_t li = item_pos(j);
            dg[j] = li < tcount ? dig(v[j]) : 0xffffffffu;
            if (dg[j] != 0xffffffffu) atomicAdd(&tfill[dg[j]], 1u);
        }
        __syncthreads();
        // ---- per partition: the whole segments of carry + tile (E, a
        // multiple of SEG) are written now; stage offsets and segment numbers
        // in one scan (c | segments << 16: both stay below 2^16)
        const uint32_t c = own ? tfill[d0] : 0;
        const uint32_t T = my_kc + c;
        uint32_t Eown = T / SEG * SEG;
        uint32_t tot;
        const uint32_t ex = block_exclusive_scan(own ? (c | ((Eown / SEG) << 16)) : 0u, scr, &tot);
        const uint32_t nseg = tot >> 16;
        unsigned long long Pown = 0;
        if (own) {
            tstart[d0] = ex & 0xffffu;
            tfill[d0] = ex & 0xffffu;
            segpre[d0] = ex >> 16;
            for (uint32_t k = 0; k < Eown / SEG; k++) segown[(ex >> 16) + k] = (uint16_t)d0;
            // reservation issued before the next tile's loads, so waiting for
            // it (after the staging below) does not wait for that prefetch
            if (Eown) Pown = atomicAdd(&cursor[(size_t)d0 * kShards], (unsigned long long)Eown);
        }
        // unconditional (clamped) loads: a fixed count in flight lets the
        // reservation results be waited for with vmcnt(ITEMS)
        load_tile(nv, nb);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < ITEMS; j++)
            if (dg[j] != 0xffffffffu) stage[atomicAdd(&tfill[dg[j]], 1u)] = pk(v[j], bad);
        if (own) {
            // an overflowing region writes nothing (the caller repeats the
            // exact partition)
            const bool ovf = Eown && Pown + Eown > my_cap;
            pos[d0] = ovf ? ~0ull : Pown;
            if (ovf) Eown = 0;
        }
        __syncthreads();
        // ---- whole segments: SEG consecutive lanes per segment, element e of
        // a partition = carry (e < kc) or its staged tuples (pair stores:
        // SEG / 2 lanes, two adjacent elements each)
        if constexpr (pack_quads<Pack>() && SEG == 4) {
            // a whole segment a lane: one 16-byte store (LayP32)
            for (uint32_t sg = threadIdx.x; sg < nseg; sg += THREADS) {
                const uint32_t d = segown[sg];
                const uint32_t e = (sg - segpre[d]) * SEG;
                const uint32_t k = kc[d];
                const uint64_t p = pos[d];
                OutT x[4];
#pragma unroll
                for (uint32_t i = 0; i < 4; i++)
                    x[i] = e + i < k ? carry[d * SEG + e + i] : stage[tstart[d] + e + i - k];
                if (p != ~0ull) {
                    if ((p & 3) == 0) {
                        Pack::store4(out, ostride, p + e, x);
                    } else {  // after an odd flush of a workgroup sharing the cursor
#pragma unroll
                        for (uint32_t i = 0; i < 4; i++) Pack::store(out, ostride, p + e + i, x[i]);
                    }
                }
            }
        } else if constexpr (Pack::kPairs) {
            constexpr uint32_t PS = SEG / 2;
            for (uint32_t q = threadIdx.x; q < nseg * PS; q += THREADS) {
                const uint32_t sg = q / PS;
                const uint32_t d = segown[sg];
                const uint32_t e = (sg - segpre[d]) * SEG + 2 * (q % PS);
                const uint32_t k = kc[d];
                const uint64_t p = pos[d];
                const OutT x0 = e < k ? carry[d * SEG + e] : stage[tstart[d] + e - k];
                const OutT x1 = e + 1 < k ? carry[d * SEG + e + 1] : stage[tstart[d] + e + 1 - k];
                // p is odd after a workgroup sharing this shard cursor flushed
                // an odd carry (the flush below): the pair store needs p + e
                // even (e is), else two element stores
                if (p != ~0ull) {
                    if ((p & 1) == 0) {
                        Pack::store2(out, ostride, p + e, x0, x1);
                    } else {
                        Pack::store(out, ostride, p + e, x0);
                        Pack::store(out, ostride, p + e + 1, x1);
                    }
                }
            }
        } else {
            for (uint32_t q = threadIdx.x; q < nseg * SEG; q += THREADS) {
                const uint32_t sg = q / SEG;
                const uint32_t d = segown[sg];
                const uint32_t e = (sg - segpre[d]) * SEG + q % SEG;
                const uint32_t k = kc[d];
                const uint64_t p = pos[d];
                const OutT x = e < k ? carry[d * SEG + e] : stage[tstart[d] + e - k];
                if (p != ~0ull) Pack::store(out, ostride, p + e, x);
            }
        }
        __syncthreads();
        // ---- leftovers (< SEG) become the partition's carry
        if (own) {
            uint32_t left = T - Eown;
            if (left > SEG - 1) left = SEG - 1;  // only after an overflow (discarded)
            for (uint32_t e = Eown; e < Eown + left; e++)
                carry[d0 * SEG + (e - Eown)] =
                    e < my_kc ? carry[d0 * SEG + e] : stage[tstart[d0] + e - my_kc];
            my_kc = left;
            kc[d0] = left;
            tfill[d0] = 0;
        }
#pragma unroll
        for (int j = 0; j < ITEMS; j++) v[j] = nv[j];
        __syncthreads();
    }
    // ---- flush the carries: reserve exactly what is left
    if (own) {
        const uint32_t d = d0;
        pos[d] = 0;
        if (kc[d]) {
            const uint64_t p = atomicAdd(&cursor[(size_t)d * kShards], (unsigned long long)kc[d]);
            pos[d] = p + kc[d] <= my_cap ? p : ~0ull;
        }
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < nbins * SEG; q += THREADS) {
        const uint32_t d = q / SEG, j = q % SEG;
        if (j < kc[d] && pos[d] != ~0ull) Pack::store(out, ostride, pos[d] + j, carry[q]);
    }
    if (bad_flag && bad) atomicOr(bad_flag, bad);
}

// pad copy for wide digits: item at unpadded position i of digit d moves to
// padded_start[d] + (i - unpadded_start[d])
template <class Digit>
__global__ void k_padcopy(const Tup* __restrict__ in, uint64_t n, Digit dig_arg,
                          const uint64_t* __restrict__ ustart,
                          const uint64_t* __restrict__ pstart,
                          Tup* __restrict__ out) {
    const auto dig = dig_arg.load();
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) {
        Tup t = in[i];
        uint32_t d = dig(t);
        out[pstart[d] + (i - ustart[d])] = t;
    }
}

// global-atomic histogram (wide digits only: test-sized inputs)
template <class Digit>
__global__ void k_hist_global(const Tup* __restrict__ in, uint64_t n, Digit dig_arg,
                              unsigned long long* __restrict__ hist) {
    const auto dig = dig_arg.load();
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) atomicAdd(&hist[dig(in[i])], 1ull);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct LowBits {
    Digit32 inner;
    uint32_t lowbits;
    __device__ __forceinline__ LowBits load() const { return *this; }
    __device__ __forceinline__ uint32_t operator()(const Tup& t) const {
        return inner(t) & ((1u << lowbits) - 1u);
    }
};
struct HighBits {
    Digit32 inner;
    uint32_t lowbits;
    __device__ __forceinline__ HighBits load() const { return *this; }
    __device__ __forceinline__ uint32_t operator()(const Tup& t) const {
        return inner(t) >> lowbits;
    }
};

// Histogram + scan + scatter over THREADS x ITEMS tiles, up to 8 workgroups
// per CU.  STABLE: k_scatter_swc (ballot ranks, write combining) where its
// LDS fits, else k_scatter; unstable: k_scatter_u (the join's exact level-1
// partition of 8-byte tuples and the exchange's packed partition).
template <int THREADS, int ITEMS, bool STABLE, class Digit, class Pack = PackNone>
static void partition_hist_scatter(Workspace* ws, const Tup* in, uint64_t n,
                                   typename Pack::OutT* out, const Digit& dig, uint32_t dbits,
                                   int padded, uint64_t* starts_dev,
                                   int64_t* hist_out, int64_t* off_out,
                                   hipStream_t st, const Pack& pk = Pack(),
                                   unsigned int* bad_flag = nullptr) {
    constexpr int TILE = THREADS * ITEMS;
    const uint32_t nbins = 1u << dbits;
    uint64_t ntiles = (n + TILE - 1) / TILE;
    if (ntiles == 0) ntiles = 1;
    const uint32_t maxwg = 256 * 8;
    uint32_t nwg = (uint32_t)(ntiles < maxwg ? ntiles : maxwg);
    const uint64_t tiles_per_wg = (ntiles + nwg - 1) / nwg;
    const uint64_t chunk = tiles_per_wg * TILE;
    nwg = (uint32_t)((ntiles + tiles_per_wg - 1) / tiles_per_wg);

    uint32_t* counts = (uint32_t*)ws->scratch("pt_counts", (size_t)nbins * nwg * 4);
    uint64_t* totals = (uint64_t*)ws->scratch("pt_totals", (size_t)nbins * 8);
    {
        TraceScope ts(ws, "k_hist", st);
        hipLaunchKernelGGL((k_hist<THREADS, ITEMS, Digit>), dim3(nwg), dim3(THREADS),
                           nbins * sizeof(uint32_t), st, in, n, chunk, dig, nbins,
                           counts, nwg);
    }
    {
        TraceScope ts(ws, "k_scan", st);
        hipLaunchKernelGGL(k_scanrow, dim3(nbins), dim3(256), 0, st, counts, nwg,
                           totals);
        hipLaunchKernelGGL(k_scandig, dim3(1), dim3(256), 0, st, totals, nbins,
                           padded, starts_dev, hist_out, off_out);
    }
    if (n == 0) return;
    if constexpr (!STABLE) {
        const size_t ldsu = scatter_u_lds<THREADS, ITEMS>(nbins);
        set_lds_attr((const void*)k_scatter_u<THREADS, ITEMS, Digit, Pack>, 160 * 1024);
        if (ldsu > 160 * 1024) {
            fprintf(stderr, "[ERROR] smj: scatter LDS %zu > 160 KiB\n", ldsu);
            abort();
        }
        TraceScope ts(ws, "k_scatter", st);
        hipLaunchKernelGGL((k_scatter_u<THREADS, ITEMS, Digit, Pack>), dim3(nwg),
                           dim3(THREADS), ldsu, st, in, n, chunk, dig, nbins,
                           counts, nwg, starts_dev, out, pk, bad_flag);
        SMJ_CHECK(hipGetLastError());
        return;
    } else {
        // write-combining stable scatter (its own 512x8 geometry; the
        // histogram's chunking, so counts[d][wg] match)
        typedef SwcGeom<512, 8> SG;
        if (nbins <= 4 * 512 && SG::lds_bytes(nbins) <= 160 * 1024) {
            set_lds_attr((const void*)k_scatter_swc<512, 8, Digit>, 160 * 1024);
            TraceScope ts(ws, "k_scatter", st);
            hipLaunchKernelGGL((k_scatter_swc<512, 8, Digit>), dim3(nwg), dim3(512),
                               SG::lds_bytes(nbins), st, in, n, chunk, dig, nbins, dbits,
                               counts, nwg, starts_dev, out);
            SMJ_CHECK(hipGetLastError());
            return;
        }
        const size_t lds = scatter_lds<THREADS, ITEMS>(nbins);
        set_lds_attr((const void*)k_scatter<THREADS, ITEMS, Digit>, 160 * 1024);
        if (lds > 160 * 1024) {
            fprintf(stderr, "[ERROR] smj: scatter LDS %zu > 160 KiB\n", lds);
            abort();
        }
        {
            TraceScope ts(ws, "k_scatter", st);
            hipLaunchKernelGGL((k_scatter<THREADS, ITEMS, Digit>), dim3(nwg),
                               dim3(THREADS), lds, st, in, n, chunk, dig, nbins, dbits,
                               counts, nwg, starts_dev, out);
        }
    }
    SMJ_CHECK(hipGetLastError());
}

// The ranks of k_scatter_swp rely on a hardware property (lanes of one LDS
// atomic that hit the same word get their old values in lane order).  It is
// checked on the device once per process, the first time a stable partition
// runs; a device without it takes the ballot ranks of k_scatter_swc.
static bool lds_order_ok(Workspace* ws, hipStream_t st) {
    static const bool ok = [&] {
        const uint64_t bad = lds_order_selfcheck(ws, st);
        if (bad)
            fprintf(stderr, "[WARN] smj: LDS atomics return %llu values out of lane order: "
                            "the stable partition uses ballot ranks\n",
                    (unsigned long long)bad);
        return bad == 0;
    }();
    return ok;
}

// histogram + scan + k_scatter_swp, one workgroup per CU (1 <= dbits <= 10).
// bench_partitioning 2^27 x 10 bits on MI355X (round 2, tools/ab_swa.sh): the
// 16-byte loads of k_hist_v took 8-byte tuples' histogram from 0.236 to
// 0.160 ms, non-temporal loads 16-byte tuples' from 0.424 to 0.317 ms.
template <class Digit>
static void stable_partition_swp(Workspace* ws, const Tup* in, uint64_t n, Tup* out,
                                 const Digit& dig, uint32_t dbits, int padded,
                                 uint64_t* starts_dev, int64_t* hist_out, int64_t* off_out,
                                 hipStream_t st) {
    constexpr int THREADS = 512;
    constexpr int ITEMS = sizeof(Tup) == 16 ? 8 : 16;
    typedef SwaGeom<THREADS, ITEMS> G;
    const uint32_t nbins = 1u << dbits;
    uint64_t ntiles = (n + G::TILE - 1) / G::TILE;
    if (ntiles == 0) ntiles = 1;
    uint32_t nwg = (uint32_t)(ntiles < 256 ? ntiles : 256);
    const uint64_t tiles_per_wg = (ntiles + nwg - 1) / nwg;
    const uint64_t chunk = tiles_per_wg * G::TILE;
    nwg = (uint32_t)((ntiles + tiles_per_wg - 1) / tiles_per_wg);
    uint32_t* counts = (uint32_t*)ws->scratch("pt_counts", (size_t)nbins * nwg * 4);
    uint64_t* totals = (uint64_t*)ws->scratch("pt_totals", (size_t)nbins * 8);
    {
        TraceScope ts(ws, "k_hist", st);
        bool vec = false;
        if constexpr (sizeof(Tup) == 8) {
            vec = ((uintptr_t)in & 15) == 0 && (chunk & 1) == 0;
            if (vec)
                hipLaunchKernelGGL((k_hist_v<512, 8, Digit>), dim3(nwg), dim3(512),
                                   nbins * sizeof(uint32_t), st, in, n, chunk, dig, nbins,
                                   counts, nwg);
        }
        if (!vec)
            hipLaunchKernelGGL((k_hist_p<512, 16, Digit, true>), dim3(nwg), dim3(512),
                               nbins * sizeof(uint32_t), st, in, n, chunk, dig, nbins, counts,
                               nwg);
    }
    {
        TraceScope ts(ws, "k_scan", st);
        hipLaunchKernelGGL(k_scanrow, dim3(nbins), dim3(256), 0, st, counts, nwg, totals);
        hipLaunchKernelGGL(k_scandig, dim3(1), dim3(256), 0, st, totals, nbins, padded,
                           starts_dev, hist_out, off_out);
    }
    if (n == 0) return;
    set_lds_attr((const void*)k_scatter_swp<THREADS, ITEMS, Digit, true>, 160 * 1024);
    TraceScope ts(ws, "k_scatter", st);
    hipLaunchKernelGGL((k_scatter_swp<THREADS, ITEMS, Digit, true>), dim3(nwg), dim3(THREADS),
                       G::lds_bytes(nbins), st, in, n, chunk, dig, nbins, counts, nwg,
                       starts_dev, out, 1);
    SMJ_CHECK(hipGetLastError());
}

template <class Digit>
static void stable_partition_narrow(Workspace* ws, const Tup* in, uint64_t n,
                                    Tup* out, const Digit& dig, uint32_t dbits,
                                    int padded, uint64_t* starts_dev,
                                    int64_t* hist_out, int64_t* off_out,
                                    hipStream_t st) {
    // positions are 32-bit inside k_scatter_swp; its LDS holds 2^10 digits
    typedef SwaGeom<512, sizeof(Tup) == 16 ? 8 : 16> SG;
    if (dbits >= 1 && dbits <= 10 && n + ((uint64_t)64 << dbits) < (1ull << 32) &&
        SG::lds_bytes(1u << dbits) <= 160 * 1024 && lds_order_ok(ws, st)) {
        stable_partition_swp(ws, in, n, out, dig, dbits, padded, starts_dev, hist_out,
                             off_out, st);
        return;
    }
    // the big tiles need the 16-bit per-wave counters and <= 160 KiB LDS
    if (dbits <= 10)
        partition_hist_scatter<512, 16, true>(ws, in, n, out, dig, dbits, padded,
                                              starts_dev, hist_out, off_out, st);
    else
        partition_hist_scatter<256, 8, true>(ws, in, n, out, dig, dbits, padded,
                                             starts_dev, hist_out, off_out, st);
}

// unstable variant (the join's exact level-1 partition): 512 x 16 tiles
// measured fastest (round 1)
template <class Digit>
static void unstable_partition(Workspace* ws, const Tup* in, uint64_t n,
                               Tup* out, const Digit& dig, uint32_t dbits,
                               uint64_t* starts_dev, int64_t* hist_out,
                               hipStream_t st) {
    if (dbits <= 10)
        partition_hist_scatter<512, 16, false>(ws, in, n, out, dig, dbits, 0, starts_dev,
                                               hist_out, nullptr, st);
    else
        partition_hist_scatter<256, 8, false>(ws, in, n, out, dig, dbits, 0, starts_dev,
                                              hist_out, nullptr, st);
}

void stable_partition(Workspace* ws, const Tup* in, uint64_t n, Tup* out,
                      const Digit32& dig, uint32_t dbits, int padded,
                      int64_t* hist_out, int64_t* off_out, hipStream_t st) {
    const uint32_t nbins = 1u << dbits;
    if (dbits <= kNarrowDigitBits) {
        uint64_t* starts = (uint64_t*)ws->scratch("pt_starts", (size_t)nbins * 8);
        stable_partition_narrow(ws, in, n, out, dig, dbits, padded, starts,
                                hist_out, off_out, st);
        return;
    }
    // wide digits: stable LSD (low part, then high part), then pad copy
    const uint32_t lowb = dbits / 2, highb = dbits - lowb;
    Tup* t1 = (Tup*)ws->scratch("pt_wide1", (n ? n : 1) * sizeof(Tup));
    Tup* t2 = (Tup*)ws->scratch("pt_wide2", (n ? n : 1) * sizeof(Tup));
    uint64_t* st1 = (uint64_t*)ws->scratch("pt_wst1", (1u << lowb) * 8);
    uint64_t* st2 = (uint64_t*)ws->scratch("pt_wst2", (1u << highb) * 8);
    LowBits lo{dig, lowb};
    HighBits hi{dig, lowb};
    stable_partition_narrow(ws, in, n, t1, lo, lowb, 0, st1, nullptr, nullptr, st);
    stable_partition_narrow(ws, t1, n, t2, hi, highb, 0, st2, nullptr, nullptr, st);
    unsigned long long* h = (unsigned long long*)ws->scratch("pt_whist", (size_t)nbins * 8);
    SMJ_CHECK(hipMemsetAsync(h, 0, (size_t)nbins * 8, st));
    if (n) hipLaunchKernelGGL(k_hist_global<Digit32>, dim3(1024), dim3(256), 0,
                              st, in, n, dig, h);
    uint64_t* ust = (uint64_t*)ws->scratch("pt_wust", (size_t)nbins * 8);
    uint64_t* pst = (uint64_t*)ws->scratch("pt_wpst", (size_t)nbins * 8);
    hipLaunchKernelGGL(k_scandig, dim3(1), dim3(256), 0, st,
                       (const uint64_t*)h, nbins, 0, ust, nullptr, nullptr);
    hipLaunchKernelGGL(k_scandig, dim3(1), dim3(256), 0, st,
                       (const uint64_t*)h, nbins, padded, pst, hist_out, off_out);
    if (n) hipLaunchKernelGGL(k_padcopy<Digit32>, dim3(2048), dim3(256), 0, st,
                              t2, n, dig, ust, pst, out);
    SMJ_CHECK(hipGetLastError());
}

// Exact level-1 partition of the join/sort (range-plan digit, unpadded; the
// order inside a partition is free: every bucket is fully sorted afterwards).
// 16-byte tuples: histogram + write-combining scatter (4-tuple segments), one
// workgroup per CU and a long chunk per workgroup (the carries pay off over
// many tiles).  8-byte tuples: k_scatter_u (write combining measured no gain
// for them, round 1).
void plan_partition(Workspace* ws, const Tup* in, uint64_t n, Tup* out,
                    const RangePlan* plan_dev, uint32_t dbits,
                    uint64_t* starts_dev, int64_t* hist_out, hipStream_t st) {
    PlanDigit1 dig{plan_dev};
    const uint32_t nbins = 1u << dbits;
    constexpr int THREADS = 512;
    constexpr int ITEMS = sizeof(Tup) == 16 ? 8 : 16;
    constexpr int TILE = THREADS * ITEMS;
    const size_t lds = scatter_wc_lds<THREADS, ITEMS>(nbins);
    if (sizeof(Tup) != 16 || dbits > 10 || lds > 160 * 1024) {
        unstable_partition(ws, in, n, out, dig, dbits, starts_dev, hist_out, st);
        return;
    }
    uint64_t ntiles = (n + TILE - 1) / TILE;
    if (ntiles == 0) ntiles = 1;
    const uint32_t maxwg = 256;  // one per CU
    uint32_t nwg = (uint32_t)(ntiles < maxwg ? ntiles : maxwg);
    const uint64_t tiles_per_wg = (ntiles + nwg - 1) / nwg;
    const uint64_t chunk = tiles_per_wg * TILE;
    nwg = (uint32_t)((ntiles + tiles_per_wg - 1) / tiles_per_wg);
    uint32_t* counts = (uint32_t*)ws->scratch("pt_counts", (size_t)nbins * nwg * 4);
    uint64_t* totals = (uint64_t*)ws->scratch("pt_totals", (size_t)nbins * 8);
    {
        // one workgroup per scatter chunk: 16 waves keep enough loads in flight
        TraceScope ts(ws, "k_hist", st);
        hipLaunchKernelGGL((k_hist<1024, 8, PlanDigit1>), dim3(nwg), dim3(1024),
                           nbins * sizeof(uint32_t), st, in, n, chunk, dig, nbins,
                           counts, nwg);
    }
    {
        TraceScope ts(ws, "k_scan", st);
        hipLaunchKernelGGL(k_scanrow, dim3(nbins), dim3(256), 0, st, counts, nwg,
                           totals);
        hipLaunchKernelGGL(k_scandig, dim3(1), dim3(256), 0, st, totals, nbins, 0,
                           starts_dev, hist_out, (int64_t*)nullptr);
    }
    if (n == 0) return;
    set_lds_attr((const void*)k_scatter_wc<THREADS, ITEMS, PlanDigit1>, 160 * 1024);
    TraceScope ts(ws, "k_scatter", st);
    hipLaunchKernelGGL((k_scatter_wc<THREADS, ITEMS, PlanDigit1>), dim3(nwg),
                       dim3(THREADS), lds, st, in, n, chunk, dig, nbins, counts,
                       nwg, starts_dev, out);
    SMJ_CHECK(hipGetLastError());
}

#ifdef KEY_8B
// plan_partition writing LayPacked words for `pack_plan` (the multi-GPU
// exchange: half the bytes on the wire); *pack_bad |= 1 when a tuple does
// not pack.  Histogram + unstable scatter (partitions back to back).
void plan_partition_packed(Workspace* ws, const Tup* in, uint64_t n, uint64_t* out,
                           const RangePlan* plan_dev, const RangePlan& pack_plan,
                           uint32_t dbits, uint64_t* starts_dev, int64_t* hist_out,
                           unsigned int* pack_bad, hipStream_t st) {
    PlanDigit1 dig{plan_dev};
    LayPacked::Pack pk;
    pk.bu = key_u(pack_plan.base);
    pk.span = pack_plan.span;
    pk.s1 = pack_plan.s1;
    // the 16-byte stage of 512x16 tiles and 2^12 bins would exceed 160 KiB
    if (dbits > 10)
        partition_hist_scatter<256, 8, false, PlanDigit1, LayPacked::Pack>(
            ws, in, n, out, dig, dbits, 0, starts_dev, hist_out, nullptr, st, pk, pack_bad);
    else
        partition_hist_scatter<512, 16, false, PlanDigit1, LayPacked::Pack>(
            ws, in, n, out, dig, dbits, 0, starts_dev, hist_out, nullptr, st, pk, pack_bad);
}
#endif

// Sampled level-1 partition (see k_scatter_res): `out` must hold
// sampled_capacity(n, dbits) tuples.  starts_dev/hist_out receive each
// partition's region start and size; *flag_dev is OR-ed with 1 when a region
// overflowed (then the output is incomplete and the exact partition must be
// used).  Nothing is read back to the host.
#ifndef SMJ_SC_THREADS
#define SMJ_SC_THREADS 1024
#endif
#ifndef SMJ_SC_ITEMS16
#define SMJ_SC_ITEMS16 4   // 16-byte tuples staged as tuples
#endif
#ifndef SMJ_SC_ITEMS16Q
#define SMJ_SC_ITEMS16Q 6  // 16-byte tuples staged as 12-byte elements (LayP96): 4 items
                           // 1.52 ms, 6 1.47, 8 1.47 (profiles/r06_lab/p12_ab.txt)
#endif
#ifndef SMJ_SC_ITEMS16P
#define SMJ_SC_ITEMS16P 8  // 16-byte tuples staged as packed 8-byte words
#endif
#ifndef SMJ_SC_ITEMS8
// even, for the 16-byte pair loads (k_scatter_res VEC): 128M x 128M 8 B join
// 3.20-3.24 -> 3.04-3.07 ms against 13 items of 8-byte loads (interleaved,
// tools/ab_scvec.sh; 14 items with pair loads 3.12-3.17)
#define SMJ_SC_ITEMS8 12
#endif
#ifndef SMJ_SC_ITEMS8W
#define SMJ_SC_ITEMS8W 16  // 8-byte tuples staged as 32-bit words (LayP32): bench_sort
                           // scatter 12 items 0.469 ms, 16 0.435, 20 0.639, 24 0.748
                           // (profiles/r06_lab/scatter_items.txt)
#endif
#ifndef SMJ_SC_WG_PER_CU
#define SMJ_SC_WG_PER_CU 1
#endif
#ifndef SMJ_SAMPLE_STRIDE
#define SMJ_SAMPLE_STRIDE 128
#endif
static constexpr uint32_t kSampleStride = SMJ_SAMPLE_STRIDE;
#ifndef SMJ_SAMPLE_WG
#define SMJ_SAMPLE_WG 128
#endif
static constexpr uint32_t kSampleWg = SMJ_SAMPLE_WG;
static constexpr uint64_t kRegionSlack = 1024;  // per shard

// Upper bound of the regions k_regions lays out, in elements of the smallest
// layout (8-byte words: the most per segment).  The blocked sample counts 4
// tuples at every 4*stride-th position, so sample[] sums to at most
// n/stride + 4 and the estimates to n + 4*stride; a shard's capacity is 9/8
// of its estimate plus the slack, rounded up to a segment:
//     sum <= (n + 4*stride) * 9/8 + 2^dbits * kShards * (slack + ALIGN - 1),
// ALIGN = kRegionAlign in elements (the capacities' rounding).
uint64_t sampled_capacity(uint64_t n, uint32_t dbits) {
    const uint64_t ALIGN = kRegionAlign / 4;  // the finest: LayP48's 4-byte plane
    return n + n / 8 + 5 * kSampleStride + 1 +
           ((uint64_t)1 << dbits) * kShards * (kRegionSlack + ALIGN);
}

// the sampled scatter's chunk of one workgroup (n > 0) and its workgroups
static uint64_t scatter_chunk(uint64_t n, uint64_t tile, uint32_t* nwg_out) {
    const uint64_t ntiles = (n + tile - 1) / tile;
    const uint32_t maxwg = 256 * SMJ_SC_WG_PER_CU;
    uint32_t nwg = (uint32_t)(ntiles < maxwg ? ntiles : maxwg);
    const uint64_t tiles_per_wg = (ntiles + nwg - 1) / nwg;
    *nwg_out = (uint32_t)((ntiles + tiles_per_wg - 1) / tiles_per_wg);
    return tiles_per_wg * tile;
}

// items per thread of the sampled scatter for Pack at nbins partitions: the
// widest tile whose LDS fits (0: none)
template <class Pack>
static int sampled_items(uint32_t nbins) {
    constexpr int THREADS = SMJ_SC_THREADS;
    constexpr int BIG = sizeof(Tup) == 16
        ? (sizeof(typename Pack::OutT) <= 8    ? SMJ_SC_ITEMS16P
           : sizeof(typename Pack::OutT) <= 12 ? SMJ_SC_ITEMS16Q
                                               : SMJ_SC_ITEMS16)
        : (sizeof(typename Pack::OutT) <= 4 ? SMJ_SC_ITEMS8W : SMJ_SC_ITEMS8);
    constexpr int SMALL = sizeof(Tup) == 16 ? 4 : 8;
    typedef typename Pack::OutT O;
    if (ScatterGeom<THREADS, BIG, O, Pack::kStoreBytes>::lds_bytes(nbins) <= 160 * 1024) return BIG;
    if (ScatterGeom<THREADS, SMALL, O, Pack::kStoreBytes>::lds_bytes(nbins) <= 160 * 1024)
        return SMALL;
    return 0;
}

template <int ITEMS, class Pack>
static bool sampled_scatter_t(Workspace* ws, const Tup* in, uint64_t n, void* out,
                              uint64_t ostride, const PlanDigit1& dig, uint32_t nbins,
                              unsigned long long* cursor, const uint64_t* cap_end,
                              const Pack& pk, unsigned int* bad_flag, hipStream_t st) {
    constexpr int THREADS = SMJ_SC_THREADS;
    constexpr int TILE = THREADS * ITEMS;
    const size_t lds = ScatterGeom<THREADS, ITEMS, typename Pack::OutT,
                                   Pack::kStoreBytes>::lds_bytes(nbins);
    if (lds > 160 * 1024) return false;
    uint32_t nwg = 0;
    const uint64_t chunk = scatter_chunk(n, TILE, &nwg);
    constexpr bool VEC_OK = sizeof(Tup) == 8 && ITEMS % 2 == 0;
    set_lds_attr((const void*)k_scatter_res<THREADS, ITEMS, PlanDigit1, Pack, false>, 160 * 1024);
    if constexpr (VEC_OK)
        set_lds_attr((const void*)k_scatter_res<THREADS, ITEMS, PlanDigit1, Pack, true>,
                     160 * 1024);
    TraceScope ts(ws, "k_scatter", st);
    bool vec = false;
    if constexpr (VEC_OK) {
        vec = n % 2 == 0 && chunk % 2 == 0 && ((uintptr_t)in & 15) == 0;
        if (vec)
            hipLaunchKernelGGL((k_scatter_res<THREADS, ITEMS, PlanDigit1, Pack, true>), dim3(nwg),
                               dim3(THREADS), lds, st, in, n, chunk, dig, nbins, cursor,
                               cap_end, out, ostride, pk, bad_flag);
    }
    if (!vec)
        hipLaunchKernelGGL((k_scatter_res<THREADS, ITEMS, PlanDigit1, Pack, false>), dim3(nwg),
                           dim3(THREADS), lds, st, in, n, chunk, dig, nbins, cursor,
                           cap_end, out, ostride, pk, bad_flag);
    return true;
}

// The LDS stage holds OutT and the carry 64 bytes per partition: the widest
// tile that fits (8-byte tuples: 12 x 1024 up to 512 partitions, 8 x 1024 at
// 1024; packed words 8 / 4 x 1024; 16-byte tuples 4 x 1024), measured best.
template <class Pack>
static void sampled_scatter(Workspace* ws, const Tup* in, uint64_t n, void* out,
                            uint64_t ostride, const PlanDigit1& dig, uint32_t nbins,
                            unsigned long long* cursor, const uint64_t* cap_end,
                            const Pack& pk, unsigned int* bad_flag, hipStream_t st) {
    constexpr int THREADS = SMJ_SC_THREADS;
    if (nbins > (uint32_t)THREADS) {
        fprintf(stderr, "[ERROR] smj: sampled scatter needs <= %d partitions\n", THREADS);
        abort();
    }
    constexpr int BIG = sizeof(Tup) == 16
        ? (sizeof(typename Pack::OutT) <= 8    ? SMJ_SC_ITEMS16P
           : sizeof(typename Pack::OutT) <= 12 ? SMJ_SC_ITEMS16Q
                                               : SMJ_SC_ITEMS16)
        : (sizeof(typename Pack::OutT) <= 4 ? SMJ_SC_ITEMS8W : SMJ_SC_ITEMS8);
    constexpr int SMALL = sizeof(Tup) == 16 ? 4 : 8;
    // the choice sampled_items makes (k_shard_hist counts with its chunking)
    const int items = sampled_items<Pack>(nbins);
    if (items == BIG && sampled_scatter_t<BIG>(ws, in, n, out, ostride, dig, nbins, cursor,
                                               cap_end, pk, bad_flag, st))
        return;
    if (items == SMALL && sampled_scatter_t<SMALL>(ws, in, n, out, ostride, dig, nbins,
                                                   cursor, cap_end, pk, bad_flag, st))
        return;
    fprintf(stderr, "[ERROR] smj: sampled scatter LDS exceeds 160 KiB (%u partitions)\n", nbins);
    abort();
}

void sampled_partition(Workspace* ws, int nrel, const Tup* const* in, const uint64_t* n,
                       void* const* out, const RangePlan* plan_dev, uint32_t dbits,
                       unsigned int* sample, uint64_t* const* starts_dev,
                       int64_t* const* hist_out, uint64_t* const* seg_start,
                       int64_t* const* seg_cnt, unsigned int* flag_dev, hipStream_t st,
                       const RangePlan* host_plan, bool packed, unsigned int* bad,
                       uint64_t p48_stride, bool p32, bool exact, bool p96) {
    PlanDigit1 dig{plan_dev};
    const uint32_t nbins = 1u << dbits;
    // p96 (16-byte tuples): LayP96 elements in two planes of p48_stride
    // elements (int64 payloads, then uint32 key offsets)
    if (p96 && (sizeof(Tup) != 16 || !host_plan || !p48_stride || p32 || exact)) {
        fprintf(stderr, "[ERROR] smj: the 96-bit layout needs 16-byte tuples, the host plan "
                        "and a plane stride\n");
        abort();
    }
    if (exact && (p48_stride || p32)) {
        fprintf(stderr, "[ERROR] smj: exact shard regions take tuples or 64-bit words\n");
        abort();
    }
#ifndef KEY_8B
    // 8-byte tuples: no 64-bit packed words, but 48- and 32-bit ones
    packed = p48_stride != 0 || p32;
#endif
    if (p32 && (p48_stride || !packed)) {
        fprintf(stderr, "[ERROR] smj: the 32-bit layout is a packed one-plane layout\n");
        abort();
    }
    // p48_stride > 0: 48-bit words in two planes of that many elements (LayP48)
    if (p48_stride && !packed) {
        fprintf(stderr, "[ERROR] smj: the 48-bit layout is a packed layout\n");
        abort();
    }
    if (packed && !host_plan) {
        fprintf(stderr, "[ERROR] smj: packed partition needs the host plan\n");
        abort();
    }
    static const char* cn[2] = {"sp_cursor0", "sp_cursor1"};
    static const char* en[2] = {"sp_capend0", "sp_capend1"};
    SampleRel S;
    RegionRel R;
    uint64_t nmax = 0;
    for (int r = 0; r < 2; r++) {
        const int rr = r < nrel ? r : 0;
        S.in[r] = in[rr];
        S.n[r] = n[rr];
        S.hist[r] = sample + (size_t)rr * nbins * (exact ? kShards : 1);
        R.sample[r] = S.hist[r];
        R.base[r] = starts_dev[rr];
        R.seg_start[r] = seg_start[rr];
        R.hist_out[r] = hist_out[rr];
        R.seg_cnt[r] = seg_cnt[rr];
        if (r < nrel) {
            R.cursor[r] = (unsigned long long*)ws->scratch(cn[r], (size_t)nbins * kShards * 8);
            R.cap_end[r] = (uint64_t*)ws->scratch(en[r], (size_t)nbins * kShards * 8);
            nmax = n[r] > nmax ? n[r] : nmax;
        } else {
            R.cursor[r] = R.cursor[0];
            R.cap_end[r] = R.cap_end[0];
        }
    }
    if (exact) {
        // exact (partition, shard) counts with the scatter's chunking, then
        // regions back to back (`sample` holds nbins * kShards per relation)
        TraceScope ts(ws, "k_hist", st);
        for (int r = 0; r < nrel; r++) {
            if (!n[r]) continue;
            int items = 0;
#ifdef KEY_8B
            if (packed)
                items = sampled_items<LayPacked::Pack>(nbins);
            else
#endif
                items = sampled_items<PackRange>(nbins);
            if (!items) {
                fprintf(stderr, "[ERROR] smj: sampled scatter LDS exceeds 160 KiB (%u "
                        "partitions)\n", nbins);
                abort();
            }
            uint32_t nwg = 0;
            const uint64_t chunk = scatter_chunk(n[r], (uint64_t)SMJ_SC_THREADS * items, &nwg);
            constexpr int HI = sizeof(Tup) == 16 ? 8 : 16;
            const uint32_t split = 4;  // workgroups counting one scatter chunk
            hipLaunchKernelGGL((k_shard_hist<1024, HI, PlanDigit1>), dim3(nwg * split),
                               dim3(1024), nbins * sizeof(unsigned int), st, in[r], n[r], chunk,
                               split, dig, nbins, S.hist[r]);
        }
        hipLaunchKernelGGL(k_regions_exact, dim3(nrel), dim3(1024), 0, st, R, nbins);
    } else {
        TraceScope ts(ws, "k_sample", st);
        const uint64_t npts = (nmax + 4 * kSampleStride - 1) / (4 * kSampleStride);
        uint32_t g = (uint32_t)((npts + 255) / 256);
        // each workgroup ends with one global add per partition: at most
        // SMJ_SAMPLE_WG workgroups per relation keep those adds (contended,
        // nbins addresses) few.  128M x 128M join, interleaved
        // (tools/ab_sample.sh): k_sample + k_regions 0.057 ms at 1024
        // workgroups, 0.038 at 256, 0.031 at 128
        if (g > kSampleWg) g = kSampleWg;
        if (g == 0) g = 1;
        hipLaunchKernelGGL((k_sample_hist<PlanDigit1>), dim3(g, nrel), dim3(256),
                           nbins * sizeof(unsigned int), st, S, kSampleStride, dig, nbins);
        // regions aligned to 128 bytes of the first plane (LayP48: 32
        // elements, so the hi plane's regions start on 64 bytes)
        hipLaunchKernelGGL(k_regions, dim3(nrel), dim3(256), 0, st, R, nbins, kSampleStride,
                           kRegionSlack,
                           p96 ? (uint32_t)SMJ_P96_SEGB : p48_stride || p32 ? 4u : packed ? 8u
                                                                     : (uint32_t)sizeof(Tup));
    }
    for (int r = 0; r < nrel; r++) {
        if (!n[r]) continue;
        if (p32) {
            LayP32::Pack pk;
            pk.bu = key_u(host_plan->base);
            pk.span = host_plan->span;
            pk.s1 = host_plan->s1;
            sampled_scatter(ws, in[r], n[r], out[r], 0, dig, nbins, R.cursor[r], R.cap_end[r],
                            pk, bad, st);
            continue;
        }
#ifdef KEY_8B
        if (p96) {
            LayP96::Pack pk;
            pk.bu = key_u(host_plan->base);
            pk.span = host_plan->span;
            sampled_scatter(ws, in[r], n[r], out[r], p48_stride, dig, nbins, R.cursor[r],
                            R.cap_end[r], pk, bad, st);
            continue;
        }
#endif
        if (p48_stride) {
            LayP48::Pack pk;
            pk.bu = key_u(host_plan->base);
            pk.span = host_plan->span;
            pk.s1 = host_plan->s1;
            sampled_scatter(ws, in[r], n[r], out[r], p48_stride, dig, nbins, R.cursor[r],
                            R.cap_end[r], pk, bad, st);
            continue;
        }
#ifdef KEY_8B
        if (packed) {
            LayPacked::Pack pk;
            pk.bu = key_u(host_plan->base);
            pk.span = host_plan->span;
            pk.s1 = host_plan->s1;
            sampled_scatter(ws, in[r], n[r], out[r], 0, dig, nbins, R.cursor[r], R.cap_end[r],
                            pk, bad, st);
            continue;
        }
#endif
        // tuples: range-checked against the host plan when a flag is given
        PackRange pk{0ull, ~0ull};
        if (bad && host_plan) {
            pk.bu = key_u(host_plan->base);
            pk.span = host_plan->span;
        }
        sampled_scatter(ws, in[r], n[r], out[r], 0, dig, nbins, R.cursor[r], R.cap_end[r], pk,
                        bad && host_plan ? bad : (unsigned int*)nullptr, st);
    }
    hipLaunchKernelGGL(k_regions_done, dim3(nrel), dim3(256), 0, st, R, nbins, flag_dev);
    SMJ_CHECK(hipGetLastError());
}

// Self-check of the hardware property k_scatter_swa's ranks rely on: the old
// values an LDS atomic add returns to lanes of one instruction that hit the
// same word are in lane order.  Every wave draws digits from K values (many
// collisions), compares each returned value with the ballot-matched
// expectation and counts violations (must be 0).
__global__ void __launch_bounds__(1024)
k_lds_order(uint32_t K, uint32_t iters, unsigned long long* bad) {
    __shared__ uint32_t ctr[16][64];
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    ctr[wid][lane] = 0;
    __syncthreads();
    const uint64_t lt = lanemask_lt();
    unsigned long long nb = 0;
    uint32_t h = blockIdx.x * 7919u + threadIdx.x * 104729u + K;
    for (uint32_t it = 0; it < iters; it++) {
        h = h * 1664525u + 1013904223u;
        const uint32_t d = (h >> 8) % K;
        uint64_t peers = ~0ull;
        for (int b = 0; b < 6; b++) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bal = __ballot(bit);
            peers &= bit ? bal : ~bal;
        }
        const uint32_t snap = ctr[wid][d];
        __builtin_amdgcn_wave_barrier();
        const uint32_t old = atomicAdd(&ctr[wid][d], 1u);
        __builtin_amdgcn_wave_barrier();
        nb += old != snap + (uint32_t)__popcll(peers & lt);
    }
    if (nb) atomicAdd(bad, nb);
}

uint64_t lds_order_selfcheck(Workspace* ws, hipStream_t st) {
    unsigned long long* bad = (unsigned long long*)ws->scratch("lds_order_bad", 8);
    SMJ_CHECK(hipMemsetAsync(bad, 0, 8, st));
    for (uint32_t K : {1u, 2u, 5u, 16u, 64u})
        hipLaunchKernelGGL(k_lds_order, dim3(512), dim3(1024), 0, st, K, 256u, bad);
    SMJ_CHECK(hipGetLastError());
    unsigned long long* h = (unsigned long long*)ws->host_pinned("lds_order_h", 8);
    SMJ_CHECK(hipMemcpyAsync(h, bad, 8, hipMemcpyDeviceToHost, st));
    SMJ_CHECK(hipStreamSynchronize(st));
    return *h;
}

// histogram-only pass + plain copy (histogram_memcpy_bench)
void hist_memcpy(Workspace* ws, const Tup* in, uint64_t n, Tup* out,
                 uint32_t dbits, hipStream_t st) {
    constexpr int THREADS = 256, ITEMS = 8, TILE = THREADS * ITEMS;
    const uint32_t nbins = 1u << dbits;
    uint64_t ntiles = (n + TILE - 1) / TILE;
    if (ntiles == 0) ntiles = 1;
    uint32_t nwg = (uint32_t)(ntiles < 2048 ? ntiles : 2048);
    const uint64_t tiles_per_wg = (ntiles + nwg - 1) / nwg;
    const uint64_t chunk = tiles_per_wg * TILE;
    nwg = (uint32_t)((ntiles + tiles_per_wg - 1) / tiles_per_wg);
    uint32_t* counts = (uint32_t*)ws->scratch("pt_counts", (size_t)nbins * nwg * 4);
    Digit32 dig{nbins - 1u, 0u};
    if (dbits > kNarrowDigitBits) {
        unsigned long long* h = (unsigned long long*)ws->scratch("pt_whist", (size_t)nbins * 8);
        SMJ_CHECK(hipMemsetAsync(h, 0, (size_t)nbins * 8, st));
        if (n) hipLaunchKernelGGL(k_hist_global<Digit32>, dim3(1024), dim3(256), 0, st, in, n, dig, h);
    } else {
        hipLaunchKernelGGL((k_hist<THREADS, ITEMS, Digit32>), dim3(nwg), dim3(THREADS),
                           nbins * sizeof(uint32_t), st, in, n, chunk, dig, nbins,
                           counts, nwg);
    }
    if (n) SMJ_CHECK(hipMemcpyAsync(out, in, n * sizeof(Tup),
                                    hipMemcpyDeviceToDevice, st));
}

}  // namespace smj
