// bucketsort.hip -- MSD bucket sort of level-1 partitions with a fused
// merge-join count (the sorting_phase + mergejoin_phase of the reference m-way
// join, src/joins/sortmergejoin_multiway.c:388-460, 559-599, re-designed for
// MI355X).
//
// After the level-1 radix partition (partition.hip) every bucket b holds the
// tuples whose key falls in one contiguous key range of the RangePlan.
//
//   k_tilepass  : every bucket is cut into tiles (tile_elems: 16384 8-byte
//                 elements, 8192 16-byte tuples).  A tile is
//                 loaded into registers, counted by its level-2 digit d2 (the
//                 "group") in an LDS histogram, staged in LDS grouped by d2 and
//                 written back linearly (fully coalesced), together with the
//                 tile's exclusive d2 prefix (uint16 per digit + a sentinel =
//                 tile length).  Traffic: 2w.
//   k_groupsort : one workgroup per group (b, d2), two workgroups per CU.  The
//                 group's piece in each tile of bucket b is one contiguous run
//                 (about 1 KiB at the default plan), so the workgroup gathers
//                 R's and S's runs with fully used 128-byte lines, all loads in
//                 flight at once (the run of an element is found with a
//                 run-start bitmap in LDS, no search).  It then counting-sorts
//                 each relation in LDS by the level-3 digit d3, fixes the
//                 (rare) equal-digit runs on the full (key, payload) order,
//                 writes the group to its final place in one contiguous
//                 stream, and counts the matching pairs from the two d3
//                 histograms (the plan makes d3 the exact key when it can) or
//                 by binary search.  Traffic: 2w; the join reads nothing more.
//
// Groups that do not fit in LDS, or whose long equal-key runs are not already
// in payload order (skew), are copied unsorted to their final place and
// finished by the segmented merge sort (mergesort.hip) and the merge-join
// count kernel.
#include <algorithm>
#include <type_traits>
#include <vector>

#include "smj_common.hpp"
#include "smj_internal.hpp"

namespace smj {

// tile-pass workgroup: TP_THREADS threads, tp_items<W>() elements each
// (tile_elems below: 16384 8-byte elements, 8192 16-byte ones).  Round 4 with
// the 48-bit layout (tools/r04_sclab.sh, profiles/r04_lab/tilelab.txt, two
// interleaved rounds on one box): 16384-element tiles against 8192 took the
// 16-byte join 3.29 -> 3.22 ms, the 8-byte join 2.69 -> 2.64, the 8-byte sort
// 1.48 -> 1.46 (the group pass gathers runs twice as long: -0.03 to -0.08 ms;
// the tile pass +0.02).  Round 3, with 64-bit words, had measured the reverse.
#ifndef SMJ_TP_THREADS
#define SMJ_TP_THREADS 1024
#endif
constexpr int TP_THREADS = SMJ_TP_THREADS;
#ifndef SMJ_TP_PERSIST
#define SMJ_TP_PERSIST 1  // persistent tile pass, next tile's loads in flight (0: one tile a workgroup)
#endif
#ifndef SMJ_GS_XCD
#define SMJ_GS_XCD 1  // XCD-aware group order in k_groupsort (0: a lab build's contiguous chunks)
#endif
#ifndef SMJ_GS_PAIR
#define SMJ_GS_PAIR 1  // one relation: two groups per group-pass iteration (0: a lab build's one)
#endif
#ifndef SMJ_GS_TWO
#define SMJ_GS_TWO 1  // both slots of a group-pass iteration in one barrier chain (sort_two)
#endif
// Group-pass metadata one iteration ahead, loaded at the top of the
// iteration (1: two ahead, prefetched while the current group sorts).  The
// prefetch kept a third metadata copy live in scalar registers; without it
// the join kernel spills 79 instead of 154 SGPRs to VGPR lanes and the group
// pass runs 0.003-0.035 ms faster (round 4, profiles/r04_lab/metalab.txt).
#ifndef SMJ_GS_META_PREFETCH
#define SMJ_GS_META_PREFETCH 0
#endif
// The group pass reads its GroupArgs from device memory (written by a
// one-thread kernel before the launch) through a constant-address pointer
// laundered every iteration: the arguments are reloaded with scalar loads
// instead of held in scalar registers across the persistent loop.  The join
// kernel then spills 13 SGPRs instead of 79; the 16-byte join's group pass
// 1.30-1.32 -> 1.26-1.28 ms, the 8-byte join's 1.03 -> 1.01-1.03 (round 4,
// interleaved on one box, profiles/r04_lab/argslab.txt).
#ifndef SMJ_GS_ARGS_MEM
#define SMJ_GS_ARGS_MEM 1
#endif
// elements a tile-pass thread holds: the stage of a tile is 128 KB of LDS, one
// tile a CU (16-byte elements: 16-byte tuples in their own layout take half
// the tile), 64 KB for 32-bit words (two a CU)
#ifndef SMJ_TP_STAGE4
#define SMJ_TP_STAGE4 (64 * 1024)  // the stage of 32-bit words (LayP32): two tiles a CU;
                                   // bench_sort tile pass 0.27 -> 0.19 ms, the step
                                   // 1.215 -> 1.155 (profiles/r06_lab/tile_stage.txt)
#endif
#ifndef SMJ_TP_STAGE8
#define SMJ_TP_STAGE8 (128 * 1024)  // the stage of 8-byte elements (words, tuples): 64 KB
                                    // moves as much into the group pass as it saves
                                    // (profiles/r06_lab/tile_stage.txt)
#endif
template <class W>
constexpr int tp_items() {
    return (int)((sizeof(W) == 4 ? SMJ_TP_STAGE4 : sizeof(W) == 8 ? SMJ_TP_STAGE8 : 128 * 1024)
                 / sizeof(W)) / TP_THREADS;
}
template <class W>
constexpr uint32_t tile_elems() {
    return (uint32_t)(TP_THREADS * tp_items<W>());
}
static_assert(tile_elems<uint64_t>() <= 65535 + 1, "u16 prefix rows");
// 48-bit words staged in LDS as two planes (u32 lo, u16 hi: 6 bytes an
// element) instead of uint64_t: SMJ_TP_STAGE6 bytes of them a tile (0: off).
// 72 KB (12288 elements) puts two tiles on a CU instead of one 16384-element
// tile: the tile pass 0.645 -> 0.570 ms, the group pass +0.05 (runs 3/4 as
// long); the 16-byte join 3.123 -> 3.100 ms, the 8-byte and the Zipf joins
// within noise, and the group pass becomes the join's longest kernel at 0.82
// of its credit instead of the scatter at 0.86 (profiles/r06_lab/tile_stage.txt).
// Off: within the noise between boxes
#ifndef SMJ_TP_STAGE6
#define SMJ_TP_STAGE6 0
#endif
template <class Lay>
struct TileStage {
    static constexpr bool kSplit = false;
    static constexpr uint32_t kBytes = sizeof(typename Lay::W);
    static constexpr int kItems = tp_items<typename Lay::W>();
};
template <>
struct TileStage<LayP48> {
    static constexpr bool kSplit = SMJ_TP_STAGE6 > 0;
    static constexpr uint32_t kBytes = kSplit ? 6 : 8;
    static constexpr int kItems = kSplit ? SMJ_TP_STAGE6 / 6 / TP_THREADS : tp_items<uint64_t>();
};
template <class Lay>
constexpr uint32_t tile_elems_l() {
    return (uint32_t)(TP_THREADS * TileStage<Lay>::kItems);
}
// the bucket-size unit of the plan (choose_levels): a level-1 bucket stays
// within 192 of these (the group pass takes up to 256 tiles of a bucket).
// 16384, the tile of 8-byte elements: the 1024M x 1024M join then plans 2^9
// level-1 partitions instead of 2^10 and its scatter takes 10.4 instead of
// 14.5 ms (31.0 -> 27.3 ms; Zipf 34.4 -> 31.6; 128M unchanged: round 4,
// profiles/r04_lab/kt_lines.txt).  16-byte tuples in their own layout keep
// 8192-element tiles: a bucket of up to 3.1M of them is 384 tiles, past the
// group pass's 256, and takes the skew path (that layout is the fallback for
// unpackable keys only).
#ifndef SMJ_PLAN_TILE
#define SMJ_PLAN_TILE 16384
#endif
const uint32_t kTileTuples = SMJ_PLAN_TILE;

#ifndef SMJ_GS_THREADS
#define SMJ_GS_THREADS 256
#endif
constexpr int GS_THREADS = SMJ_GS_THREADS;      // one workgroup per group
// resident group-pass workgroups per CU: 16-byte elements (LDS- and
// VGPR-bound) and 8-byte ones (tuples or packed words)
#ifndef SMJ_GS_WG_PER_CU
#define SMJ_GS_WG_PER_CU 2
#endif
#ifndef SMJ_GS_WG_PER_CU8
#define SMJ_GS_WG_PER_CU8 4
#endif
// 12-byte elements (LayP96): a workgroup's group buffer is 30 KB, so three
// fit the 160 KB of LDS
#ifndef SMJ_GS_WG_PER_CU12
#define SMJ_GS_WG_PER_CU12 3
#endif
// 32-bit words (LayP32) in pair mode (one relation: the sort): the kernel
// needs ~85 VGPRs and 26 KB of LDS a workgroup, so more fit
#ifndef SMJ_GS_WG_PER_CU4P
#define SMJ_GS_WG_PER_CU4P 5  // 4: sort 2^27 group pass 0.474 ms, 5: 0.447, 6: 0.440 (r05_lab/p32_ab.txt)
#endif
template <class W, bool PAIR = false>
constexpr int gs_wg_per_cu() {
    return sizeof(W) == 16 ? SMJ_GS_WG_PER_CU
         : sizeof(W) == 12 ? SMJ_GS_WG_PER_CU12
         : (sizeof(W) == 4 && PAIR) ? SMJ_GS_WG_PER_CU4P : SMJ_GS_WG_PER_CU8;
}
// 2560 elements per relation: the plan's groups average 2048, so a group's
// run in an 8192-element tile was ~64 words (512 B; 16384-element tiles since
// round 4: ~128) and the gathers waste less
// of the partial 128-byte lines at run ends than with 1280 (1024 on average,
// 256 B runs): 128M x 128M join, group pass 16 B 1.50 -> 1.39 ms, 8 B 1.29 ->
// 1.16 ms; 3072 loses (3 workgroups per CU)
#ifndef SMJ_GS_ITEMS
#define SMJ_GS_ITEMS (2560 / SMJ_GS_THREADS)
#endif
constexpr int GS_ITEMS = SMJ_GS_ITEMS;          // tuples per thread per relation
constexpr int GS_CAP = GS_THREADS * GS_ITEMS;   // tuples per group per relation
constexpr int GS_D3MAX = GS_CAP >= 2048 ? 11 : 10;  // level-3 bits sorted in LDS
constexpr int GS_BPT = (1 << GS_D3MAX) / GS_THREADS;  // d3 bins per thread
constexpr int GS_NB3 = 1 << GS_D3MAX;
// tiles per bucket on the fast path: TPL per lane of the relation's wave
// (k_groupsort<Lay, TPL>, TPL = 2 or 4: 128 or 256 tiles)
constexpr int GS_TMAX = 256;
constexpr int GS_WIN = GS_CAP / 64;
constexpr int GS_RUNMAX = 32;   // longest equal-digit run fixed serially
static_assert(GS_CAP % 64 == 0 && GS_CAP % GS_THREADS == 0, "group capacity");

#ifdef KEY_8B
typedef int64_t KeyT;
#else
typedef int32_t KeyT;
#endif

struct TileTable {
    uint64_t* off;     // tile start in `part`
    uint32_t* len;     // tile length
    uint32_t* bucket;  // owning bucket
    uint32_t* btile0;  // first tile of every bucket (nbuckets + 1)
    uint16_t* pref;    // [tile][nb2 + 1] exclusive prefix, sentinel = length
    uint16_t* prefT;   // the same, digit-major: [d2][tstride] (k_preft)
    uint32_t tstride;  // tiles per prefT row (>= the tile count)
};

struct OvfEntry {
    uint32_t bucket, d2;
    uint32_t nr[2];
    uint64_t off[2];   // offset of the group inside its bucket
    uint32_t counted;  // 1: its matches were already added (exact digits)
    uint32_t pad;
};

// ---------------------------------------------------------------------------
// tile table: block b writes the tiles of bucket b, numbered from btile0[b]
// (uploaded by the host): consecutive tsz-element chunks of each of its segments
// (one segment = the whole bucket, or kShards of a sampled partition).
__global__ void __launch_bounds__(64)
k_tiles(const uint64_t* __restrict__ bstart, const int64_t* __restrict__ bcount,
        const uint64_t* __restrict__ seg_start, const int64_t* __restrict__ seg_cnt,
        uint32_t nseg, TileTable tt, uint32_t tsz) {
    const uint32_t b = blockIdx.x;
    uint32_t t0 = tt.btile0[b];
    for (uint32_t q = 0; q < nseg; q++) {
        const uint64_t s0 = seg_start ? seg_start[(size_t)b * nseg + q] : bstart[b];
        const int64_t cnt = seg_cnt ? seg_cnt[(size_t)b * nseg + q] : bcount[b];
        const uint32_t nt = (uint32_t)((cnt + tsz - 1) / tsz);
        for (uint32_t i = threadIdx.x; i < nt; i += 64) {
            const uint64_t o = (uint64_t)i * tsz;
            const int64_t rem = cnt - (int64_t)o;
            tt.off[t0 + i] = s0 + o;
            tt.len[t0 + i] = (uint32_t)(rem < (int64_t)tsz ? rem : tsz);
            tt.bucket[t0 + i] = b;
        }
        t0 += nt;
    }
}

// ---------------------------------------------------------------------------
// One launch covers the tiles [t0[r], t0[r] + nt[r]) of both relations
// (blocks [0, nt[0]) are R's, the rest S's).  A tile at part offset `off` is
// written to tmp[r][off]: `tmp` is either the partition buffer itself (in
// place) or any buffer of the same layout.
struct TilePassArgs {
    const void* part[2];  // Lay::W elements
    void* tmp[2];
    TileTable tt[2];
    uint32_t t0[2];
    uint32_t nt[2];               // blocks of relation r (an upper bound when...)
    const uint32_t* ntiles[2];    // ...the tile count is only known on the device
    RangePlan plan;  // by value: kernel arguments live in SGPRs
    uint32_t nb2;
    const unsigned int* pack_bad;  // set: the packed partition is void, exit
    uint32_t d2_fast;              // Lay::fast_ok for the level-2 digit (host)
    uint64_t pstride[2] = {0, 0};  // plane stride of part/tmp (LayP48)
    uint64_t ostride[2] = {0, 0};  // of tmp when it is written in another layout (LayP40)
};

// Lay: the partition's layout; LayO: the layout the grouped tiles are written
// in (LayP40 after LayP48: the group's digit is not stored)
template <class Lay, class LayO = Lay>
__global__ void __launch_bounds__(TP_THREADS)
k_tilepass(TilePassArgs A) {
    typedef typename Lay::W W;
    static_assert(std::is_same<W, typename LayO::W>::value, "one element type");
    typedef TileStage<Lay> TS;
    constexpr int TP_ITEMS = TS::kItems;
    constexpr uint32_t TSZ = tile_elems_l<Lay>();
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    if (A.pack_bad && *A.pack_bad) return;
    const RangePlan& P = A.plan;
    const uint32_t nb2 = A.nb2;
    W* stage = reinterpret_cast<W*>(lds_raw);
    uint32_t* stage_lo = reinterpret_cast<uint32_t*>(lds_raw);        // kSplit
    uint16_t* stage_hi = reinterpret_cast<uint16_t*>(lds_raw + TSZ * 4);
    uint32_t* hist = reinterpret_cast<uint32_t*>(lds_raw + ((TSZ * TS::kBytes + 15) & ~15u));
    uint32_t* scr = hist + nb2;

    const int r = blockIdx.x < A.nt[0] ? 0 : 1;
    const uint32_t t = A.t0[r] + (r ? blockIdx.x - A.nt[0] : blockIdx.x);
    if (A.ntiles[r] && t >= *A.ntiles[r]) return;
    const TileTable& tt = A.tt[r];
    const typename Lay::CView part = Lay::cview(A.part[r], A.pstride[r]);
    const typename LayO::View tmp =
        LayO::view(A.tmp[r], std::is_same<Lay, LayO>::value ? A.pstride[r] : A.ostride[r]);
    const uint64_t off = tt.off[t];
    const uint32_t len = tt.len[t];
    const uint32_t b = tt.bucket[t];

    for (uint32_t d = threadIdx.x; d < nb2; d += TP_THREADS) hist[d] = 0;
    W v[TP_ITEMS];
    uint32_t dg[TP_ITEMS];
#pragma unroll
    for (int j = 0; j < TP_ITEMS; j++) {
        uint32_t i = j * TP_THREADS + threadIdx.x;
        if (i < len) v[j] = part[off + i];
    }
    __syncthreads();
    // keys outside the plan range (clamped by plan_rel) only sit in the first
    // and the last bucket: every other tile takes the 32-bit digit
    if (A.d2_fast && b != 0 && b != (1u << P.D1) - 1) {
        const uint32_t base_lo = (uint32_t)P.base, mask = nb2 - 1;
#pragma unroll
        for (int j = 0; j < TP_ITEMS; j++) {
            uint32_t i = j * TP_THREADS + threadIdx.x;
            if (i < len) {
                dg[j] = Lay::digit_fast(v[j], base_lo, P.s1, P.s2, mask);
                atomicAdd(&hist[dg[j]], 1u);
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < TP_ITEMS; j++) {
            uint32_t i = j * TP_THREADS + threadIdx.x;
            if (i < len) {
                dg[j] = plan_d2(P, Lay::rel(P, v[j], b), b);
                atomicAdd(&hist[dg[j]], 1u);
            }
        }
    }
    __syncthreads();
    // exclusive scan of the nb2 bins (contiguous range per thread)
    const uint32_t per = (nb2 + TP_THREADS - 1) / TP_THREADS;
    const uint32_t d0 = threadIdx.x * per;
    uint32_t loc = 0;
    for (uint32_t k = 0; k < per; k++)
        if (d0 + k < nb2) loc += hist[d0 + k];
    uint32_t tot;
    uint32_t ex = block_exclusive_scan(loc, scr, &tot);
    // row of nb2 + 1 entries: the sentinel pref[nb2] = tile length lets the
    // bucket pass read [pref[d2], pref[d2+1]) without a select
    uint16_t* pref = tt.pref + (uint64_t)t * (nb2 + 1);
    for (uint32_t k = 0; k < per; k++) {
        uint32_t d = d0 + k;
        if (d < nb2) {
            uint32_t c = hist[d];
            hist[d] = ex;
            pref[d] = (uint16_t)ex;
            ex += c;
        }
    }
    if (threadIdx.x == 0) pref[nb2] = (uint16_t)len;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < TP_ITEMS; j++) {
        uint32_t i = j * TP_THREADS + threadIdx.x;
        if (i < len) {
            uint32_t pos = atomicAdd(&hist[dg[j]], 1u);
            if constexpr (TS::kSplit) {
                stage_lo[pos] = (uint32_t)v[j];
                stage_hi[pos] = (uint16_t)(v[j] >> 32);
            } else {
                stage[pos] = v[j];
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < TP_ITEMS; j++) {
        uint32_t i = j * TP_THREADS + threadIdx.x;
        if constexpr (TS::kSplit) {
            if (i < len) st_w(tmp + off + i, (W)stage_lo[i] | ((W)stage_hi[i] << 32));
        } else {
            if (i < len) st_w(tmp + off + i, stage[i]);
        }
    }
}

// ---------------------------------------------------------------------------
// The tile pass as a persistent kernel (round 5): one workgroup per CU walks
// the tiles idx = blockIdx.x + k * gridDim.x of both relations, and the next
// tile's loads are issued before the current tile's LDS phases, so they fly
// under its ranking, staging and stores.  (One tile per workgroup, as in
// k_tilepass, holds 128 KB of LDS: a CU runs one workgroup at a time and every
// tile's loads start only when the previous workgroup has gone.)  Two
// register tiles alternate (the loop is unrolled by two: no register copy
// waits for loads).  LDS phases per tile: digits + histogram | scan + prefix
// row | ranks + stage | histogram cleared, stage -> HBM.
template <class Lay, class LayO>
struct TilePassP {
    typedef typename Lay::W W;
    static constexpr int ITEMS = tp_items<W>();
    // element j of a thread
    __device__ static __forceinline__ uint32_t elem(int j) {
        return (uint32_t)j * TP_THREADS + threadIdx.x;
    }
    const TilePassArgs& A;
    W* stage;
    uint32_t* hist;
    uint32_t* scr;
    uint32_t n0, total;

    struct Meta {
        uint64_t off;
        uint32_t len, b, t;
        int r;
    };
    // tile idx's place; past the last tile, the last tile's place with no
    // elements (its loads then read one valid element, discarded)
    __device__ __forceinline__ Meta meta(uint32_t idx) const {
        const bool none = idx >= total;
        if (none) idx = total - 1;
        Meta m;
        m.r = idx < n0 ? 0 : 1;
        m.t = A.t0[m.r] + (m.r ? idx - n0 : idx);
        // the tile table is read-only here: scalar loads through the constant
        // address space (a vector load's wait would drain the previous tile's
        // stores before the next tile's loads are issued)
        const TileTable& tt = A.tt[m.r];
        typedef const __attribute__((address_space(4))) uint64_t* C64;
        typedef const __attribute__((address_space(4))) uint32_t* C32;
        m.off = ((C64)tt.off)[m.t];
        m.len = none ? 0u : ((C32)tt.len)[m.t];
        m.b = ((C32)tt.bucket)[m.t];
        return m;
    }
    // unconditional loads (clamped to the tile): a fixed count in flight, no
    // branches around them
    __device__ __forceinline__ void load(W (&v)[ITEMS], const Meta& m) const {
        const typename Lay::CView part = Lay::cview(A.part[m.r], A.pstride[m.r]) + m.off;
        const uint32_t lim = m.len ? m.len - 1 : 0u;
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint32_t i = elem(j);
            v[j] = part[i < lim ? i : lim];
        }
    }
    // the level-2 digits of the tile's elements, hist[d] += 1 (RANK false)
    // or the element staged at hist[d]++ (RANK true); recomputed in both
    // phases instead of held (the two register tiles leave no room)
    template <bool RANK>
    __device__ __forceinline__ void digits(const W (&v)[ITEMS], const Meta& m) const {
        const RangePlan& P = A.plan;
        if (A.d2_fast && m.b != 0 && m.b != (1u << P.D1) - 1) {
            const uint32_t base_lo = (uint32_t)P.base, mask = A.nb2 - 1;
#pragma unroll
            for (int j = 0; j < ITEMS; j++) {
                const uint32_t i = elem(j);
                if (i < m.len) {
                    const uint32_t d = Lay::digit_fast(v[j], base_lo, P.s1, P.s2, mask);
                    if (RANK)
                        stage[atomicAdd(&hist[d], 1u)] = v[j];
                    else
                        atomicAdd(&hist[d], 1u);
                }
            }
        } else {
#pragma unroll
            for (int j = 0; j < ITEMS; j++) {
                const uint32_t i = elem(j);
                if (i < m.len) {
                    const uint32_t d = plan_d2(P, Lay::rel(P, v[j], m.b), m.b);
                    if (RANK)
                        stage[atomicAdd(&hist[d], 1u)] = v[j];
                    else
                        atomicAdd(&hist[d], 1u);
                }
            }
        }
    }
    __device__ __forceinline__ void tile(const W (&v)[ITEMS], const Meta& m) const {
        const uint32_t nb2 = A.nb2;
        __syncthreads();  // the histogram is clear, the previous stage read out
        digits<false>(v, m);
        __syncthreads();
        const uint32_t per = (nb2 + TP_THREADS - 1) / TP_THREADS;
        const uint32_t d0 = threadIdx.x * per;
        uint32_t loc = 0;
        for (uint32_t k = 0; k < per; k++)
            if (d0 + k < nb2) loc += hist[d0 + k];
        uint32_t tot;
        uint32_t ex = block_exclusive_scan(loc, scr, &tot);
        uint16_t* pref = A.tt[m.r].pref + (uint64_t)m.t * (nb2 + 1);
        for (uint32_t k = 0; k < per; k++) {
            const uint32_t d = d0 + k;
            if (d < nb2) {
                const uint32_t c = hist[d];
                hist[d] = ex;
                pref[d] = (uint16_t)ex;
                ex += c;
            }
        }
        if (threadIdx.x == 0) pref[nb2] = (uint16_t)m.len;
        __syncthreads();
        digits<true>(v, m);
        __syncthreads();
        for (uint32_t d = threadIdx.x; d < nb2; d += TP_THREADS) hist[d] = 0;
        const typename LayO::View tmp = LayO::view(
            A.tmp[m.r], std::is_same<Lay, LayO>::value ? A.pstride[m.r] : A.ostride[m.r]) + m.off;
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint32_t i = elem(j);
            if (i < m.len) st_w(tmp + i, stage[i]);
        }
    }
};

template <class Lay, class LayO = Lay>
__global__ void __launch_bounds__(TP_THREADS)
k_tilepass_p(TilePassArgs A) {
    typedef TilePassP<Lay, LayO> TP;
    typedef typename TP::W W;
    static_assert(std::is_same<W, typename LayO::W>::value, "one element type");
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    if (A.pack_bad && *A.pack_bad) return;
    TP s{A};
    s.stage = reinterpret_cast<W*>(lds_raw);
    s.hist = reinterpret_cast<uint32_t*>(lds_raw + tile_elems<W>() * sizeof(W));
    s.scr = s.hist + A.nb2;
    uint32_t n[2];
    for (int r = 0; r < 2; r++)
        n[r] = A.nt[r] == 0 ? 0u : A.ntiles[r] ? min(*A.ntiles[r], A.nt[r]) : A.nt[r];
    s.n0 = n[0];
    s.total = n[0] + n[1];
    uint32_t idx = blockIdx.x;
    if (idx >= s.total) return;
    for (uint32_t d = threadIdx.x; d < A.nb2; d += TP_THREADS) s.hist[d] = 0;
    W a[TP::ITEMS], b[TP::ITEMS];
    typename TP::Meta ma = s.meta(idx), mb;
    s.load(a, ma);
    for (;;) {
        mb = s.meta(idx + gridDim.x);
        s.load(b, mb);
        s.tile(a, ma);
        if ((idx += gridDim.x) >= s.total) break;
        ma = s.meta(idx + gridDim.x);
        s.load(a, ma);
        s.tile(b, mb);
        if ((idx += gridDim.x) >= s.total) break;
    }
}

// ---------------------------------------------------------------------------
// prefix rows -> digit-major (prefT[d][t]): a group reads one entry per tile
// of its bucket, and the bucket's tiles are consecutive, so the group pass
// loads its run table with one or two lines per relation instead of one
// line per tile.  One block per 64 tiles of one relation (upper-bound grid
// when the tile count is only known on the device).
constexpr int PT_TILES = 64;
__global__ void __launch_bounds__(256)
k_preft(TileTable tt0, TileTable tt1, uint32_t nb0, const uint32_t* __restrict__ ntiles0,
        const uint32_t* __restrict__ ntiles1, uint32_t nt0_host, uint32_t nt1_host,
        uint32_t nb2) {
    extern __shared__ uint16_t sp[];  // [PT_TILES][nb2 + 1]
    const int r = blockIdx.x < nb0 ? 0 : 1;
    const TileTable& tt = r ? tt1 : tt0;
    const uint32_t ntl = (r ? ntiles1 : ntiles0) ? *(r ? ntiles1 : ntiles0)
                                                 : (r ? nt1_host : nt0_host);
    const uint32_t tb = (r ? blockIdx.x - nb0 : blockIdx.x) * PT_TILES;
    if (tb >= ntl) return;
    const uint32_t nt = min((uint32_t)PT_TILES, ntl - tb);
    const uint32_t row = nb2 + 1;
    const uint16_t* src = tt.pref + (uint64_t)tb * row;
    for (uint32_t i = threadIdx.x; i < nt * row; i += 256) sp[i] = src[i];
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < row * PT_TILES; i += 256) {
        const uint32_t d = i / PT_TILES, t = i % PT_TILES;
        if (t < nt) tt.prefT[(uint64_t)d * tt.tstride + tb + t] = sp[t * row + d];
    }
}

// ---------------------------------------------------------------------------
struct GroupArgs {
    const void* tmp[2];  // Lay::W elements (tile-pass output)
    Tup* out[2];
    const uint64_t* bstart[2];  // bucket start in the partition / tmp buffer
    const uint64_t* ostart[2];  // bucket start in the (dense) output
    TileTable tt[2];
    int nrel;
    RangePlan plan;  // by value: kernel arguments live in SGPRs
    unsigned long long* count_dev;
    uint32_t nb2;             // groups per bucket (= 1 << plan.D2 = pref stride - 1)
    uint32_t g_begin, g_end;  // groups b * nb2 + d2 of this launch
    uint32_t per;             // consecutive groups per workgroup
    OvfEntry* ovf;
    uint32_t* novf;
    uint32_t ovf_cap;
    const unsigned int* pack_bad;  // set: the packed partition is void, exit
    uint32_t d3_fast;              // Lay::fast_ok for the level-3 digit (host)
    uint64_t pstride[2] = {0, 0};  // plane stride of tmp (LayP48)
    // one relation (nrel == 1): two groups per loop iteration, one in each
    // relation slot (the slots' tables alias relation 0), so that a group's
    // gather flies under the other slot's sort as in the join
    uint32_t pair;
};

// threadIdx.x behind an empty asm: per-thread LDS addresses are recomputed
// where they are used instead of being hoisted out of the group loop (which
// ran the persistent kernel out of VGPRs)
__device__ __forceinline__ uint32_t otid() {
    uint32_t t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

template <class W>
struct GroupLDS {
    W B[GS_CAP + 1];                      // one relation's group (+ a dump slot)
    uint32_t cnt[2][GS_NB3 / 2];          // d3 histograms of R and S (2 x u16)
    uint32_t cur[GS_NB3 / 2];             // placement cursors (2 x u16)
    // the group's non-empty tile runs, numbered in position order: group
    // position j of run k sits at bucket offset j + run[k] (mod 2^32)
    uint32_t run[2][GS_TMAX];
    // per 64-position window w: bit i of m: a run starts at position 64 w + i;
    // wk: runs starting before the window, minus one (one 16-byte LDS read)
    struct alignas(16) Win {  // one 16-byte LDS read
        unsigned long long m;
        uint32_t wk, pad;
    } win[2][GS_WIN];
    uint32_t wtot[2][GS_THREADS / 64];
    uint32_t flags;  // sort_two's block vote: any repeated d3 digit (slot 0, 1), a clamped key
    unsigned long long scan64[GS_THREADS / 64 + 1];
    uint32_t n[2];
    uint32_t off[2];
};

// Where the group pass reads a tile's prefix entries (the digit-major uint16
// table of k_preft) and its elements.  A policy, so that another producer of
// the tiles (an earlier, fused form of the two passes: DESIGN.md §4) could
// plug in its own.
struct SrcPlain {
    // run [lo, lo + len) of group g in tile t
    __device__ static __forceinline__ void run(const TileTable& tt, uint32_t nb2, uint32_t t,
                                               uint32_t g, uint32_t& lo, uint32_t& len) {
        const uint16_t* pf = tt.prefT + (uint64_t)g * tt.tstride + t;
        lo = pf[0];
        len = (uint32_t)(pf[tt.tstride] - pf[0]);
    }
    template <class V>
    __device__ static __forceinline__ auto load(const V& p) { return p[0]; }
};

// A group and, for the calling thread, its tile run: wave r < nslot owns
// slot r (relation r; in pair mode the r-th group of the iteration), lane t
// its tile t (lo = run start in the tile, len = length).
template <int TPL>
struct GroupMeta {
    uint32_t b[2], g[2];    // bucket and level-2 digit of slot r's group
    uint32_t t0[2], nt[2];  // first tile and tile count of the bucket
    uint64_t bst[2];        // bucket start (partition buffer)
    uint64_t ost[2];        // bucket start (output)
    uint32_t lo[TPL], len[TPL];  // tiles lane + 64 h
    uint32_t toff[TPL];          // their offsets from the bucket start
};

// (PAIR, a template parameter of the kernel and the functions below, is the
// launch's A.pair)
template <bool PAIR>
__device__ __forceinline__ int group_slots(const GroupArgs& A) { return PAIR ? 2 : A.nrel; }

// Metadata of loop iteration j of a workgroup whose groups are g0, g0 +
// stride, ... (cnt of them): slot r holds group j (both relations) or, in
// pair mode, group 2j + r; a slot past the end is empty (no tiles).
template <class Src, bool PAIR, int TPL>
__device__ __forceinline__ void load_meta(const GroupArgs& A, uint32_t g0, uint32_t stride,
                                          uint32_t cnt, uint32_t j, GroupMeta<TPL>& M,
                                          bool same_bucket) {
    const int nslot = group_slots<PAIR>(A);
    auto bucket_meta = [&](int r, uint32_t b) {
        // uniform: keep them in SGPRs
        M.t0[r] = __builtin_amdgcn_readfirstlane(A.tt[r].btile0[b]);
        M.nt[r] = __builtin_amdgcn_readfirstlane(A.tt[r].btile0[b + 1]) - M.t0[r];
        const uint64_t bs = A.bstart[r][b];
        M.bst[r] = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(bs >> 32)) << 32) |
                   __builtin_amdgcn_readfirstlane((uint32_t)bs);
        const uint64_t os = A.ostart[r][b];
        M.ost[r] = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(os >> 32)) << 32) |
                   __builtin_amdgcn_readfirstlane((uint32_t)os);
    };
    if (!PAIR) {
        // both relations of one group: slot 0's b and g stand for both
        const uint32_t gi = g0 + j * stride;
        const uint32_t b = gi / A.nb2;
        M.g[0] = gi % A.nb2;
        if (!same_bucket || b != M.b[0]) {
#pragma unroll
            for (int r = 0; r < 2; r++) {
                M.t0[r] = M.nt[r] = 0;
                M.bst[r] = M.ost[r] = 0;
                if (r < A.nrel) bucket_meta(r, b);
            }
        }
        M.b[0] = b;
    } else {
#pragma unroll
        for (int r = 0; r < 2; r++) {
            const uint32_t k = 2 * j + r;
            const bool valid = k < cnt;  // uniform
            const uint32_t gi = g0 + k * stride;
            const uint32_t b = valid ? gi / A.nb2 : 0xffffffffu;
            M.g[r] = valid ? gi % A.nb2 : 0u;
            if (!valid) {
                M.t0[r] = M.nt[r] = 0;
                M.bst[r] = M.ost[r] = 0;
            } else if (!same_bucket || b != M.b[r]) {
                bucket_meta(r, b);
            }
            M.b[r] = b;
        }
    }
    // the wave index is uniform: table pointers stay scalar
    const uint32_t wid = __builtin_amdgcn_readfirstlane(otid() >> 6), lane = otid() & 63;
#pragma unroll
    for (int h = 0; h < TPL; h++) M.lo[h] = M.len[h] = M.toff[h] = 0;
    if (wid < (uint32_t)nslot) {
        const uint32_t nt = wid ? M.nt[1] : M.nt[0];
        const uint32_t t0 = wid ? M.t0[1] : M.t0[0];
        const uint32_t g = PAIR && wid ? M.g[1] : M.g[0];
#pragma unroll
        for (int h = 0; h < TPL; h++) {
            const uint32_t t = lane + 64 * h;
            if (nt <= 64 * TPL && t < nt) {
                // digit-major prefix (SrcPlain): lanes read consecutive entries
                Src::run(A.tt[wid], A.nb2, t0 + t, g, M.lo[h], M.len[h]);
                M.toff[h] = (uint32_t)(A.tt[wid].off[t0 + t] - (wid ? M.bst[1] : M.bst[0]));
            }
        }
    }
}

__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t x) {
    const int lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x;
}

__device__ __forceinline__ unsigned long long wave_incl_scan64(unsigned long long x) {
    const int lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x;
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// block-wide exclusive scan of one uint64 per thread
__device__ __forceinline__ unsigned long long block_scan64(unsigned long long v,
                                                           unsigned long long* scr,
                                                           unsigned long long* total) {
    const int lane = lane_id(), wid = otid() >> 6, nw = blockDim.x >> 6;
    const unsigned long long x = wave_incl_scan64(v);
    if (lane == 63) scr[wid] = x;
    __syncthreads();
    if (otid() == 0) {
        unsigned long long run = 0;
        for (int w = 0; w < nw; w++) {
            const unsigned long long t = scr[w];
            scr[w] = run;
            run += t;
        }
        scr[nw] = run;
    }
    __syncthreads();
    const unsigned long long r = scr[wid] + x - v;
    *total = scr[nw];
    __syncthreads();
    return r;
}

template <class Lay>
__device__ __forceinline__ void insertion_sort(typename Lay::W* a, uint32_t n) {
    for (uint32_t i = 1; i < n; i++) {
        typename Lay::W x = a[i];
        uint32_t j = i;
        while (j > 0 && Lay::less(x, a[j - 1])) {
            a[j] = a[j - 1];
            j--;
        }
        a[j] = x;
    }
}

// Group tables in LDS: wave r builds relation r's table of non-empty runs
// (compacted by ballot), the run-start bitmap and, per 64-position window,
// the number of runs that start before it (no block barrier inside; one at
// the end).  The run of position j is then wk[j/64] + (starts in its window
// up to j) - 1: two LDS round trips per gathered element, no search.
template <bool PAIR, int TPL, class LDS>
__device__ __forceinline__ void build_tables(const GroupArgs& A, LDS& L,
                                             const GroupMeta<TPL>& M) {
    const uint32_t wid = otid() >> 6, lane = otid() & 63;
    if (wid < (uint32_t)group_slots<PAIR>(A)) {
        const int r = wid;
        const uint32_t nt = r ? M.nt[1] : M.nt[0];
        if (lane < GS_WIN) L.win[r][lane].m = 0ull;
        // tiles lane + 64 h: scan of (start in tile << 32 | length), and the
        // non-empty runs compacted in tile order = position order (run starts
        // at or past GS_CAP only occur in groups that overflow: never gathered)
        unsigned long long acc = 0;
        uint32_t kacc = 0;
        uint32_t s[TPL], k[TPL];
        bool e[TPL];
#pragma unroll
        for (int h = 0; h < TPL; h++) {
            const unsigned long long p = ((unsigned long long)M.lo[h] << 32) | M.len[h];
            const unsigned long long incl = wave_incl_scan64(p) + acc;
            acc = __shfl(incl, 63, 64);
            s[h] = (uint32_t)(incl - p);
            e[h] = lane + 64 * h < nt && M.len[h] > 0 && s[h] < GS_CAP;
            const uint64_t bal = __ballot(e[h]);
            k[h] = kacc + (uint32_t)__popcll(bal & lanemask_lt());
            kacc += (uint32_t)__popcll(bal);
        }
#pragma unroll
        for (int h = 0; h < TPL; h++)
            if (e[h]) L.run[r][k[h]] = M.toff[h] + M.lo[h] - s[h];
        if (lane == 0) {
            L.n[r] = nt <= 64 * TPL ? (uint32_t)acc : 0xffffffffu;
            L.off[r] = (uint32_t)(acc >> 32);
        }
        wave_lds_sync();
#pragma unroll
        for (int h = 0; h < TPL; h++)
            if (e[h]) atomicOr(&L.win[r][s[h] >> 6].m, 1ull << (s[h] & 63));
        wave_lds_sync();
        const uint32_t c = lane < GS_WIN ? (uint32_t)__popcll(L.win[r][lane].m) : 0u;
        const uint32_t incl = wave_incl_scan32(c);
        if (lane < GS_WIN) L.win[r][lane].wk = incl - c - 1u;
    }
    __syncthreads();
}

// A group too large for LDS (or with long equal-digit runs out of order) is
// queued: its size and offset in each relation come from the prefix table,
// its tuples are sorted and counted afterwards by the skew kernels below, over
// many workgroups.  Called by the whole workgroup (uniform control flow).
// In pair mode `slot` names the one slot whose group is queued (as relation
// 0 of its entry); otherwise both relations of the group are.
template <class Src, bool PAIR, class LDS, class Meta>
__device__ __forceinline__ void group_overflow(const GroupArgs& A, LDS& L,
                                               const Meta& M, int slot = 0) {
    uint32_t nn[2] = {0, 0};
    uint64_t oo[2] = {0, 0};
    const uint32_t tid = otid();
    const int nq = PAIR ? 1 : A.nrel;
#pragma unroll
    for (int q = 0; q < 2; q++) {
        if (q >= nq) break;
        const int r = PAIR ? slot : q;
        const uint32_t t0 = r ? M.t0[1] : M.t0[0], nt = r ? M.nt[1] : M.nt[0];
        const uint32_t g = PAIR && r ? M.g[1] : M.g[0];
        unsigned long long acc = 0;
        for (uint32_t t = tid; t < nt; t += GS_THREADS) {
            uint32_t lo, len;
            Src::run(A.tt[r], A.nb2, t0 + t, g, lo, len);
            acc += ((unsigned long long)lo << 32) | len;
        }
        unsigned long long tot;
        (void)block_scan64(acc, L.scan64, &tot);
        nn[q] = (uint32_t)tot;
        oo[q] = tot >> 32;
    }
    if (tid == 0) {
        const uint32_t k = atomicAdd(A.novf, 1u);
        if (k < A.ovf_cap) {
            OvfEntry e;
            e.bucket = PAIR && slot ? M.b[1] : M.b[0];
            e.d2 = PAIR && slot ? M.g[1] : M.g[0];
            e.nr[0] = nn[0];
            e.nr[1] = nn[1];
            e.off[0] = oo[0];
            e.off[1] = oo[1];
            e.counted = 0;
            e.pad = 0;
            A.ovf[k] = e;
        }
    }
    __syncthreads();
}

// gather relation r's group into registers (loads only: every load in
// flight at once).  Position j = k * GS_THREADS + thread: a wave's 64
// positions are one bitmap window (broadcast read), so the run of the lane's
// position is the window's earlier runs plus the run starts below the lane
// (mbcnt) and at it.  Branch-free (the compiler may then keep several
// elements' LDS reads in flight): a position past the end has every run start
// below it, so its run is the last one, and it re-reads the group's last
// element (p = n - 1).
template <class Lay, class Src, class Meta>
__device__ __forceinline__ void gather_group(const GroupArgs& A, GroupLDS<typename Lay::W>& L,
                                             const Meta& C, int r, uint32_t grp, uint32_t n,
                                             typename Lay::W (&v)[GS_ITEMS]) {
    if (n == 0) return;
    const typename Lay::CView tp =
        with_group(Lay::cview(A.tmp[r], A.pstride[r]), grp, A.plan) + C.bst[r];
    const uint32_t lane = lane_id();
    const uint32_t wid = __builtin_amdgcn_readfirstlane(otid() >> 6);
    typedef uint32_t U4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int k = 0; k < GS_ITEMS; k++) {
        const uint32_t w = k * (GS_THREADS / 64) + wid;  // uniform
        const U4 win = *reinterpret_cast<const U4*>(&L.win[r][w]);
        const uint32_t below = __builtin_amdgcn_mbcnt_hi(win.y, __builtin_amdgcn_mbcnt_lo(win.x, 0u));
        const uint32_t at = (uint32_t)((((uint64_t)win.y << 32) | win.x) >> lane) & 1u;
        const uint32_t j = w * 64 + lane;
        v[k] = Src::load(tp + (min(j, n - 1) + L.run[r][win.z + below + at]));
    }
}

// Sort relation r's group (in registers) by the level-3 digit in LDS and
// write it to out at offset `off` of its bucket.  `after_place` runs as soon
// as the elements sit in LDS (the registers are free): the persistent loop
// issues the next group's gather there.  Returns false when the group must
// take the skew path.
template <class Lay, bool PAIR, class Meta, typename Hook>
__device__ __forceinline__ bool sort_group(const GroupArgs& A, GroupLDS<typename Lay::W>& L,
                                           const Meta& C, const RangePlan& P,
                                           int r, uint32_t nr, uint32_t off,
                                           typename Lay::W (&v)[GS_ITEMS], bool& clamped,
                                           Hook&& after_place) {
    const uint32_t tid = otid(), wid = tid >> 6, lane = tid & 63;
    const uint32_t cb = PAIR && r ? C.b[1] : C.b[0], cg = PAIR && r ? C.g[1] : C.g[0];
    const uint32_t d12 = (cb << P.D2) | cg;
    // ---- level-3 digits, histogram (two u16 counters per word).  Only the
    // first and the last group of the plan can hold keys outside its range
    // (plan_rel clamps them there); every other group takes the 32-bit digit.
    uint32_t dg[GS_ITEMS];
    const bool edge = (cb == 0 && cg == 0) ||
                      (cb == (1u << P.D1) - 1 && cg == A.nb2 - 1);
    if (A.d3_fast && !edge) {
        const uint32_t base_lo = (uint32_t)P.base, mask = (1u << P.D3) - 1;
#pragma unroll
        for (int k = 0; k < GS_ITEMS; k++) {
            const bool valid = k * GS_THREADS + tid < nr;
            dg[k] = Lay::digit_fast(v[k], base_lo, P.s1, P.s3, mask);
            if (valid) atomicAdd(&L.cnt[r][dg[k] >> 1], 1u << ((dg[k] & 1) * 16));
        }
    } else {
#pragma unroll
        for (int k = 0; k < GS_ITEMS; k++) {
            const bool valid = k * GS_THREADS + tid < nr;
            clamped |= valid && Lay::clamped(P, v[k]);
            dg[k] = plan_d3(P, Lay::rel(P, v[k], cb), d12);
            if (valid) atomicAdd(&L.cnt[r][dg[k] >> 1], 1u << ((dg[k] & 1) * 16));
        }
    }
    __syncthreads();
    // ---- exclusive scan of the bins: thread owns GS_BPT consecutive bins;
    // wave totals meet in LDS (two barriers, one carries the "any equal-digit
    // run" vote)
    uint32_t c[GS_BPT];
    uint32_t loc = 0, mx = 0;
#pragma unroll
    for (int q = 0; q < GS_BPT / 2; q++) {
        const uint32_t wv = L.cnt[r][tid * (GS_BPT / 2) + q];
        c[2 * q] = wv & 0xffffu;
        c[2 * q + 1] = wv >> 16;
        loc += c[2 * q] + c[2 * q + 1];
        mx = max(mx, max(c[2 * q], c[2 * q + 1]));
    }
    const uint32_t incl = wave_incl_scan32(loc);
    if (lane == 63) L.wtot[0][wid] = incl;
    const bool dup = __syncthreads_or(mx > 1);
    uint32_t ex = incl - loc;
#pragma unroll
    for (uint32_t w = 0; w < GS_THREADS / 64; w++)
        if (w < wid) ex += L.wtot[0][w];
    const uint32_t first = ex;
#pragma unroll
    for (int q = 0; q < GS_BPT / 2; q++) {
        const uint32_t lo16 = ex;
        ex += c[2 * q];
        L.cur[tid * (GS_BPT / 2) + q] = lo16 | (ex << 16);
        ex += c[2 * q + 1];
    }
    __syncthreads();
    // ---- place (lanes past the end drop their element in the dump slot).
    // Every digit at most once (no equal-digit run: a PK relation's groups):
    // the bin's start is the element's place, read without an atomic.
#pragma unroll
    for (int k = 0; k < GS_ITEMS; k++) {
        const bool valid = k * GS_THREADS + tid < nr;
        const uint32_t sh = (dg[k] & 1) * 16;
        const uint32_t old = dup ? atomicAdd(&L.cur[dg[k] >> 1], valid ? 1u << sh : 0u)
                                 : L.cur[valid ? dg[k] >> 1 : 0u];
        L.B[valid ? (old >> sh) & 0xffffu : GS_CAP] = v[k];
    }
    after_place();
    __syncthreads();
    if (dup) {
        // ---- equal-digit runs.  The group is ordered by digit, so an
        // inversion can only sit inside such a run: one parallel pass finds
        // out whether any needs sorting (never for equal tuples of a hot key).
        // If so, short runs are insertion-sorted by their bin's thread; long
        // ones must already be in order, otherwise the skew path.
        bool ok = true;
        for (uint32_t i = tid + 1; i < nr; i += GS_THREADS)
            ok &= !Lay::less(L.B[i], L.B[i - 1]);
        if (__syncthreads_or(!ok)) {
            uint32_t e = first;
            bool has_long = false;
#pragma unroll
            for (int q = 0; q < GS_BPT; q++) {
                const uint32_t b0 = e;
                e += c[q];
                if (c[q] > 1) {
                    if (c[q] <= GS_RUNMAX)
                        insertion_sort<Lay>(L.B + b0, c[q]);
                    else
                        has_long = true;
                }
            }
            if (__syncthreads_or(has_long)) {
                ok = true;
                for (uint32_t i = tid + 1; i < nr; i += GS_THREADS)
                    ok &= !Lay::less(L.B[i], L.B[i - 1]);
                if (__syncthreads_or(!ok)) return false;
            }
        }
    }
    // ---- write the sorted group: one contiguous stream
    Tup* dst = A.out[r] + C.ost[r] + off;
#pragma unroll
    for (int k = 0; k < GS_ITEMS; k++) {
        const uint32_t j = k * GS_THREADS + tid;
        if (j < nr) st_stream(dst + j, Lay::unpack(P, L.B[j], cb));
    }
    return true;
}

// Hide a value from the optimiser (an empty asm that "changes" its words):
// the value is recomputed from it instead of being kept alive.
template <class T>
__device__ __forceinline__ void launder(T& x) {
    static_assert(sizeof(T) % 4 == 0, "word-sized");
    uint32_t* w = reinterpret_cast<uint32_t*>(&x);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); i++) asm volatile("" : "+v"(w[i]));
}

// Equal-digit runs of one sorted slot in B (see sort_group): false when a
// long run is out of order (the skew path).  c / first: the calling thread's
// bins' counts and the start of its first bin.
template <class Lay>
__device__ __forceinline__ bool fix_runs(GroupLDS<typename Lay::W>& L, uint32_t nr,
                                         const uint32_t (&c)[GS_BPT], uint32_t first) {
    const uint32_t tid = otid();
    bool ok = true;
    for (uint32_t i = tid + 1; i < nr; i += GS_THREADS) ok &= !Lay::less(L.B[i], L.B[i - 1]);
    if (!__syncthreads_or(!ok)) return true;
    uint32_t e = first;
    bool has_long = false;
#pragma unroll
    for (int q = 0; q < GS_BPT; q++) {
        const uint32_t b0 = e;
        e += c[q];
        if (c[q] > 1) {
            if (c[q] <= GS_RUNMAX)
                insertion_sort<Lay>(L.B + b0, c[q]);
            else
                has_long = true;
        }
    }
    if (__syncthreads_or(has_long)) {
        ok = true;
        for (uint32_t i = tid + 1; i < nr; i += GS_THREADS) ok &= !Lay::less(L.B[i], L.B[i - 1]);
        if (__syncthreads_or(!ok)) return false;
    }
    return true;
}

// Both slots' groups (R and S of one group, or pair mode's two groups of one
// relation) through ONE chain of barriers (round 4): the two d3 histograms,
// their scans and cursors are built together, then slot 0 is placed, fixed
// and written, then slot 1.  sort_group ran the whole chain once per slot
// (hist | scan | cursors | place | write, twice: 8 block barriers per join
// group); here it is 6.  LDS is unchanged: slot 1's cursors overwrite its
// counts in L.cnt[1] (the owning thread keeps the counts in registers, and
// computes the exact-key match count from them during the scan), and every
// thread zeroes its own bins at the end, so no barrier clears the histograms.
// Only called when both slots' groups fit.  join: nrel == 2 (a failed slot 0
// skips slot 1, the caller queues both, as sort_group's callers do).
// Returns bit r set = slot r must take the skew path; `exact` reports whether
// `matches` got the exact-key count (otherwise the caller counts by search).
template <class Lay, bool PAIR, class Meta, typename Hook0, typename Hook1>
__device__ __forceinline__ uint32_t sort_two(const GroupArgs& A, GroupLDS<typename Lay::W>& L,
                                             const Meta& C, const RangePlan& P,
                                             const uint32_t (&nr)[2], const uint32_t (&off)[2],
                                             typename Lay::W (&v0)[GS_ITEMS],
                                             typename Lay::W (&v1)[GS_ITEMS], bool join,
                                             unsigned long long& matches, bool& exact,
                                             Hook0&& after0, Hook1&& after1) {
    typedef typename Lay::W W;
    const uint32_t tid = otid(), wid = tid >> 6, lane = tid & 63;
    // the d3 digit of slot r's elements: the fast form unless the group is
    // an edge group of the plan (the branch is uniform: taken outside the
    // loops, as in sort_group).  Recomputed where needed (two digit arrays
    // held over the scans would push the kernel past 128 VGPRs).
    auto fast = [&](int r) {
        const uint32_t cb = PAIR && r ? C.b[1] : C.b[0], cg = PAIR && r ? C.g[1] : C.g[0];
        const bool edge = (cb == 0 && cg == 0) || (cb == (1u << P.D1) - 1 && cg == A.nb2 - 1);
        return A.d3_fast && !edge;
    };
    auto slow_digit = [&](int r, const W& x) -> uint32_t {
        const uint32_t cb = PAIR && r ? C.b[1] : C.b[0], cg = PAIR && r ? C.g[1] : C.g[0];
        return plan_d3(P, Lay::rel(P, x, cb), (cb << P.D2) | cg);
    };
    const uint32_t base_lo = (uint32_t)P.base, mask3 = (1u << P.D3) - 1;
    bool clamped = false;
    auto hist = [&](int r, const W(&v)[GS_ITEMS]) {
        if (fast(r)) {
            const typename Lay::FastDigit fd(P, P.s3, P.D3);
#pragma unroll
            for (int k = 0; k < GS_ITEMS; k++) {
                const uint32_t d = fd(v[k]);
                if (k * GS_THREADS + tid < nr[r])
                    atomicAdd(&L.cnt[r][d >> 1], 1u << ((d & 1) * 16));
            }
        } else {
#pragma unroll
            for (int k = 0; k < GS_ITEMS; k++) {
                const bool valid = k * GS_THREADS + tid < nr[r];
                clamped |= valid && Lay::clamped(P, v[k]);
                const uint32_t d = slow_digit(r, v[k]);
                if (valid) atomicAdd(&L.cnt[r][d >> 1], 1u << ((d & 1) * 16));
            }
        }
    };
    hist(0, v0);
    hist(1, v1);
    __syncthreads();
    // ---- both scans
    uint32_t w0[GS_BPT / 2], w1[GS_BPT / 2];
    uint32_t loc0 = 0, loc1 = 0, mx0 = 0, mx1 = 0;
#pragma unroll
    for (int q = 0; q < GS_BPT / 2; q++) {
        w0[q] = L.cnt[0][tid * (GS_BPT / 2) + q];
        w1[q] = L.cnt[1][tid * (GS_BPT / 2) + q];
        const uint32_t a0 = w0[q] & 0xffffu, a1 = w0[q] >> 16;
        const uint32_t b0 = w1[q] & 0xffffu, b1 = w1[q] >> 16;
        loc0 += a0 + a1;
        loc1 += b0 + b1;
        mx0 = max(mx0, max(a0, a1));
        mx1 = max(mx1, max(b0, b1));
    }
    const uint32_t incl0 = wave_incl_scan32(loc0), incl1 = wave_incl_scan32(loc1);
    if (lane == 63) {
        L.wtot[0][wid] = incl0;
        L.wtot[1][wid] = incl1;
    }
    const uint32_t vote = (mx0 > 1 ? 1u : 0u) | (mx1 > 1 ? 2u : 0u) | (clamped ? 4u : 0u);
    if (vote) atomicOr(&L.flags, vote);
    __syncthreads();
    const uint32_t fl = __builtin_amdgcn_readfirstlane(L.flags);
    exact = join && P.s3 == 0 && !(fl & 4);
    // the level-3 digit is the exact key: sum_k |R_k| * |S_k| over the owned
    // bins, added once both slots are sorted (the skew path counts a queued
    // group itself)
    unsigned long long m = 0;
    if (exact) {
#pragma unroll
        for (int q = 0; q < GS_BPT / 2; q++)
            m += (unsigned long long)(w0[q] & 0xffffu) * (w1[q] & 0xffffu) +
                 (unsigned long long)(w0[q] >> 16) * (w1[q] >> 16);
    }
    uint32_t ex0 = incl0 - loc0, ex1 = incl1 - loc1;
#pragma unroll
    for (uint32_t w = 0; w < GS_THREADS / 64; w++)
        if (w < wid) {
            ex0 += L.wtot[0][w];
            ex1 += L.wtot[1][w];
        }
#pragma unroll
    for (int q = 0; q < GS_BPT / 2; q++) {
        uint32_t lo16 = ex0;
        ex0 += w0[q] & 0xffffu;
        L.cur[tid * (GS_BPT / 2) + q] = lo16 | (ex0 << 16);
        ex0 += w0[q] >> 16;
        lo16 = ex1;
        ex1 += w1[q] & 0xffffu;
        L.cnt[1][tid * (GS_BPT / 2) + q] = lo16 | (ex1 << 16);
        ex1 += w1[q] >> 16;
    }
    __syncthreads();
    // the vote has been read by every thread (before the barrier above)
    if (tid == 0) L.flags = 0;
    auto place1 = [&](uint32_t* cur, bool dup, bool valid, uint32_t d, const W& x) {
        const uint32_t sh = (d & 1) * 16;
        const uint32_t old = dup ? atomicAdd(&cur[d >> 1], valid ? 1u << sh : 0u)
                                 : cur[valid ? d >> 1 : 0u];
        L.B[valid ? (old >> sh) & 0xffffu : GS_CAP] = x;
    };
    // one loop per (digit form, placement form): `dup` is uniform, and
    // tested inside the element loop it made every element wait for the LDS
    // queue before and after its cursor read; unswitched, the plain reads of
    // the no-repeat form are in flight together
    auto place_loop = [&](int r, uint32_t* cur, const W(&v)[GS_ITEMS], auto&& digit,
                          auto dupc) {
#pragma unroll
        for (int k = 0; k < GS_ITEMS; k++) {
            // an opaque copy of each element: otherwise the compiler keeps the
            // histogram's digits alive over the scans instead of recomputing
            W x = v[k];
            launder(x);
            place1(cur, decltype(dupc)::value, k * GS_THREADS + tid < nr[r], digit(x), v[k]);
        }
    };
    auto place = [&](int r, uint32_t* cur, bool dup, const W(&v)[GS_ITEMS]) {
        typedef std::integral_constant<bool, true> Dup;
        typedef std::integral_constant<bool, false> NoDup;
        if (fast(r)) {
            const typename Lay::FastDigit fd(P, P.s3, P.D3);
            if (dup) place_loop(r, cur, v, fd, Dup());
            else place_loop(r, cur, v, fd, NoDup());
        } else {
            auto sd = [&](const W& x) { return slow_digit(r, x); };
            if (dup) place_loop(r, cur, v, sd, Dup());
            else place_loop(r, cur, v, sd, NoDup());
        }
    };
    // after a placement by atomics every cursor word holds its two bins'
    // ends: the owned bins' counts come back from them and the thread's
    // first start (no count registers held over the placement)
    auto fix = [&](int r, const uint32_t* cur) {
        uint32_t c[GS_BPT];
        // the first owned bin starts where the previous thread's last ends
        const uint32_t first = tid ? cur[tid * (GS_BPT / 2) - 1] >> 16 : 0u;
        uint32_t prev = first;
#pragma unroll
        for (int q = 0; q < GS_BPT / 2; q++) {
            const uint32_t e = cur[tid * (GS_BPT / 2) + q];
            c[2 * q] = (e & 0xffffu) - prev;
            c[2 * q + 1] = (e >> 16) - (e & 0xffffu);
            prev = e >> 16;
        }
        return fix_runs<Lay>(L, nr[r], c, first);
    };
    auto write = [&](int r) {
        const uint32_t cb = PAIR && r ? C.b[1] : C.b[0];
        Tup* dst = A.out[r] + C.ost[r] + off[r];
        const typename Lay::Unpack up(P, cb);
#pragma unroll
        for (int k = 0; k < GS_ITEMS; k++) {
            const uint32_t j = k * GS_THREADS + tid;
            if (j < nr[r]) st_stream(dst + j, up(L.B[j]));
        }
    };
    uint32_t failed = 0;
    // ---- slot 0
    place(0, L.cur, fl & 1, v0);
    after0();
    __syncthreads();
    if ((fl & 1) && !fix(0, L.cur)) failed |= 1;
    if (!failed) write(0);
    // ---- slot 1 (a join whose R failed leaves S to the skew path too)
    if (!(join && failed)) {
        __syncthreads();  // B is free again
        place(1, L.cnt[1], fl & 2, v1);
        after1();
        __syncthreads();
        if ((fl & 2) && !fix(1, L.cnt[1])) failed |= 2;
        if (!(failed & 2)) write(1);
    } else {
        after1();
        __syncthreads();  // slot 1's cursors are read no more
    }
    // the owned bins: zero for the next group (cursors and counts read no more)
#pragma unroll
    for (int q = 0; q < GS_BPT / 2; q++) {
        L.cnt[0][tid * (GS_BPT / 2) + q] = 0u;
        L.cnt[1][tid * (GS_BPT / 2) + q] = 0u;
    }
    if (!failed) matches += m;
    return failed;
}

// Merge-join count of a group whose last digit is not the exact key: S's
// sorted group is still in B, R's is in out (written by this workgroup before
// a barrier, so visible); every S key run binary-searches R.
template <class Lay, class Meta>
__device__ __forceinline__ void count_by_search(const GroupArgs& A, GroupLDS<typename Lay::W>& L,
                                                const Meta& C, const RangePlan& P,
                                                const uint32_t (&cn)[2], const uint32_t (&co)[2],
                                                unsigned long long& matches) {
    const uint32_t tid = otid();
    const Tup* Rs = A.out[0] + C.ost[0] + co[0];
    const uint32_t nR = cn[0], nS = cn[1];
    for (uint32_t i = tid; i < nS; i += GS_THREADS) {
        const int64_t k = tup_key(Lay::unpack(P, L.B[i], C.b[0]));
        if (i > 0 && tup_key(Lay::unpack(P, L.B[i - 1], C.b[0])) == k) continue;
        uint32_t e = i + 1;
        while (e < nS && tup_key(Lay::unpack(P, L.B[e], C.b[0])) == k) e++;
        uint32_t lo = 0, hi = nR;
        while (lo < hi) {
            const uint32_t m = (lo + hi) >> 1;
            if (tup_key(Rs[m]) < k) lo = m + 1; else hi = m;
        }
        const uint32_t lb = lo;
        hi = nR;
        while (lo < hi) {
            const uint32_t m = (lo + hi) >> 1;
            if (tup_key(Rs[m]) <= k) lo = m + 1; else hi = m;
        }
        matches += (unsigned long long)(lo - lb) * (e - i);
    }
}

// Groups g0, g0 + stride, ... (cnt of them) in order, software-pipelined
// across groups: the next group's tables are built while the current one's
// data is in registers, its R is gathered as soon as the current R sits in
// LDS and its S as soon as the current S does, so both gathers fly under the
// current sort, write-out and count; the tile runs of the group after next are
// loaded one group further ahead.  Matches are added to `matches`.  In pair
// mode (one relation) an iteration takes two consecutive groups of the
// sequence, one per slot, pipelined the same way.
template <class Lay, int TPL, class Src, bool PAIR>
__device__ __forceinline__ void group_loop(const GroupArgs& A0, GroupLDS<typename Lay::W>& L,
                                           uint32_t g0, uint32_t stride, uint32_t cnt,
                                           unsigned long long& matches) {
    typedef typename Lay::W W;
    const GroupArgs& A = A0;
    const RangePlan& P = A.plan;
    const uint32_t tid = otid();
    const int nrel = A.nrel;
    constexpr bool pair = PAIR;
    const int nslot = group_slots<PAIR>(A);
    if (cnt == 0) return;
    const uint32_t nit = pair ? (cnt + 1) / 2 : cnt;
    // a slot's group fits in LDS; without pair mode a group fits when both
    // of its relations do
    auto fits = [&](const uint32_t (&n)[2], bool f[2]) {
        f[0] = n[0] <= GS_CAP;
        f[1] = n[1] <= GS_CAP;
        if (!pair) f[0] = f[1] = f[0] && f[1];
    };

    for (uint32_t i = tid; i < GS_NB3; i += GS_THREADS) (&L.cnt[0][0])[i] = 0u;
    if (tid == 0) L.flags = 0u;
    GroupMeta<TPL> M;
    load_meta<Src, PAIR>(A, g0, stride, cnt, 0, M, false);
    build_tables<PAIR>(A, L, M);
    GroupMeta<TPL> C = M;
    uint32_t cn[2], co[2];
#pragma unroll
    for (int r = 0; r < 2; r++) {
        cn[r] = r < nslot ? __builtin_amdgcn_readfirstlane(L.n[r]) : 0;
        co[r] = r < nslot ? __builtin_amdgcn_readfirstlane(L.off[r]) : 0;
    }
    bool cf[2];
    fits(cn, cf);
    W vr[GS_ITEMS], vs[GS_ITEMS];
    // slot r's group digit (both slots hold one group in a join)
    auto slot_g = [&](const GroupMeta<TPL>& X, int r) { return PAIR && r ? X.g[1] : X.g[0]; };
    if (cf[0]) gather_group<Lay, Src>(A, L, C, 0, slot_g(C, 0), cn[0], vr);
    if (cf[1] && nslot > 1) gather_group<Lay, Src>(A, L, C, 1, slot_g(C, 1), cn[1], vs);
    if (nit > 1 && SMJ_GS_META_PREFETCH) load_meta<Src, PAIR>(A, g0, stride, cnt, 1, M, true);

    for (uint32_t j = 0; j < nit; j++) {
#if SMJ_GS_ARGS_MEM
        // the arguments again, from memory (opaque pointer: not hoisted)
        typedef const __attribute__((address_space(4))) GroupArgs* ConstArgs;
        ConstArgs Aj = (ConstArgs)&A0;  // constant memory: scalar loads
        asm volatile("" : "+s"(Aj));
        const GroupArgs& A = *(const GroupArgs*)Aj;
        const RangePlan& P = A.plan;
#endif
        const bool has_next = j + 1 < nit;
        if (!SMJ_GS_META_PREFETCH && has_next) load_meta<Src, PAIR>(A, g0, stride, cnt, j + 1, M, true);
        // every lane's gather of group gi has read the tables: rebuild them
        __syncthreads();
        const GroupMeta<TPL> N = M;
        uint32_t nn[2] = {0, 0}, no[2] = {0, 0};
        if (has_next) {
            build_tables<PAIR>(A, L, N);
#pragma unroll
            for (int r = 0; r < 2; r++) {
                nn[r] = r < nslot ? __builtin_amdgcn_readfirstlane(L.n[r]) : 0;
                no[r] = r < nslot ? __builtin_amdgcn_readfirstlane(L.off[r]) : 0;
            }
        }
        if (SMJ_GS_META_PREFETCH && j + 2 < nit)
            load_meta<Src, PAIR>(A, g0, stride, cnt, j + 2, M, true);
        bool nf[2];
        fits(nn, nf);
        nf[0] &= has_next;
        nf[1] &= has_next;
        auto gather_next_r = [&]() {
            if (nf[0]) gather_group<Lay, Src>(A, L, N, 0, slot_g(N, 0), nn[0], vr);
        };
        auto gather_next_s = [&]() {
            if (nf[1] && nslot > 1) gather_group<Lay, Src>(A, L, N, 1, slot_g(N, 1), nn[1], vs);
        };
        bool cleared = false;  // sort_two zeroed the histograms itself
        if (SMJ_GS_TWO && nslot == 2 && (pair || (cf[0] && cf[1]))) {
            // ---- both slots in one barrier chain (sort_two).  Pair mode: a
            // slot whose group does not fit goes in empty and is queued below
            const bool join = !pair;
            bool exact = false;
            const uint32_t nr2[2] = {cf[0] ? cn[0] : 0u, cf[1] ? cn[1] : 0u};
            const uint32_t failed = sort_two<Lay, PAIR>(A, L, C, P, nr2, co, vr, vs, join, matches,
                                                         exact, gather_next_r, gather_next_s);
            cleared = true;
            if (join) {
                if (failed) {
                    __syncthreads();
                    group_overflow<Src, PAIR>(A, L, C);
                } else if (!exact) {
                    count_by_search<Lay>(A, L, C, P, cn, co, matches);
                }
            } else {
                for (int q = 0; q < 2; q++)
                    if (!cf[q] || (failed & (1u << q))) {
                        __syncthreads();
                        group_overflow<Src, PAIR>(A, L, C, q);
                    }
            }
        } else if (pair && !SMJ_GS_TWO) {
            // ---- two groups of one relation, independently: a group that
            // does not fit or fails is queued for the skew path on its own
            bool clamped = false;
            bool ok = cf[0] && sort_group<Lay, PAIR>(A, L, C, P, 0, cn[0], co[0], vr, clamped,
                                               gather_next_r);
            if (!cf[0]) gather_next_r();
            if (!ok) {
                __syncthreads();
                group_overflow<Src, PAIR>(A, L, C, 0);
            }
            ok = cf[1] && sort_group<Lay, PAIR>(A, L, C, P, 1, cn[1], co[1], vs, clamped,
                                          gather_next_s);
            if (!cf[1]) gather_next_s();
            if (!ok) {
                __syncthreads();
                group_overflow<Src, PAIR>(A, L, C, 1);
            }
        } else if (!cf[0] || (SMJ_GS_TWO && SMJ_GS_PAIR)) {
            // With sort_two and pair mode, a non-pair kernel only runs joins
            // (nrel 2), whose groups reach here only when they do not fit:
            // the per-slot path below is then compiled out (kept in, it
            // pushes the join kernel past 128 VGPRs into scratch)
            group_overflow<Src, PAIR>(A, L, C);
            gather_next_r();
            gather_next_s();
        } else {
            bool clamped = false;
            bool ok = sort_group<Lay, PAIR>(A, L, C, P, 0, cn[0], co[0], vr, clamped, gather_next_r);
            bool s_issued = false;
            if (ok && nrel > 1) {
                ok = sort_group<Lay, PAIR>(A, L, C, P, 1, cn[1], co[1], vs, clamped, gather_next_s);
                s_issued = true;
            }
            if (!ok) {
                __syncthreads();
                group_overflow<Src, PAIR>(A, L, C);
                if (!s_issued) gather_next_s();
            } else if (nrel == 2) {
                // ---- merge-join count of the two groups
                const bool exact = P.s3 == 0 && !__syncthreads_or(clamped);
                if (exact) {
                    // the level-3 digit is the exact key: sum_k |R_k| * |S_k|
#pragma unroll
                    for (int q = 0; q < GS_BPT / 2; q++) {
                        const uint32_t a0 = L.cnt[0][tid * (GS_BPT / 2) + q];
                        const uint32_t a1 = L.cnt[1][tid * (GS_BPT / 2) + q];
                        matches += (unsigned long long)(a0 & 0xffffu) * (a1 & 0xffffu) +
                                   (unsigned long long)(a0 >> 16) * (a1 >> 16);
                    }
                } else {
                    count_by_search<Lay>(A, L, C, P, cn, co, matches);
                }
            }
        }
        if (!cleared) {
            __syncthreads();  // histograms and B are reused by the next group
            for (uint32_t i = tid; i < GS_NB3; i += GS_THREADS) (&L.cnt[0][0])[i] = 0u;
        }
        C = N;
        cn[0] = nn[0];
        cn[1] = nn[1];
        co[0] = no[0];
        co[1] = no[1];
        cf[0] = nf[0];
        cf[1] = nf[1];
    }
}

// Persistent: every workgroup sorts `per` groups in order (group_loop).
// XCD-aware: blocks b and b + 8 share an XCD and its L2 (MI355X_MICROARCH
// [G]: observed placement, used for speed only).  The blocks of one XCD take
// one contiguous range of groups, interleaved (block k of the XCD: groups
// lo + k, lo + k + nx, ...), so at any moment they sort neighbouring groups:
// the 128-byte line that two neighbouring groups' runs share in a tile is
// fetched into that L2 once instead of once per XCD.  The grid is a multiple
// of 8 (launch_groupsort).
#if SMJ_GS_ARGS_MEM
typedef const GroupArgs* __restrict__ GroupArgsParam;
#define SMJ_GS_ARGS_REF(p) (*(p))
#else
typedef GroupArgs GroupArgsParam;
#define SMJ_GS_ARGS_REF(p) (p)
#endif

__global__ void k_put_args(GroupArgs G, GroupArgs* dst) { *dst = G; }

template <class Lay, int TPL, bool PAIR>
__global__ void __launch_bounds__(GS_THREADS,
                                  (gs_wg_per_cu<typename Lay::W, PAIR>() * GS_THREADS / 256))
k_groupsort(GroupArgsParam Ap) {
    typedef typename Lay::W W;
    const GroupArgs& A = SMJ_GS_ARGS_REF(Ap);
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    if (A.pack_bad && *A.pack_bad) return;
    GroupLDS<W>& L = *reinterpret_cast<GroupLDS<W>*>(lds_raw);
#if SMJ_GS_XCD
    const uint32_t nx = gridDim.x / 8, k = blockIdx.x / 8;
    const uint32_t lo = A.g_begin + (blockIdx.x % 8) * nx * A.per;
    const uint32_t g0 = lo + k, stride = nx;
    const uint32_t hi = min(lo + nx * A.per, A.g_end);
    const uint32_t cnt = g0 < hi ? (hi - g0 + nx - 1) / nx : 0u;
#else
    const uint32_t g0 = A.g_begin + blockIdx.x * A.per, stride = 1;
    const uint32_t cnt = g0 < A.g_end ? min(A.per, A.g_end - g0) : 0u;
#endif
    unsigned long long matches = 0;
    if (cnt == 0) return;
    group_loop<Lay, TPL, SrcPlain, PAIR>(A, L, g0, stride, cnt, matches);
    if (A.nrel == 2) {
        matches = wave_sum(matches);
        if ((otid() & 63) == 0 && matches) atomicAdd(A.count_dev, matches);
    }
}

// ---------------------------------------------------------------------------
// Skew path on the device: the queued groups (too large for LDS, e.g. the
// groups of hot Zipf keys) are counting-sorted by the last digit through HBM.
// The host sorts the queue by size once it has read it:
//   k_skew_small : one workgroup per group of up to kSkewSmall tuples per
//                  relation: d3 histograms in LDS (exact digits give the
//                  match count sum_k |R_k|*|S_k|), cursors, placement in
//                  `out`, then a check that equal-key runs came out in
//                  (key, payload) order
//   larger groups are split over many workgroups, one work item = one
//   relation of one group and every ts-th tile run of it:
//   k_skew_hist  : d3 histogram of the item's runs -> the group's global
//                  histogram; flags keys outside the plan (digit not exact)
//   k_skew_scan  : per group: match count, histograms -> cursors
//   k_skew_place : every run chunk reserves its digits' ranges at the group's
//                  cursors and places its tuples (inexact groups: the run is
//                  copied unsorted to its place in the group)
//   k_skew_check : per group: equal-key runs in (key, payload) order?
// What is left (inexact digits, equal-key runs out of payload order) goes to
// the host-driven merge sort and merge-join count.
#ifndef SMJ_SK_THREADS
#define SMJ_SK_THREADS 256
#endif
constexpr int SK_THREADS = SMJ_SK_THREADS;
constexpr int SK_ITEMS = 8;
constexpr int SK_CHUNK = SK_THREADS * SK_ITEMS;
constexpr uint32_t kSkewSmall = SK_THREADS * 64;  // tuples per relation, one workgroup
#ifndef SMJ_SKEW_ITEM
#define SMJ_SKEW_ITEM 8192  // tuples per work item of a large skew group (2048 measured slower)
#endif
constexpr int SK_TM = 256;              // tile runs in LDS tables (small groups)

struct SkewArgs {
    GroupArgs G;
    OvfEntry* q;            // every queued group
    const uint32_t* list;   // k_skew_small / _scan / _check: group indices
    const uint4* items;     // large groups: {group, slot, r << 16 | s, ts}
    uint32_t n;             // list or item count
    uint32_t* ghist;        // [slot][2][GS_NB3]: histograms, then cursors
    const uint32_t* slot;   // k_skew_scan / _check: slot of list[i]
    uint32_t* gflag;        // [group] bit 0: key outside the plan, bit 1: run out of order
};

// tile t of group (b, g) in relation r: run [src, src + len)
template <class Lay>
__device__ __forceinline__ typename Lay::CView skew_run(const GroupArgs& G, int r, uint32_t g,
                                                      uint32_t t0, uint32_t t, uint32_t& len) {
    const TileTable& tt = G.tt[r];
    const uint16_t* pf = tt.prefT + (uint64_t)g * tt.tstride + t0 + t;
    const uint32_t lo = pf[0];
    len = (uint32_t)(pf[tt.tstride] - lo);
    return with_group(Lay::cview(G.tmp[r], G.pstride[r]), g, G.plan) + (tt.off[t0 + t] + lo);
}

constexpr uint32_t SK_WIN = kSkewSmall / 64;  // 64-position windows of a small group
static_assert(SK_WIN == SK_THREADS, "one window per thread when the run tables are built");

struct SkewSmallLDS {
    uint32_t h[2][GS_NB3];
    unsigned long long first[GS_NB3];  // pass 2: an element seen per digit
    // one relation's non-empty tile runs in position order (the group pass's
    // tables, build_tables; rebuilt per relation and pass, so that four
    // workgroups fit a CU): group position j of run k is tmp[j + base[k]]
    // (mod 2^64); window w: bit i of m = a run starts at 64 w + i, wk = runs
    // starting before the window, minus one
    uint64_t base[SK_TM];
    struct Win {
        unsigned long long m;
        uint32_t wk, pad;
    } win[SK_WIN];
    unsigned long long scr[SK_THREADS / 64 + 1];
};

// apply f(x) to every tuple of relation r's group, SK_ITEMS loads in flight
// per thread (groups of more than SK_TM runs: run by run)
template <class Lay, class F>
__device__ __forceinline__ void skew_for_each(const GroupArgs& G, const SkewSmallLDS& L, int r,
                                              uint32_t g, uint32_t t0, uint32_t nt, uint32_t n,
                                              F&& f) {
    typedef typename Lay::W W;
    if (nt <= SK_TM) {
        const typename Lay::CView tmp = with_group(Lay::cview(G.tmp[r], G.pstride[r]), g, G.plan);
        const uint32_t lane = lane_id();
        const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        for (uint32_t c = 0; c < n; c += SK_CHUNK) {
            W v[SK_ITEMS];
#pragma unroll
            for (int k = 0; k < SK_ITEMS; k++) {
                // a wave's 64 positions are one window (broadcast read): the
                // run of the lane's position is the window's earlier runs plus
                // the starts below the lane (mbcnt) and at it; positions past
                // the end re-read position 0 (unconditional loads: a
                // conditional one waits alone)
                const uint32_t w = (c + k * SK_THREADS) / 64 + wid;  // uniform
                const uint32_t j = w * 64 + lane;
                const bool ok = j < n;
                const auto win = L.win[ok ? w : 0u];
                const uint32_t below = __builtin_amdgcn_mbcnt_hi(
                    (uint32_t)(win.m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)win.m, 0u));
                const uint32_t at = (uint32_t)(win.m >> lane) & 1u;
                const uint32_t q = ok ? win.wk + below + at : 0u;
                v[k] = tmp[(uint64_t)(ok ? j : 0u) + L.base[q]];
            }
#pragma unroll
            for (int k = 0; k < SK_ITEMS; k++) f(v[k], c + k * SK_THREADS + threadIdx.x < n);
        }
    } else {
        for (uint32_t t = 0; t < nt; t++) {
            uint32_t len;
            const typename Lay::CView src = skew_run<Lay>(G, r, g, t0, t, len);
            for (uint32_t i0 = 0; i0 < len; i0 += SK_THREADS) {
                const uint32_t i = i0 + threadIdx.x;
                f(src[i < len ? i : len - 1], i < len);
            }
        }
    }
}

// any i in [lo, hi) with out[i] < out[i - 1]  (lo >= 1)
__device__ __forceinline__ bool skew_inversion(const Tup* dst, uint32_t lo, uint32_t hi) {
    bool inv = false;
    for (uint32_t c = lo; c < hi; c += SK_CHUNK) {
        Tup a[SK_ITEMS], b[SK_ITEMS];
#pragma unroll
        for (int k = 0; k < SK_ITEMS; k++) {
            const uint32_t i = min(c + k * SK_THREADS + threadIdx.x, hi - 1);
            a[k] = dst[i - 1];
            b[k] = dst[i];
        }
#pragma unroll
        for (int k = 0; k < SK_ITEMS; k++)
            if (c + k * SK_THREADS + threadIdx.x < hi) inv |= tup_less(b[k], a[k]);
    }
    return inv;
}

template <class Lay>
__global__ void __launch_bounds__(SK_THREADS)
k_skew_small(SkewArgs K) {
    typedef typename Lay::W W;
    __shared__ SkewSmallLDS L;
    const GroupArgs& G = K.G;
    const RangePlan& P = G.plan;
    const uint32_t qi = K.list[blockIdx.x];
    const OvfEntry e = K.q[qi];
    const uint32_t d12 = (e.bucket << P.D2) | e.d2;
    const uint32_t tid = threadIdx.x;
    uint32_t t0[2] = {0, 0}, nt[2] = {0, 0};
    for (uint32_t i = tid; i < 2 * GS_NB3; i += SK_THREADS) (&L.h[0][0])[i] = 0;
    __syncthreads();
    for (int r = 0; r < G.nrel; r++) {
        t0[r] = G.tt[r].btile0[e.bucket];
        nt[r] = G.tt[r].btile0[e.bucket + 1] - t0[r];
    }
    // ---- run tables of relation r: one scan gives every tile run its start
    // in the group (low half) and its index among the non-empty runs (high
    // half).  Uniform control flow (barriers inside).
    auto tables = [&](int r) {
        if (nt[r] > SK_TM) return;  // run by run (skew_for_each)
        __syncthreads();            // the previous tables are no longer read
        L.win[tid].m = 0ull;        // SK_WIN == SK_THREADS
        uint32_t len = 0;
        uint64_t src = 0;
        if (tid < nt[r]) {
            const TileTable& tt = G.tt[r];
            const uint16_t* pf = tt.prefT + (uint64_t)e.d2 * tt.tstride + t0[r] + tid;
            len = (uint32_t)(pf[tt.tstride] - pf[0]);
            src = tt.off[t0[r] + tid] + pf[0];
        }
        const unsigned long long acc = ((unsigned long long)(len ? 1u : 0u) << 32) | len;
        unsigned long long tot;
        const unsigned long long ex = block_scan64(acc, L.scr, &tot);  // barriers: m is zero
        const uint32_t st = (uint32_t)ex, k = (uint32_t)(ex >> 32);
        if (len) {
            L.base[k] = src - st;
            atomicOr(&L.win[st >> 6].m, 1ull << (st & 63));
        }
        __syncthreads();
        // window prefix counts (one window per thread)
        const uint32_t cw = (uint32_t)__popcll(L.win[tid].m);
        unsigned long long wt;
        const uint32_t wex = (uint32_t)block_scan64(cw, L.scr, &wt);  // ends with a barrier
        L.win[tid].wk = wex - 1u;
        __syncthreads();
    };
    // ---- pass 1: d3 histograms
    bool clamped = false;
    for (int r = 0; r < G.nrel; r++) {
        tables(r);
        skew_for_each<Lay>(G, L, r, e.d2, t0[r], nt[r], e.nr[r], [&](const W& x, bool ok) {
            clamped |= ok && Lay::clamped(P, x);
            if (ok) atomicAdd(&L.h[r][plan_d3(P, Lay::rel(P, x, e.bucket), d12)], 1u);
        });
    }
    const bool exact = P.s3 == 0 && !__syncthreads_or(clamped);
    if (!exact) {
        // inexact digits: copy the runs unsorted to the group's place
        for (int r = 0; r < G.nrel; r++) {
            Tup* dst = G.out[r] + G.ostart[r][e.bucket] + e.off[r];
            uint32_t pos = 0;
            for (uint32_t t = 0; t < nt[r]; t++) {
                uint32_t len;
                const typename Lay::CView src = skew_run<Lay>(G, r, e.d2, t0[r], t, len);
                for (uint32_t i = tid; i < len; i += SK_THREADS)
                    dst[pos + i] = Lay::unpack(P, src[i], e.bucket);
                pos += len;
            }
        }
        if (tid == 0) K.gflag[qi] |= 1u;
        return;
    }
    if (G.nrel == 2) {
        unsigned long long m = 0;
        for (uint32_t d = tid; d < GS_NB3; d += SK_THREADS)
            m += (unsigned long long)L.h[0][d] * L.h[1][d];
        m = wave_sum(m);
        if ((tid & 63) == 0 && m) atomicAdd(G.count_dev, m);
        if (tid == 0) K.q[qi].counted = 1;
    }
    bool inv = false;
    for (int r = 0; r < G.nrel; r++) {
        Tup* dst = G.out[r] + G.ostart[r][e.bucket] + e.off[r];
        // ---- cursors: exclusive scan of the bins (thread owns a range)
        constexpr int BPT = GS_NB3 / SK_THREADS;
        uint32_t c[BPT];
        unsigned long long loc = 0;
#pragma unroll
        for (int k = 0; k < BPT; k++) {
            c[k] = L.h[r][tid * BPT + k];
            loc += c[k];
        }
        unsigned long long tot;
        unsigned long long ex = block_scan64(loc, L.scr, &tot);
#pragma unroll
        for (int k = 0; k < BPT; k++) {
            L.h[r][tid * BPT + k] = (uint32_t)ex;
            ex += c[k];
        }
        __syncthreads();
        for (uint32_t d = tid; d < GS_NB3; d += SK_THREADS) L.first[d] = ~0ull;
        tables(r);  // (barriers inside; without tables one barrier)
        __syncthreads();
        // ---- pass 2: place; and note whether some key holds differing
        // elements (the first element seen per digit is kept: ~0 is the
        // empty mark, an element equal to it just counts as differing)
        bool differ = false;
        skew_for_each<Lay>(G, L, r, e.d2, t0[r], nt[r], e.nr[r], [&](const W& x, bool ok) {
            const uint32_t d = plan_d3(P, Lay::rel(P, x, e.bucket), d12);
            if (ok) {
                dst[atomicAdd(&L.h[r][d], 1u)] = Lay::unpack(P, x, e.bucket);
                const unsigned long long id = Lay::same_key_id(x);
                const unsigned long long old = atomicCAS(&L.first[d], ~0ull, id);
                differ |= id == ~0ull || (old != ~0ull && old != id);
            }
        });
        __threadfence_block();
        // ---- pass 3 (only when a key holds differing elements): ordered by
        // key, an inversion sits inside an equal-key run
        if (__syncthreads_or(differ)) inv |= skew_inversion(dst, 1, e.nr[r]);
    }
    if (__syncthreads_or(inv) && tid == 0) K.gflag[qi] |= 2u;
}

template <class Lay>
__global__ void __launch_bounds__(SK_THREADS)
k_skew_hist(SkewArgs K) {
    typedef typename Lay::W W;
    __shared__ uint32_t h[GS_NB3];
    const GroupArgs& G = K.G;
    const RangePlan& P = G.plan;
    const uint4 it = K.items[blockIdx.x];
    const uint32_t qi = it.x, sl = it.y, r = it.z >> 16, s = it.z & 0xffffu, ts = it.w;
    const OvfEntry e = K.q[qi];  // a copy: a reference is re-read after every store
    const uint32_t t0 = G.tt[r].btile0[e.bucket];
    const uint32_t nt = G.tt[r].btile0[e.bucket + 1] - t0;
    if (s >= nt) return;
    for (uint32_t d = threadIdx.x; d < GS_NB3; d += SK_THREADS) h[d] = 0;
    __syncthreads();
    const uint32_t d12 = (e.bucket << P.D2) | e.d2;
    bool clamped = false;
    for (uint32_t t = s; t < nt; t += ts) {
        uint32_t len;
        const typename Lay::CView src = skew_run<Lay>(G, (int)r, e.d2, t0, t, len);
        for (uint32_t c = 0; c < len; c += SK_CHUNK) {
            W v[SK_ITEMS];
#pragma unroll
            for (int k = 0; k < SK_ITEMS; k++) {
                const uint32_t i = c + k * SK_THREADS + threadIdx.x;
                v[k] = src[i < len ? i : len - 1];  // unconditional: all in flight
            }
#pragma unroll
            for (int k = 0; k < SK_ITEMS; k++) {
                const uint32_t i = c + k * SK_THREADS + threadIdx.x;
                const bool ok = i < len;
                clamped |= ok && Lay::clamped(P, v[k]);
                if (ok) atomicAdd(&h[plan_d3(P, Lay::rel(P, v[k], e.bucket), d12)], 1u);
            }
        }
    }
    const bool any = __syncthreads_or(clamped);
    uint32_t* gh = K.ghist + ((size_t)sl * 2 + r) * GS_NB3;
    for (uint32_t d = threadIdx.x; d < GS_NB3; d += SK_THREADS)
        if (h[d]) atomicAdd(&gh[d], h[d]);
    if (any && threadIdx.x == 0) atomicOr(&K.gflag[qi], 1u);
}

__global__ void __launch_bounds__(SK_THREADS)
k_skew_scan(SkewArgs K) {
    __shared__ unsigned long long scr[SK_THREADS / 64 + 1];
    const uint32_t qi = K.list[blockIdx.x], sl = K.slot[blockIdx.x];
    const RangePlan& P = K.G.plan;
    const bool exact = P.s3 == 0 && !(K.gflag[qi] & 1u);
    if (!exact) return;
    uint32_t* gh = K.ghist + (size_t)sl * 2 * GS_NB3;
    if (K.G.nrel == 2) {
        unsigned long long m = 0;
        for (uint32_t d = threadIdx.x; d < GS_NB3; d += SK_THREADS)
            m += (unsigned long long)gh[d] * gh[GS_NB3 + d];
        m = wave_sum(m);
        if ((threadIdx.x & 63) == 0 && m) atomicAdd(K.G.count_dev, m);
        if (threadIdx.x == 0) K.q[qi].counted = 1;
    }
    constexpr int BPT = GS_NB3 / SK_THREADS;
    for (int r = 0; r < K.G.nrel; r++) {
        uint32_t* h = gh + r * GS_NB3;
        uint32_t c[BPT];
        unsigned long long loc = 0;
#pragma unroll
        for (int k = 0; k < BPT; k++) {
            c[k] = h[threadIdx.x * BPT + k];
            loc += c[k];
        }
        unsigned long long tot;
        unsigned long long ex = block_scan64(loc, scr, &tot);
#pragma unroll
        for (int k = 0; k < BPT; k++) {
            h[threadIdx.x * BPT + k] = (uint32_t)ex;
            ex += c[k];
        }
    }
}

template <class Lay>
__global__ void __launch_bounds__(SK_THREADS)
k_skew_place(SkewArgs K) {
    typedef typename Lay::W W;
    __shared__ uint32_t h[GS_NB3];
    __shared__ unsigned long long scr[SK_THREADS / 64 + 1];
    const GroupArgs& G = K.G;
    const RangePlan& P = G.plan;
    const uint4 it = K.items[blockIdx.x];
    const uint32_t qi = it.x, sl = it.y, r = it.z >> 16, s = it.z & 0xffffu, ts = it.w;
    const OvfEntry e = K.q[qi];  // a copy: a reference is re-read after every store
    const uint32_t t0 = G.tt[r].btile0[e.bucket];
    const uint32_t nt = G.tt[r].btile0[e.bucket + 1] - t0;
    if (s >= nt) return;
    Tup* dst = G.out[r] + G.ostart[r][e.bucket] + e.off[r];
    const bool exact = P.s3 == 0 && !(K.gflag[qi] & 1u);
    if (!exact) {
        // copy the runs unsorted: run t starts after the runs before it
        for (uint32_t t = s; t < nt; t += ts) {
            unsigned long long acc = 0;
            for (uint32_t u = threadIdx.x; u < t; u += SK_THREADS) {
                uint32_t l;
                (void)skew_run<Lay>(G, (int)r, e.d2, t0, u, l);
                acc += l;
            }
            unsigned long long pos;
            (void)block_scan64(acc, scr, &pos);
            uint32_t len;
            const typename Lay::CView src = skew_run<Lay>(G, (int)r, e.d2, t0, t, len);
            for (uint32_t i = threadIdx.x; i < len; i += SK_THREADS)
                dst[pos + i] = Lay::unpack(P, src[i], e.bucket);
        }
        return;
    }
    const uint32_t d12 = (e.bucket << P.D2) | e.d2;
    uint32_t* gcur = K.ghist + ((size_t)sl * 2 + r) * GS_NB3;
    for (uint32_t t = s; t < nt; t += ts) {
        uint32_t len;
        const typename Lay::CView src = skew_run<Lay>(G, (int)r, e.d2, t0, t, len);
        for (uint32_t c = 0; c < len; c += SK_CHUNK) {
            for (uint32_t d = threadIdx.x; d < GS_NB3; d += SK_THREADS) h[d] = 0;
            W v[SK_ITEMS];
            uint32_t dg[SK_ITEMS];
#pragma unroll
            for (int k = 0; k < SK_ITEMS; k++) {
                const uint32_t i = c + k * SK_THREADS + threadIdx.x;
                v[k] = src[i < len ? i : len - 1];  // unconditional: all in flight
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < SK_ITEMS; k++) {
                const uint32_t i = c + k * SK_THREADS + threadIdx.x;
                dg[k] = i < len ? plan_d3(P, Lay::rel(P, v[k], e.bucket), d12) : 0u;
                if (i < len) atomicAdd(&h[dg[k]], 1u);
            }
            __syncthreads();
            // reserve this chunk's share of every digit at the cursors: a
            // thread's atomics all in flight, their results used only after
            // the last one (one returned atomic at a time waited ~8 global
            // round trips per chunk)
            constexpr int RPT = GS_NB3 / SK_THREADS;
            uint32_t res[RPT];
#pragma unroll
            for (int k = 0; k < RPT; k++) {
                const uint32_t d = threadIdx.x + k * SK_THREADS;
                const uint32_t n = h[d];
                res[k] = n ? atomicAdd(&gcur[d], n) : 0u;
            }
#pragma unroll
            for (int k = 0; k < RPT; k++) h[threadIdx.x + k * SK_THREADS] = res[k];
            __syncthreads();
#pragma unroll
            for (int k = 0; k < SK_ITEMS; k++) {
                const bool ok = c + k * SK_THREADS + threadIdx.x < len;
                if (ok) dst[atomicAdd(&h[dg[k]], 1u)] = Lay::unpack(P, v[k], e.bucket);
            }
            __syncthreads();
        }
    }
}

__global__ void __launch_bounds__(SK_THREADS)
k_skew_check(SkewArgs K) {
    const uint4 it = K.items[blockIdx.x];
    const uint32_t qi = it.x, r = it.z >> 16, s = it.z & 0xffffu, ts = it.w;
    const RangePlan& P = K.G.plan;
    if (!(P.s3 == 0 && !(K.gflag[qi] & 1u))) return;
    const OvfEntry e = K.q[qi];  // a copy: a reference is re-read after every store
    const Tup* dst = K.G.out[r] + K.G.ostart[r][e.bucket] + e.off[r];
    const uint32_t n = e.nr[r];
    const uint32_t lo = max(1u, (uint32_t)((uint64_t)n * s / ts));
    const uint32_t hi = (uint32_t)((uint64_t)n * (s + 1) / ts);
    if (__syncthreads_or(skew_inversion(dst, lo, hi)) && threadIdx.x == 0)
        atomicOr(&K.gflag[qi], 2u);
}

// The queued groups [0, no): device skew kernels, then whatever they could
// not finish (inexact digits, equal-key runs out of payload order) through
// the segmented merge sort and the merge-join count.  hdst[r * nb + b] is
// bucket b's output start.
template <class Lay>
static void skew_path(Workspace* ws, const GroupArgs& G, OvfEntry* ovf, uint32_t no,
                      const uint64_t* hdst, uint32_t nb, hipStream_t st) {
    const int nrel = G.nrel;
    // pinned host copies (a pageable destination makes each copy a staged,
    // blocking transfer)
    OvfEntry* he = (OvfEntry*)ws->host_pinned("sk_he", (size_t)no * sizeof(OvfEntry));
    SMJ_CHECK(hipMemcpyAsync(he, ovf, no * sizeof(OvfEntry), hipMemcpyDeviceToHost, st));
    ws->wait_stream(st);
    // small groups: one workgroup each; large ones: work items over their runs
    std::vector<uint32_t> small, large, lslot;
    std::vector<uint4> items;
    for (uint32_t i = 0; i < no; i++) {
        const uint32_t m = std::max(he[i].nr[0], nrel > 1 ? he[i].nr[1] : 0u);
        if (m <= kSkewSmall) {
            small.push_back(i);
            continue;
        }
        const uint32_t sl = (uint32_t)large.size();
        large.push_back(i);
        lslot.push_back(sl);
        for (int r = 0; r < nrel; r++) {
            // about SMJ_SKEW_ITEM tuples per item (runs are strided over the
            // items; an item past the bucket's runs exits)
            const uint32_t ts =
                std::min<uint32_t>(std::max<uint32_t>(he[i].nr[r] / SMJ_SKEW_ITEM, 1), 256);
            for (uint32_t s = 0; s < ts; s++)
                items.push_back(make_uint4(i, sl, ((uint32_t)r << 16) | s, ts));
        }
    }
    const size_t nl = large.size();
    const size_t lbytes = (small.size() + 2 * nl) * 4;
    const size_t ibytes = items.size() * sizeof(uint4);
    unsigned char* hbuf = (unsigned char*)ws->host_pinned("sk_h", lbytes + ibytes + 16);
    unsigned char* dbuf = (unsigned char*)ws->scratch("sk_d", lbytes + ibytes + 16);
    uint32_t* hl = (uint32_t*)hbuf;
    std::copy(small.begin(), small.end(), hl);
    std::copy(large.begin(), large.end(), hl + small.size());
    std::copy(lslot.begin(), lslot.end(), hl + small.size() + nl);
    const size_t ioff = (lbytes + 15) / 16 * 16;
    std::copy(items.begin(), items.end(), (uint4*)(hbuf + ioff));
    SMJ_CHECK(hipMemcpyAsync(dbuf, hbuf, ioff + ibytes, hipMemcpyHostToDevice, st));
    uint32_t* gflag = (uint32_t*)ws->scratch("sk_flag", (size_t)no * 4);
    SMJ_CHECK(hipMemsetAsync(gflag, 0, (size_t)no * 4, st));
    SkewArgs K;
    K.G = G;
    K.q = ovf;
    K.gflag = gflag;
    K.ghist = nullptr;
    K.slot = nullptr;
    K.items = nullptr;
    if (!small.empty()) {
        K.list = (const uint32_t*)dbuf;
        K.n = (uint32_t)small.size();
        TraceScope ts(ws, "k_skew_small", st);
        hipLaunchKernelGGL(k_skew_small<Lay>, dim3(K.n), dim3(SK_THREADS), 0, st, K);
    }
    if (nl) {
        K.ghist = (uint32_t*)ws->scratch("sk_hist", nl * 2 * GS_NB3 * 4);
        SMJ_CHECK(hipMemsetAsync(K.ghist, 0, nl * 2 * GS_NB3 * 4, st));
        K.list = (const uint32_t*)dbuf + small.size();
        K.slot = K.list + nl;
        K.items = (const uint4*)(dbuf + ioff);
        const uint32_t ni = (uint32_t)items.size();
        {
            TraceScope ts(ws, "k_skew_hist", st);
            hipLaunchKernelGGL(k_skew_hist<Lay>, dim3(ni), dim3(SK_THREADS), 0, st, K);
        }
        hipLaunchKernelGGL(k_skew_scan, dim3((uint32_t)nl), dim3(SK_THREADS), 0, st, K);
        {
            TraceScope ts(ws, "k_skew_place", st);
            hipLaunchKernelGGL(k_skew_place<Lay>, dim3(ni), dim3(SK_THREADS), 0, st, K);
        }
        hipLaunchKernelGGL(k_skew_check, dim3(ni), dim3(SK_THREADS), 0, st, K);
    }
    SMJ_CHECK(hipGetLastError());
    uint32_t* flags = (uint32_t*)ws->host_pinned("sk_flags", (size_t)no * 4);
    SMJ_CHECK(hipMemcpyAsync(flags, gflag, (size_t)no * 4, hipMemcpyDeviceToHost, st));
    SMJ_CHECK(hipMemcpyAsync(he, ovf, no * sizeof(OvfEntry), hipMemcpyDeviceToHost, st));
    ws->wait_stream(st);
    // what the device could not finish
    std::vector<uint32_t> rest;
    for (uint32_t i = 0; i < no; i++)
        if (flags[i] != 0 || G.plan.s3 != 0) rest.push_back(i);
    if (rest.empty()) return;
    for (int r = 0; r < nrel; r++) {
        std::vector<uint64_t> so, sl;
        for (uint32_t i : rest) {
            so.push_back(hdst[(size_t)r * nb + he[i].bucket] + he[i].off[r]);
            sl.push_back(he[i].nr[r]);
        }
        segmented_sort(ws, G.out[r], so.data(), sl.data(), (uint32_t)rest.size(), st);
    }
    if (nrel == 2) {
        std::vector<const Tup*> rp, sp;
        std::vector<uint64_t> nr, ns;
        for (uint32_t i : rest) {
            if (he[i].counted || !he[i].nr[0] || !he[i].nr[1]) continue;
            rp.push_back(G.out[0] + hdst[he[i].bucket] + he[i].off[0]);
            sp.push_back(G.out[1] + hdst[nb + he[i].bucket] + he[i].off[1]);
            nr.push_back(he[i].nr[0]);
            ns.push_back(he[i].nr[1]);
        }
        merge_join_count_batch(ws, rp.data(), nr.data(), sp.data(), ns.data(),
                               (uint32_t)rp.size(), G.count_dev, st);
    }
}

// ---------------------------------------------------------------------------
// range plan from a strided sample of the relations (or from hints)
__global__ void __launch_bounds__(256)
k_plan(const Tup* r0, uint64_t n0, const Tup* r1, uint64_t n1, uint32_t D1,
       uint32_t D2, uint32_t D2cap, int64_t hmin, int64_t hmax, RangePlan* plan) {
    __shared__ int64_t smin[4], smax[4];
    int64_t mn = INT64_MAX, mx = INT64_MIN;
    const int S = 4096;
    for (int rel = 0; rel < 2; rel++) {
        const Tup* p = rel ? r1 : r0;
        uint64_t n = rel ? n1 : n0;
        if (!p || n == 0) continue;
        for (int i = threadIdx.x; i < S; i += 256) {
            // golden-ratio stride sample, deterministic
            uint64_t idx = __umul64hi((uint64_t)i * 0x9E3779B97F4A7C15ull, n);
            if (i == 0) idx = 0;
            if (i == 1) idx = n - 1;
            int64_t k = tup_key(p[idx]);
            mn = k < mn ? k : mn;
            mx = k > mx ? k : mx;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        int64_t a = __shfl_xor(mn, o, 64), c = __shfl_xor(mx, o, 64);
        mn = a < mn ? a : mn;
        mx = c > mx ? c : mx;
    }
    if (lane_id() == 0) {
        smin[threadIdx.x >> 6] = mn;
        smax[threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 0; w < 4; w++) {
            mn = smin[w] < mn ? smin[w] : mn;
            mx = smax[w] > mx ? smax[w] : mx;
        }
        int64_t lo, hi;
        if (hmin <= hmax) {
            lo = hmin;
            hi = hmax;
        } else if (mn > mx) {
            lo = 0;
            hi = 0;
        } else {
            // widen the sampled range by 1/64 on both sides (saturating)
            uint64_t w = key_u(mx) - key_u(mn);
            uint64_t m = w / 64 + 1;
            uint64_t lu = key_u(mn) > m ? key_u(mn) - m : 0;
            uint64_t hu = (~0ull - key_u(mx)) > m ? key_u(mx) + m : ~0ull;
            lo = (int64_t)(lu ^ 0x8000000000000000ull);
            hi = (int64_t)(hu ^ 0x8000000000000000ull);
        }
        *plan = make_plan(lo, hi, D1, D2, D2cap, GS_D3MAX);
    }
}

void plan_from_sample(Workspace* ws, const Tup* const* rels, const uint64_t* ns,
                      int nrel, uint32_t D1, uint32_t D2, uint32_t D2cap,
                      int64_t hint_min, int64_t hint_max, RangePlan* plan_dev,
                      hipStream_t st) {
    (void)ws;
    hipLaunchKernelGGL(k_plan, dim3(1), dim3(256), 0, st, rels[0], ns[0],
                       nrel > 1 ? rels[1] : (const Tup*)nullptr,
                       nrel > 1 ? ns[1] : 0, D1, D2, D2cap, hint_min, hint_max,
                       plan_dev);
    SMJ_CHECK(hipGetLastError());
}

const uint32_t kGroupD3Max = GS_D3MAX;
// expected group size the plan aims for (capi.hip choose_levels)
const uint32_t kGroupTarget = GS_CAP * 4 / 5 >= 2048 ? 2048 : (GS_CAP * 4 / 5 >= 1024 ? 1024 : 512);

// ---------------------------------------------------------------------------
// device-side tile numbering of a segmented (sampled) partition: per bucket
// the tiles of its segments, their exclusive scan (btile0, total in
// btile0[nb] and *ntiles) and the dense output start of every bucket
struct SegRel {
    const int64_t* seg_cnt[2];
    const int64_t* bcount[2];
    const uint64_t* bstart[2];
    const uint64_t* seg_start[2];
    uint32_t* ntiles[2];
    uint64_t* ostart[2];
    TileTable tt[2];
};

// blockIdx.x = relation
__global__ void __launch_bounds__(256)
k_seg_scan(SegRel S, uint32_t nb, uint32_t nseg, uint32_t tsz) {
    const int r = blockIdx.x;
    const int64_t* __restrict__ seg_cnt = S.seg_cnt[r];
    const int64_t* __restrict__ bcount = S.bcount[r];
    uint32_t* __restrict__ btile0 = S.tt[r].btile0;
    uint64_t* __restrict__ ostart = S.ostart[r];
    __shared__ unsigned long long scr[5];
    __shared__ unsigned long long base;
    if (threadIdx.x == 0) base = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < nb; b0 += 256) {
        const uint32_t b = b0 + threadIdx.x;
        uint32_t nt = 0;
        uint64_t cnt = 0;
        if (b < nb) {
            for (uint32_t q = 0; q < nseg; q++)
                nt += (uint32_t)((seg_cnt[(size_t)b * nseg + q] + tsz - 1) / tsz);
            cnt = (uint64_t)bcount[b];
        }
        // (tiles << 40 | count): both exclusive scans in one
        unsigned long long tot;
        const unsigned long long ex =
            block_scan64(((unsigned long long)nt << 40) | cnt, scr, &tot);
        const unsigned long long run = base;
        if (b < nb) {
            btile0[b] = (uint32_t)((run >> 40) + (ex >> 40));
            ostart[b] = (run & ((1ull << 40) - 1)) + (ex & ((1ull << 40) - 1));
        }
        __syncthreads();
        if (threadIdx.x == 0) base = run + tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        btile0[nb] = (uint32_t)(base >> 40);
        *S.ntiles[r] = (uint32_t)(base >> 40);
    }
}

// k_tiles of both relations (blockIdx.y = relation)
__global__ void __launch_bounds__(64)
k_tiles2(SegRel S, uint32_t nseg, uint32_t tsz) {
    const int r = blockIdx.y;
    const uint32_t b = blockIdx.x;
    const TileTable& tt = S.tt[r];
    uint32_t t0 = tt.btile0[b];
    for (uint32_t q = 0; q < nseg; q++) {
        const uint64_t s0 = S.seg_start[r] ? S.seg_start[r][(size_t)b * nseg + q] : S.bstart[r][b];
        const int64_t cnt = S.seg_cnt[r] ? S.seg_cnt[r][(size_t)b * nseg + q] : S.bcount[r][b];
        const uint32_t nt = (uint32_t)((cnt + tsz - 1) / tsz);
        for (uint32_t i = threadIdx.x; i < nt; i += 64) {
            const uint64_t o = (uint64_t)i * tsz;
            const int64_t rem = cnt - (int64_t)o;
            tt.off[t0 + i] = s0 + o;
            tt.len[t0 + i] = (uint32_t)(rem < (int64_t)tsz ? rem : tsz);
            tt.bucket[t0 + i] = b;
        }
        t0 += nt;
    }
}

// digit-major prefix tables of both relations (k_preft); `ub` bounds the
// tile count, `ntiles` holds it on the device (nullptr: ub is exact)
static void launch_preft(const TileTable* tt, int nrel, const uint32_t* ub,
                         uint32_t* const* ntiles, uint32_t nb2, hipStream_t st) {
    const uint32_t nb0 = (ub[0] + PT_TILES - 1) / PT_TILES;
    const uint32_t nb1 = nrel > 1 ? (ub[1] + PT_TILES - 1) / PT_TILES : 0;
    if (nb0 + nb1 == 0) return;
    const size_t lds = (size_t)PT_TILES * (nb2 + 1) * 2;
    hipLaunchKernelGGL(k_preft, dim3(nb0 + nb1), dim3(256), lds, st, tt[0],
                       tt[nrel > 1 ? 1 : 0], nb0, ntiles[0], nrel > 1 ? ntiles[1] : nullptr,
                       ub[0], nrel > 1 ? ub[1] : 0u, nb2);
}

// the tiles [t0, t0 + nt) of one tile-pass batch: shift the tables so the
// batch's first tile is tile 0 of the launch
static void launch_preft_range(const TilePassArgs& T, int nrel, uint32_t nb2,
                               hipStream_t st) {
    TileTable tt[2];
    uint32_t ub[2] = {0, 0};
    uint32_t* nt[2] = {nullptr, nullptr};
    for (int r = 0; r < 2; r++) {
        tt[r] = T.tt[r];
        if (r < nrel) {
            tt[r].pref += (uint64_t)T.t0[r] * (nb2 + 1);
            tt[r].prefT += T.t0[r];
            ub[r] = T.nt[r];
        }
    }
    launch_preft(tt, nrel, ub, nt, nb2, st);
}

// the tile pass over the tiles [0, nt[r]) of both relations (device counts:
// at most ntiles[r]); persistent, one workgroup per CU (SMJ_TP_PERSIST) for
// 16-byte tuples
template <class Lay, class LayO>
static void launch_tilepass(const TilePassArgs& T, size_t lds, hipStream_t st) {
    const uint32_t nblk = T.nt[0] + T.nt[1];
    // measured (profiles/r05_lab/tp_ab.txt): 16-byte tuples 1.63 -> 1.52 ms;
    // words (8-byte elements, two loads and two stores each for the 48-bit
    // planes) 0.65 -> 0.68-0.71 ms, the prefetch and the stores together
    // saturating the 63 outstanding memory operations; 32-bit words spill
    if (SMJ_TP_PERSIST && sizeof(typename Lay::W) >= 12) {
        hipLaunchKernelGGL((k_tilepass_p<Lay, LayO>), dim3(nblk < 256 ? nblk : 256),
                           dim3(TP_THREADS), lds, st, T);
    } else {
        hipLaunchKernelGGL((k_tilepass<Lay, LayO>), dim3(nblk), dim3(TP_THREADS), lds, st, T);
    }
}

// dynamic LDS limits of the tile and group passes (per layout)
template <class Lay>
static void set_pass_attrs() {
    set_lds_attr((const void*)k_tilepass<Lay>, 160 * 1024);
    set_lds_attr((const void*)k_tilepass_p<Lay>, 160 * 1024);
    // several workgroups per CU (launch bounds): ask for what one needs
    const void* gs[4] = {(const void*)k_groupsort<Lay, 2, false>,
                         (const void*)k_groupsort<Lay, 4, false>,
                         (const void*)k_groupsort<Lay, 2, true>,
                         (const void*)k_groupsort<Lay, 4, true>};
    for (const void* f : gs) set_lds_attr(f, (int)sizeof(GroupLDS<typename Lay::W>));
}

// Tile runs per lane of the group pass: 2 (128 tiles per bucket) unless the
// expected largest bucket (mean + 1/4, plus one partial tile per segment)
// needs more, then 4 (256).  A bucket beyond that takes the skew path.
static uint64_t expected_tiles(uint64_t nmax, uint32_t nb, uint32_t nseg, uint32_t tsz) {
    const uint64_t per = nmax / (nb ? nb : 1);
    return (per + per / 4) / tsz + nseg + 1;
}
static int group_tpl(uint64_t nmax, uint32_t nb, uint32_t nseg, uint32_t tsz) {
    return expected_tiles(nmax, nb, nseg, tsz) <= 128 ? 2 : 4;
}

// persistent grid of the group pass: `per` groups per workgroup, at most
// maxwg (a multiple of 8) workgroups, rounded up to a multiple of 8 for the
// XCD-aware order (blocks past the last group exit)
static uint32_t groupsort_grid(uint32_t ngroups, uint32_t maxwg, uint32_t& per) {
    per = (ngroups + maxwg - 1) / maxwg;
    const uint32_t nwg = (ngroups + per - 1) / per;
    return (nwg + 7) & ~7u;
}

template <class Lay>
static void launch_groupsort(Workspace* ws, int tpl, uint32_t nwg, hipStream_t st,
                             const GroupArgs& G0) {
    const size_t lds = sizeof(GroupLDS<typename Lay::W>);
#if SMJ_GS_ARGS_MEM
    // one argument slot per workspace: a workspace serves one stream at a
    // time (smj.h: one per stream/thread), so the group pass of the previous
    // call on it has read its arguments before k_put_args rewrites them
    GroupArgs* G = (GroupArgs*)ws->scratch("gs_args", sizeof(GroupArgs));
    hipLaunchKernelGGL(k_put_args, dim3(1), dim3(1), 0, st, G0, G);
#else
    const GroupArgs& G = G0;
#endif
#if SMJ_GS_XCD
    // k_groupsort's XCD-aware order splits the groups into 8 ranges of
    // gridDim.x / 8 blocks each: any other grid would sort some groups twice
    // (counting their matches twice) and leave others unsorted
    if (nwg % 8 != 0) {
        fprintf(stderr, "[ERROR] smj: group pass grid %u is not a multiple of 8\n", nwg);
        abort();
    }
#endif
    if (G0.pair) {
        if (tpl == 4)
            hipLaunchKernelGGL((k_groupsort<Lay, 4, true>), dim3(nwg), dim3(GS_THREADS), lds, st, G);
        else
            hipLaunchKernelGGL((k_groupsort<Lay, 2, true>), dim3(nwg), dim3(GS_THREADS), lds, st, G);
    } else {
        if (tpl == 4)
            hipLaunchKernelGGL((k_groupsort<Lay, 4, false>), dim3(nwg), dim3(GS_THREADS), lds, st, G);
        else
            hipLaunchKernelGGL((k_groupsort<Lay, 2, false>), dim3(nwg), dim3(GS_THREADS), lds, st, G);
    }
}

// Bucket pass without a host synchronisation before the kernels (sampled
// partition + host-known plan): launch sizes are upper bounds, the tile
// numbering is computed on the device.  One synchronisation at the end (skew
// queue and the partition's overflow flag).
#ifndef SMJ_P40
#define SMJ_P40 1  // the tile pass writes 48-bit words without their group digit
#endif
// Lay: the level-1 partition's layout; LayG: the layout the tile pass
// writes and the group pass reads (LayP40 after LayP48)
template <class Lay, class LayG = Lay>
static bool bucket_sort_nosync(Workspace* ws, const BucketSortArgs& a, hipStream_t st) {
    typedef typename Lay::W W;
    set_pass_attrs<Lay>();
    set_pass_attrs<LayG>();
    constexpr bool p40 = !std::is_same<Lay, LayG>::value;
    if (p40) {
        set_lds_attr((const void*)k_tilepass<Lay, LayG>, 160 * 1024);
        set_lds_attr((const void*)k_tilepass_p<Lay, LayG>, 160 * 1024);
    }
    const uint32_t nb = a.nbuckets;
    const int nrel = a.nrel;
    const uint32_t nb2 = 1u << a.host_plan->D2;
    const uint64_t nmax = nrel > 1 && a.n[1] > a.n[0] ? a.n[1] : a.n[0];
    const uint32_t tsz = tile_elems_l<Lay>();
    TileTable tt[2];
    static const char* names[2][8] = {
        {"bs_off0", "bs_len0", "bs_bkt0", "bs_bt00", "bs_pref0", "bs_ost0", "bs_nt0", "bs_preft0"},
        {"bs_off1", "bs_len1", "bs_bkt1", "bs_bt01", "bs_pref1", "bs_ost1", "bs_nt1", "bs_preft1"}};
    uint64_t* ostart[2] = {nullptr, nullptr};
    uint32_t* ntiles[2] = {nullptr, nullptr};
    uint32_t ub[2] = {0, 0};
    for (int r = 0; r < nrel; r++) {
        ub[r] = (uint32_t)((a.n[r] + tsz - 1) / tsz + (uint64_t)nb * a.nseg);
        tt[r].off = (uint64_t*)ws->scratch(names[r][0], (size_t)ub[r] * 8);
        tt[r].len = (uint32_t*)ws->scratch(names[r][1], (size_t)ub[r] * 4);
        tt[r].bucket = (uint32_t*)ws->scratch(names[r][2], (size_t)ub[r] * 4);
        tt[r].btile0 = (uint32_t*)ws->scratch(names[r][3], (nb + 1) * 4);
        tt[r].pref = (uint16_t*)ws->scratch(names[r][4], (size_t)ub[r] * (nb2 + 1) * 2);
        tt[r].prefT = (uint16_t*)ws->scratch(names[r][7], (size_t)ub[r] * (nb2 + 1) * 2);
        tt[r].tstride = ub[r];
        ostart[r] = (uint64_t*)ws->scratch(names[r][5], (size_t)nb * 8);
        ntiles[r] = (uint32_t*)ws->scratch(names[r][6], 4);
    }
    if (nrel == 1) tt[1] = tt[0];
    // the relations whose tile stage this call runs, as launch slots 0..ns-1
    int sel[2] = {0, 0}, ns = 0;
    for (int r = 0; r < nrel; r++)
        if (a.stage & (1u << r)) sel[ns++] = r;
    if (ns) {
        // tile numbering of the selected relations: two launches
        SegRel S;
        for (int i = 0; i < 2; i++) {
            const int rr = sel[i < ns ? i : 0];
            S.seg_cnt[i] = a.seg_cnt[rr];
            S.bcount[i] = a.bcount[rr];
            S.bstart[i] = a.bstart[rr];
            S.seg_start[i] = a.seg_start[rr];
            S.ntiles[i] = ntiles[rr];
            S.ostart[i] = ostart[rr];
            S.tt[i] = tt[rr];
        }
        hipLaunchKernelGGL(k_seg_scan, dim3(ns), dim3(256), 0, st, S, nb, a.nseg, tsz);
        hipLaunchKernelGGL(k_tiles2, dim3(nb, ns), dim3(64), 0, st, S, a.nseg, tsz);
    }
    if (a.ev_tile) SMJ_CHECK(hipEventRecord(a.ev_tile, st));

    const uint32_t ngroups = nb * nb2;
    const uint32_t ovf_cap = ngroups;
    OvfEntry* ovf = (OvfEntry*)ws->scratch("bs_ovf", (size_t)ovf_cap * sizeof(OvfEntry));
    uint32_t* novf = a.status ? a.status + 2 : (uint32_t*)ws->scratch("bs_novf", 4);
    if (!a.status && (a.stage & 4)) SMJ_CHECK(hipMemsetAsync(novf, 0, 4, st));
    TilePassArgs T;
    GroupArgs G;
    for (int i = 0; i < 2; i++) {
        const int rr = sel[i < ns ? i : 0];
        T.part[i] = a.part[rr];
        T.tmp[i] = a.tmp[rr];
        T.pstride[i] = a.pstride[rr];
        T.tt[i] = tt[rr];
        T.t0[i] = 0;
        T.nt[i] = i < ns ? ub[rr] : 0;
        T.ntiles[i] = ntiles[rr];
    }
    // LayP40: the grouped tiles' byte plane, a buffer of the workspace per
    // relation (kept across the calls of a staged join); its offset from the
    // lo plane is the layout's "stride"
    uint64_t hoff[2] = {0, 0};
    if (p40) {
        static const char* hn[2] = {"p40_hi0", "p40_hi1"};
        for (int r = 0; r < nrel; r++) {
            const uint8_t* hb = (const uint8_t*)ws->scratch(hn[r], a.pstride[r] ? a.pstride[r] : 1);
            hoff[r] = (uint64_t)((uintptr_t)hb - (uintptr_t)a.tmp[r]);
        }
        for (int i = 0; i < 2; i++) T.ostride[i] = hoff[sel[i < ns ? i : 0]];
    }
    for (int r = 0; r < 2; r++) {
        const int rr = r < nrel ? r : 0;
        G.tmp[r] = a.tmp[rr];
        G.pstride[r] = p40 ? hoff[rr] : a.pstride[rr];
        G.out[r] = a.out[rr];
        G.bstart[r] = a.bstart[rr];
        G.ostart[r] = ostart[rr];
        G.tt[r] = tt[rr];
    }
    T.plan = *a.host_plan;
    T.nb2 = nb2;
    T.pack_bad = a.pack_bad;
    T.d2_fast = a.digit_fast && Lay::fast_ok(T.plan, T.plan.s2, T.plan.D2);
    G.pack_bad = a.pack_bad;
    G.d3_fast = a.digit_fast && Lay::fast_ok(T.plan, T.plan.s3, T.plan.D3);
    G.nrel = nrel;
    G.pair = SMJ_GS_PAIR && nrel == 1;
    G.plan = *a.host_plan;
    G.count_dev = a.count_dev;
    G.nb2 = nb2;
    G.ovf = ovf;
    G.novf = novf;
    G.ovf_cap = ovf_cap;
    G.g_begin = 0;
    G.g_end = ngroups;
    if (ns) {
        {
            TraceScope ts(ws, "k_tilepass", st);
            const size_t tp_lds =
                (((size_t)tsz * TileStage<Lay>::kBytes + 15) & ~(size_t)15) + nb2 * 4 + 64;
            launch_tilepass<Lay, LayG>(T, tp_lds, st);
        }
        const uint32_t ubs[2] = {T.nt[0], T.nt[1]};
        uint32_t* nts[2] = {ntiles[sel[0]], ntiles[sel[ns > 1 ? 1 : 0]]};
        launch_preft(T.tt, ns, ubs, nts, nb2, st);
    }
    if (!(a.stage & 4)) {
        SMJ_CHECK(hipGetLastError());
        return true;  // the group pass comes with a later call
    }
    if (a.ev_bucket) SMJ_CHECK(hipEventRecord(a.ev_bucket, st));
    {
        const uint32_t maxwg =
            (G.pair ? gs_wg_per_cu<W, true>() : gs_wg_per_cu<W, false>()) * 256;
        const uint32_t nwg = groupsort_grid(ngroups, maxwg, G.per);
        TraceScope ts(ws, "k_groupsort", st);
        launch_groupsort<LayG>(ws, group_tpl(nmax, nb, a.nseg, tsz), nwg, st, G);
    }
    SMJ_CHECK(hipGetLastError());
    if (a.ev_ovf) SMJ_CHECK(hipEventRecord(a.ev_ovf, st));

    // ---- the one synchronisation: partition overflow flag + skew queue
    uint32_t* h = (uint32_t*)ws->host_pinned("bs_h_flagovf", 16);
    h[0] = h[1] = h[2] = h[3] = 0;
    if (a.status) {
        SMJ_CHECK(hipMemcpyAsync(h, a.status, 16, hipMemcpyDeviceToHost, st));
    } else {
        SMJ_CHECK(hipMemcpyAsync(h, a.part_flag, 4, hipMemcpyDeviceToHost, st));
        SMJ_CHECK(hipMemcpyAsync(h + 2, novf, 4, hipMemcpyDeviceToHost, st));
        if (a.pack_bad)
            SMJ_CHECK(hipMemcpyAsync(h + 1, a.pack_bad, 4, hipMemcpyDeviceToHost, st));
    }
    ws->wait_stream(st);
    if (a.status_out) {
        a.status_out[0] = h[0];
        a.status_out[1] = h[1];
    }
    // the caller repeats with exact partitions (region overflow), on tuples
    // (not packable) or with the exact plan (a key outside a guessed one); the
    // tile and group passes exited at once on the latter two
    if (h[0] || h[1]) return false;
    const uint32_t no = h[2];
    if (no == 0) return true;
    if (no > ovf_cap) {
        fprintf(stderr, "[ERROR] smj: overflow table too small\n");
        abort();
    }
    uint64_t* hdst = (uint64_t*)ws->host_pinned("sk_hdst", (size_t)2 * nb * 8);
    for (int r = 0; r < nrel; r++)
        SMJ_CHECK(hipMemcpyAsync(hdst + (size_t)r * nb, ostart[r], (size_t)nb * 8,
                                 hipMemcpyDeviceToHost, st));
    skew_path<LayG>(ws, G, ovf, no, hdst, nb, st);
    SMJ_CHECK(hipGetLastError());
    return true;
}

bool bucket_sort(Workspace* ws, const BucketSortArgs& a, hipStream_t st) {
    const uint32_t nb = a.nbuckets;
    const int nrel = a.nrel;
    set_lds_attr((const void*)k_preft, PT_TILES * ((1 << kMaxD2) + 1) * 2);
    set_pass_attrs<LayTup>();
    if (a.host_plan && a.seg_start[0] && a.part_flag) {
        if (a.p32) return bucket_sort_nosync<LayP32>(ws, a, st);
        // 16-byte tuples only: with 8-byte tuples the group pass gained
        // less than the byte plane cost it (the join 2.542-2.551 ms either
        // way, the group pass 0.911-0.921 -> 0.930 ms, its SQ wait share
        // 0.49 -> 0.56; profiles/r05_lab/p40_ab.txt, r05_sq_join8*)
        if (a.p48)
            return SMJ_P40 && sizeof(Tup) == 16 && LayP40::holds(*a.host_plan)
                ? bucket_sort_nosync<LayP48, LayP40>(ws, a, st)
                : bucket_sort_nosync<LayP48>(ws, a, st);
#ifdef KEY_8B
        if (a.packed) return bucket_sort_nosync<LayPacked>(ws, a, st);
        if (a.p96) return bucket_sort_nosync<LayP96>(ws, a, st);
#endif
        return bucket_sort_nosync<LayTup>(ws, a, st);
    }
    if (a.packed || a.stage != 7) {
        fprintf(stderr, "[ERROR] smj: packed or staged bucket sorts need the host plan\n");
        abort();
    }

    // ---- host view of the plan and the bucket counts (one synchronisation):
    // launch sizes and the tile numbering are derived from them
    const uint32_t tsz = tile_elems<Tup>();
    uint64_t* hcnt = (uint64_t*)ws->host_pinned("bs_hcnt", (size_t)2 * nb * 8);
    RangePlan* hplan = (RangePlan*)ws->host_pinned("bs_hplan", sizeof(RangePlan));
    const bool segs = a.seg_start[0] != nullptr;
    const uint32_t nseg = segs ? a.nseg : 1;
    int64_t* hseg = (int64_t*)ws->host_pinned("bs_hseg", (size_t)2 * nb * nseg * 8);
    for (int r = 0; r < nrel; r++) {
        SMJ_CHECK(hipMemcpyAsync(hcnt + r * nb, a.bcount[r], nb * 8,
                                 hipMemcpyDeviceToHost, st));
        if (segs)
            SMJ_CHECK(hipMemcpyAsync(hseg + (size_t)r * nb * nseg, a.seg_cnt[r],
                                     (size_t)nb * nseg * 8, hipMemcpyDeviceToHost, st));
    }
    SMJ_CHECK(hipMemcpyAsync(hplan, a.plan_dev, sizeof(RangePlan),
                             hipMemcpyDeviceToHost, st));
    unsigned int* hflag = (unsigned int*)ws->host_pinned("bs_hflag", 4);
    *hflag = 0;
    if (a.part_flag)
        SMJ_CHECK(hipMemcpyAsync(hflag, a.part_flag, 4, hipMemcpyDeviceToHost, st));
    SMJ_CHECK(hipStreamSynchronize(st));
    if (*hflag) return false;
    const uint32_t nb2 = 1u << hplan->D2;  // groups per bucket

    TileTable tt[2];
    static const char* names[2][6] = {
        {"bs_off0", "bs_len0", "bs_bkt0", "bs_bt00", "bs_pref0", "bs_preft0"},
        {"bs_off1", "bs_len1", "bs_bkt1", "bs_bt01", "bs_pref1", "bs_preft1"}};
    uint32_t* hbt = (uint32_t*)ws->host_pinned("bs_hbt", (size_t)2 * (nb + 1) * 4);
    // dense output start of every bucket (partition regions may have slack)
    uint64_t* hdst = (uint64_t*)ws->host_pinned("bs_hdst", (size_t)2 * nb * 8);
    uint64_t* ostart[2] = {nullptr, nullptr};
    for (int r = 0; r < nrel; r++) {
        uint32_t* bt0 = hbt + r * (nb + 1);
        uint32_t acc = 0;
        uint64_t dacc = 0;
        for (uint32_t b = 0; b < nb; b++) {
            hdst[r * nb + b] = dacc;
            dacc += hcnt[r * nb + b];
            bt0[b] = acc;
            if (segs) {
                for (uint32_t q = 0; q < nseg; q++)
                    acc += (uint32_t)((hseg[((size_t)r * nb + b) * nseg + q] + tsz - 1) / tsz);
            } else {
                acc += (uint32_t)((hcnt[r * nb + b] + tsz - 1) / tsz);
            }
        }
        bt0[nb] = acc;
        const uint64_t ntl = acc ? acc : 1;
        tt[r].off = (uint64_t*)ws->scratch(names[r][0], ntl * 8);
        tt[r].len = (uint32_t*)ws->scratch(names[r][1], ntl * 4);
        tt[r].bucket = (uint32_t*)ws->scratch(names[r][2], ntl * 4);
        tt[r].btile0 = (uint32_t*)ws->scratch(names[r][3], (nb + 1) * 4);
        tt[r].pref = (uint16_t*)ws->scratch(names[r][4], ntl * (nb2 + 1) * 2);
        tt[r].prefT = (uint16_t*)ws->scratch(names[r][5], ntl * (nb2 + 1) * 2);
        tt[r].tstride = (uint32_t)ntl;
        SMJ_CHECK(hipMemcpyAsync(tt[r].btile0, bt0, (nb + 1) * 4,
                                 hipMemcpyHostToDevice, st));
        ostart[r] = (uint64_t*)ws->scratch(r ? "bs_ost1" : "bs_ost0", (size_t)nb * 8);
        SMJ_CHECK(hipMemcpyAsync(ostart[r], hdst + r * nb, (size_t)nb * 8,
                                 hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_tiles, dim3(nb), dim3(64), 0, st, a.bstart[r],
                           a.bcount[r], a.seg_start[r], a.seg_cnt[r], nseg, tt[r], tsz);
    }
    if (nrel == 1) tt[1] = tt[0];
    if (a.ev_tile) SMJ_CHECK(hipEventRecord(a.ev_tile, st));

    const uint32_t ngroups = nb * nb2;
    const uint32_t ovf_cap = ngroups;
    OvfEntry* ovf = (OvfEntry*)ws->scratch("bs_ovf", (size_t)ovf_cap * sizeof(OvfEntry));
    uint32_t* novf = (uint32_t*)ws->scratch("bs_novf", 4);
    SMJ_CHECK(hipMemsetAsync(novf, 0, 4, st));
    const size_t tp_lds = (size_t)tsz * sizeof(Tup) + nb2 * 4 + 64;

    TilePassArgs T;
    GroupArgs G;
    for (int r = 0; r < 2; r++) {
        const int rr = r < nrel ? r : 0;
        T.part[r] = a.part[rr];
        T.tt[r] = tt[rr];
        T.t0[r] = 0;
        T.nt[r] = 0;
        T.ntiles[r] = nullptr;
        G.out[r] = a.out[rr];
        G.bstart[r] = a.bstart[rr];
        G.ostart[r] = ostart[rr];
        G.tt[r] = tt[rr];
    }
    T.plan = *hplan;
    T.nb2 = nb2;
    T.pack_bad = nullptr;
    T.d2_fast = a.digit_fast && LayTup::fast_ok(*hplan, hplan->s2, hplan->D2);
    G.pack_bad = nullptr;
    G.d3_fast = a.digit_fast && LayTup::fast_ok(*hplan, hplan->s3, hplan->D3);
    G.nrel = nrel;
    G.pair = SMJ_GS_PAIR && nrel == 1;
    G.plan = *hplan;
    G.count_dev = a.count_dev;
    G.nb2 = nb2;
    G.ovf = ovf;
    G.novf = novf;
    G.ovf_cap = ovf_cap;
    uint32_t ntiles = 0;
    for (int r = 0; r < 2; r++) {
        const int rr = r < nrel ? r : 0;
        T.tmp[r] = a.tmp[rr];
        G.tmp[r] = a.tmp[rr];
        if (r < nrel) {
            T.t0[r] = 0;
            T.nt[r] = hbt[r * (nb + 1) + nb];
            ntiles += T.nt[r];
        }
    }
    if (ntiles) {
        {
            TraceScope ts(ws, "k_tilepass", st);
            launch_tilepass<LayTup, LayTup>(T, tp_lds, st);
        }
        launch_preft_range(T, nrel, nb2, st);
    }
    if (a.ev_bucket) SMJ_CHECK(hipEventRecord(a.ev_bucket, st));
    G.g_begin = 0;
    G.g_end = nb * nb2;
    {
        // persistent: gs_wg_per_cu workgroups per CU, consecutive groups each
        const uint32_t ng = G.g_end - G.g_begin;
        const uint32_t maxwg = gs_wg_per_cu<Tup>() * 256;
        const uint32_t nwg = groupsort_grid(ng, maxwg, G.per);
        TraceScope ts(ws, "k_groupsort", st);
        const uint64_t nmax = nrel > 1 && a.n[1] > a.n[0] ? a.n[1] : a.n[0];
        launch_groupsort<LayTup>(ws, group_tpl(nmax, nb, nseg, tsz), nwg, st, G);
    }
    SMJ_CHECK(hipGetLastError());
    if (a.ev_ovf) SMJ_CHECK(hipEventRecord(a.ev_ovf, st));

    // ---- overflow path (synchronises once)
    uint32_t* h_novf = (uint32_t*)ws->host_pinned("bs_h_novf", 4);
    SMJ_CHECK(hipMemcpyAsync(h_novf, novf, 4, hipMemcpyDeviceToHost, st));
    ws->wait_stream(st);
    const uint32_t no = *h_novf;
    if (no == 0) return true;
    if (no > ovf_cap) {
        fprintf(stderr, "[ERROR] smj: overflow table too small\n");
        abort();
    }
    skew_path<LayTup>(ws, G, ovf, no, hdst, nb, st);
    SMJ_CHECK(hipGetLastError());
    return true;
}

}  // namespace smj
