// bucketsort.hip -- MSD bucket sort of level-1 partitions with a fused
// merge-join count (the sorting_phase + mergejoin_phase of the reference m-way
// join, src/joins/sortmergejoin_multiway.c:388-460, 559-599, re-designed for
// MI355X).
//
// After the level-1 radix partition (partition.hip) every bucket b holds the
// tuples whose key falls in one contiguous key range of the RangePlan.
//
//   k_tilepass : every bucket is cut into tiles of TILE2 tuples.  A tile is
//                loaded into registers, counted by its level-2 digit d2 in an
//                LDS histogram, staged in LDS grouped by d2 and written back in
//                place, linearly (fully coalesced), together with the tile's
//                exclusive d2 prefix (uint16 per digit + a sentinel = length).
//                Traffic: 2w.
//   k_subwave  : ONE WAVE per sub-bucket (b, d2) at a time, twelve independent
//                waves per CU, no workgroup barriers.  The wave gathers the
//                sub-bucket's piece from every tile of bucket b (contiguous
//                runs read by consecutive lanes; the piece of a lane is found
//                with one ballot over a piece-start map instead of a search),
//                counting-sorts it in its private LDS slice by the level-3
//                digit, fixes equal-digit runs with an insertion sort on the
//                full (key, payload) order and writes the sorted sub-bucket to
//                its final position -- R first, then S in the same LDS slice --
//                and, for a join, counts the matching pairs of the two
//                sub-buckets from their level-3 histograms (exact digits) or
//                by binary search in R's sorted keys.  Traffic: 2w; the join
//                reads nothing more.  The eight-to-twelve waves of a workgroup
//                take neighbouring sub-buckets at the same time, so the cache
//                lines shared at piece boundaries and the 128-byte lines of the
//                prefix table are served from L1/L2, not refetched.
//
// Sub-buckets that do not fit the per-wave LDS capacity, or that hold long
// runs of equal digits (skew, e.g. Zipf hot keys), are queued and finished by
// the segmented merge sort (mergesort.hip) and the merge-join count kernel.
#include "smj_common.hpp"
#include "smj_internal.hpp"

namespace smj {

constexpr int TP_THREADS = 256;
constexpr int TP_ITEMS = 16;
constexpr int TILE2 = TP_THREADS * TP_ITEMS;  // 4096 tuples per tile

#ifdef KEY_8B
constexpr int SW_CAP = 384;  // tuples per sub-bucket per relation in LDS
typedef int64_t KeyT;
#else
constexpr int SW_CAP = 768;
typedef int32_t KeyT;
#endif
constexpr int SW_ITEMS = SW_CAP / 64;
constexpr int SW_D3MAX = 8;  // level-3 bins per wave (256)
constexpr int SW_NB3 = 1 << SW_D3MAX;
constexpr int SW_PMAX = 64;    // tiles per bucket handled by the wave path
constexpr int SW_RUNMAX = 32;  // longest equal-digit run fixed in LDS

struct TileTable {
    uint64_t* off;     // tile start in `part`
    uint32_t* len;     // tile length
    uint32_t* bucket;  // owning bucket
    uint32_t* btile0;  // first tile of every bucket (nbuckets + 1)
    uint16_t* pref;    // [tile][nb2 + 1] exclusive prefix, sentinel = length
    uint32_t* ntiles;  // device scalar
};

struct OvfEntry {
    uint32_t bucket, d2;
    uint32_t nr[2];
    uint64_t off[2];  // offset of the sub-bucket inside its bucket
};

// ---------------------------------------------------------------------------
// tile table: one workgroup scans the per-bucket tile counts.  The tiles of a
// bucket are consecutive TILE2-sized chunks of it.
__global__ void __launch_bounds__(256)
k_tiles(const uint64_t* __restrict__ bstart, const int64_t* __restrict__ bcount,
        uint32_t nb, TileTable tt) {
    __shared__ uint32_t scr[8];
    __shared__ uint32_t base_sh;
    if (threadIdx.x == 0) base_sh = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < nb; b0 += 256) {
        uint32_t b = b0 + threadIdx.x;
        uint32_t nt = 0;
        if (b < nb) nt = (uint32_t)((bcount[b] + TILE2 - 1) / TILE2);
        uint32_t tot;
        uint32_t ex = block_exclusive_scan(nt, scr, &tot);
        uint32_t t0 = base_sh + ex;
        if (b < nb) {
            tt.btile0[b] = t0;
            for (uint32_t i = 0; i < nt; i++) {
                uint64_t o = (uint64_t)i * TILE2;
                int64_t rem = bcount[b] - (int64_t)o;
                tt.off[t0 + i] = bstart[b] + o;
                tt.len[t0 + i] = (uint32_t)(rem < TILE2 ? rem : TILE2);
                tt.bucket[t0 + i] = b;
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) base_sh += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        tt.btile0[nb] = base_sh;
        *tt.ntiles = base_sh;
    }
}

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(TP_THREADS)
k_tilepass(const Tup* __restrict__ part, Tup* __restrict__ tmp, TileTable tt,
           const RangePlan* __restrict__ plan_dev, uint32_t nb2) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    const RangePlan P = *plan_dev;
    Tup* stage = reinterpret_cast<Tup*>(lds_raw);
    uint32_t* hist = reinterpret_cast<uint32_t*>(lds_raw + TILE2 * sizeof(Tup));
    uint32_t* scr = hist + nb2;

    const uint32_t t = blockIdx.x;
    if (t >= *tt.ntiles) return;
    const uint64_t off = tt.off[t];
    const uint32_t len = tt.len[t];
    const uint32_t b = tt.bucket[t];

    for (uint32_t d = threadIdx.x; d < nb2; d += TP_THREADS) hist[d] = 0;
    Tup v[TP_ITEMS];
    uint32_t dg[TP_ITEMS];
#pragma unroll
    for (int j = 0; j < TP_ITEMS; j++) {
        uint32_t i = j * TP_THREADS + threadIdx.x;
        if (i < len) v[j] = part[off + i];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < TP_ITEMS; j++) {
        uint32_t i = j * TP_THREADS + threadIdx.x;
        if (i < len) {
            dg[j] = plan_d2(P, plan_rel(P, tup_key(v[j])), b);
            atomicAdd(&hist[dg[j]], 1u);
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
            stage[pos] = v[j];
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < TP_ITEMS; j++) {
        uint32_t i = j * TP_THREADS + threadIdx.x;
        if (i < len) tmp[off + i] = stage[i];
    }
}

// ---------------------------------------------------------------------------
struct SubWaveArgs {
    const Tup* tmp[2];
    Tup* out[2];
    const uint64_t* bstart[2];
    TileTable tt[2];
    int nrel;
    const RangePlan* plan_dev;
    unsigned long long* count_dev;
    uint32_t nb2;   // level-2 table stride (>= 1 << plan.D2)
    uint32_t nsub;  // nbuckets * nb2
    uint32_t spw;   // sub-buckets per wave
    OvfEntry* ovf;
    uint32_t* novf;
    uint32_t ovf_cap;
};

// per-wave LDS slice; R and S pass through B one after the other
struct WaveLDS {
    Tup B[SW_CAP];
    KeyT rkey[SW_CAP];       // R's sorted keys (generic join)
    uint32_t h[2][SW_NB3];   // level-3 bin starts of R and S
    uint32_t fill[SW_NB3];
    uint32_t psrc[SW_PMAX];  // piece start, relative to the bucket start
    uint32_t pdst[SW_PMAX];  // piece position inside the sub-bucket
    uint8_t pat[SW_CAP];     // piece starting at a position, 0xff = none
};
constexpr int SW_WAVES_RAW = (160 * 1024) / (int)sizeof(WaveLDS);
constexpr int SW_WAVES = SW_WAVES_RAW > 16 ? 16 : SW_WAVES_RAW;
constexpr int SW_THREADS = SW_WAVES * 64;
static_assert(SW_WAVES >= 8, "LDS slice too large");

// order this wave's LDS accesses (LDS executes one wave's instructions in
// order; the fences stop the compiler from moving accesses across)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    const int lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x;
}

__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        uint32_t y = __shfl_xor(x, o, 64);
        x = y > x ? y : x;
    }
    return x;
}

__device__ __forceinline__ void lds_insertion_sort(Tup* a, uint32_t n) {
    for (uint32_t i = 1; i < n; i++) {
        Tup x = a[i];
        uint32_t j = i;
        while (j > 0 && tup_less(x, a[j - 1])) {
            a[j] = a[j - 1];
            j--;
        }
        a[j] = x;
    }
}

__device__ void sub_overflow(const SubWaveArgs& A, uint32_t b, uint32_t d2,
                             const uint32_t* n, const uint64_t* off,
                             bool sizes_known, int lane) {
    if (lane != 0) return;
    uint32_t n2[2] = {0, 0};
    uint64_t o2[2] = {0, 0};
    for (int r = 0; r < A.nrel; r++) {
        if (sizes_known) {
            n2[r] = n[r];
            o2[r] = off[r];
            continue;
        }
        const TileTable& tt = A.tt[r];
        for (uint32_t t = tt.btile0[b]; t < tt.btile0[b + 1]; t++) {
            const uint16_t* pf = tt.pref + (uint64_t)t * (A.nb2 + 1);
            n2[r] += (uint32_t)pf[d2 + 1] - pf[d2];
            o2[r] += pf[d2];
        }
    }
    const uint32_t k = atomicAdd(A.novf, 1u);
    if (k < A.ovf_cap) {
        OvfEntry e;
        e.bucket = b;
        e.d2 = d2;
        e.nr[0] = n2[0];
        e.nr[1] = n2[1];
        e.off[0] = o2[0];
        e.off[1] = o2[1];
        A.ovf[k] = e;
    }
}

__global__ void __launch_bounds__(SW_THREADS)
k_subwave(SubWaveArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    WaveLDS& L = reinterpret_cast<WaveLDS*>(lds_raw)[threadIdx.x >> 6];
    const RangePlan P = *A.plan_dev;
    const uint32_t nb2 = A.nb2;
    const uint32_t nb3 = 1u << P.D3;
    const uint32_t d2lim = 1u << P.D2;
    const int lane = lane_id();
    const uint64_t lmask_le = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    const uint64_t bu = key_u(P.base);

    // the workgroup owns [g0, s_end); its waves take them interleaved
    const uint32_t g0 = blockIdx.x * SW_WAVES * A.spw;
    uint32_t s_end = g0 + SW_WAVES * A.spw;
    if (s_end > A.nsub) s_end = A.nsub;
    unsigned long long matches = 0;
    uint32_t cur_b = 0xffffffffu;
    uint32_t t0[2] = {0, 0}, nt[2] = {0, 0};
    uint64_t bst[2] = {0, 0};

    for (uint32_t s = g0 + (threadIdx.x >> 6); s < s_end; s += SW_WAVES) {
        const uint32_t b = s / nb2;
        const uint32_t d2 = s % nb2;
        if (d2 >= d2lim) continue;  // a table column no digit maps to
        if (b != cur_b) {
            cur_b = b;
#pragma unroll
            for (int r = 0; r < 2; r++) {
                if (r < A.nrel) {
                    t0[r] = A.tt[r].btile0[b];
                    nt[r] = A.tt[r].btile0[b + 1] - t0[r];
                    bst[r] = A.bstart[r][b];
                }
            }
        }
        // ---- sizes of the sub-bucket in both relations (one round trip)
        uint32_t n[2] = {0, 0}, plo[2] = {0, 0}, pcnt[2] = {0, 0}, pincl[2] = {0, 0};
        uint64_t off[2] = {0, 0};
        bool ovf = false, known = true;
#pragma unroll
        for (int r = 0; r < 2; r++) {
            if (r >= A.nrel) break;
            if (nt[r] > SW_PMAX) {
                ovf = true;
                known = false;
                continue;
            }
            if ((uint32_t)lane < nt[r]) {
                const uint16_t* pf =
                    A.tt[r].pref + (uint64_t)(t0[r] + lane) * (nb2 + 1) + d2;
                plo[r] = pf[0];
                pcnt[r] = (uint32_t)pf[1] - plo[r];
            }
        }
#pragma unroll
        for (int r = 0; r < 2; r++) {
            if (r >= A.nrel || nt[r] > SW_PMAX) continue;
            pincl[r] = wave_incl_scan(pcnt[r]);
            n[r] = __shfl(pincl[r], 63, 64);
            off[r] = wave_sum((unsigned long long)plo[r]);
            if (n[r] > SW_CAP) ovf = true;
        }
        if (ovf) {
            sub_overflow(A, b, d2, n, off, known, lane);
            continue;
        }

        const uint32_t d12 = (b << P.D2) | d2;
        bool clamped = false;
#pragma unroll
        for (int r = 0; r < 2; r++) {
            if (r >= A.nrel) break;
            const uint32_t nr = n[r];
            // ---- piece tables and the piece-start map
            if ((uint32_t)lane < nt[r]) {
                L.psrc[lane] = lane * (uint32_t)TILE2 + plo[r];
                L.pdst[lane] = pincl[r] - pcnt[r];
            }
            for (uint32_t j = lane; j < SW_CAP / 4; j += 64)
                reinterpret_cast<uint32_t*>(L.pat)[j] = 0xffffffffu;
#pragma unroll
            for (int q = 0; q < SW_NB3 / 64; q++) L.h[r][lane * (SW_NB3 / 64) + q] = 0;
            wave_lds_sync();
            if ((uint32_t)lane < nt[r] && pcnt[r] > 0)
                L.pat[pincl[r] - pcnt[r]] = (uint8_t)lane;
            wave_lds_sync();

            // ---- gather: the piece of position i is the last piece start <= i
            Tup v[SW_ITEMS];
            uint32_t dg[SW_ITEMS];
            const Tup* tp = A.tmp[r] + bst[r];
            uint32_t carry = 0;
#pragma unroll
            for (int k = 0; k < SW_ITEMS; k++) {
                const uint32_t i = k * 64 + lane;
                const bool valid = i < nr;
                const uint32_t m = valid ? L.pat[i] : 0xffu;
                const uint64_t starts = __ballot(m != 0xffu) & lmask_le;
                const uint32_t src_lane = starts ? 63 - __clzll(starts) : 0;
                const uint32_t pm = __shfl(m, src_lane, 64);
                const uint32_t p = starts ? pm : carry;
                carry = __shfl(p, 63, 64);
                if (valid) v[k] = tp[L.psrc[p] + (i - L.pdst[p])];
            }
            // ---- level-3 digits, histogram
#pragma unroll
            for (int k = 0; k < SW_ITEMS; k++) {
                const uint32_t i = k * 64 + lane;
                if (i < nr) {
                    const int64_t key = tup_key(v[k]);
                    const uint64_t ku = key_u(key);
                    clamped |= (ku < bu) || (ku - bu > P.span);
                    dg[k] = plan_d3(P, plan_rel(P, key), d12);
                    atomicAdd(&L.h[r][dg[k]], 1u);
                }
            }
            wave_lds_sync();
            // ---- exclusive scan of the bins: lane owns 4 consecutive bins
            uint32_t c[SW_NB3 / 64];
            uint32_t loc = 0, mx = 0;
#pragma unroll
            for (int q = 0; q < SW_NB3 / 64; q++) {
                c[q] = L.h[r][lane * (SW_NB3 / 64) + q];
                loc += c[q];
                mx = c[q] > mx ? c[q] : mx;
            }
            uint32_t ex = wave_incl_scan(loc) - loc;
#pragma unroll
            for (int q = 0; q < SW_NB3 / 64; q++) {
                L.h[r][lane * (SW_NB3 / 64) + q] = ex;
                L.fill[lane * (SW_NB3 / 64) + q] = ex;
                ex += c[q];
            }
            if (wave_max(mx) > SW_RUNMAX) {
                ovf = true;
                break;
            }
            wave_lds_sync();
            // ---- place, fix equal-digit runs, write
#pragma unroll
            for (int k = 0; k < SW_ITEMS; k++) {
                const uint32_t i = k * 64 + lane;
                if (i < nr) L.B[atomicAdd(&L.fill[dg[k]], 1u)] = v[k];
            }
            wave_lds_sync();
            for (uint32_t d = lane; d < nb3; d += 64) {
                const uint32_t s0 = L.h[r][d];
                const uint32_t e0 = (d + 1 < nb3) ? L.h[r][d + 1] : nr;
                if (e0 - s0 > 1) lds_insertion_sort(L.B + s0, e0 - s0);
            }
            wave_lds_sync();
            Tup* dst = A.out[r] + bst[r] + off[r];
            for (uint32_t i = lane; i < nr; i += 64) {
                const Tup t = L.B[i];
                dst[i] = t;
                if (r == 0) L.rkey[i] = (KeyT)tup_key(t);
            }
            wave_lds_sync();
        }
        if (ovf) {
            // a long equal-digit run: the fallback re-sorts the sub-bucket of
            // both relations (an R already written here is simply rewritten)
            sub_overflow(A, b, d2, n, off, true, lane);
            continue;
        }

        // ---- merge-join count of the two sub-buckets
        if (A.nrel == 2) {
            const uint32_t nR = n[0], nS = n[1];
            if (P.s3 == 0 && !__any(clamped)) {
                // the level-3 digit is the exact key: sum_k |R_k| * |S_k|
                for (uint32_t d = lane; d < nb3; d += 64) {
                    const uint32_t cr = ((d + 1 < nb3) ? L.h[0][d + 1] : nR) - L.h[0][d];
                    const uint32_t cs = ((d + 1 < nb3) ? L.h[1][d + 1] : nS) - L.h[1][d];
                    matches += (unsigned long long)cr * cs;
                }
            } else {
                // S is still in B, R's sorted keys in rkey
                for (uint32_t i = lane; i < nS; i += 64) {
                    const int64_t k = tup_key(L.B[i]);
                    if (i > 0 && tup_key(L.B[i - 1]) == k) continue;
                    uint32_t e = i + 1;
                    while (e < nS && tup_key(L.B[e]) == k) e++;
                    uint32_t lo = 0, hi = nR;
                    while (lo < hi) {
                        const uint32_t m = (lo + hi) >> 1;
                        if ((int64_t)L.rkey[m] < k) lo = m + 1; else hi = m;
                    }
                    const uint32_t lb = lo;
                    hi = nR;
                    while (lo < hi) {
                        const uint32_t m = (lo + hi) >> 1;
                        if ((int64_t)L.rkey[m] <= k) lo = m + 1; else hi = m;
                    }
                    matches += (unsigned long long)(lo - lb) * (e - i);
                }
            }
            wave_lds_sync();
        }
    }
    if (A.nrel == 2) {
        matches = wave_sum(matches);
        if (lane == 0 && matches) atomicAdd(A.count_dev, matches);
    }
}

// ---------------------------------------------------------------------------
// overflow: copy the pieces of a sub-bucket, unsorted, into its output slot
__global__ void __launch_bounds__(256)
k_gather_sub(const Tup* __restrict__ tmp, Tup* __restrict__ out,
             const uint64_t* __restrict__ bstart, TileTable tt,
             const OvfEntry* __restrict__ ovf, int r, uint32_t nb2) {
    const OvfEntry e = ovf[blockIdx.x];
    const uint32_t b = e.bucket, d2 = e.d2;
    Tup* dst = out + bstart[b] + e.off[r];
    uint32_t pos = 0;
    for (uint32_t t = tt.btile0[b]; t < tt.btile0[b + 1]; t++) {
        const uint16_t* pf = tt.pref + (uint64_t)t * (nb2 + 1);
        uint32_t lo = pf[d2];
        uint32_t hi = pf[d2 + 1];
        const Tup* src = tmp + tt.off[t] + lo;
        for (uint32_t i = threadIdx.x; i < hi - lo; i += 256) dst[pos + i] = src[i];
        pos += hi - lo;
    }
}

// ---------------------------------------------------------------------------
// range plan from a strided sample of the relations (or from hints)
__global__ void __launch_bounds__(256)
k_plan(const Tup* r0, uint64_t n0, const Tup* r1, uint64_t n1, uint32_t D1,
       uint32_t D2, int64_t hmin, int64_t hmax, RangePlan* plan) {
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
        *plan = make_plan(lo, hi, D1, D2, SW_D3MAX);
    }
}

void plan_from_sample(Workspace* ws, const Tup* const* rels, const uint64_t* ns,
                      int nrel, uint32_t D1, uint32_t D2, int64_t hint_min,
                      int64_t hint_max, RangePlan* plan_dev, hipStream_t st) {
    (void)ws;
    hipLaunchKernelGGL(k_plan, dim3(1), dim3(256), 0, st, rels[0], ns[0],
                       nrel > 1 ? rels[1] : (const Tup*)nullptr,
                       nrel > 1 ? ns[1] : 0, D1, D2, hint_min, hint_max,
                       plan_dev);
    SMJ_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
void bucket_sort(Workspace* ws, const BucketSortArgs& a, uint32_t D2,
                 hipStream_t st) {
    const uint32_t nb = a.nbuckets;
    const uint32_t nb2 = 1u << D2;
    TileTable tt[2];
    static const char* names[2][6] = {
        {"bs_off0", "bs_len0", "bs_bkt0", "bs_bt00", "bs_pref0", "bs_nt0"},
        {"bs_off1", "bs_len1", "bs_bkt1", "bs_bt01", "bs_pref1", "bs_nt1"}};
    uint64_t maxt[2] = {0, 0};
    for (int r = 0; r < a.nrel; r++) {
        maxt[r] = (a.n[r] + TILE2 - 1) / TILE2 + nb + 1;
        tt[r].off = (uint64_t*)ws->scratch(names[r][0], maxt[r] * 8);
        tt[r].len = (uint32_t*)ws->scratch(names[r][1], maxt[r] * 4);
        tt[r].bucket = (uint32_t*)ws->scratch(names[r][2], maxt[r] * 4);
        tt[r].btile0 = (uint32_t*)ws->scratch(names[r][3], (nb + 1) * 4);
        tt[r].pref = (uint16_t*)ws->scratch(names[r][4], maxt[r] * (nb2 + 1) * 2);
        tt[r].ntiles = (uint32_t*)ws->scratch(names[r][5], 4);
        hipLaunchKernelGGL(k_tiles, dim3(1), dim3(256), 0, st, a.bstart[r],
                           a.bcount[r], nb, tt[r]);
    }
    if (a.ev_tile) SMJ_CHECK(hipEventRecord(a.ev_tile, st));
    static bool attr = false;
    if (!attr) {
        SMJ_CHECK(hipFuncSetAttribute((const void*)k_tilepass,
                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                      160 * 1024));
        SMJ_CHECK(hipFuncSetAttribute((const void*)k_subwave,
                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                      160 * 1024));
        attr = true;
    }
    const size_t tp_lds = TILE2 * sizeof(Tup) + nb2 * 4 + 64;
    for (int r = 0; r < a.nrel; r++) {
        TraceScope ts(ws, "k_tilepass", st);
        hipLaunchKernelGGL(k_tilepass, dim3((uint32_t)maxt[r]), dim3(TP_THREADS),
                           tp_lds, st, a.part[r], a.tmp[r], tt[r], a.plan_dev, nb2);
    }
    if (a.ev_bucket) SMJ_CHECK(hipEventRecord(a.ev_bucket, st));

    const uint32_t nsub = nb * nb2;
    const uint32_t ovf_cap = nsub;
    OvfEntry* ovf = (OvfEntry*)ws->scratch("bs_ovf", (size_t)ovf_cap * sizeof(OvfEntry));
    uint32_t* novf = (uint32_t*)ws->scratch("bs_novf", 4);
    SMJ_CHECK(hipMemsetAsync(novf, 0, 4, st));
    SubWaveArgs B;
    for (int r = 0; r < 2; r++) {
        int rr = r < a.nrel ? r : 0;
        B.tmp[r] = a.tmp[rr];
        B.out[r] = a.out[rr];
        B.bstart[r] = a.bstart[rr];
        B.tt[r] = tt[rr];
    }
    B.nrel = a.nrel;
    B.plan_dev = a.plan_dev;
    B.count_dev = a.count_dev;
    B.nb2 = nb2;
    B.nsub = nsub;
    // one workgroup of SW_WAVES waves per CU, several sub-buckets per wave
    const uint32_t target_waves = 256 * SW_WAVES;
    B.spw = (nsub + target_waves - 1) / target_waves;
    if (B.spw == 0) B.spw = 1;
    const uint32_t nwg = (nsub + SW_WAVES * B.spw - 1) / (SW_WAVES * B.spw);
    B.ovf = ovf;
    B.novf = novf;
    B.ovf_cap = ovf_cap;
    {
        TraceScope ts(ws, "k_subwave", st);
        hipLaunchKernelGGL(k_subwave, dim3(nwg), dim3(SW_THREADS),
                           sizeof(WaveLDS) * SW_WAVES, st, B);
    }
    SMJ_CHECK(hipGetLastError());
    if (a.ev_ovf) SMJ_CHECK(hipEventRecord(a.ev_ovf, st));

    // ---- overflow path (synchronises once)
    uint32_t* h_novf = (uint32_t*)ws->host_pinned("bs_h_novf", 4);
    SMJ_CHECK(hipMemcpyAsync(h_novf, novf, 4, hipMemcpyDeviceToHost, st));
    SMJ_CHECK(hipStreamSynchronize(st));
    const uint32_t no = *h_novf;
    if (no == 0) return;
    if (no > ovf_cap) {
        fprintf(stderr, "[ERROR] smj: overflow table too small\n");
        abort();
    }
    std::vector<OvfEntry> he(no);
    SMJ_CHECK(hipMemcpyAsync(he.data(), ovf, no * sizeof(OvfEntry),
                             hipMemcpyDeviceToHost, st));
    std::vector<uint64_t> hbstart[2];
    for (int r = 0; r < a.nrel; r++) {
        hbstart[r].resize(nb);
        SMJ_CHECK(hipMemcpyAsync(hbstart[r].data(), a.bstart[r], nb * 8,
                                 hipMemcpyDeviceToHost, st));
    }
    SMJ_CHECK(hipStreamSynchronize(st));
    for (int r = 0; r < a.nrel; r++) {
        hipLaunchKernelGGL(k_gather_sub, dim3(no), dim3(256), 0, st, a.tmp[r],
                           a.out[r], a.bstart[r], tt[r], ovf, r, nb2);
        std::vector<uint64_t> so(no), sl(no);
        for (uint32_t i = 0; i < no; i++) {
            so[i] = hbstart[r][he[i].bucket] + he[i].off[r];
            sl[i] = he[i].nr[r];
        }
        segmented_sort(ws, a.out[r], so.data(), sl.data(), no, st);
    }
    if (a.nrel == 2) {
        for (uint32_t i = 0; i < no; i++) {
            const Tup* rp = a.out[0] + hbstart[0][he[i].bucket] + he[i].off[0];
            const Tup* sp = a.out[1] + hbstart[1][he[i].bucket] + he[i].off[1];
            if (he[i].nr[0] && he[i].nr[1])
                merge_join_count(rp, he[i].nr[0], sp, he[i].nr[1], a.count_dev, st);
        }
    }
    SMJ_CHECK(hipGetLastError());
}

}  // namespace smj
