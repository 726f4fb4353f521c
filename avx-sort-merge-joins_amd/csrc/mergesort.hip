// mergesort.hip -- merge-path kernels: 2-way merge (avx_merge_*), k-way merge
// tree (avx_multiway_merge), segmented merge sort (skew fallback of the bucket
// sort) and the merge-join count (merge_join).
//
// Reference counterparts: src/merge/merge.c:106-235 (bitonic 2-way merge
// kernels), src/merge/avx_multiwaymerge.c:199-338 (FIFO merge tree),
// src/avxsort/avxsort_core.h:1276-1399 (in-cache block sort with bitonic
// networks), src/joins/joincommon.c:239-312 (merge_join).
//
// GPU form: every merge is split into output tiles along the merge path
// (co-rank binary search on the two inputs), so each workgroup reads exactly
// the slices of A and B that produce its 2048 outputs with coalesced 16-byte
// lane loads, merges them in LDS and writes a contiguous output tile.  Block
// sorts run a bitonic network in registers (lane shuffles, LDS only across
// waves).
#include <string.h>

#include <algorithm>

#include "smj_common.hpp"
#include "smj_internal.hpp"

namespace smj {

constexpr int MG_THREADS = 256;
constexpr int MG_TILE = 2048;  // outputs per merge tile
constexpr int MG_IPT = MG_TILE / MG_THREADS;
constexpr int BS_THREADS = 256;
constexpr int BS_BLOCK = 2048;  // block-sort tile (power of two)

struct MergeTile {
    const Tup* a;
    const Tup* b;
    Tup* out;
    uint64_t na, nb;
    uint64_t d0, d1;  // output diagonal range of this tile
};

// co-rank: number of A items among the first d outputs (A first on ties)
template <class GetA, class GetB>
__device__ __forceinline__ uint64_t corank(uint64_t d, uint64_t na,
                                           uint64_t nb, GetA A, GetB B) {
    uint64_t lo = d > nb ? d - nb : 0;
    uint64_t hi = d < na ? d : na;
    while (lo < hi) {
        uint64_t mid = (lo + hi) >> 1;
        // A[mid] precedes B[d-1-mid]  <=>  !(B < A)
        if (!tup_less(B(d - 1 - mid), A(mid)))
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(MG_THREADS)
k_mergetile(const MergeTile* __restrict__ tiles) {
    __shared__ __attribute__((aligned(16))) Tup sm[MG_TILE];
    __shared__ uint64_t sh_ab[2];
    const MergeTile T = tiles[blockIdx.x];
    if (threadIdx.x < 2) {
        const uint64_t d = threadIdx.x == 0 ? T.d0 : T.d1;
        sh_ab[threadIdx.x] = corank(
            d, T.na, T.nb, [&](uint64_t i) { return ld_g(T.a + i); },
            [&](uint64_t i) { return ld_g(T.b + i); });
    }
    __syncthreads();
    const uint64_t a0 = sh_ab[0], a1 = sh_ab[1];
    const uint64_t b0 = T.d0 - a0, b1 = T.d1 - a1;
    const uint32_t la = (uint32_t)(a1 - a0), lb = (uint32_t)(b1 - b0);
    for (uint32_t i = threadIdx.x; i < la; i += MG_THREADS) sm[i] = ld_g(T.a + a0 + i);
    for (uint32_t i = threadIdx.x; i < lb; i += MG_THREADS) sm[la + i] = ld_g(T.b + b0 + i);
    __syncthreads();
    const Tup* As = sm;
    const Tup* Bs = sm + la;
    const uint32_t len = la + lb;
    uint32_t p = threadIdx.x * MG_IPT;
    Tup res[MG_IPT];
    if (p < len) {
        uint32_t i = (uint32_t)corank(
            p, la, lb, [&](uint64_t x) { return As[x]; },
            [&](uint64_t x) { return Bs[x]; });
        uint32_t j = p - i;
        // branch-free, selecting values (selecting LDS references sent res
        // to scratch); past the end both runs are exhausted and the result
        // is not stored
#pragma unroll
        for (int k = 0; k < MG_IPT; k++) {
            const Tup av = sm[min(i, len - 1)];
            const Tup bv = sm[min(la + j, len - 1)];
            const bool takeA = i < la && (j >= lb || !tup_less(bv, av));
            res[k] = tup_sel(takeA, av, bv);
            i += takeA ? 1 : 0;
            j += takeA ? 0 : 1;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < MG_IPT; k++)
        if (p + k < len) sm[p + k] = res[k];
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < len; i += MG_THREADS) st_g(T.out + T.d0 + i, sm[i]);
}

// ---------------------------------------------------------------------------
struct SortBlock {
    uint64_t off;
    uint32_t len;
};

__device__ __forceinline__ Tup shfl_xor_tup(const Tup& v, int m) {
#ifdef KEY_8B
    Tup r;
    r.payload = __shfl_xor(v.payload, m, 64);
    r.key = __shfl_xor(v.key, m, 64);
    return r;
#else
    return (Tup)__shfl_xor((unsigned long long)v, m, 64);
#endif
}

// compare-exchange of element e with its partner of stage (k, j): keep the
// minimum when e is the pair's lower index of an ascending run (or the upper
// index of a descending one), else the maximum
__device__ __forceinline__ void bs_keep(Tup& x, const Tup& y, uint32_t e, uint32_t j,
                                        uint32_t k) {
    const bool keep_min = ((e & j) == 0) == ((e & k) == 0);
    if (keep_min ? tup_less(y, x) : tup_less(x, y)) x = y;
}

// Bitonic sort of one block of up to BS_BLOCK tuples, in registers: thread t
// holds elements [BS_IPT t, BS_IPT (t + 1)); stages whose partner is inside
// the thread swap registers, stages with a partner in another lane of the
// wave exchange through __shfl_xor, and only the stages across waves
// (j >= 64 BS_IPT: three of the 66 at 2048 elements) go through LDS.
// (avxsort_core.h:1276-1399 sorts its cache-sized blocks with in-register
// AVX networks the same way.)
constexpr uint32_t BS_IPT = BS_BLOCK / BS_THREADS;
static_assert(BS_IPT == 8, "k_blocksort's in-thread stages are j = 4, 2, 1");
template <uint32_t J>
__device__ __forceinline__ void bs_inthread(Tup (&v)[BS_IPT], uint32_t t, uint32_t k) {
#pragma unroll
    for (uint32_t i = 0; i < BS_IPT; i++) {
        const uint32_t i2 = i ^ J;
        if (i2 > i) {
            const bool up = ((t * BS_IPT + i) & k) == 0;
            if (tup_less(v[i2], v[i]) == up) {
                const Tup x = v[i];
                v[i] = v[i2];
                v[i2] = x;
            }
        }
    }
}
__global__ void __launch_bounds__(BS_THREADS)
k_blocksort(Tup* __restrict__ data, const SortBlock* __restrict__ blocks) {
    __shared__ __attribute__((aligned(16))) Tup sm[BS_BLOCK];
    const SortBlock blk = blocks[blockIdx.x];
    const Tup sent = tup_max_sentinel();
    const uint32_t t = threadIdx.x;
    // coalesced load (sentinels past the end), then BS_IPT consecutive
    // elements per thread
    for (uint32_t i = t; i < BS_BLOCK; i += BS_THREADS) {
        Tup x = sent;  // a value, not a select between references (scratch)
        if (i < blk.len) x = ld_g(data + blk.off + i);
        sm[i] = x;
    }
    __syncthreads();
    Tup v[BS_IPT];
#pragma unroll
    for (uint32_t i = 0; i < BS_IPT; i++) v[i] = sm[t * BS_IPT + i];
    for (uint32_t k = 2; k <= BS_BLOCK; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            if (j >= 64 * BS_IPT) {  // partner in another wave
                __syncthreads();
#pragma unroll
                for (uint32_t i = 0; i < BS_IPT; i++) sm[t * BS_IPT + i] = v[i];
                __syncthreads();
#pragma unroll
                for (uint32_t i = 0; i < BS_IPT; i++) {
                    const uint32_t e = t * BS_IPT + i;
                    bs_keep(v[i], sm[e ^ j], e, j, k);
                }
            } else if (j >= BS_IPT) {  // partner in lane ^ (j / BS_IPT)
#pragma unroll
                for (uint32_t i = 0; i < BS_IPT; i++) {
                    const uint32_t e = t * BS_IPT + i;
                    bs_keep(v[i], shfl_xor_tup(v[i], (int)(j / BS_IPT)), e, j, k);
                }
            } else {  // partner in this thread: a compile-time j, so that v
                      // stays in registers (a runtime index sends it to scratch)
                if (j == 4) bs_inthread<4>(v, t, k);
                else if (j == 2) bs_inthread<2>(v, t, k);
                else bs_inthread<1>(v, t, k);
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t i = 0; i < BS_IPT; i++) sm[t * BS_IPT + i] = v[i];
    __syncthreads();
    for (uint32_t i = t; i < blk.len; i += BS_THREADS) data[blk.off + i] = sm[i];
}

// ---------------------------------------------------------------------------
// merge-join count: sum over keys of |R_k| * |S_k| for sorted R and S
__global__ void __launch_bounds__(256)
k_mjcount(const Tup* __restrict__ R, uint64_t nr, const Tup* __restrict__ S,
          uint64_t ns, unsigned long long* __restrict__ count) {
    unsigned long long c = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ns;
         i += stride) {
        const int64_t k = tup_key(S[i]);
        if (i > 0 && tup_key(S[i - 1]) == k) continue;
        // end of this key's run in S
        uint64_t lo = i + 1, hi = ns;
        while (lo < hi) {
            uint64_t m = (lo + hi) >> 1;
            if (tup_key(S[m]) <= k) lo = m + 1; else hi = m;
        }
        const uint64_t sc = lo - i;
        lo = 0;
        hi = nr;
        while (lo < hi) {
            uint64_t m = (lo + hi) >> 1;
            if (tup_key(R[m]) < k) lo = m + 1; else hi = m;
        }
        const uint64_t rl = lo;
        hi = nr;
        while (lo < hi) {
            uint64_t m = (lo + hi) >> 1;
            if (tup_key(R[m]) <= k) lo = m + 1; else hi = m;
        }
        c += (unsigned long long)(lo - rl) * sc;
    }
    c = wave_sum(c);
    if (lane_id() == 0 && c) atomicAdd(count, c);
}

// one block per pair of sorted runs: k_mjcount's counting, grid-batched
struct JoinPair {
    const Tup* r;
    const Tup* s;
    uint64_t nr, ns;
};

__global__ void __launch_bounds__(256)
k_mjcount_batch(const JoinPair* __restrict__ pairs, unsigned long long* __restrict__ count) {
    const JoinPair P = pairs[blockIdx.x];
    unsigned long long c = 0;
    for (uint64_t i = threadIdx.x; i < P.ns; i += 256) {
        const int64_t k = tup_key(ld_g(P.s + i));
        if (i > 0 && tup_key(ld_g(P.s + i - 1)) == k) continue;
        uint64_t lo = i + 1, hi = P.ns;
        while (lo < hi) {
            const uint64_t m = (lo + hi) >> 1;
            if (tup_key(ld_g(P.s + m)) <= k) lo = m + 1; else hi = m;
        }
        const uint64_t sc = lo - i;
        lo = 0;
        hi = P.nr;
        while (lo < hi) {
            const uint64_t m = (lo + hi) >> 1;
            if (tup_key(ld_g(P.r + m)) < k) lo = m + 1; else hi = m;
        }
        const uint64_t rl = lo;
        hi = P.nr;
        while (lo < hi) {
            const uint64_t m = (lo + hi) >> 1;
            if (tup_key(ld_g(P.r + m)) <= k) lo = m + 1; else hi = m;
        }
        c += (unsigned long long)(lo - rl) * sc;
    }
    c = wave_sum(c);
    if (lane_id() == 0 && c) atomicAdd(count, c);
}

__global__ void k_copy(const Tup* __restrict__ a, Tup* __restrict__ b,
                       uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += stride)
        b[i] = a[i];
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static void launch_tiles(Workspace* ws, const std::vector<MergeTile>& tiles,
                         hipStream_t st) {
    if (tiles.empty()) return;
    // tables live in their own scratch slot; the host copy is staged through
    // pinned memory so the upload is stream ordered
    const size_t bytes = tiles.size() * sizeof(MergeTile);
    MergeTile* dev = (MergeTile*)ws->scratch("mg_tiles", bytes);
    uint32_t slot;
    MergeTile* h = (MergeTile*)ws->ring_acquire("mg_tiles_h", bytes, &slot);
    std::copy(tiles.begin(), tiles.end(), h);
    SMJ_CHECK(hipMemcpyAsync(dev, h, bytes, hipMemcpyHostToDevice, st));
    ws->ring_release("mg_tiles_h", slot, st);
    hipLaunchKernelGGL(k_mergetile, dim3((uint32_t)tiles.size()),
                       dim3(MG_THREADS), 0, st, dev);
    SMJ_CHECK(hipGetLastError());
}

static void add_pair_tiles(std::vector<MergeTile>& v, const Tup* a,
                           uint64_t na, const Tup* b, uint64_t nb, Tup* out) {
    const uint64_t n = na + nb;
    for (uint64_t d = 0; d < n; d += MG_TILE) {
        MergeTile t;
        t.a = a;
        t.b = b;
        t.out = out;
        t.na = na;
        t.nb = nb;
        t.d0 = d;
        t.d1 = std::min<uint64_t>(n, d + MG_TILE);
        v.push_back(t);
    }
}

void merge2(Workspace* ws, const Tup* a, uint64_t na, const Tup* b, uint64_t nb, Tup* out,
            hipStream_t st) {
    std::vector<MergeTile> v;
    add_pair_tiles(v, a, na, b, nb, out);
    launch_tiles(ws, v, st);  // the caller's workspace: one per thread/stream
}

void merge_join_count(const Tup* r, uint64_t nr, const Tup* s, uint64_t ns,
                      unsigned long long* count_dev, hipStream_t st) {
    if (nr == 0 || ns == 0) return;
    uint64_t blocks = (ns + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_mjcount, dim3((uint32_t)blocks), dim3(256), 0, st, r,
                       nr, s, ns, count_dev);
    SMJ_CHECK(hipGetLastError());
}

void merge_join_count_batch(Workspace* ws, const Tup* const* r, const uint64_t* nr,
                            const Tup* const* s, const uint64_t* ns, uint32_t k,
                            unsigned long long* count_dev, hipStream_t st) {
    if (k == 0) return;
    const size_t bytes = (size_t)k * sizeof(JoinPair);
    JoinPair* dev = (JoinPair*)ws->scratch("mj_pairs", bytes);
    uint32_t slot;
    JoinPair* h = (JoinPair*)ws->ring_acquire("mj_pairs_h", bytes, &slot);
    for (uint32_t i = 0; i < k; i++) h[i] = JoinPair{r[i], s[i], nr[i], ns[i]};
    SMJ_CHECK(hipMemcpyAsync(dev, h, bytes, hipMemcpyHostToDevice, st));
    ws->ring_release("mj_pairs_h", slot, st);
    hipLaunchKernelGGL(k_mjcount_batch, dim3(k), dim3(256), 0, st, dev, count_dev);
    SMJ_CHECK(hipGetLastError());
}

// Sort every segment [off, off+len) of `data` in place.
void segmented_sort(Workspace* ws, Tup* data, const uint64_t* seg_off,
                    const uint64_t* seg_len, uint32_t nseg, hipStream_t st) {
    std::vector<SortBlock> blocks;
    uint64_t total = 0, maxlen = 0;
    for (uint32_t s = 0; s < nseg; s++) {
        for (uint64_t o = 0; o < seg_len[s]; o += BS_BLOCK) {
            SortBlock b;
            b.off = seg_off[s] + o;
            b.len = (uint32_t)std::min<uint64_t>(BS_BLOCK, seg_len[s] - o);
            blocks.push_back(b);
        }
        total += seg_len[s];
        maxlen = std::max(maxlen, seg_len[s]);
    }
    if (blocks.empty()) return;
    {
        const size_t bytes = blocks.size() * sizeof(SortBlock);
        SortBlock* dev = (SortBlock*)ws->scratch("ms_blocks", bytes);
        uint32_t slot;
        SortBlock* h = (SortBlock*)ws->ring_acquire("ms_blocks_h", bytes, &slot);
        std::copy(blocks.begin(), blocks.end(), h);
        SMJ_CHECK(hipMemcpyAsync(dev, h, bytes, hipMemcpyHostToDevice, st));
        ws->ring_release("ms_blocks_h", slot, st);
        hipLaunchKernelGGL(k_blocksort, dim3((uint32_t)blocks.size()),
                           dim3(BS_THREADS), 0, st, data, dev);
        SMJ_CHECK(hipGetLastError());
    }
    if (maxlen <= (uint64_t)BS_BLOCK) return;
    // merge passes: ping-pong between `data` (at seg_off) and a packed temp
    std::vector<uint64_t> tmp_off(nseg);
    uint64_t acc = 0;
    for (uint32_t s = 0; s < nseg; s++) {
        tmp_off[s] = acc;
        acc += seg_len[s];
    }
    Tup* tmp = (Tup*)ws->scratch("ms_tmp", acc * sizeof(Tup));
    bool in_data = true;
    for (uint64_t w = BS_BLOCK; w < maxlen; w <<= 1) {
        std::vector<MergeTile> tiles;
        for (uint32_t s = 0; s < nseg; s++) {
            if (seg_len[s] <= BS_BLOCK && w > BS_BLOCK) {
                // already fully sorted; it is copied along when it has to move
            }
            const Tup* src = in_data ? data + seg_off[s] : tmp + tmp_off[s];
            Tup* dst = in_data ? tmp + tmp_off[s] : data + seg_off[s];
            const uint64_t L = seg_len[s];
            for (uint64_t o = 0; o < L; o += 2 * w) {
                const uint64_t na = std::min<uint64_t>(w, L - o);
                const uint64_t nb = std::min<uint64_t>(w, L - o - na);
                add_pair_tiles(tiles, src + o, na, src + o + na, nb, dst + o);
            }
        }
        launch_tiles(ws, tiles, st);
        in_data = !in_data;
    }
    if (!in_data) {
        // copy every segment back in one launch (a merge with an empty run)
        std::vector<MergeTile> tiles;
        for (uint32_t s = 0; s < nseg; s++)
            if (seg_len[s]) add_pair_tiles(tiles, tmp + tmp_off[s], seg_len[s],
                                           tmp + tmp_off[s], 0, data + seg_off[s]);
        launch_tiles(ws, tiles, st);
    }
}

// ---------------------------------------------------------------------------
// One-pass k-way merge (avx_multiway_merge, src/merge/avx_multiwaymerge.c:
// 199-338).  The reference streams k runs through an L3-resident FIFO tree;
// here the key range of the runs is cut into 2^D value buckets and, because
// every run is sorted, the part of run i in bucket b is ONE contiguous slice
// whose ends are two binary searches away.  So:
//   k_km_bounds : the key range from the runs' first and last elements, and
//                 off[i][b] = first element of run i in bucket >= b (k x (B+1)
//                 binary searches, no data pass; a streaming pass that wrote
//                 the boundaries where consecutive buckets differ measured
//                 slower: 0.76 against 0.57 ms for 64 runs of 2M; the two
//                 searches of a slice done by the merge's own workgroups,
//                 round 5, took the merge 0.026 -> 0.066 ms: each workgroup
//                 waits for a chain of dependent loads);
//   k_km_merge  : one workgroup per bucket sums its slice starts (= its place
//                 in the output: no size / scan kernels), gathers its k slices with
//                 coalesced loads (all in flight), counting-sorts them in LDS
//                 by the top 12 bits of the key's offset in the bucket (the
//                 exact key when the bucket spans <= 4096 keys), fixes the
//                 equal-digit runs on the full (key, payload) order and writes
//                 the bucket to its place in the output in one stream.
// Traffic: each tuple read once and written once (2w).  A long unsorted
// equal-digit run is sorted in LDS (bitonic, on the full order); a bucket
// larger than LDS (a hot key) is queued for k_km_over, which ranks its
// elements by binary searches across the runs' slices (round 5: no host
// decision, so the merge needs no host synchronisation).
constexpr int KM_THREADS = 256;
constexpr uint32_t KM_CAP = sizeof(Tup) == 8 ? 4096 : 2048;  // bucket capacity (32 KB)
constexpr uint32_t KM_IPT = KM_CAP / KM_THREADS;
constexpr uint32_t KM_KMAX = KM_THREADS;  // runs per one-pass merge
constexpr uint32_t KM_LOGNB = 12;         // digit bits sorted in LDS
constexpr uint32_t KM_NB = 1u << KM_LOGNB;
constexpr uint32_t KM_BPT = KM_NB / KM_THREADS;  // bins per thread
constexpr uint32_t KM_RUNMAX = 64;               // longest equal-digit run fixed serially

struct KmRun {
    const Tup* p;
    uint64_t n;
};

// the runs' key range (their first and last elements), computed by every
// workgroup for itself (k <= 256 cached loads) instead of by a kernel of its own
__device__ __forceinline__ void km_range(const KmRun* __restrict__ runs, uint32_t k,
                                         uint64_t& lo, uint64_t& hi) {
    __shared__ unsigned long long rl[KM_THREADS / 64], rh[KM_THREADS / 64];
    lo = ~0ull;
    hi = 0;
    for (uint32_t i = threadIdx.x; i < k; i += KM_THREADS) {
        const KmRun r = runs[i];
        if (r.n == 0) continue;
        lo = min(lo, key_u(tup_key(ld_g(r.p))));
        hi = max(hi, key_u(tup_key(ld_g(r.p + r.n - 1))));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t a = __shfl_xor(lo, o, 64), c = __shfl_xor(hi, o, 64);
        lo = a < lo ? a : lo;
        hi = c > hi ? c : hi;
    }
    if (lane_id() == 0) {
        rl[threadIdx.x >> 6] = lo;
        rh[threadIdx.x >> 6] = hi;
    }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < KM_THREADS / 64; w++) {
        lo = rl[w] < lo ? rl[w] : lo;
        hi = rh[w] > hi ? rh[w] : hi;
    }
}

// bucket shift: 2^D buckets over the key range [lo, hi]
__device__ __forceinline__ uint32_t km_shift(uint64_t lo, uint64_t hi, uint32_t D) {
    const uint64_t w = hi >= lo ? hi - lo : 0;
    const uint32_t L = w ? 64 - __clzll((long long)w) : 0;
    return L > D ? L - D : 0;
}

// off[i][b] = first element of run i in bucket >= b (binary search); thread
// i * (B + 1) + b, so the lanes of a wave search neighbouring ranges of one
// run and store adjacent entries (run-major table).  Workgroup 0 publishes
// the key range for k_km_merge.
__global__ void __launch_bounds__(KM_THREADS)
k_km_bounds(const KmRun* __restrict__ runs, uint32_t k, uint32_t D,
            unsigned long long* __restrict__ mm, uint32_t* __restrict__ off,
            unsigned int* __restrict__ queue) {
    uint64_t minu, maxu;
    km_range(runs, k, minu, maxu);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        mm[0] = minu;
        mm[1] = maxu;
        queue[0] = 0;  // k_km_merge's overflow queue (it runs after this kernel)
    }
    const uint32_t B = 1u << D;
    const uint64_t idx = (uint64_t)blockIdx.x * KM_THREADS + threadIdx.x;
    if (idx >= (uint64_t)(B + 1) * k) return;
    const uint32_t i = (uint32_t)(idx / (B + 1)), b = (uint32_t)(idx % (B + 1));
    const KmRun r = runs[i];
    uint64_t pos;
    if (b == 0) {
        pos = 0;
    } else if (b == B) {
        pos = r.n;
    } else {
        const uint32_t s = km_shift(minu, maxu, D);
        uint64_t lo = 0, hi = r.n;
        while (lo < hi) {  // first element whose bucket is >= b
            const uint64_t m = (lo + hi) >> 1;
            if (((key_u(tup_key(ld_g(r.p + m))) - minu) >> s) < b) lo = m + 1; else hi = m;
        }
        pos = lo;
    }
    off[idx] = (uint32_t)pos;
}

// sort buf[0, total) in LDS on the full order (bitonic over the next power of
// two, the tail filled with the largest tuple): the rare bucket with a long
// equal-digit run out of order
__device__ __forceinline__ Tup km_max_tup() {
#ifdef KEY_8B
    Tup t;
    t.key = INT64_MAX;
    t.payload = INT64_MAX;
    return t;
#else
    return (Tup)INT64_MAX;
#endif
}
__device__ void km_bitonic(Tup* buf, uint32_t total) {
    uint32_t n = 1;
    while (n < total) n <<= 1;
    for (uint32_t i = total + threadIdx.x; i < n; i += KM_THREADS) buf[i] = km_max_tup();
    __syncthreads();
    for (uint32_t k = 2; k <= n; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < n; i += KM_THREADS) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const Tup a = buf[i], c = buf[l];
                    const bool up = (i & k) == 0;
                    if (up ? tup_less(c, a) : tup_less(a, c)) {
                        buf[i] = c;
                        buf[l] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
}

__global__ void __launch_bounds__(KM_THREADS)
k_km_merge(const KmRun* __restrict__ runs, uint32_t k, uint32_t D,
           const unsigned long long* __restrict__ mm, const uint32_t* __restrict__ off,
           unsigned int* __restrict__ flag, Tup* __restrict__ out) {
    // flag: [0] queued buckets, [2 + q] the q-th (k_km_over)
    __shared__ __attribute__((aligned(16))) Tup buf[KM_CAP];
    __shared__ uint32_t cnt[KM_NB / 2];     // digit histogram, two u16 per word
    __shared__ uint32_t cur[KM_NB / 2];     // placement cursors
    // the non-empty slices in run (= position) order: slice q's element for
    // bucket position j is sptr[q][j]; smap bit j: a slice starts at j; wk[w]:
    // slices starting before position 64 w
    __shared__ const Tup* sptr[KM_KMAX];
    __shared__ unsigned long long smap[KM_CAP / 64];
    __shared__ uint32_t wk[KM_CAP / 64];
    __shared__ uint32_t wt[KM_THREADS / 64];
    __shared__ unsigned long long wo[KM_THREADS / 64];
    const uint32_t b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (uint32_t i = tid; i < KM_NB / 2; i += KM_THREADS) cnt[i] = 0;
    for (uint32_t i = tid; i < KM_CAP / 64; i += KM_THREADS) smap[i] = 0ull;
    // ---- slices: run tid's part of bucket b; one scan gives its position in
    // the bucket (low 21 bits; lengths clamped to KM_CAP + 1, so a sum over
    // 256 runs fits) and its index among the non-empty slices (high bits).
    // The bucket's place in the output is the sum of the slice starts: every
    // element before it lies in a lower bucket of some run.
    uint32_t lo = 0, len = 0;
    if (tid < k) {
        const uint32_t* orow = off + (uint64_t)tid * ((1u << D) + 1);
        lo = orow[b];
        len = orow[b + 1] - lo;
    }
    const uint32_t pk = min(len, KM_CAP + 1) | ((len ? 1u : 0u) << 21);
    uint32_t x = pk;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    const uint64_t lsum = wave_sum((uint64_t)lo);
    if (lane == 63) wt[wid] = x;
    if (lane == 0) wo[wid] = lsum;
    __syncthreads();
    uint32_t ex = x - pk, tot2 = 0;
    uint64_t o = 0;
#pragma unroll
    for (int w = 0; w < KM_THREADS / 64; w++) {
        if (w < (int)wid) ex += wt[w];
        tot2 += wt[w];
        o += wo[w];
    }
    const uint32_t total = tot2 & 0x1fffffu;
    if (total == 0) return;  // uniform: an empty bucket
    if (total > KM_CAP) {    // a bucket larger than LDS: k_km_over merges it
        if (tid == 0) {
            const uint32_t q = atomicAdd(flag, 1u);
            flag[2 + q] = b;  // the queue (room for every bucket)
        }
        return;
    }
    if (len) {
        const uint32_t p0 = ex & 0x1fffffu;
        sptr[ex >> 21] = runs[tid].p + ((int64_t)lo - (int64_t)p0);
        atomicOr(&smap[p0 >> 6], 1ull << (p0 & 63));
    }
    __syncthreads();
    if (tid < KM_CAP / 64) {  // window prefix counts (KM_CAP / 64 <= 64: one wave)
        const uint32_t c = (uint32_t)__popcll(smap[tid]);
        uint32_t y = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t z = __shfl_up(y, o, 64);
            if (lane >= o) y += z;
        }
        wk[tid] = y - c;
    }
    __syncthreads();
    // ---- gather (every load in flight at once: the run of position j by a
    // fixed-step search over the slice starts) and the level digit: the
    // bucket's key offset, its top KM_LOGNB bits (exact keys for buckets no
    // wider than KM_NB keys)
    const uint32_t s = km_shift(mm[0], mm[1], D);
    const uint64_t base = mm[0] + ((uint64_t)b << s);
    const uint32_t s3 = s > KM_LOGNB ? s - KM_LOGNB : 0;
    Tup v[KM_IPT];
    uint32_t dg[KM_IPT];
    auto gather = [&](int q) {
        const uint32_t j = min(q * KM_THREADS + tid, total - 1);
        const uint32_t w = j >> 6;
        const uint32_t sl = wk[w] + (uint32_t)__popcll(smap[w] & (~0ull >> (63 - (j & 63)))) - 1u;
        v[q] = ld_g(sptr[sl] + j);
    };
    // buckets average KM_CAP / 2: the upper half of the loads (and of the
    // counting and placing below) only when the bucket reaches it; rows past
    // the end would otherwise be same-address LDS atomics, serialised
#pragma unroll
    for (int q = 0; q < (int)KM_IPT / 2; q++) gather(q);
    if (total > KM_CAP / 2) {
#pragma unroll
        for (int q = KM_IPT / 2; q < (int)KM_IPT; q++) gather(q);
    }
#pragma unroll
    for (int q = 0; q < (int)KM_IPT; q++) {
        if (q * KM_THREADS >= total) break;  // uniform
        const bool valid = q * KM_THREADS + tid < total;
        dg[q] = (uint32_t)min((key_u(tup_key(v[q])) - base) >> s3, (uint64_t)KM_NB - 1);
        if (valid) atomicAdd(&cnt[dg[q] >> 1], 1u << ((dg[q] & 1) * 16));
    }
    __syncthreads();
    // ---- exclusive scan of the bins: thread tid owns KM_BPT consecutive bins
    uint32_t c[KM_BPT];
    uint32_t loc = 0, mx = 0;
#pragma unroll
    for (int q = 0; q < (int)KM_BPT / 2; q++) {
        const uint32_t wv = cnt[tid * (KM_BPT / 2) + q];
        c[2 * q] = wv & 0xffffu;
        c[2 * q + 1] = wv >> 16;
        loc += c[2 * q] + c[2 * q + 1];
        mx = max(mx, max(c[2 * q], c[2 * q + 1]));
    }
    x = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    __syncthreads();  // wt is reused
    if (lane == 63) wt[wid] = x;
    const bool dup = __syncthreads_or(mx > 1);
    ex = x - loc;
#pragma unroll
    for (int w = 0; w < KM_THREADS / 64; w++)
        if (w < (int)wid) ex += wt[w];
    const uint32_t first = ex;
#pragma unroll
    for (int q = 0; q < (int)KM_BPT / 2; q++) {
        const uint32_t lo16 = ex;
        ex += c[2 * q];
        cur[tid * (KM_BPT / 2) + q] = lo16 | (ex << 16);
        ex += c[2 * q + 1];
    }
    __syncthreads();
    // ---- place
#pragma unroll
    for (int q = 0; q < (int)KM_IPT; q++) {
        if (q * KM_THREADS >= total) break;  // uniform
        if (q * KM_THREADS + tid < total) {
            const uint32_t sh = (dg[q] & 1) * 16;
            const uint32_t old = atomicAdd(&cur[dg[q] >> 1], 1u << sh);
            buf[(old >> sh) & 0xffffu] = v[q];
        }
    }
    __syncthreads();
    if (dup) {
        // equal-digit runs arrive in any order: one parallel inversion check,
        // then short runs are insertion-sorted by their bin's thread; a long
        // unsorted run flags the merge for the merge-path tree
        bool ok = true;
        for (uint32_t i = tid + 1; i < total; i += KM_THREADS) ok &= !tup_less(buf[i], buf[i - 1]);
        if (__syncthreads_or(!ok)) {
            uint32_t e = first;
#pragma unroll
            for (int q = 0; q < (int)KM_BPT; q++) {
                const uint32_t b0 = e;
                e += c[q];
                if (c[q] > 1 && c[q] <= KM_RUNMAX) {
                    for (uint32_t i = b0 + 1; i < b0 + c[q]; i++) {
                        const Tup t = buf[i];
                        uint32_t jj = i;
                        while (jj > b0 && tup_less(t, buf[jj - 1])) {
                            buf[jj] = buf[jj - 1];
                            jj--;
                        }
                        buf[jj] = t;
                    }
                }
            }
            __syncthreads();
            ok = true;
            for (uint32_t i = tid + 1; i < total; i += KM_THREADS)
                ok &= !tup_less(buf[i], buf[i - 1]);
            if (__syncthreads_or(!ok)) km_bitonic(buf, total);  // a long run out of order
        }
    }
    // ---- the bucket, in order, to its place in the output
    for (uint32_t j = tid; j < total; j += KM_THREADS) out[o + j] = buf[j];
}

// Buckets too large for LDS (queued by k_km_merge): every workgroup takes
// its share of every queued bucket's elements (the queue's length is only
// known on the device; a hot key can put most of the input in one bucket).
// Element p of run i's slice goes to its rank among the bucket's elements:
// its position in its slice plus, in every other slice j, the elements below
// it (equal ones too when j < i) -- binary searches, no LDS; ties keep run
// order, so the output is the merged order whatever the tie.
__global__ void __launch_bounds__(KM_THREADS)
k_km_over(const KmRun* __restrict__ runs, uint32_t k, uint32_t D,
          const uint32_t* __restrict__ off, const unsigned int* __restrict__ flag,
          Tup* __restrict__ out) {
    __shared__ uint32_t slo[KM_KMAX], sln[KM_KMAX], sst[KM_KMAX];
    __shared__ uint32_t scr[KM_THREADS / 64 + 1];
    __shared__ unsigned long long wsum[KM_THREADS / 64];
    const uint32_t nq = flag[0];
    const uint32_t tid = threadIdx.x;
    for (uint32_t q = 0; q < nq; q++) {
        const uint32_t b = flag[2 + q];
        uint32_t lo = 0, len = 0;
        if (tid < k) {
            const uint32_t* orow = off + (uint64_t)tid * ((1u << D) + 1);
            lo = orow[b];
            len = orow[b + 1] - lo;
        }
        // the slices' starts in the bucket (block scan) and the bucket's
        // place in the output: the sum of the slice starts
        uint32_t total;
        const uint32_t ex = block_exclusive_scan(len, scr, &total);
        const unsigned long long ls = wave_sum((unsigned long long)lo);
        if ((tid & 63) == 0) wsum[tid >> 6] = ls;
        if (tid < k) {
            slo[tid] = lo;
            sln[tid] = len;
            sst[tid] = ex;
        }
        __syncthreads();
        uint64_t o = 0;
#pragma unroll
        for (int w = 0; w < KM_THREADS / 64; w++) o += wsum[w];
        for (uint32_t e = blockIdx.x * KM_THREADS + tid; e < total; e += gridDim.x * KM_THREADS) {
            // the slice of e: the last start <= e (binary search over k)
            uint32_t a = 0, z = k - 1;
            while (a < z) {
                const uint32_t m = (a + z + 1) >> 1;
                if (sst[m] <= e) a = m; else z = m - 1;
            }
            while (a + 1 < k && sln[a] == 0) a++;  // (an empty slice shares its start)
            const uint32_t i = a, p = e - sst[i];
            const Tup x = ld_g(runs[i].p + slo[i] + p);
            uint64_t rank = p;
            for (uint32_t j = 0; j < k; j++) {
                if (j == i || sln[j] == 0) continue;
                const Tup* sj = runs[j].p + slo[j];
                uint32_t l = 0, h = sln[j];
                while (l < h) {  // j < i: elements <= x; j > i: elements < x
                    const uint32_t m = (l + h) >> 1;
                    const Tup y = ld_g(sj + m);
                    if (j < i ? !tup_less(x, y) : tup_less(y, x)) l = m + 1; else h = m;
                }
                rank += l;
            }
            out[o + rank] = x;
        }
        __syncthreads();
    }
}

// true when the one-pass merge ran (queued buckets included); false: k is
// outside the one-pass range and nothing was written
static bool multiway_merge_buckets(Workspace* ws, const Tup* const* runs, const uint64_t* lens,
                                   uint32_t k, uint64_t total, Tup* out, hipStream_t st) {
    if (k < 3 || k > KM_KMAX) return false;
    for (uint32_t i = 0; i < k; i++)
        if (lens[i] >= (1ull << 32)) return false;
    // buckets of KM_CAP / 2 tuples on average
    uint32_t D = 0;
    while (D < 24 && (total >> D) > KM_CAP / 2) D++;
    const uint32_t B = 1u << D;
    // one pinned block, one copy: the key-range words (written by
    // k_km_bounds), then the runs -- skipped when this workspace uploaded the
    // same table to the same place last time.  No host synchronisation
    // follows, so the staging block comes from a ring (its copy has finished
    // before the block is written again).
    const size_t hdr = 32, bytes = hdr + (size_t)k * sizeof(KmRun);
    unsigned long long* mm = (unsigned long long*)ws->scratch("km_hdr", bytes);
    const KmRun* dr = (const KmRun*)((char*)mm + hdr);
    uint32_t* off = (uint32_t*)ws->scratch("km_off", (size_t)(B + 1) * k * 4);
    // the overflow queue: [0] length (zeroed by k_km_bounds), [2..] bucket
    // numbers (k_km_merge)
    unsigned int* q = (unsigned int*)ws->scratch("km_queue", ((size_t)B + 2) * 4);
    uint32_t slot = 0;
    unsigned long long* h = (unsigned long long*)ws->ring_acquire("km_hdr_h", bytes, &slot);
    h[0] = ~0ull;
    h[1] = 0;
    h[2] = 0;
    h[3] = 0;
    KmRun* hr = (KmRun*)((char*)h + hdr);
    for (uint32_t i = 0; i < k; i++) hr[i] = KmRun{runs[i], lens[i]};
    const size_t rb = (size_t)k * sizeof(KmRun);
    if (ws->km_last_dev != (const void*)mm || ws->km_last.size() != rb ||
        memcmp(ws->km_last.data(), hr, rb) != 0) {
        SMJ_CHECK(hipMemcpyAsync(mm, h, bytes, hipMemcpyHostToDevice, st));
        ws->ring_release("km_hdr_h", slot, st);
        ws->km_last.assign((const unsigned char*)hr, (const unsigned char*)hr + rb);
        ws->km_last_dev = mm;
    }
    const uint64_t nb = (uint64_t)(B + 1) * k;
    {
        traced_launch(ws, "k_km_bounds", k_km_bounds,
                      dim3((uint32_t)((nb + KM_THREADS - 1) / KM_THREADS)), dim3(KM_THREADS), 0,
                      st, dr, k, D, mm, off, q);
    }
    {
        traced_launch(ws, "k_km_merge", k_km_merge, dim3(B), dim3(KM_THREADS), 0, st, dr, k,
                      D, mm, off, q, out);
    }
    // the queued buckets (usually none: every workgroup exits at once)
    hipLaunchKernelGGL(k_km_over, dim3(B < 64 ? B : 64), dim3(KM_THREADS), 0, st, dr, k, D, off,
                       q, out);
    SMJ_CHECK(hipGetLastError());
    return true;
}

// k-way merge: one pass by value buckets (above; buckets too big for LDS
// finished by k_km_over); otherwise (k > 256, one run, two runs) a tree of
// 2-way merge-path passes.
void multiway_merge(Workspace* ws, const Tup* const* runs, const uint64_t* lens,
                    uint32_t k, Tup* out, hipStream_t st) {
    uint64_t total = 0;
    for (uint32_t i = 0; i < k; i++) total += lens[i];
    if (total == 0) return;
    if (multiway_merge_buckets(ws, runs, lens, k, total, out, st)) return;
    multiway_merge_tree(ws, runs, lens, k, out, st);
}

// the merge-path tree alone: ceil(log2 k) passes of pairwise 2-way merges
void multiway_merge_tree(Workspace* ws, const Tup* const* runs, const uint64_t* lens,
                         uint32_t k, Tup* out, hipStream_t st) {
    uint64_t total = 0;
    for (uint32_t i = 0; i < k; i++) total += lens[i];
    if (total == 0) return;
    std::vector<const Tup*> cur(runs, runs + k);
    std::vector<uint64_t> cl(lens, lens + k);
    Tup* bufs[2] = {(Tup*)ws->scratch("mw_a", total * sizeof(Tup)),
                    (Tup*)ws->scratch("mw_b", total * sizeof(Tup))};
    int which = 0;
    while (cur.size() > 1) {
        const bool last = cur.size() <= 2;
        Tup* dstbase = last ? out : bufs[which];
        std::vector<MergeTile> tiles;
        std::vector<const Tup*> nxt;
        std::vector<uint64_t> nl;
        uint64_t o = 0;
        for (size_t i = 0; i < cur.size(); i += 2) {
            const uint64_t na = cl[i];
            const uint64_t nb = i + 1 < cur.size() ? cl[i + 1] : 0;
            const Tup* b = i + 1 < cur.size() ? cur[i + 1] : cur[i];
            add_pair_tiles(tiles, cur[i], na, b, nb, dstbase + o);
            nxt.push_back(dstbase + o);
            nl.push_back(na + nb);
            o += na + nb;
        }
        launch_tiles(ws, tiles, st);
        cur.swap(nxt);
        cl.swap(nl);
        which ^= 1;
    }
    if (k == 1) {
        hipLaunchKernelGGL(k_copy, dim3(1024), dim3(256), 0, st, runs[0], out,
                           lens[0]);
        SMJ_CHECK(hipGetLastError());
    }
}

}  // namespace smj
