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
// sorts run a bitonic sorting network over an LDS tile.
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
            d, T.na, T.nb, [&](uint64_t i) { return T.a[i]; },
            [&](uint64_t i) { return T.b[i]; });
    }
    __syncthreads();
    const uint64_t a0 = sh_ab[0], a1 = sh_ab[1];
    const uint64_t b0 = T.d0 - a0, b1 = T.d1 - a1;
    const uint32_t la = (uint32_t)(a1 - a0), lb = (uint32_t)(b1 - b0);
    for (uint32_t i = threadIdx.x; i < la; i += MG_THREADS) sm[i] = T.a[a0 + i];
    for (uint32_t i = threadIdx.x; i < lb; i += MG_THREADS) sm[la + i] = T.b[b0 + i];
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
#pragma unroll
        for (int k = 0; k < MG_IPT; k++) {
            if (p + k < len) {
                bool takeA;
                if (i >= la) takeA = false;
                else if (j >= lb) takeA = true;
                else takeA = !tup_less(Bs[j], As[i]);
                res[k] = takeA ? As[i] : Bs[j];
                if (takeA) i++; else j++;
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < MG_IPT; k++)
        if (p + k < len) sm[p + k] = res[k];
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < len; i += MG_THREADS) T.out[T.d0 + i] = sm[i];
}

// ---------------------------------------------------------------------------
struct SortBlock {
    uint64_t off;
    uint32_t len;
};

__global__ void __launch_bounds__(BS_THREADS)
k_blocksort(Tup* __restrict__ data, const SortBlock* __restrict__ blocks) {
    __shared__ __attribute__((aligned(16))) Tup sm[BS_BLOCK];
    const SortBlock blk = blocks[blockIdx.x];
    uint32_t P2 = 2;
    while (P2 < blk.len) P2 <<= 1;
    const Tup sent = tup_max_sentinel();
    for (uint32_t i = threadIdx.x; i < P2; i += BS_THREADS)
        sm[i] = i < blk.len ? data[blk.off + i] : sent;
    __syncthreads();
    // bitonic sorting network over P2 items (ascending)
    for (uint32_t k = 2; k <= P2; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t t = threadIdx.x; t < P2 / 2; t += BS_THREADS) {
                const uint32_t i = 2 * t - (t & (j - 1));  // lower index
                const uint32_t l = i + j;
                const bool up = (i & k) == 0;
                Tup x = sm[i], y = sm[l];
                if (tup_less(y, x) == up) {
                    sm[i] = y;
                    sm[l] = x;
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t i = threadIdx.x; i < blk.len; i += BS_THREADS)
        data[blk.off + i] = sm[i];
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
        const int64_t k = tup_key(P.s[i]);
        if (i > 0 && tup_key(P.s[i - 1]) == k) continue;
        uint64_t lo = i + 1, hi = P.ns;
        while (lo < hi) {
            const uint64_t m = (lo + hi) >> 1;
            if (tup_key(P.s[m]) <= k) lo = m + 1; else hi = m;
        }
        const uint64_t sc = lo - i;
        lo = 0;
        hi = P.nr;
        while (lo < hi) {
            const uint64_t m = (lo + hi) >> 1;
            if (tup_key(P.r[m]) < k) lo = m + 1; else hi = m;
        }
        const uint64_t rl = lo;
        hi = P.nr;
        while (lo < hi) {
            const uint64_t m = (lo + hi) >> 1;
            if (tup_key(P.r[m]) <= k) lo = m + 1; else hi = m;
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
    MergeTile* h = (MergeTile*)ws->host_pinned("mg_tiles_h", bytes);
    SMJ_CHECK(hipStreamSynchronize(st));  // pinned staging buffer is reused
    std::copy(tiles.begin(), tiles.end(), h);
    SMJ_CHECK(hipMemcpyAsync(dev, h, bytes, hipMemcpyHostToDevice, st));
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

void merge2(const Tup* a, uint64_t na, const Tup* b, uint64_t nb, Tup* out,
            hipStream_t st) {
    static Workspace ws2;
    std::vector<MergeTile> v;
    add_pair_tiles(v, a, na, b, nb, out);
    launch_tiles(&ws2, v, st);
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
    JoinPair* h = (JoinPair*)ws->host_pinned("mj_pairs_h", bytes);
    SMJ_CHECK(hipStreamSynchronize(st));  // the pinned table is reused
    for (uint32_t i = 0; i < k; i++) h[i] = JoinPair{r[i], s[i], nr[i], ns[i]};
    SMJ_CHECK(hipMemcpyAsync(dev, h, bytes, hipMemcpyHostToDevice, st));
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
        SortBlock* h = (SortBlock*)ws->host_pinned("ms_blocks_h", bytes);
        SMJ_CHECK(hipStreamSynchronize(st));
        std::copy(blocks.begin(), blocks.end(), h);
        SMJ_CHECK(hipMemcpyAsync(dev, h, bytes, hipMemcpyHostToDevice, st));
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

// k-way merge as a tree of 2-way merge-path passes.
void multiway_merge(Workspace* ws, const Tup* const* runs, const uint64_t* lens,
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
