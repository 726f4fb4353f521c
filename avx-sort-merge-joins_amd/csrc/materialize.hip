// materialize.hip -- materialised merge-join output.
//
// Reference: src/joins/joincommon.c:239-312 (merge_join built with
// JOIN_MATERIALIZE): for every match the reference appends <S.key, S.payload>
// to a chained tuple buffer, R-major -- for each R tuple of a key run, the
// whole S run of that key (joincommon.c:267-287).  Over sorted inputs the
// output of key k is therefore the S run of k repeated |R_k| times, keys in
// ascending order.  (The chained buffer's header, tuple_buffer.h, is absent
// from the reference tree; the output here is one flat tuple array.)
//
// GPU form, over sorted R and S:
//   k_mat_bounds one thread per S tile: the tile's R window (the R range of
//                its key range) and the S extent of its first and last key
//                runs -- the long binary searches, all in flight at once;
//   k_mat_count  one workgroup per S tile: |R_k| of every S element, searched
//                in the R window staged in LDS (galloping from the previous
//                key), summed per tile; a tile whose elements match at most
//                once (R unique) also leaves its match bitmap;
//   k_mat_part/pscan/down  tile output offsets, and the work items (each
//                tile's output cut into pieces of kMatPiece outputs);
//   k_mat_write  one workgroup per work item: recomputes its tile's counts,
//                scans them in LDS and writes its piece output-major, so the
//                stores are coalesced and a hot key spreads over many
//                workgroups instead of serialising one thread (bitmap tiles:
//                an ordered copy of the set elements, nothing recomputed).
#include "smj_common.hpp"
#include "smj_internal.hpp"

namespace smj {

constexpr int MT_THREADS = 256;
// small tiles keep the LDS per workgroup at 18 KB (8 workgroups per CU), so
// the staging loads of some workgroups overlap the searches of others
// (16 B, 128M x 128M, before the bitmap path: 2048-element tiles 6.6 ms,
// 1024: 4.6 ms, 512: 4.2 ms; with it: 1024: 2.9 ms, 512: 2.4 ms, 256: 3.7 ms
// -- more, smaller tiles lose to the per-tile searches and launch width)
constexpr int MT_IPT = 2;
constexpr uint32_t MT_TILE = MT_THREADS * MT_IPT;  // S elements per tile
constexpr uint32_t MT_RWIN = 2 * MT_TILE;          // R keys staged in LDS
constexpr uint64_t kMatPiece = 8192;                // outputs per work item

// first index of [lo, hi) whose key is >= k (UPPER: > k); K(i) = key i
template <bool UPPER, class K>
__device__ __forceinline__ uint64_t key_search(K key, uint64_t lo, uint64_t hi,
                                               int64_t k) {
    while (lo < hi) {
        const uint64_t m = (lo + hi) >> 1;
        const int64_t x = key(m);
        if (UPPER ? x <= k : x < k) lo = m + 1; else hi = m;
    }
    return lo;
}

// the same answer, galloping forward from lo (consecutive keys of a tile sit
// close together in R)
template <bool UPPER, class K>
__device__ __forceinline__ uint64_t key_gallop(K key, uint64_t lo, uint64_t hi,
                                               int64_t k) {
    uint64_t step = 1;
    while (true) {
        const uint64_t e = lo + step - 1;
        if (e >= hi) return key_search<UPPER>(key, lo, hi, k);
        const int64_t x = key(e);
        if (!(UPPER ? x <= k : x < k)) return key_search<UPPER>(key, lo, e, k);
        lo = e + 1;
        step <<= 1;
    }
}

struct TupKey {
    const Tup* a;
    __device__ __forceinline__ int64_t operator()(uint64_t i) const { return tup_key(a[i]); }
};

// per tile: R window [lo, hi), S start of the first key run, S end of the last
__global__ void __launch_bounds__(256)
k_mat_bounds(const Tup* __restrict__ R, uint64_t nR, const Tup* __restrict__ S,
             uint64_t nS, uint64_t ntiles, uint64_t* __restrict__ bounds) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntiles) return;
    const uint64_t tb = t * MT_TILE;
    const uint64_t te = min(tb + MT_TILE, nS);
    const TupKey rk{R}, sk{S};
    const int64_t kf = sk(tb), kl = sk(te - 1);
    const uint64_t rlo = key_search<false>(rk, 0, nR, kf);
    const uint64_t rhi = key_search<true>(rk, rlo, nR, kl);
    const uint64_t s0 = (tb > 0 && sk(tb - 1) == kf) ? key_search<false>(sk, 0, tb, kf) : tb;
    const uint64_t se = (te < nS && sk(te) == kl) ? key_search<true>(sk, te, nS, kl) : te;
    bounds[4 * t + 0] = rlo;
    bounds[4 * t + 1] = rhi;
    bounds[4 * t + 2] = s0;
    bounds[4 * t + 3] = se;
}

struct MatLDS {
    int64_t key[MT_TILE];
    uint64_t rc[MT_TILE];    // |R_k| of the element; inclusive prefix (write)
    uint16_t s0[MT_TILE];    // tile index of the element's run start (0: ends[2])
    uint16_t se[MT_TILE];    // tile index of its run end (MT_TILE... len: ends[3])
    int64_t rkey[MT_RWIN];   // the R window's keys, when it fits
    uint64_t ends[4];
    uint64_t wsum[MT_THREADS / 64 + 1];
};

template <class K>
__device__ __forceinline__ void mat_runs(K rkey, uint64_t Rlo, uint64_t Rhi,
                                         uint32_t i0, uint32_t i1, uint32_t len,
                                         MatLDS& L) {
    // run start of the thread's first element, run end of its last (LDS)
    uint32_t a = 0, b = i0;
    {
        const int64_t k = L.key[i0];
        while (a < b) {
            const uint32_t m = (a + b) >> 1;
            if (L.key[m] < k) a = m + 1; else b = m;
        }
    }
    uint32_t c = i1, d = len;
    {
        const int64_t k = L.key[i1 - 1];
        while (c < d) {
            const uint32_t m = (c + d) >> 1;
            if (L.key[m] <= k) c = m + 1; else d = m;
        }
    }
    uint32_t s0 = a;
    uint64_t rlo, rhi = Rlo;
    uint32_t i = i0;
    while (i < i1) {
        const int64_t k = L.key[i];
        uint32_t j = i + 1;
        while (j < i1 && L.key[j] == k) j++;
        if (i != i0) s0 = i;
        rlo = key_gallop<false>(rkey, rhi, Rhi, k);
        rhi = key_gallop<true>(rkey, rlo, Rhi, k);
        const uint32_t e = j < i1 ? j : c;
        for (uint32_t u = i; u < j; u++) {
            L.rc[u] = rhi - rlo;
            L.s0[u] = (uint16_t)s0;
            L.se[u] = (uint16_t)e;
        }
        i = j;
    }
}

// key runs and R match counts of S[tb, tb + len)
__device__ void mat_tile(const Tup* __restrict__ R, const Tup* __restrict__ S,
                         const uint64_t* __restrict__ bounds, uint64_t t,
                         uint64_t tb, uint32_t len, MatLDS& L) {
    const uint32_t tid = threadIdx.x;
    if (tid < 4) L.ends[tid] = bounds[4 * t + tid];
    for (uint32_t i = tid; i < len; i += MT_THREADS) L.key[i] = tup_key(S[tb + i]);
    __syncthreads();
    const uint64_t Rlo = L.ends[0], Rhi = L.ends[1];
    const bool staged = Rhi - Rlo <= MT_RWIN;
    if (staged)
        for (uint32_t i = tid; i < Rhi - Rlo; i += MT_THREADS) L.rkey[i] = tup_key(R[Rlo + i]);
    __syncthreads();
    const uint32_t i0 = tid * MT_IPT;
    if (i0 >= len) return;
    const uint32_t i1 = min(i0 + (uint32_t)MT_IPT, len);
    if (staged) {
        const int64_t* rk = L.rkey;
        mat_runs([rk](uint64_t i) { return rk[i]; }, 0, Rhi - Rlo, i0, i1, len, L);
    } else {
        mat_runs(TupKey{R}, Rlo, Rhi, i0, i1, len, L);
    }
}

// block-wide exclusive scan of one uint64 per thread
__device__ __forceinline__ uint64_t block_scan64(uint64_t v, uint64_t* wsum,
                                                 uint64_t* total) {
    const int lane = lane_id(), wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up((unsigned long long)x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t run = 0;
        for (int w = 0; w < nw; w++) {
            const uint64_t t = wsum[w];
            wsum[w] = run;
            run += t;
        }
        wsum[nw] = run;
    }
    __syncthreads();
    const uint64_t res = wsum[wid] + x - v;
    if (total) *total = wsum[nw];
    __syncthreads();
    return res;
}

__global__ void __launch_bounds__(MT_THREADS)
k_mat_count(const Tup* __restrict__ R, const Tup* __restrict__ S, uint64_t nS,
            const uint64_t* __restrict__ bounds, uint64_t* __restrict__ tile_out,
            uint64_t* __restrict__ bitmap, uint32_t* __restrict__ multi_out) {
    __shared__ MatLDS L;
    const uint64_t tb = (uint64_t)blockIdx.x * MT_TILE;
    const uint32_t len = (uint32_t)min((uint64_t)MT_TILE, nS - tb);
    mat_tile(R, S, bounds, blockIdx.x, tb, len, L);
    uint64_t s = 0;
    int multi = 0;
    const uint32_t i0 = threadIdx.x * MT_IPT;
    for (uint32_t u = i0; u < min(i0 + (uint32_t)MT_IPT, len); u++) {
        s += L.rc[u];
        multi |= L.rc[u] > 1;
    }
    multi = __syncthreads_or(multi);
    if (!multi) {
        // every element matches at most once (a key join): its matches as a
        // bitmap, so the write pass copies them without the R window
#pragma unroll
        for (uint32_t p = 0; p < MT_IPT; p++) {
            const uint32_t e = p * MT_THREADS + threadIdx.x;
            const uint64_t bal = __ballot(e < len && L.rc[e] != 0);
            if (lane_id() == 0) bitmap[blockIdx.x * (MT_TILE / 64) + e / 64] = bal;
        }
    }
    if (threadIdx.x == 0) multi_out[blockIdx.x] = (uint32_t)multi;
    s = wave_sum(s);
    if (lane_id() == 0) L.wsum[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int w = 0; w < MT_THREADS / 64; w++) t += L.wsum[w];
        tile_out[blockIdx.x] = t;
    }
}

__device__ __forceinline__ uint64_t mat_items(uint64_t c) {
    return (c + kMatPiece - 1) / kMatPiece;
}

// tile output bases and work-item bases (exclusive) in three launches:
// per 1024 tiles the sums (k_mat_part), one workgroup scanning those
// (k_mat_pscan, totals into tot[0..1]), per 1024 tiles the bases (k_mat_down)
constexpr uint32_t MS_BLOCK = 1024;

__global__ void __launch_bounds__(MS_BLOCK)
k_mat_part(const uint64_t* __restrict__ cnt, uint64_t ntiles, uint64_t* __restrict__ part) {
    __shared__ uint64_t ws[2][MS_BLOCK / 64];
    const uint64_t t = (uint64_t)blockIdx.x * MS_BLOCK + threadIdx.x;
    const uint64_t c = t < ntiles ? cnt[t] : 0;
    const uint64_t so = wave_sum(c), si = wave_sum(mat_items(c));
    if (lane_id() == 0) {
        ws[0][threadIdx.x >> 6] = so;
        ws[1][threadIdx.x >> 6] = si;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        uint64_t a = 0;
        for (uint32_t w = 0; w < MS_BLOCK / 64; w++) a += ws[threadIdx.x][w];
        part[2 * blockIdx.x + threadIdx.x] = a;
    }
}

// exclusive scan of the (outputs, items) pairs of nb blocks, in place
__global__ void __launch_bounds__(MS_BLOCK)
k_mat_pscan(uint64_t* __restrict__ part, uint32_t nb, uint64_t* __restrict__ tot) {
    __shared__ uint64_t ws[MS_BLOCK / 64 + 1];
    uint64_t carry_o = 0, carry_i = 0;
    for (uint32_t r0 = 0; r0 < nb; r0 += MS_BLOCK) {
        const uint32_t b = r0 + threadIdx.x;
        const uint64_t vo = b < nb ? part[2 * b] : 0, vi = b < nb ? part[2 * b + 1] : 0;
        uint64_t to, ti;
        const uint64_t eo = block_scan64(vo, ws, &to), ei = block_scan64(vi, ws, &ti);
        if (b < nb) {
            part[2 * b] = carry_o + eo;
            part[2 * b + 1] = carry_i + ei;
        }
        carry_o += to;
        carry_i += ti;
    }
    if (threadIdx.x == 0) {
        tot[0] = carry_o;
        tot[1] = carry_i;
    }
}

__global__ void __launch_bounds__(MS_BLOCK)
k_mat_down(const uint64_t* __restrict__ cnt, uint64_t ntiles,
           const uint64_t* __restrict__ part, uint64_t* __restrict__ base,
           uint64_t* __restrict__ ibase) {
    __shared__ uint64_t ws[MS_BLOCK / 64 + 1];
    const uint64_t t = (uint64_t)blockIdx.x * MS_BLOCK + threadIdx.x;
    const uint64_t c = t < ntiles ? cnt[t] : 0;
    const uint64_t eo = block_scan64(c, ws, nullptr);
    const uint64_t ei = block_scan64(mat_items(c), ws, nullptr);
    if (t < ntiles) {
        base[t] = part[2 * blockIdx.x] + eo;
        ibase[t] = part[2 * blockIdx.x + 1] + ei;
    }
}

__global__ void __launch_bounds__(MT_THREADS)
k_mat_write(const Tup* __restrict__ R, const Tup* __restrict__ S, uint64_t nS,
            const uint64_t* __restrict__ bounds, const uint64_t* __restrict__ cnt,
            const uint64_t* __restrict__ base, const uint64_t* __restrict__ ibase,
            uint64_t ntiles, const uint64_t* __restrict__ bitmap,
            const uint32_t* __restrict__ multi, Tup* __restrict__ out, uint64_t out_cap) {
    __shared__ MatLDS L;
    __shared__ uint64_t sh_t;
    const uint64_t w = blockIdx.x;
    if (threadIdx.x == 0) {
        // the last tile whose first item is <= w owns item w
        uint64_t lo = 0, hi = ntiles;
        while (lo < hi) {
            const uint64_t m = (lo + hi) >> 1;
            if (ibase[m] <= w) lo = m + 1; else hi = m;
        }
        sh_t = lo - 1;
    }
    __syncthreads();
    const uint64_t t = sh_t;
    const uint64_t q0 = (w - ibase[t]) * kMatPiece;
    const uint64_t q1 = min(q0 + kMatPiece, cnt[t]);
    const uint64_t ob = base[t];
    if (ob + q0 >= out_cap) return;  // uniform over the workgroup
    const uint64_t tb = t * MT_TILE;
    const uint32_t len = (uint32_t)min((uint64_t)MT_TILE, nS - tb);
    if (!multi[t]) {
        // key join tile (one piece): copy the matching elements in order
        constexpr uint32_t NW = MT_TILE / 64;
        uint64_t bw[NW];
#pragma unroll
        for (uint32_t k = 0; k < NW; k++) bw[k] = bitmap[t * NW + k];
#pragma unroll
        for (uint32_t p = 0; p < MT_IPT; p++) {
            const uint32_t e = p * MT_THREADS + threadIdx.x;
            uint32_t rank = 0;
            bool hit = false;
#pragma unroll
            for (uint32_t k = 0; k < NW; k++) {
                if (k < e / 64) rank += __popcll(bw[k]);
                if (k == e / 64) {
                    rank += __popcll(bw[k] & ((1ull << (e & 63)) - 1));
                    hit = (bw[k] >> (e & 63)) & 1;
                }
            }
            if (hit && e < len && ob + rank < out_cap) st_stream(out + ob + rank, S[tb + e]);
        }
        return;
    }
    mat_tile(R, S, bounds, t, tb, len, L);
    // inclusive prefix of the counts over the tile
    const uint32_t i0 = threadIdx.x * MT_IPT;
    const uint32_t i1 = min(i0 + (uint32_t)MT_IPT, len);
    uint64_t s = 0;
    for (uint32_t u = i0; u < i1; u++) s += L.rc[u];
    uint64_t run = block_scan64(s, L.wsum, nullptr);
    for (uint32_t u = i0; u < i1; u++) {
        run += L.rc[u];
        L.rc[u] = run;
    }
    __syncthreads();
    const int64_t first_s0 = (int64_t)L.ends[2], last_se = (int64_t)L.ends[3];
    for (uint64_t q = q0 + threadIdx.x; q < q1; q += MT_THREADS) {
        if (ob + q >= out_cap) break;
        // element j: the first inclusive prefix above q
        uint32_t lo = 0, hi = len - 1;
        while (lo < hi) {
            const uint32_t m = (lo + hi) >> 1;
            if (L.rc[m] <= q) lo = m + 1; else hi = m;
        }
        const uint32_t j = lo;
        const uint64_t excl = j ? L.rc[j - 1] : 0;
        const uint64_t rcj = L.rc[j] - excl;
        const uint32_t a = L.s0[j], c = L.se[j];
        const int64_t s0 = a == 0 ? first_s0 : (int64_t)(tb + a);
        const int64_t se = c == len ? last_se : (int64_t)(tb + c);
        const uint64_t sc = (uint64_t)(se - s0);
        // the run's output starts (tb + j - s0) * rcj outputs before element
        // j's first (mod 2^64 when the run began in an earlier tile)
        const uint64_t off = q - (excl - (uint64_t)((int64_t)(tb + j) - s0) * rcj);
        const uint64_t src = (uint64_t)s0 + (sc == 1 ? 0 : off % sc);
        st_stream(out + ob + q, S[src]);
    }
}

uint64_t materialize(Workspace* ws, const Tup* R, uint64_t nR, const Tup* S,
                     uint64_t nS, Tup* out, uint64_t out_cap, hipStream_t st) {
    if (nR == 0 || nS == 0) return 0;
    const uint64_t ntiles = (nS + MT_TILE - 1) / MT_TILE;
    uint64_t* tab = (uint64_t*)ws->scratch("mat_tab", (7 * ntiles + 2) * 8);
    uint64_t* bitmap = (uint64_t*)ws->scratch("mat_bits", ntiles * (MT_TILE / 8));
    uint32_t* multi = (uint32_t*)ws->scratch("mat_multi", ntiles * 4);
    uint64_t* cnt = tab;
    uint64_t* base = tab + ntiles;
    uint64_t* ibase = tab + 2 * ntiles;
    uint64_t* bounds = tab + 3 * ntiles;  // 4 per tile
    uint64_t* tot = tab + 7 * ntiles;
    {
        TraceScope ts(ws, "k_mat_bounds", st);
        hipLaunchKernelGGL(k_mat_bounds, dim3((uint32_t)((ntiles + 255) / 256)), dim3(256),
                           0, st, R, nR, S, nS, ntiles, bounds);
        SMJ_CHECK(hipGetLastError());
    }
    {
        TraceScope ts(ws, "k_mat_count", st);
        hipLaunchKernelGGL(k_mat_count, dim3((uint32_t)ntiles), dim3(MT_THREADS), 0,
                           st, R, S, nS, bounds, cnt, bitmap, multi);
        SMJ_CHECK(hipGetLastError());
    }
    {
        TraceScope ts(ws, "k_mat_scan", st);
        const uint32_t nb = (uint32_t)((ntiles + MS_BLOCK - 1) / MS_BLOCK);
        uint64_t* part = (uint64_t*)ws->scratch("mat_part", (size_t)nb * 16);
        hipLaunchKernelGGL(k_mat_part, dim3(nb), dim3(MS_BLOCK), 0, st, cnt, ntiles, part);
        SMJ_CHECK(hipGetLastError());
        hipLaunchKernelGGL(k_mat_pscan, dim3(1), dim3(MS_BLOCK), 0, st, part, nb, tot);
        SMJ_CHECK(hipGetLastError());
        hipLaunchKernelGGL(k_mat_down, dim3(nb), dim3(MS_BLOCK), 0, st, cnt, ntiles, part,
                           base, ibase);
        SMJ_CHECK(hipGetLastError());
    }
    uint64_t* h = (uint64_t*)ws->host_pinned("mat_tot_h", 16);
    SMJ_CHECK(hipMemcpyAsync(h, tot, 16, hipMemcpyDeviceToHost, st));
    SMJ_CHECK(hipStreamSynchronize(st));
    const uint64_t total = h[0], items = h[1];
    // work items run in output order and every tile's items but its last
    // hold kMatPiece outputs: the items below out_cap number at most one per
    // tile plus out_cap / kMatPiece (a small buffer for a huge skewed join
    // launches no more than that)
    const uint64_t need = ntiles + out_cap / kMatPiece + 1;
    const uint64_t launch = items < need ? items : need;
    if (launch && out_cap) {
        TraceScope ts(ws, "k_mat_write", st);
        hipLaunchKernelGGL(k_mat_write, dim3((uint32_t)launch), dim3(MT_THREADS), 0,
                           st, R, S, nS, bounds, cnt, base, ibase, ntiles, bitmap, multi,
                           out, out_cap);
        SMJ_CHECK(hipGetLastError());
    }
    return total;
}

}  // namespace smj
