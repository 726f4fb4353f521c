// exchange.hip -- the table side of the multi-GPU join's exchange step
// (smj/dist.py; the reference's analogue is the
// redistribution of co-partitions between threads before the multiway merge,
// src/joins/sortmergejoin_multiway.c:463-556).
//
// After a rank range-partitions a relation into F partitions (K shard regions
// each, exact partitions use shard 0 only), partition p belongs to rank
// owner(p) = p * G / U, the last rank also owning [U, F) (contiguous ranges,
// dist.py owners()).  U = the partitions the plan's key range reaches: F is a
// power of two, the key span is not (keys 1..1024M at F = 2^10 reach 977
// partitions), so splitting F would leave the last rank short.  Two one-
// workgroup kernels turn the region tables into
//   xsend: the message to every rank g -- [chunk size, used elements, the
//          sender's two flags, the owned regions' offsets inside the chunk,
//          their counts] -- rank after rank, plus the chunk starts/sizes;
//   xrecv: from the G messages received (an all-to-all), the local join's
//          segment tables (bucket-major, G * K segments per bucket) with the
//          rank's own chunk read in place inside its partition buffer and the
//          other ranks' rows after it, and a small summary the host reads in
//          one copy (chunk starts and sizes, receive sizes, used elements,
//          the flags OR-ed over the ranks).
// They replace two dozen small framework ops (and their host round trips) per
// relation and step.
#include "smj_common.hpp"
#include "smj_internal.hpp"

namespace smj {

// the first partition of rank g (g = G: F); U = the partitions holding keys
__device__ __forceinline__ uint32_t owned_lo(uint32_t F, uint32_t G, uint32_t U, uint32_t g) {
    return g >= G ? F : (uint32_t)(((uint64_t)g * U + G - 1) / G);
}
__device__ __forceinline__ uint32_t owner_of(uint32_t G, uint32_t U, uint32_t p) {
    return p < U ? (uint32_t)((uint64_t)p * G / U) : G - 1;
}

constexpr uint32_t kXHead = 4;  // chunk size, used, flag0 (not packable), flag1 (overflow)

__global__ void __launch_bounds__(256)
k_xsend(const int64_t* __restrict__ start, const int64_t* __restrict__ cnt,
        const unsigned int* __restrict__ flags, uint32_t F, uint32_t K, uint32_t G, uint32_t U,
        int64_t* __restrict__ msg, int64_t* __restrict__ chunk) {
    __shared__ unsigned long long wend[4];
    __shared__ int64_t used[1024];
    for (uint32_t g = threadIdx.x; g < G; g += 256) used[g] = 0;
    __syncthreads();
    // end of the last region (thread maxima, then waves) and every
    // destination's used elements: a thread's partitions are consecutive, so
    // it adds one run per owner it meets
    const uint32_t per = (F + 255) / 256;
    const uint32_t p0 = threadIdx.x * per, p1 = min(p0 + per, F);
    unsigned long long e = 0;
    int64_t acc = 0;
    uint32_t cur = 0xffffffffu;
    for (uint32_t p = p0; p < p1; p++) {
        const uint32_t g = owner_of(G, U, p);
        if (g != cur) {
            if (acc) atomicAdd((unsigned long long*)&used[cur], (unsigned long long)acc);
            cur = g;
            acc = 0;
        }
        for (uint32_t q = 0; q < K; q++) {
            const size_t i = (size_t)p * K + q;
            e = max(e, (unsigned long long)(start[i] + cnt[i]));
            acc += cnt[i];
        }
    }
    if (acc) atomicAdd((unsigned long long*)&used[cur], (unsigned long long)acc);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long x = __shfl_xor(e, o, 64);
        e = x > e ? x : e;
    }
    if ((threadIdx.x & 63) == 0) wend[threadIdx.x >> 6] = e;
    __syncthreads();
    const int64_t cend = (int64_t)max(max(wend[0], wend[1]), max(wend[2], wend[3]));
    // chunk of g: from its first partition's first region to the next rank's
    for (uint32_t g = threadIdx.x; g < G; g += 256) {
        const int64_t cs = start[(size_t)owned_lo(F, G, U, g) * K];
        const int64_t ce = g + 1 < G ? start[(size_t)owned_lo(F, G, U, g + 1) * K] : cend;
        chunk[g] = cs;
        chunk[G + g] = ce - cs;
    }
    // messages: rank g's at sum over earlier ranks of (head + 2 K owned); the
    // region entries of all ranks in one sweep, the heads by one thread each
    for (uint32_t i = threadIdx.x; i < F * K; i += 256) {
        const uint32_t p = i / K;
        const uint32_t g = owner_of(G, U, p);
        const uint32_t lo = owned_lo(F, G, U, g), hi = owned_lo(F, G, U, g + 1);
        const uint64_t m0 = (uint64_t)g * kXHead + 2ull * K * lo;
        const uint32_t nreg = (hi - lo) * K, j = i - lo * K;
        const int64_t cs = start[(size_t)lo * K];
        msg[m0 + kXHead + j] = cnt[i] > 0 ? start[i] - cs : 0;
        msg[m0 + kXHead + nreg + j] = cnt[i];
    }
    for (uint32_t g = threadIdx.x; g < G; g += 256) {
        const uint32_t lo = owned_lo(F, G, U, g), hi = owned_lo(F, G, U, g + 1);
        const uint64_t m0 = (uint64_t)g * kXHead + 2ull * K * lo;
        const int64_t cs = start[(size_t)lo * K];
        const int64_t ce = g + 1 < G ? start[(size_t)hi * K] : cend;
        msg[m0 + 0] = ce - cs;
        msg[m0 + 1] = used[g];
        msg[m0 + 2] = flags[1];  // not packable
        msg[m0 + 3] = flags[0];  // region overflow
    }
}

// msg: G rows of (head + 2 * mine * K), row s from rank s.  tstart/tcnt:
// (2^lbits) x (G * K), bucket b = owned partition b, segment (s, q).
// summary: [chunk start (G) | chunk size = send (G) | receive (G) | used
// received (G) | flag0 | flag1, each OR-ed over the ranks]
__global__ void __launch_bounds__(256)
k_xrecv(const int64_t* __restrict__ msg, const int64_t* __restrict__ chunk, uint32_t G,
        uint32_t rank, uint32_t mine, uint32_t K, uint32_t nb, uint64_t cap,
        int64_t* __restrict__ tstart, int64_t* __restrict__ tcnt, int64_t* __restrict__ summary) {
    const uint32_t row = kXHead + 2 * mine * K;
    __shared__ int64_t base[1024];
    if (threadIdx.x == 0) {
        // the own chunk stays in place in the partition buffer; the others
        // follow the partition buffer (its first `cap` elements), rank order
        int64_t ro = (int64_t)cap, f0 = 0, f1 = 0;
        for (uint32_t s = 0; s < G; s++) {
            const int64_t rl = msg[(size_t)s * row];
            base[s] = s == rank ? chunk[rank] : ro;
            if (s != rank) ro += rl;
            summary[2 * G + s] = rl;
            summary[3 * G + s] = msg[(size_t)s * row + 1];
            f0 |= msg[(size_t)s * row + 2];  // bit masks: every rank's reasons
            f1 |= msg[(size_t)s * row + 3];
        }
        summary[4 * G] = f0;
        summary[4 * G + 1] = f1;
    }
    for (uint32_t g = threadIdx.x; g < G; g += 256) {
        summary[g] = chunk[g];
        summary[G + g] = chunk[G + g];
    }
    __syncthreads();
    const uint32_t GK = G * K;
    for (uint32_t i = threadIdx.x; i < nb * GK; i += 256) {
        const uint32_t b = i / GK, j = i % GK, s = j / K, q = j % K;
        int64_t st = 0, ct = 0;
        if (b < mine) {
            const size_t m = (size_t)s * row + kXHead + (size_t)b * K + q;
            ct = msg[m + (size_t)mine * K];
            st = msg[m] + base[s];
        }
        tstart[i] = st;
        tcnt[i] = ct;
    }
}

// The tables of an exact range partition (partitions back to back, hist[p]
// elements each) in the sampled partition's shape: shard 0 of partition p
// starts at the exclusive prefix sum of hist, the other K - 1 shards are
// empty.  One workgroup of 1024 threads, F <= 1024.
__global__ void __launch_bounds__(1024)
k_hist_tables(const int64_t* __restrict__ hist, uint32_t F, uint32_t K,
              int64_t* __restrict__ start, int64_t* __restrict__ cnt) {
    __shared__ int64_t sc[2][1024];
    const uint32_t p = threadIdx.x;
    const int64_t h = p < F ? hist[p] : 0;
    int cur = 0;
    sc[0][p] = h;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan
        sc[cur ^ 1][p] = sc[cur][p] + (p >= o ? sc[cur][p - o] : 0);
        cur ^= 1;
        __syncthreads();
    }
    if (p < F) {
        for (uint32_t q = 0; q < K; q++) {
            start[(size_t)p * K + q] = q == 0 ? sc[cur][p] - h : 0;
            cnt[(size_t)p * K + q] = q == 0 ? h : 0;
        }
    }
}

void hist_tables(const int64_t* hist, uint32_t F, uint32_t K, int64_t* start, int64_t* cnt,
                 hipStream_t st) {
    hipLaunchKernelGGL(k_hist_tables, dim3(1), dim3(1024), 0, st, hist, F, K, start, cnt);
    SMJ_CHECK(hipGetLastError());
}

void xsend(const int64_t* start, const int64_t* cnt, const unsigned int* flags, uint32_t F,
           uint32_t K, uint32_t G, uint32_t U, int64_t* msg, int64_t* chunk, hipStream_t st) {
    hipLaunchKernelGGL(k_xsend, dim3(1), dim3(256), 0, st, start, cnt, flags, F, K, G, U, msg,
                       chunk);
    SMJ_CHECK(hipGetLastError());
}

void xrecv(const int64_t* msg, const int64_t* chunk, uint32_t G, uint32_t rank, uint32_t mine,
           uint32_t K, uint32_t nb, uint64_t cap, int64_t* tstart, int64_t* tcnt,
           int64_t* summary, hipStream_t st) {
    hipLaunchKernelGGL(k_xrecv, dim3(1), dim3(256), 0, st, msg, chunk, G, rank, mine, K, nb,
                       cap, tstart, tcnt, summary);
    SMJ_CHECK(hipGetLastError());
}

}  // namespace smj
