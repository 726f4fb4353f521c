// mgpu_orch.hpp -- the multi-GPU m-way join behind sortmergejoin_mpsm: one
// rank (a host thread and its streams) per GPU inside one process.
//
// The reference scales the m-way join over the T threads of one host
// (src/joins/sortmergejoin_multiway.c:129-328, threads spawned by
// src/joins/joincommon.c:118-165, each on a contiguous chunk of R and S,
// :127-139).  Each thread radix-partitions its chunks, the threads then
// exchange co-partitions so that thread t owns whole partitions
// (multiwaymerge_phase, :463-556: thread t gathers its partitions' runs from
// every thread, in the NUMA order of src/util/numa_shuffle.c:83, NEXT =
// (t + i) % T), merges and joins them, and the counts are summed.  Here a rank
// plays a thread and its GPU plays the thread's NUMA region:
//   1. range-partition the rank's slices of R and S on its GPU into
//      F = 2^pbits partitions of the GLOBAL key range; of the U partitions the
//      key range reaches, partition p belongs to rank owner(p) = p * G / U
//      (the ones above U to the last rank), so every rank owns one contiguous
//      key range of about 1/G of the keys;
//   2. a table message (the owned regions' offsets and counts, two flags) to
//      every rank over the collective, the receive tables built on the device,
//      one small summary read by the host (every flag is OR-ed over all
//      ranks, so every rank takes the same decisions);
//   3. the rows: grouped send/recv of each chunk to its owner, peers in NEXT
//      order, pieces of at most 512 MB;
//   4. the received partitions ARE the level-1 buckets of the local sort: the
//      local join starts at its tile pass (R's tile stage while S's rows are
//      still in flight) and the count is all-reduced.
// This is the protocol of smj/dist.py (one process per GPU over
// torch.distributed) in C++, reachable from the reference's C API.
//
// The template does not include HIP.  `Ops` is the device work of one rank
// and `Coll` its collectives: mgpu.hip instantiates them with the library's
// kernels and RCCL (or device copies when ranks share a GPU), and
// tests/orch_host/ with host stand-ins, so the CPU tests run this exact code
// at G = 2, 3 and 8.
//
// Ops (one rank; every call below is stream-ordered on kMain unless a stream
// is named; pointers are the rank's "device" memory):
//   static constexpr int kTupleBytes;          8 or 16
//   bool can_pack() const;                      64-bit packed words (16 B only)
//   void* alloc(size_t); void release(void*);   (release after the streams drained)
//   void* host_alloc(size_t); void host_release(void*);
//   void copy(void* dst, const void* src, size_t bytes, int stream);
//   void to_host(void* h, const void* d, size_t bytes, int stream);
//   void to_dev(void* d, const void* h, size_t bytes, int stream);
//   void fill_u32(void* p, uint32_t v, size_t count, int stream);
//   void record(int ev, int stream); void wait(int stream, int ev);
//   void host_wait(int ev); void sync(int stream);
//   void tmark(int mark, int stream);           a timing mark (TMark)
//   double tspan(int a, int b);                 ms between two completed marks
//   uint32_t shards(); uint64_t sampled_capacity(uint64_t n, uint32_t nbits);
//   int  part_planes(in, n, out, stride, nbits, kmin, kmax, ss, sc, flags);
//   int  part_sampled(in, n, out, nbits, kmin, kmax, packed, ss, sc, flags);
//   int  part_shards(in, n, out, nbits, kmin, kmax, packed, ss, sc, flags);
//                                               exact shard regions, no slack
//   void part_exact(in, n, out, nbits, kmin, kmax, hist);
//   int  part_exact_packed(in, n, out, nbits, kmin, kmax, hist, bad);
//   void hist_tables(hist, F, K, ss, sc);       exact partition -> shard-0 tables
//   void xsend(...), xrecv(...);                smj_dev_xsend / smj_dev_xrecv
//   void join(lay, R, strideR, nR, tsR, tcR, S, strideS, nS, tsS, tcS, nseg,
//             lbits, key_lo, key_hi, stage, sortedR, sortedS, count);
//   bool key_range(R, nR, S, nS, int64_t* lo, int64_t* hi);   host result
// Coll (one rank of G; every rank issues the same calls in the same order):
//   void exchange(int stream, const std::vector<Piece>& sends,
//                 const std::vector<Piece>& recvs);
//   void allreduce_sum_u64(int stream, unsigned long long* dev);
//   int64_t reduce(int64_t v, int op);   host value over the ranks (0 sum,
//                                        1 min, 2 max), every rank gets it
#pragma once
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace smj {
namespace mg {

// ---------------------------------------------------------------------------
// plan arithmetic (the same functions as smj/dist.py, which documents them)
// ---------------------------------------------------------------------------
constexpr uint32_t kMaxPartBits = 10;   // widest exchange partition (2^10)
constexpr uint32_t kPlaneMaxBits = 10;  // the 48-bit scatter's LDS carries (16-byte segments)
constexpr uint64_t kLocalBucketCap = 192ull * 16384;  // tiles of the tile pass
constexpr uint32_t kHead = 4;           // message head (exchange.hip kXHead)
constexpr uint32_t kBadPayload = 1, kBadRange = 2, kBadPayload48 = 4;
constexpr uint64_t kPieceBytes = 512ull << 20;  // RCCL message limit

// exchange layouts, narrowest last (dist.py LAYOUTS)
enum Layout : int { kTuples = 0, kWords = 1, kPlanes = 2 };
inline const char* layout_name(int l) {
    return l == kPlanes ? "planes" : l == kWords ? "words" : "tuples";
}
enum Stream : int { kMain = 0, kRows = 1 };
// events of one rank (Ops::record / wait)
enum Event : int { kEvAttemptR = 0, kEvAttemptS = 1, kEvRowsR = 2, kEvRowsS = 3, kEvMain = 4,
                   kNumEvents = 5 };
// timing marks of one rank (Ops::tmark / tspan), the phases of Stats: the
// start and end of the call on kMain; per relation r the start of its range
// partition, its end, the end of its table messages (kTPart0 + 3 r + 0/1/2);
// per relation its row exchange on kRows (kTRows0 + 2 r + 0/1); the local
// join (one call: J0-J1; staged: J0-J1 and J2-J3)
enum TMark : int { kTStart = 0, kTPart0 = 1, kTRows0 = 7, kTJoin0 = 11, kTJoin1 = 12,
                   kTJoin2 = 13, kTJoin3 = 14, kTEnd = 15, kNumTMarks = 16 };

typedef __int128 i128;

inline uint32_t bitlen(uint64_t x) {
    uint32_t L = 0;
    while (L < 64 && (x >> L) != 0) L++;
    return L;
}
inline uint32_t ceil_log2(uint64_t x) { return x <= 1 ? 0 : bitlen(x - 1); }
inline uint64_t span_of(int64_t kmin, int64_t kmax) {
    return kmax > kmin ? (uint64_t)kmax - (uint64_t)kmin : 0;
}
// [owned_lo(g), owned_lo(g + 1)) = the partitions of rank g (dist.py owned):
// the U partitions the key range reaches split evenly, the rest of the F to
// the last rank (exchange.hip owner_of)
inline uint32_t owned_lo(uint32_t F, uint32_t G, uint32_t U, uint32_t g) {
    return g >= G ? F : (uint32_t)(((uint64_t)g * U + G - 1) / G);
}
// s1 of the range plan: partition p covers [kmin + p 2^s1, kmin + (p+1) 2^s1)
inline uint32_t plan_shift(int64_t kmin, int64_t kmax, uint32_t bits) {
    const uint32_t L = bitlen(span_of(kmin, kmax));
    return L > bits ? L - bits : 0;
}
// the plan's base: kmin, moved down when base + 2^L - 1 would pass INT64_MAX
inline int64_t plan_base(int64_t kmin, int64_t kmax) {
    const uint32_t L = bitlen(span_of(kmin, kmax));
    const i128 one = 1, i64max = (i128)INT64_MAX;
    i128 base = kmin;
    if (base + (one << L) - 1 > i64max) base = i64max - (one << L) + 1;
    return (int64_t)base;
}
// the partitions [0, U) the key range reaches (dist.py used_parts)
inline uint32_t used_parts(int64_t kmin, int64_t kmax, uint32_t pbits) {
    const int64_t base = plan_base(kmin, kmax);
    const uint32_t s1 = plan_shift(base, kmax, pbits);
    const uint64_t u = (span_of(base, kmax) >> s1) + 1;
    return (uint32_t)std::min<uint64_t>(u, 1ull << pbits);
}
// 48-bit words worth trying: s1 key bits plus payloads up to the key span
inline bool planes_hold(int64_t kmin, int64_t kmax, uint32_t pbits) {
    const uint32_t s1 = plan_shift(kmin, kmax, pbits);
    return s1 >= 1 && s1 <= 32 && span_of(kmin, kmax) < (1ull << (48 - s1));
}
// exchange partition width (dist.py partition_bits); n_hint = elements per
// rank and relation (0: unknown)
inline uint32_t partition_bits(uint32_t bucket_bits, uint32_t G, bool planes, uint64_t n_hint,
                               bool have_range, int64_t kmin, int64_t kmax) {
    uint32_t pbits = std::min(bucket_bits + ceil_log2(G), kMaxPartBits);
    if (planes && pbits > kPlaneMaxBits && n_hint) {
        const int lbits = (int)kPlaneMaxBits - (int)ceil_log2(G);
        const bool fits = !have_range || planes_hold(kmin, kmax, kPlaneMaxBits);
        if (fits && lbits >= 6 && (n_hint + (1ull << lbits) - 1) >> lbits <= kLocalBucketCap)
            pbits = kPlaneMaxBits;
    }
    return pbits;
}

struct LocalRange {
    int64_t base;    // the global plan's key_min (moved down near INT64_MAX)
    int64_t key_lo;  // the rank's local plan
    int64_t key_hi;
    uint32_t lbits;  // local buckets = 2^lbits >= the rank's partitions
};
// dist.py local_range: the rank's partitions [p_lo, p_hi) are the level-1
// buckets of its local plan, whose width keeps the global partition width
inline LocalRange local_range(int64_t kmin, int64_t kmax, uint32_t pbits, uint32_t G,
                              uint32_t rank) {
    const uint32_t L = bitlen(span_of(kmin, kmax));
    const i128 one = 1;
    const i128 base = plan_base(kmin, kmax);
    const uint32_t F = 1u << pbits, U = used_parts(kmin, kmax, pbits);
    const uint32_t p_lo = owned_lo(F, G, U, rank), p_hi = owned_lo(F, G, U, rank + 1);
    LocalRange r;
    r.lbits = ceil_log2(std::max<uint32_t>(p_hi - p_lo, 1));
    const uint32_t s1 = plan_shift((int64_t)base, kmax, pbits);
    i128 klo = base + ((i128)p_lo << s1);
    i128 khi = r.lbits ? klo + (one << (s1 + r.lbits - 1)) : klo + (one << s1) - 1;
    const i128 top = base + (one << L) - 1;
    klo = std::min(klo, top);
    khi = std::min(khi, top);
    r.base = (int64_t)base;
    r.key_lo = (int64_t)klo;
    r.key_hi = (int64_t)khi;
    return r;
}

// the layout and form an invalid attempt repeats with, on every rank alike
// (bad / ovf are OR-ed over the ranks; dist.py _next_layout)
inline void next_layout(int& lay, bool& sampled, uint32_t bad, uint32_t ovf, bool can_pack,
                        bool default_sampled) {
    if (lay == kPlanes) {
        const bool wide_only = bad && !(bad & (kBadPayload | kBadRange));
        lay = can_pack && (wide_only || !bad) ? kWords : kTuples;
        sampled = default_sampled && !ovf;
        return;
    }
    if (lay == kWords && bad) lay = kTuples;
    sampled = sampled && !ovf;
}

// ---------------------------------------------------------------------------
// host side of one process's ranks: a barrier and small reductions (the
// reference's threads share pthread_barrier_t the same way,
// sortmergejoin_multiway.c BARRIER_ARRIVE)
// ---------------------------------------------------------------------------
struct Piece {
    int peer;
    void* ptr;
    uint64_t bytes;
};

struct HostGroup {
    explicit HostGroup(int g) : G(g), posted((size_t)g * g), vals((size_t)g) {}
    int G;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    std::vector<std::vector<Piece>> posted;  // [from * G + to]: pieces in order
    std::vector<int64_t> vals;

    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t g = gen;
        if (++arrived == G) {
            arrived = 0;
            gen++;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != g; });
        }
    }
    // op 0 = sum, 1 = min, 2 = max over the ranks' values (every rank gets it)
    int64_t reduce(int me, int64_t v, int op) {
        vals[me] = v;
        barrier();
        int64_t r = vals[0];
        for (int g = 1; g < G; g++)
            r = op == 0 ? r + vals[g] : op == 1 ? std::min(r, vals[g]) : std::max(r, vals[g]);
        barrier();  // vals may be rewritten after every rank read them
        return r;
    }
};

// Collectives by copies between the ranks' buffers (pull: the receiver copies
// from the sender's buffer).  The CPU tests' stand-in for RCCL, and the
// library's form when several ranks share one GPU (RCCL takes one rank per
// device).  Every exchange synchronises.
template <class Ops>
struct CopyColl {
    HostGroup* grp;
    Ops* ops;
    int me;
    void exchange(int stream, const std::vector<Piece>& sends, const std::vector<Piece>& recvs) {
        const int G = grp->G;
        ops->sync(stream);  // the bytes to send are written
        for (int g = 0; g < G; g++) grp->posted[(size_t)me * G + g].clear();
        for (const Piece& p : sends) grp->posted[(size_t)me * G + p.peer].push_back(p);
        grp->barrier();
        std::vector<size_t> next((size_t)G, 0);
        for (const Piece& r : recvs) {
            const std::vector<Piece>& from = grp->posted[(size_t)r.peer * G + me];
            const size_t k = next[r.peer]++;
            if (k >= from.size() || from[k].bytes != r.bytes) {
                fprintf(stderr, "[ERROR] smj mpsm: rank %d expects %llu bytes from rank %d "
                        "(piece %zu), the sender posted %llu\n", me,
                        (unsigned long long)r.bytes, r.peer, k,
                        (unsigned long long)(k < from.size() ? from[k].bytes : 0));
                abort();
            }
            if (r.bytes) ops->copy(r.ptr, from[k].ptr, r.bytes, stream);
        }
        ops->sync(stream);
        grp->barrier();  // senders may reuse their buffers
    }
    void allreduce_sum_u64(int stream, unsigned long long* dev) {
        unsigned long long v = 0;
        ops->to_host(&v, dev, 8, stream);
        ops->sync(stream);
        v = (unsigned long long)grp->reduce(me, (int64_t)v, 0);
        ops->to_dev(dev, &v, 8, stream);
        ops->sync(stream);
    }
    int64_t reduce(int64_t v, int op) { return grp->reduce(me, v, op); }
};

// ---------------------------------------------------------------------------
// one rank
// ---------------------------------------------------------------------------
struct Options {
    uint32_t bucket_bits = 8;  // level-1 buckets per rank
    bool planes = true;        // offer the 48-bit planes
    bool staged = true;        // R's tile stage while S's rows fly (G > 1)
    int sampled = -1;          // sampled exchange partition: -1 = G == 1 (dist.py)
    // key range: given (kmin <= kmax), or guessed as 1..guess_max (the
    // reference's assumption, sortmergejoin_multiway.c:372-376) and verified
    // by the 48-bit partition, else measured (one read pass on every rank)
    int64_t kmin = 1, kmax = 0;
    uint64_t guess_max = 0;
};

struct Stats {
    int layout = kTuples;       // of the exchange that reached the local join
    uint32_t pbits = 0;
    int attempts = 0;           // exchange attempts (both relations)
    int replans = 0;            // guessed range replaced by the measured one
    uint64_t sent_B = 0, recv_B = 0;
    int64_t kmin = 0, kmax = 0; // the global plan's range
    // device phases of the call in ms (Ops::tspan).  On kMain they are
    // consecutive, so part + tables + wait + join + reduce = busy: wait is
    // kMain idle (host decisions, the key-range pass of a re-plan, and the
    // part of the row exchange the local work did not hide).  rows is the
    // row exchange on kRows, which overlaps the others.
    double part_ms = 0, tables_ms = 0, wait_ms = 0, join_ms = 0, reduce_ms = 0, busy_ms = 0,
           rows_ms = 0;
};

template <class Ops, class Coll>
struct Rank {
    Ops* ops;
    Coll* coll;
    int me = 0, G = 1;

    // buffers kept across calls (sticky sizes, like dist.py's)
    struct RelState {
        void* xb[3] = {nullptr, nullptr, nullptr};
        uint64_t xcap[3] = {0, 0, 0};       // capacity in elements
        uint64_t recv_hint[3] = {0, 0, 0};  // remote rows received last time
        void* small = nullptr;
        size_t small_bytes = 0;
        int64_t* host = nullptr;
        size_t host_bytes = 0;
    } rel[2];
    void* sorted[2] = {nullptr, nullptr};
    size_t sorted_bytes[2] = {0, 0};
    unsigned long long* count = nullptr;  // [0] local join, [1] all-reduced
    unsigned long long* count_h = nullptr;

    // this call
    const void* in[2] = {nullptr, nullptr};
    uint64_t n[2] = {0, 0};
    Options opt;
    Stats stats;
    uint32_t pbits = 0, F = 0, U = 0, K = 1;  // U: the partitions the keys reach
    LocalRange lr{};
    int64_t kmax = 0;
    bool default_sampled = true, guessed = false;
    std::vector<uint32_t> per_rank;  // partitions owned by each rank
    uint32_t mine = 0;

    struct Attempt {
        int lay = kTuples;
        bool sampled = false;
        uint64_t cap = 0;  // the rank's own partition: elements [0, cap) of xb
        int64_t *ss, *sc, *hist, *msg_in, *chunk, *msg, *tstart, *tcnt, *summary;
        uint32_t* flags;
    };
    struct Valid {
        int lay;
        uint64_t cap, nused;  // elements inside the received segments
        void* xb;
        uint64_t stride;      // planes
        int64_t *tstart, *tcnt;
    };

    static uint64_t elem_bytes(int lay) {
        return lay == kTuples ? Ops::kTupleBytes : lay == kWords ? 8 : 6;
    }
    static uint64_t round32(uint64_t x) { return (x + 31) & ~31ull; }
    static uint64_t buf_bytes(int lay, uint64_t elems) {
        if (elems == 0) elems = 1;
        return lay == kPlanes ? round32(elems) * 6 : elems * elem_bytes(lay);
    }

    template <class T>
    static T* carve(char*& p, size_t count) {
        T* r = (T*)p;
        p += (count * sizeof(T) + 255) & ~(size_t)255;
        return r;
    }

    // The exchange buffer of relation r in layout `lay` with room for `need`
    // elements; a grown buffer keeps the first `keep` elements (the rank's own
    // partition, copied on kMain).  Returns true when it moved.
    bool xbuf(int r, int lay, uint64_t need, uint64_t keep) {
        RelState& s = rel[r];
        if (s.xb[lay] && s.xcap[lay] >= need) return false;
        const uint64_t cap = lay == kPlanes ? round32(need ? need : 1) : (need ? need : 1);
        void* nb = ops->alloc(buf_bytes(lay, cap));
        if (s.xb[lay]) {
            if (keep) {
                if (lay == kPlanes) {
                    ops->copy(nb, s.xb[lay], keep * 4, kMain);
                    ops->copy((char*)nb + cap * 4, (char*)s.xb[lay] + s.xcap[lay] * 4, keep * 2,
                              kMain);
                } else {
                    ops->copy(nb, s.xb[lay], keep * elem_bytes(lay), kMain);
                }
            }
            ops->sync(kMain);
            ops->sync(kRows);
            ops->release(s.xb[lay]);
        }
        s.xb[lay] = nb;
        s.xcap[lay] = cap;
        return true;
    }

    // device tables of relation r for this call's F, K, G
    Attempt tables(int r) {
        RelState& s = rel[r];
        const size_t FK = (size_t)F * K, nb = (size_t)1 << lr.lbits;
        const size_t row = kHead + 2ull * K * mine;
        const size_t msg_len = (size_t)G * kHead + 2ull * K * F;
        const size_t words[] = {FK, FK, F, 1, msg_len, 2ull * G, (size_t)G * row, nb * G * K,
                                nb * G * K, 4ull * G + 2};
        size_t bytes = 0;
        for (size_t w : words) bytes += (w * 8 + 255) & ~(size_t)255;
        if (s.small_bytes < bytes) {
            if (s.small) {
                ops->sync(kMain);
                ops->release(s.small);
            }
            s.small = ops->alloc(bytes);
            s.small_bytes = bytes;
        }
        const size_t hb = (4ull * G + 2) * 8;
        if (s.host_bytes < hb) {
            if (s.host) ops->host_release(s.host);
            s.host = (int64_t*)ops->host_alloc(hb);
            s.host_bytes = hb;
        }
        char* p = (char*)s.small;
        Attempt a;
        a.ss = carve<int64_t>(p, FK);
        a.sc = carve<int64_t>(p, FK);
        a.hist = carve<int64_t>(p, F);
        a.flags = (uint32_t*)carve<int64_t>(p, 1);
        a.msg_in = carve<int64_t>(p, msg_len);
        a.chunk = carve<int64_t>(p, 2ull * G);
        a.msg = carve<int64_t>(p, (size_t)G * row);
        a.tstart = carve<int64_t>(p, nb * G * K);
        a.tcnt = carve<int64_t>(p, nb * G * K);
        a.summary = carve<int64_t>(p, 4ull * G + 2);
        return a;
    }

    // Enqueue one exchange attempt of relation r: its range partition, the
    // table messages and their exchange, the receive tables and the summary
    // copy (recorded on kEvAttemptR + r).  64-bit words the plan does not
    // allow become tuples (words_ok, the same on every rank).
    void attempt(int r, int lay, bool sampled, Attempt& a) {
        if (lay == kWords && !words_ok()) lay = kTuples;
        a = tables(r);
        const uint64_t nn = n[r];
        sampled = sampled || lay == kPlanes;
        a.lay = lay;
        a.sampled = sampled;
        a.cap = sampled ? ops->sampled_capacity(nn, pbits) : nn;
        RelState& s = rel[r];
        const uint64_t extra = s.recv_hint[lay]
            ? s.recv_hint[lay] : (G > 1 ? a.cap * (G - 1) / G + a.cap / 8 : 0);
        xbuf(r, lay, a.cap + extra, 0);
        void* xb = s.xb[lay];
        const size_t FK = (size_t)F * K;
        bool done = false;
        ops->tmark(kTPart0 + 3 * r, kMain);
        if (nn == 0) {  // nothing to partition: empty tables
            ops->fill_u32(a.ss, 0, 2 * FK, kMain);
            ops->fill_u32(a.sc, 0, 2 * FK, kMain);
            ops->fill_u32(a.flags, 0, 2, kMain);
            done = true;
        } else if (lay == kPlanes) {
            if (!ops->part_planes(in[r], nn, xb, s.xcap[lay], pbits, lr.base, kmax, a.ss, a.sc,
                                  a.flags)) {
                // the form does not apply on this rank: empty tables flagged
                // as too wide for 48 bits, so every rank drops the layout.  A
                // guessed range was not checked then, so the flag also asks
                // for the measured range (the other forms do not check it)
                ops->fill_u32(a.ss, 0, 2 * FK, kMain);
                ops->fill_u32(a.sc, 0, 2 * FK, kMain);
                ops->fill_u32(a.flags, 0, 1, kMain);
                ops->fill_u32(a.flags + 1, kBadPayload48 | (guessed ? kBadRange : 0u), 1, kMain);
            }
            done = true;
        } else if (sampled) {
            done = ops->part_sampled(in[r], nn, xb, pbits, lr.base, kmax, lay == kWords ? 1 : 0,
                                     a.ss, a.sc, a.flags) != 0;
            if (!done) a.cap = nn;  // the exact form below
        }
        if (!done) {
            // exact: the sampled scatter with exactly sized regions (one count
            // pass, no slack to travel); else histogram + scatter
            done = ops->part_shards(in[r], nn, xb, pbits, lr.base, kmax, lay == kWords ? 1 : 0,
                                    a.ss, a.sc, a.flags) != 0;
        }
        if (!done) {
            ops->fill_u32(a.flags, 0, 2, kMain);
            if (lay == kWords) {
                if (!ops->part_exact_packed(in[r], nn, xb, pbits, lr.base, kmax, a.hist,
                                            a.flags + 1)) {
                    fprintf(stderr, "[ERROR] smj mpsm: packed words refused a plan that "
                            "allows them\n");
                    abort();
                }
            } else {
                ops->part_exact(in[r], nn, xb, pbits, lr.base, kmax, a.hist);
            }
            ops->hist_tables(a.hist, F, K, a.ss, a.sc);
        }
        ops->tmark(kTPart0 + 3 * r + 1, kMain);
        ops->xsend(a.ss, a.sc, a.flags, F, K, (uint32_t)G, U, a.msg_in, a.chunk);
        const uint64_t row = kHead + 2ull * K * mine;
        const int64_t* msg = a.msg_in;
        if (G > 1) {
            std::vector<Piece> sends, recvs;
            uint64_t off = 0;
            for (int g = 0; g < G; g++) {
                const uint64_t len = kHead + 2ull * K * per_rank[g];
                sends.push_back({g, a.msg_in + off, len * 8});
                recvs.push_back({g, a.msg + (size_t)g * row, row * 8});
                off += len;
            }
            coll->exchange(kMain, sends, recvs);
            msg = a.msg;
        }
        ops->xrecv(msg, a.chunk, (uint32_t)G, (uint32_t)me, mine, K, 1u << lr.lbits, a.cap,
                   a.tstart, a.tcnt, a.summary);
        ops->to_host(s.host, a.summary, (4ull * G + 2) * 8, kMain);
        ops->tmark(kTPart0 + 3 * r + 2, kMain);
        ops->record(kEvAttemptR + r, kMain);
        stats.attempts++;
    }

    // Wait for relation r's attempt; repeat it until every rank agrees it is
    // valid, then issue its rows on kRows (recorded on kEvRowsR + r).
    // Returns 1, or 0 when a key lies outside a guessed range (the caller
    // replans: every rank sees the same flag).
    int finish(int r, Attempt& a, Valid& v) {
        RelState& s = rel[r];
        for (;;) {
            ops->host_wait(kEvAttemptR + r);
            stats.part_ms += ops->tspan(kTPart0 + 3 * r, kTPart0 + 3 * r + 1);
            stats.tables_ms += ops->tspan(kTPart0 + 3 * r + 1, kTPart0 + 3 * r + 2);
            const int64_t* h = s.host;
            const uint32_t bad = (uint32_t)h[4 * G], ovf = (uint32_t)h[4 * G + 1];
            if (!ovf && !(a.lay != kTuples && bad)) break;
            if (guessed && (bad & kBadRange)) return 0;
            int lay = a.lay;
            bool sampled = a.sampled;
            next_layout(lay, sampled, bad, ovf, words_ok(), default_sampled);
            attempt(r, lay, sampled, a);
        }
        const int64_t* h = s.host;
        const int64_t *cs = h, *sl = h + G, *rl = h + 2 * G, *ru = h + 3 * G;
        uint64_t remote = 0, used = 0, sent = 0;
        for (int g = 0; g < G; g++) {
            used += (uint64_t)ru[g];
            if (g != me) {
                remote += (uint64_t)rl[g];
                sent += (uint64_t)sl[g];
            }
        }
        const int lay = a.lay;
        s.recv_hint[lay] = std::max(s.recv_hint[lay], remote);
        const bool moved = xbuf(r, lay, a.cap + remote, a.cap);
        v.lay = lay;
        v.cap = a.cap;
        v.nused = used;
        v.xb = s.xb[lay];
        v.stride = s.xcap[lay];
        v.tstart = a.tstart;
        v.tcnt = a.tcnt;
        stats.sent_B += sent * elem_bytes(lay);
        stats.recv_B += remote * elem_bytes(lay);
        if (G > 1) {
            // the rows leave from kRows, ordered after this attempt only (not
            // after work queued behind it: the other relation's partition);
            // after a grown buffer's copy on kMain
            if (moved) ops->record(kEvMain, kMain);
            ops->wait(kRows, moved ? kEvMain : kEvAttemptR + r);
            rows_time(r);
            ops->tmark(kTRows0 + 2 * r, kRows);
            rows(v, cs, sl, rl);
            ops->tmark(kTRows0 + 2 * r + 1, kRows);
            rows_marked[r] = true;
            ops->record(kEvRowsR + r, kRows);
        }
        return 1;
    }

    // The rows of one relation: rank g gets xb[cs[g], cs[g] + sl[g]); the
    // other ranks' rows land after the own partition (xb[cap:], rank order);
    // the own chunk is not copied.  Peers in NEXT order, (me + i) % G
    // (numa_shuffle.c:83); pieces of at most kPieceBytes, cut the same way on
    // both sides.
    void rows(const Valid& v, const int64_t* cs, const int64_t* sl, const int64_t* rl) {
        std::vector<uint64_t> roff((size_t)G);
        uint64_t ro = v.cap;
        for (int g = 0; g < G; g++) {
            roff[g] = ro;
            if (g != me) ro += (uint64_t)rl[g];
        }
        struct Plane {
            char* base;
            uint64_t eb;
        };
        std::vector<Plane> planes;
        if (v.lay == kPlanes) {
            planes.push_back({(char*)v.xb, 4});
            planes.push_back({(char*)v.xb + v.stride * 4, 2});
        } else {
            planes.push_back({(char*)v.xb, elem_bytes(v.lay)});
        }
        std::vector<Piece> sends, recvs;
        auto cut = [&](std::vector<Piece>& out, int peer, char* p, uint64_t bytes) {
            for (uint64_t o = 0; o < bytes; o += kPieceBytes)
                out.push_back({peer, p + o, std::min(kPieceBytes, bytes - o)});
        };
        for (int i = 1; i < G; i++) {
            const int to = (me + i) % G, from = (me - i + G) % G;
            for (const Plane& pl : planes) {
                cut(sends, to, pl.base + (uint64_t)cs[to] * pl.eb, (uint64_t)sl[to] * pl.eb);
                cut(recvs, from, pl.base + roff[from] * pl.eb, (uint64_t)rl[from] * pl.eb);
            }
        }
        coll->exchange(kRows, sends, recvs);
    }

    // the row exchange of relation r timed so far (before its marks are
    // recorded again, and at the end of the call)
    bool rows_marked[2] = {false, false};
    void rows_time(int r) {
        if (!rows_marked[r]) return;
        ops->sync(kRows);
        stats.rows_ms += ops->tspan(kTRows0 + 2 * r, kTRows0 + 2 * r + 1);
        rows_marked[r] = false;
    }

    void set_plan(int64_t kmin_, int64_t kmax_) {
        const uint64_t n_hint = std::max(n[0], n[1]);
        const bool offer = opt.planes;
        pbits = partition_bits(opt.bucket_bits, (uint32_t)G, offer, n_hint, true, kmin_, kmax_);
        if ((1u << pbits) < (uint32_t)G) pbits = ceil_log2((uint64_t)G);
        F = 1u << pbits;
        U = used_parts(kmin_, kmax_, pbits);
        lr = local_range(kmin_, kmax_, pbits, (uint32_t)G, (uint32_t)me);
        kmax = kmax_;
        per_rank.assign((size_t)G, 0);
        for (int g = 0; g < G; g++)
            per_rank[g] = owned_lo(F, (uint32_t)G, U, (uint32_t)g + 1) -
                          owned_lo(F, (uint32_t)G, U, (uint32_t)g);
        mine = per_rank[me];
        stats.pbits = pbits;
        stats.kmin = lr.base;
        stats.kmax = kmax_;
    }

    // 64-bit packed words apply to the plan (16-byte tuples, 1 <= s1 <= 32):
    // a property of the plan, so every rank computes the same answer
    bool words_ok() const {
        const uint32_t s1 = plan_shift(lr.base, kmax, pbits);
        return ops->can_pack() && s1 >= 1 && s1 <= 32;
    }
    int first_layout() const {
        if (opt.planes && pbits <= kPlaneMaxBits && planes_hold(lr.base, kmax, pbits))
            return kPlanes;
        return words_ok() ? kWords : kTuples;
    }

    // The global key range measured on every rank (one read pass each).
    void measured_range(int64_t* lo, int64_t* hi) {
        int64_t l = INT64_MAX, h = INT64_MIN;
        int64_t a, b;
        if (ops->key_range(in[0], n[0], in[1], n[1], &a, &b)) {
            l = a;
            h = b;
        }
        *lo = coll->reduce(l, 1);
        *hi = coll->reduce(h, 2);
    }

    // One join of this rank's slices R[0, nR) and S[0, nS).  Returns the
    // global match count; sorted[0 / 1] hold the rank's sorted share
    // (*nR_out / *nS_out tuples: one contiguous key range, ranks in order),
    // *local the rank's own count.
    uint64_t run(const void* R, uint64_t nR, const void* S, uint64_t nS, const Options& o,
                 uint64_t* nR_out, uint64_t* nS_out, uint64_t* local) {
        in[0] = R;
        in[1] = S;
        n[0] = nR;
        n[1] = nS;
        opt = o;
        stats = Stats();
        rows_marked[0] = rows_marked[1] = false;
        ops->tmark(kTStart, kMain);
        K = ops->shards();
        default_sampled = o.sampled < 0 ? G == 1 : o.sampled != 0;
        if (!count) {
            count = (unsigned long long*)ops->alloc(16);
            count_h = (unsigned long long*)ops->host_alloc(16);
        }
        int64_t kmin_ = o.kmin, kmax_ = o.kmax;
        guessed = false;
        if (kmin_ > kmax_ && o.guess_max) {
            kmin_ = 1;
            kmax_ = (int64_t)std::min<uint64_t>(o.guess_max, (uint64_t)INT64_MAX);
            guessed = true;
        }
        if (kmin_ > kmax_) measured_range(&kmin_, &kmax_);
        if (kmin_ > kmax_) kmin_ = kmax_ = 0;  // every relation empty
        set_plan(kmin_, kmax_);
        // a guessed range is verified by the 48-bit partition only
        if (guessed && first_layout() != kPlanes) {
            guessed = false;
            measured_range(&kmin_, &kmax_);
            if (kmin_ > kmax_) kmin_ = kmax_ = 0;
            set_plan(kmin_, kmax_);
        }
        Valid v[2];
        for (;;) {
            Attempt a[2];
            const int lay0 = first_layout();
            for (int r = 0; r < 2; r++) attempt(r, lay0, default_sampled, a[r]);
            int ok = finish(0, a[0], v[0]);
            if (ok) ok = finish(1, a[1], v[1]);
            if (ok) {
                // both relations must reach the local join in one layout: the
                // one that went out narrower is exchanged again in the other's
                while (ok && v[0].lay != v[1].lay) {
                    const int r = v[0].lay > v[1].lay ? 0 : 1;
                    ops->sync(kRows);
                    attempt(r, v[1 - r].lay, default_sampled, a[r]);
                    ok = finish(r, a[r], v[r]);
                }
            }
            if (ok) break;
            // a key outside the guessed range (the same on every rank):
            // the measured range, attempts from the top
            ops->sync(kRows);
            ops->sync(kMain);
            guessed = false;
            stats.replans++;
            measured_range(&kmin_, &kmax_);
            set_plan(kmin_, kmax_);
        }
        stats.layout = v[0].lay;
        const uint64_t TB = Ops::kTupleBytes;
        for (int r = 0; r < 2; r++) {
            const size_t b = (v[r].nused ? v[r].nused : 1) * TB;
            if (sorted_bytes[r] < b) {
                if (sorted[r]) {
                    ops->sync(kMain);
                    ops->release(sorted[r]);
                }
                sorted[r] = ops->alloc(b);
                sorted_bytes[r] = b;
            }
        }
        const uint32_t nseg = (uint32_t)G * K;
        auto join = [&](int stage) {
            ops->join(v[0].lay, v[0].xb, v[0].stride, v[0].nused, v[0].tstart, v[0].tcnt, v[1].xb,
                      v[1].stride, v[1].nused, v[1].tstart, v[1].tcnt, nseg, lr.lbits, lr.key_lo,
                      lr.key_hi, stage, sorted[0], sorted[1], count);
        };
        bool two = false;
        if (v[0].nused == 0 && v[1].nused == 0) {
            if (G > 1) {
                ops->wait(kMain, kEvRowsR);
                ops->wait(kMain, kEvRowsS);
            }
            ops->tmark(kTJoin0, kMain);
            ops->fill_u32(count, 0, 2, kMain);
            ops->tmark(kTJoin1, kMain);
        } else if (G > 1 && opt.staged) {
            ops->wait(kMain, kEvRowsR);
            ops->tmark(kTJoin0, kMain);
            join(1);
            ops->tmark(kTJoin1, kMain);
            ops->wait(kMain, kEvRowsS);
            ops->tmark(kTJoin2, kMain);
            join(2);
            ops->tmark(kTJoin3, kMain);
            two = true;
        } else {
            if (G > 1) {
                ops->wait(kMain, kEvRowsR);
                ops->wait(kMain, kEvRowsS);
            }
            ops->tmark(kTJoin0, kMain);
            join(0);
            ops->tmark(kTJoin1, kMain);
        }
        ops->copy(count + 1, count, 8, kMain);
        coll->allreduce_sum_u64(kMain, count + 1);
        ops->tmark(kTEnd, kMain);
        ops->to_host(count_h, count, 16, kMain);
        ops->sync(kMain);
        // the phases (every mark on kMain has completed; the rows' marks too:
        // kMain waited for the rows)
        stats.join_ms = ops->tspan(kTJoin0, kTJoin1) + (two ? ops->tspan(kTJoin2, kTJoin3) : 0.0);
        stats.reduce_ms = ops->tspan(two ? kTJoin3 : kTJoin1, kTEnd);
        stats.busy_ms = ops->tspan(kTStart, kTEnd);
        stats.wait_ms = std::max(0.0, stats.busy_ms - stats.part_ms - stats.tables_ms -
                                          stats.join_ms - stats.reduce_ms);
        for (int r = 0; r < 2; r++) rows_time(r);
        *nR_out = last_n[0] = v[0].nused;
        *nS_out = last_n[1] = v[1].nused;
        *local = count_h[0];
        return count_h[1];
    }
    uint64_t last_n[2] = {0, 0};
    void sorted_sizes(uint64_t* nr, uint64_t* ns) const {
        *nr = last_n[0];
        *ns = last_n[1];
    }

    void release_all() {
        ops->sync(kMain);
        ops->sync(kRows);
        for (int r = 0; r < 2; r++) {
            for (int l = 0; l < 3; l++)
                if (rel[r].xb[l]) ops->release(rel[r].xb[l]);
            if (rel[r].small) ops->release(rel[r].small);
            if (rel[r].host) ops->host_release(rel[r].host);
            if (sorted[r]) ops->release(sorted[r]);
            rel[r] = RelState();
            sorted[r] = nullptr;
            sorted_bytes[r] = 0;
        }
        if (count) ops->release(count);
        if (count_h) ops->host_release(count_h);
        count = nullptr;
        count_h = nullptr;
    }
};

// Runs fn(rank) on G threads (rank 0 on the calling thread) and joins them.
inline void run_ranks(int G, const std::function<void(int)>& fn) {
    std::vector<std::thread> th;
    for (int g = 1; g < G; g++) th.emplace_back(fn, g);
    fn(0);
    for (auto& t : th) t.join();
}

}  // namespace mg
}  // namespace smj
