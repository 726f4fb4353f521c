// host_orch.cpp -- CPU test harness of the multi-GPU join's C++ orchestration
// (avx-sort-merge-joins_amd/csrc/mgpu_orch.hpp, the code sortmergejoin_mpsm
// runs on G GPUs).  TEST INFRASTRUCTURE: built by tests/test_mgpu_host.py
// with g++ (-DKEY_8B for 16-byte tuples), never linked into the library.
//
// HostOps restates, on the host, the contracts of the device functions the
// orchestration calls (include/smj.h): the range partitions in their three
// layouts (tuples, 64-bit words, 48-bit words in two planes; sampled regions
// with garbage-filled slack, or exact), the exchange table kernels
// (exchange.hip k_xsend / k_xrecv, k_hist_tables), and the segmented local
// join (gather the bucket's segments, decode, check that every element sits
// in the bucket of its local digit, sort, count).  Ranks run as threads and
// exchange through mg::CopyColl (memcpy between the ranks' buffers), so the
// orchestration's table exchange, layout agreement, retries, buffer growth
// and row placement run exactly as on the GPUs.  Failure injection: one
// rank's sampled regions overflow, or one rank's sampled/planes partition
// does not apply.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "../../avx-sort-merge-joins_amd/csrc/mgpu_orch.hpp"

namespace mg = smj::mg;
typedef mg::i128 i128;

#ifdef KEY_8B
struct Tup {
    int64_t payload, key;
};
static inline uint64_t pay_u(const Tup& t) { return (uint64_t)t.payload; }
static inline Tup make_tup(int64_t key, uint64_t pay) { return Tup{(int64_t)pay, key}; }
#else
struct Tup {
    int32_t payload, key;
};
static inline uint64_t pay_u(const Tup& t) { return (uint32_t)t.payload; }
static inline Tup make_tup(int64_t key, uint64_t pay) {
    return Tup{(int32_t)(uint32_t)pay, (int32_t)key};
}
#endif

// the library's order: 16 B (key, payload) signed; 8 B the signed 64-bit word
// key << 32 | (uint32) payload
static inline bool tup_less(const Tup& a, const Tup& b) {
    if (a.key != b.key) return a.key < b.key;
#ifdef KEY_8B
    return a.payload < b.payload;
#else
    return (uint32_t)a.payload < (uint32_t)b.payload;
#endif
}

static std::mutex g_err_mu;
static std::string g_err;
static std::atomic<int> g_nerr{0};
#define CHECK(cond, ...)                                          \
    do {                                                          \
        if (!(cond)) {                                            \
            char b_[512];                                         \
            snprintf(b_, sizeof b_, __VA_ARGS__);                 \
            std::lock_guard<std::mutex> lk_(g_err_mu);            \
            if (g_nerr++ == 0) g_err = b_;                        \
        }                                                         \
    } while (0)

struct Range {  // the plan arithmetic of make_plan for D1 = bits
    int64_t kmin;
    uint32_t L, s1;
    Range(int64_t kmin_, int64_t kmax_, uint32_t bits)
        : kmin(kmin_), L(mg::bitlen(mg::span_of(kmin_, kmax_))),
          s1(mg::plan_shift(kmin_, kmax_, bits)) {}
    bool inside(int64_t k) const {
        const i128 r = (i128)k - kmin;
        return r >= 0 && r <= (((i128)1 << L) - 1);
    }
    uint64_t rel(int64_t k) const {  // clamped to the plan
        i128 r = (i128)k - kmin;
        if (r < 0) r = 0;
        const i128 top = ((i128)1 << L) - 1;
        if (r > top) r = top;
        return (uint64_t)r;
    }
    uint32_t digit(int64_t k) const { return (uint32_t)(rel(k) >> s1); }
};

struct HostOps {
    static constexpr int kTupleBytes = (int)sizeof(Tup);
    static constexpr uint32_t K = 3;  // shards of the sampled layout
    int rank = 0;
    bool overflow = false;        // report a sampled region overflow
    bool not_applicable = false;  // sampled / planes forms return 0
    // the staged join protocol: an R call, then a REST call with the same tables
    const void* staged = nullptr;
    const int64_t* staged_ts = nullptr;
    int stage_calls = 0, whole_calls = 0;

    bool can_pack() const { return sizeof(Tup) == 16; }
    void* alloc(size_t b) {
        void* p = nullptr;
        if (posix_memalign(&p, 256, b ? b : 16)) abort();
        memset(p, 0xA5, b ? b : 16);  // never-written bytes must not be read
        return p;
    }
    void release(void* p) { free(p); }
    void* host_alloc(size_t b) { return alloc(b); }
    void host_release(void* p) { free(p); }
    void copy(void* d, const void* s, size_t b, int) { memmove(d, s, b); }
    void to_host(void* h, const void* d, size_t b, int) { memcpy(h, d, b); }
    void to_dev(void* d, const void* h, size_t b, int) { memcpy(d, h, b); }
    void fill_u32(void* p, uint32_t v, size_t n, int) {
        for (size_t i = 0; i < n; i++) ((uint32_t*)p)[i] = v;
    }
    void record(int, int) {}
    void wait(int, int) {}
    void host_wait(int) {}
    void sync(int) {}
    // timing marks: a logical clock, so the phases' arithmetic is checked
    // (every mark one unit after the previous one)
    double clock = 0, mark_t[smj::mg::kNumTMarks] = {};
    void tmark(int m, int) { mark_t[m] = (clock += 1.0); }
    double tspan(int a, int b) { return mark_t[b] - mark_t[a]; }
    uint32_t shards() { return K; }
    uint64_t sampled_capacity(uint64_t n, uint32_t nbits) {
        return n + n / 8 + ((uint64_t)1 << nbits) * K * 5 + 16;
    }

    // the sampled layout: partition p = K consecutive shard regions (shard =
    // position * K / n), each followed by slack; element i goes to pos[i]
    void place(const Tup* in, uint64_t n, uint32_t nbits, const Range& rg, int64_t* ss,
               int64_t* sc, uint32_t* flags, std::vector<uint64_t>& pos, bool slack = true) {
        const uint64_t FK = ((uint64_t)1 << nbits) * K;
        std::vector<uint64_t> cnt(FK, 0), start(FK, 0), fill(FK, 0);
        std::vector<uint64_t> idx(n);
        for (uint64_t i = 0; i < n; i++) {
            idx[i] = (uint64_t)rg.digit(in[i].key) * K + i * K / n;
            cnt[idx[i]]++;
        }
        uint64_t acc = 0;
        for (uint64_t j = 0; j < FK; j++) {
            start[j] = acc;
            acc += cnt[j] + (slack ? cnt[j] / 8 + j % 5 : 0);
            ss[j] = (int64_t)start[j];
            sc[j] = (int64_t)cnt[j];
        }
        pos.resize(n);
        for (uint64_t i = 0; i < n; i++) pos[i] = start[idx[i]] + fill[idx[i]]++;
        flags[0] = overflow && slack ? 1u : 0u;
    }
    // smj_dev_partition_range_shards: the sampled layout with exactly sized
    // regions back to back (no slack, never an overflow); `out` holds n
    int part_shards(const void* inv, uint64_t n, void* out, uint32_t nbits, int64_t kmin,
                    int64_t kmax, int packed, int64_t* ss, int64_t* sc, uint32_t* flags) {
        const Tup* in = (const Tup*)inv;
        Range rg(kmin, kmax, nbits);
        shards_calls++;
        if (not_applicable || nbits > 10) return 0;
        if (packed && (!can_pack() || rg.s1 < 1 || rg.s1 > 32)) return 0;
        std::vector<uint64_t> pos;
        place(in, n, nbits, rg, ss, sc, flags, pos, false);
        flags[1] = 0;
        for (uint64_t i = 0; i < n; i++) {
            CHECK(pos[i] < n, "shards position %llu of %llu", (unsigned long long)pos[i],
                  (unsigned long long)n);
            if (packed) {
                uint32_t bad = 0;
                ((uint64_t*)out)[pos[i]] = word64(in[i], rg, &bad);
                flags[1] |= bad ? 1u : 0u;
            } else {
                ((Tup*)out)[pos[i]] = in[i];
            }
        }
        return 1;
    }
    int shards_calls = 0;
    int part_sampled(const void* inv, uint64_t n, void* out, uint32_t nbits, int64_t kmin,
                     int64_t kmax, int packed, int64_t* ss, int64_t* sc, uint32_t* flags) {
        const Tup* in = (const Tup*)inv;
        Range rg(kmin, kmax, nbits);
        if (not_applicable || nbits > 10) return 0;
        if (packed && (!can_pack() || rg.s1 < 1 || rg.s1 > 32)) return 0;
        std::vector<uint64_t> pos;
        place(in, n, nbits, rg, ss, sc, flags, pos);
        flags[1] = 0;
        const uint64_t cap = sampled_capacity(n, nbits);
        if (packed) {
            uint64_t* w = (uint64_t*)out;
            for (uint64_t i = 0; i < cap; i++) w[i] = (uint64_t)-7;  // slack
            for (uint64_t i = 0; i < n; i++) {
                uint32_t bad = 0;
                w[pos[i]] = word64(in[i], rg, &bad);
                flags[1] |= bad ? 1u : 0u;
            }
        } else {
            Tup* t = (Tup*)out;
            for (uint64_t i = 0; i < cap; i++) t[i] = make_tup(-7, (uint64_t)-7);
            for (uint64_t i = 0; i < n; i++) t[pos[i]] = in[i];
        }
        return 1;
    }
    uint64_t word64(const Tup& t, const Range& rg, uint32_t* bad) const {
        const uint64_t p = pay_u(t);
        if (!rg.inside(t.key) || (rg.s1 < 64 && (p >> (64 - rg.s1)) != 0)) *bad = 1;
        return ((rg.rel(t.key) & ((1ull << rg.s1) - 1)) << (64 - rg.s1)) | p;
    }
    int part_planes(const void* inv, uint64_t n, void* out, uint64_t stride, uint32_t nbits,
                    int64_t kmin, int64_t kmax, int64_t* ss, int64_t* sc, uint32_t* flags) {
        const Tup* in = (const Tup*)inv;
        Range rg(kmin, kmax, nbits);
        if (not_applicable || nbits > 10 || rg.s1 < 1 || rg.s1 > 32) return 0;
        CHECK(stride % 32 == 0 && stride >= sampled_capacity(n, nbits),
              "planes stride %llu", (unsigned long long)stride);
        std::vector<uint64_t> pos;
        place(in, n, nbits, rg, ss, sc, flags, pos);
        uint32_t* lo = (uint32_t*)out;
        uint16_t* hi = (uint16_t*)(lo + stride);
        for (uint64_t i = 0; i < stride; i++) {
            lo[i] = 0xFFFFFFF9u;
            hi[i] = 0xFFF9u;
        }
        uint32_t bad = 0;
        const uint32_t s1 = rg.s1;
        for (uint64_t i = 0; i < n; i++) {
            const uint64_t p = pay_u(in[i]);
            if (!rg.inside(in[i].key)) bad |= mg::kBadRange;
            if ((p >> (64 - s1)) != 0) bad |= mg::kBadPayload;
            if ((p >> (48 - s1)) != 0) bad |= mg::kBadPayload48;
            const uint64_t w = ((rg.rel(in[i].key) & ((1ull << s1) - 1)) << (48 - s1)) |
                               (p & ((1ull << (48 - s1)) - 1));
            lo[pos[i]] = (uint32_t)w;
            hi[pos[i]] = (uint16_t)(w >> 32);
        }
        flags[1] = bad;
        return 1;
    }
    void part_exact(const void* inv, uint64_t n, void* out, uint32_t nbits, int64_t kmin,
                    int64_t kmax, int64_t* hist) {
        const Tup* in = (const Tup*)inv;
        Range rg(kmin, kmax, nbits);
        const uint32_t F = 1u << nbits;
        std::vector<uint64_t> start(F, 0);
        for (uint32_t p = 0; p < F; p++) hist[p] = 0;
        for (uint64_t i = 0; i < n; i++) hist[rg.digit(in[i].key)]++;
        for (uint32_t p = 1; p < F; p++) start[p] = start[p - 1] + (uint64_t)hist[p - 1];
        for (uint64_t i = 0; i < n; i++) ((Tup*)out)[start[rg.digit(in[i].key)]++] = in[i];
    }
    int part_exact_packed(const void* inv, uint64_t n, void* out, uint32_t nbits, int64_t kmin,
                          int64_t kmax, int64_t* hist, uint32_t* bad) {
        const Tup* in = (const Tup*)inv;
        Range rg(kmin, kmax, nbits);
        if (!can_pack() || rg.s1 < 1 || rg.s1 > 32) return 0;
        const uint32_t F = 1u << nbits;
        std::vector<uint64_t> start(F, 0);
        for (uint32_t p = 0; p < F; p++) hist[p] = 0;
        for (uint64_t i = 0; i < n; i++) hist[rg.digit(in[i].key)]++;
        for (uint32_t p = 1; p < F; p++) start[p] = start[p - 1] + (uint64_t)hist[p - 1];
        uint32_t b = 0;
        for (uint64_t i = 0; i < n; i++)
            ((uint64_t*)out)[start[rg.digit(in[i].key)]++] = word64(in[i], rg, &b);
        if (b) *bad |= 1u;
        return 1;
    }
    // exchange.hip k_hist_tables
    void hist_tables(const int64_t* hist, uint32_t F, uint32_t Kk, int64_t* ss, int64_t* sc) {
        int64_t acc = 0;
        for (uint32_t p = 0; p < F; p++) {
            for (uint32_t q = 0; q < Kk; q++) {
                ss[(size_t)p * Kk + q] = q == 0 ? acc : 0;
                sc[(size_t)p * Kk + q] = q == 0 ? hist[p] : 0;
            }
            acc += hist[p];
        }
    }
    // exchange.hip k_xsend
    void xsend(const int64_t* start, const int64_t* cnt, const uint32_t* flags, uint32_t F,
               uint32_t Kk, uint32_t G, uint32_t U, int64_t* msg, int64_t* chunk) {
        int64_t cend = 0;
        std::vector<int64_t> used(G, 0);
        for (uint32_t p = 0; p < F; p++)
            for (uint32_t q = 0; q < Kk; q++) {
                const size_t i = (size_t)p * Kk + q;
                cend = std::max(cend, start[i] + cnt[i]);
                used[p < U ? (uint64_t)p * G / U : G - 1] += cnt[i];
            }
        for (uint32_t g = 0; g < G; g++) {
            const uint32_t lo = mg::owned_lo(F, G, U, g), hi = mg::owned_lo(F, G, U, g + 1);
            const int64_t cs = start[(size_t)lo * Kk];
            const int64_t ce = g + 1 < G ? start[(size_t)hi * Kk] : cend;
            chunk[g] = cs;
            chunk[G + g] = ce - cs;
            const uint64_t m0 = (uint64_t)g * mg::kHead + 2ull * Kk * lo;
            const uint32_t nreg = (hi - lo) * Kk;
            msg[m0 + 0] = ce - cs;
            msg[m0 + 1] = used[g];
            msg[m0 + 2] = flags[1];
            msg[m0 + 3] = flags[0];
            for (uint32_t j = 0; j < nreg; j++) {
                const size_t i = (size_t)lo * Kk + j;
                msg[m0 + mg::kHead + j] = cnt[i] > 0 ? start[i] - cs : 0;
                msg[m0 + mg::kHead + nreg + j] = cnt[i];
            }
        }
    }
    // exchange.hip k_xrecv
    void xrecv(const int64_t* msg, const int64_t* chunk, uint32_t G, uint32_t me, uint32_t mine,
               uint32_t Kk, uint32_t nb, uint64_t cap, int64_t* ts, int64_t* tc,
               int64_t* summary) {
        const uint64_t row = mg::kHead + 2ull * mine * Kk;
        std::vector<int64_t> base(G);
        int64_t ro = (int64_t)cap, f0 = 0, f1 = 0;
        for (uint32_t s = 0; s < G; s++) {
            const int64_t rl = msg[s * row];
            base[s] = s == me ? chunk[me] : ro;
            if (s != me) ro += rl;
            summary[2 * G + s] = rl;
            summary[3 * G + s] = msg[s * row + 1];
            f0 |= msg[s * row + 2];
            f1 |= msg[s * row + 3];
        }
        summary[4 * G] = f0;
        summary[4 * G + 1] = f1;
        for (uint32_t g = 0; g < G; g++) {
            summary[g] = chunk[g];
            summary[G + g] = chunk[G + g];
        }
        const uint32_t GK = G * Kk;
        for (uint32_t i = 0; i < nb * GK; i++) {
            const uint32_t b = i / GK, j = i % GK, s = j / Kk, q = j % Kk;
            int64_t st = 0, ct = 0;
            if (b < mine) {
                const size_t m = (size_t)s * row + mg::kHead + (size_t)b * Kk + q;
                ct = msg[m + (size_t)mine * Kk];
                st = msg[m] + base[s];
            }
            ts[i] = st;
            tc[i] = ct;
        }
    }
    // the segmented local join: gather, decode, check the bucket, sort, count
    void join(int lay, void* R, uint64_t strideR, uint64_t nR, const int64_t* tsR,
              const int64_t* tcR, void* S, uint64_t strideS, uint64_t nS, const int64_t* tsS,
              const int64_t* tcS, uint32_t nseg, uint32_t lbits, int64_t klo, int64_t khi,
              int stage, void* sortedR, void* sortedS, unsigned long long* count) {
        if (stage == 1) {
            CHECK(staged == nullptr, "rank %d: two R stages", rank);
            staged = R;
            staged_ts = tsR;
            stage_calls++;
            return;
        }
        if (stage == 2) {
            CHECK(staged == R && staged_ts == tsR, "rank %d: REST without its R stage", rank);
            staged = nullptr;
        } else {
            whole_calls++;
        }
        const uint32_t nb = 1u << lbits;
        Range loc(klo, khi, lbits);
        std::vector<Tup> rel[2];
        void* X[2] = {R, S};
        const uint64_t strides[2] = {strideR, strideS}, ns[2] = {nR, nS};
        const int64_t* ts[2] = {tsR, tsS};
        const int64_t* tc[2] = {tcR, tcS};
        for (int r = 0; r < 2; r++) {
            for (uint32_t b = 0; b < nb; b++)
                for (uint32_t j = 0; j < nseg; j++) {
                    const int64_t a = ts[r][(size_t)b * nseg + j], c = tc[r][(size_t)b * nseg + j];
                    for (int64_t e = a; e < a + c; e++) {
                        Tup t = decode(lay, X[r], strides[r], (uint64_t)e, b, loc, klo);
                        CHECK(!(lay == mg::kTuples && t.key == -7 && t.payload == (int64_t)-7),
                              "rank %d: a slack element was read", rank);
                        if (loc.inside(t.key))
                            CHECK(loc.digit(t.key) == b, "rank %d: key %lld in bucket %u, "
                                  "its digit is %u", rank, (long long)t.key, b,
                                  loc.digit(t.key));
                        rel[r].push_back(t);
                    }
                }
            CHECK(rel[r].size() == ns[r], "rank %d rel %d: %zu elements in the segments, n %llu",
                  rank, r, rel[r].size(), (unsigned long long)ns[r]);
            std::sort(rel[r].begin(), rel[r].end(), tup_less);
        }
        unsigned long long c = 0;
        size_t i = 0, j = 0;
        while (i < rel[0].size() && j < rel[1].size()) {
            if (rel[0][i].key < rel[1][j].key) i++;
            else if (rel[0][i].key > rel[1][j].key) j++;
            else {
                const auto k = rel[0][i].key;
                size_t a = i, b = j;
                while (a < rel[0].size() && rel[0][a].key == k) a++;
                while (b < rel[1].size() && rel[1][b].key == k) b++;
                c += (unsigned long long)(a - i) * (b - j);
                i = a;
                j = b;
            }
        }
        memcpy(sortedR, rel[0].data(), rel[0].size() * sizeof(Tup));
        memcpy(sortedS, rel[1].data(), rel[1].size() * sizeof(Tup));
        count[0] = c;
    }
    static Tup decode(int lay, const void* X, uint64_t stride, uint64_t e, uint32_t b,
                      const Range& loc, int64_t klo) {
        if (lay == mg::kTuples) return ((const Tup*)X)[e];
        uint64_t w;
        uint32_t bits;
        if (lay == mg::kWords) {
            w = ((const uint64_t*)X)[e];
            bits = 64;
        } else {
            const uint32_t* lo = (const uint32_t*)X;
            const uint16_t* hi = (const uint16_t*)(lo + stride);
            w = (uint64_t)lo[e] | ((uint64_t)hi[e] << 32);
            bits = 48;
        }
        const uint32_t s1 = loc.s1;
        const uint64_t rel = ((uint64_t)b << s1) | (w >> (bits - s1));
        return make_tup((int64_t)((uint64_t)klo + rel), w & ((1ull << (bits - s1)) - 1));
    }
    bool key_range(const void* R, uint64_t nR, const void* S, uint64_t nS, int64_t* lo,
                   int64_t* hi) {
        if (nR + nS == 0) return false;
        int64_t l = INT64_MAX, h = INT64_MIN;
        for (uint64_t i = 0; i < nR; i++) {
            l = std::min<int64_t>(l, ((const Tup*)R)[i].key);
            h = std::max<int64_t>(h, ((const Tup*)R)[i].key);
        }
        for (uint64_t i = 0; i < nS; i++) {
            l = std::min<int64_t>(l, ((const Tup*)S)[i].key);
            h = std::max<int64_t>(h, ((const Tup*)S)[i].key);
        }
        *lo = l;
        *hi = h;
        return true;
    }
};

typedef mg::CopyColl<HostOps> HostColl;
typedef mg::Rank<HostOps, HostColl> HostRank;

// flags: 1 no planes, 2 one-call join, 4 sampled, 8 exact
// info (out, 8 + 2 G int64): layout, pbits, attempts (rank 0), replans,
//   stage calls (all ranks), whole calls, errors, rank-0 bytes sent, then the
//   per-rank sorted sizes of R and S, then rank 0's phases (mg::Stats: part,
//   tables, wait, join, reduce, busy, rows) in HostOps::tmark clock units
extern "C" int64_t host_mpsm_join(const void* R, uint64_t nR, const void* S, uint64_t nS, int G,
                                  uint32_t flags, uint32_t bucket_bits, int64_t kmin, int64_t kmax, int ovf_rank,
                                  int na_rank, int calls, void* sortedR, void* sortedS,
                                  int64_t* info, char* err, int errcap) {
    g_nerr = 0;
    g_err.clear();
    mg::HostGroup grp(G);
    std::vector<HostOps> ops((size_t)G);
    std::vector<HostColl> coll((size_t)G);
    std::vector<HostRank> ranks((size_t)G);
    for (int g = 0; g < G; g++) {
        ops[g].rank = g;
        ops[g].overflow = g == ovf_rank;
        ops[g].not_applicable = g == na_rank;
        coll[g].grp = &grp;
        coll[g].ops = &ops[g];
        coll[g].me = g;
        ranks[g].ops = &ops[g];
        ranks[g].coll = &coll[g];
        ranks[g].me = g;
        ranks[g].G = G;
    }
    mg::Options o;
    if (kmin <= kmax) {
        o.kmin = kmin;
        o.kmax = kmax;
    } else {
        o.guess_max = nR;
    }
    o.planes = !(flags & 1);
    o.staged = !(flags & 2);
    o.sampled = (flags & 4) ? 1 : (flags & 8) ? 0 : -1;
    o.bucket_bits = bucket_bits;
    std::vector<int64_t> total((size_t)G), onR((size_t)G), onS((size_t)G);
    const uint64_t perR = nR / G, perS = nS / G;
    for (int c = 0; c < calls; c++) {  // a later call reuses the grown buffers
        mg::run_ranks(G, [&](int g) {
            const uint64_t nr = g == G - 1 ? nR - perR * g : perR;
            const uint64_t ns = g == G - 1 ? nS - perS * g : perS;
            uint64_t a = 0, b = 0, loc = 0;
            total[g] = (int64_t)ranks[g].run((const Tup*)R + perR * g, nr,
                                              (const Tup*)S + perS * g, ns, o, &a, &b, &loc);
            onR[g] = (int64_t)a;
            onS[g] = (int64_t)b;
        });
    }
    uint64_t oR = 0, oS = 0;
    for (int g = 0; g < G; g++) {
        CHECK(total[g] == total[0], "ranks disagree on the count");
        memcpy((Tup*)sortedR + oR, ranks[g].sorted[0], onR[g] * sizeof(Tup));
        memcpy((Tup*)sortedS + oS, ranks[g].sorted[1], onS[g] * sizeof(Tup));
        oR += onR[g];
        oS += onS[g];
    }
    int sc = 0, wc = 0;
    for (int g = 0; g < G; g++) {
        sc += ops[g].stage_calls;
        wc += ops[g].whole_calls;
    }
    info[0] = ranks[0].stats.layout;
    info[1] = ranks[0].stats.pbits;
    info[2] = ranks[0].stats.attempts;
    info[3] = ranks[0].stats.replans;
    info[4] = sc;
    info[5] = wc;
    info[6] = g_nerr.load();
    info[7] = (int64_t)ranks[0].stats.sent_B;
    for (int g = 0; g < G; g++) {
        info[8 + 2 * g] = onR[g];
        info[9 + 2 * g] = onS[g];
    }
    // rank 0's phases on the logical clock of HostOps::tmark (units)
    const mg::Stats& st = ranks[0].stats;
    const double ph[7] = {st.part_ms, st.tables_ms, st.wait_ms, st.join_ms, st.reduce_ms,
                          st.busy_ms, st.rows_ms};
    for (int i = 0; i < 7; i++) info[8 + 2 * G + i] = (int64_t)ph[i];
    if (err && errcap > 0) {
        snprintf(err, errcap, "%s", g_err.c_str());
    }
    for (int g = 0; g < G; g++) ranks[g].release_all();
    return total[0];
}
