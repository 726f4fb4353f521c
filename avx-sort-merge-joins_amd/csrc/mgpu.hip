// mgpu.hip -- the multi-GPU join on the device: sortmergejoin_mpsm and
// smj_mgpu_join (include/smj.h).
//
// One process drives G GPUs: rank g is a host thread with device g, two HIP
// streams (kMain: partitions, tables, the local join; kRows: the row
// exchange) and two RCCL communicators over the same devices, one per stream
// (ncclCommInitAll), so that R's rows travel while S is partitioned and S's
// rows while R's tiles are sorted.  The orchestration is mgpu_orch.hpp
// (shared with the CPU tests' host stand-ins); this file gives it
//   DevOps   -- the library's kernels on one rank's device and streams
//               (smj_dev_partition_range_{planes,sampled,...}, the exchange
//               tables, smj_dev_join_segmented_{tables,planes});
//   DevColl  -- grouped ncclSend/ncclRecv (peers in NEXT order) and
//               ncclAllReduce, or, when several ranks share one device (the
//               single-GPU tests of the G-rank protocol), device copies
//               between the ranks' buffers (mg::CopyColl).
// Reference structure: the T join threads of joincommon.c:118-165 on their
// chunks (:127-139), the co-partition exchange of
// sortmergejoin_multiway.c:463-556, NEXT peer order numa_shuffle.c:83.
#include <string.h>
#include <sys/time.h>

#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include <rccl/rccl.h>

#include "../../include/smj.h"
#include "mgpu_orch.hpp"
#include "smj_common.hpp"
#include "smj_internal.hpp"

namespace smj {
bool key_range(Workspace* ws, const Tup* const* rels, const uint64_t* ns, int nrel,
               int64_t* lo, int64_t* hi, hipStream_t st);
uint64_t materialize_append_on(Workspace* ws, hipStream_t st, const Tup* r, uint64_t nR,
                               const Tup* s, uint64_t nS, chainedtuplebuffer_t* cb);
bool materialize_on();
}  // namespace smj

using namespace smj;

#define SMJ_NCCL(call)                                                              \
    do {                                                                            \
        ncclResult_t r_ = (call);                                                   \
        if (r_ != ncclSuccess) {                                                    \
            fprintf(stderr, "[ERROR] smj mpsm: RCCL %s at %s:%d: %s\n", #call,     \
                    __FILE__, __LINE__, ncclGetErrorString(r_));                    \
            abort();                                                                \
        }                                                                           \
    } while (0)

namespace {

// ---------------------------------------------------------------------------
// the device work of one rank
// ---------------------------------------------------------------------------
struct DevOps {
    static constexpr int kTupleBytes = (int)sizeof(Tup);
    int device = 0;
    hipStream_t st[2] = {nullptr, nullptr};
    hipEvent_t ev[mg::kNumEvents] = {};
    hipEvent_t tev[mg::kNumTMarks] = {};  // timing marks (the phases of mg::Stats)
    uint32_t tset = 0;                    // marks recorded since the rank was made
    Workspace* ws = nullptr;

    smj_workspace* w() const { return (smj_workspace*)ws; }
    bool can_pack() const { return sizeof(Tup) == 16; }
    void* alloc(size_t b) {
        void* p = nullptr;
        SMJ_CHECK(hipMalloc(&p, b ? b : 16));
        return p;
    }
    void release(void* p) { SMJ_CHECK(hipFree(p)); }
    void* host_alloc(size_t b) {
        void* p = nullptr;
        SMJ_CHECK(hipHostMalloc(&p, b ? b : 16, hipHostMallocDefault));
        return p;
    }
    void host_release(void* p) { SMJ_CHECK(hipHostFree(p)); }
    void copy(void* d, const void* s, size_t b, int sid) {
        if (b) SMJ_CHECK(hipMemcpyAsync(d, s, b, hipMemcpyDefault, st[sid]));
    }
    void to_host(void* h, const void* d, size_t b, int sid) {
        if (b) SMJ_CHECK(hipMemcpyAsync(h, d, b, hipMemcpyDeviceToHost, st[sid]));
    }
    void to_dev(void* d, const void* h, size_t b, int sid) {
        if (b) SMJ_CHECK(hipMemcpyAsync(d, h, b, hipMemcpyHostToDevice, st[sid]));
    }
    void fill_u32(void* p, uint32_t v, size_t count, int sid) {
        if (count) SMJ_CHECK(hipMemsetD32Async((hipDeviceptr_t)p, (int)v, count, st[sid]));
    }
    void record(int e, int sid) { SMJ_CHECK(hipEventRecord(ev[e], st[sid])); }
    void wait(int sid, int e) { SMJ_CHECK(hipStreamWaitEvent(st[sid], ev[e], 0)); }
    void host_wait(int e) { SMJ_CHECK(hipEventSynchronize(ev[e])); }
    void sync(int sid) { SMJ_CHECK(hipStreamSynchronize(st[sid])); }
    void tmark(int m, int sid) {
        SMJ_CHECK(hipEventRecord(tev[m], st[sid]));
        tset |= 1u << m;
    }
    double tspan(int a, int b) {
        if (!((tset >> a) & 1) || !((tset >> b) & 1)) return 0.0;
        float ms = 0.f;
        SMJ_CHECK(hipEventElapsedTime(&ms, tev[a], tev[b]));
        return ms;
    }
    uint32_t shards() { return smj_sampled_shards(); }
    uint64_t sampled_capacity(uint64_t n, uint32_t nbits) { return smj_sampled_capacity(n, nbits); }
    int part_planes(const void* in, uint64_t n, void* out, uint64_t stride, uint32_t nbits,
                    int64_t kmin, int64_t kmax, int64_t* ss, int64_t* sc, uint32_t* flags) {
        return smj_dev_partition_range_planes(w(), (const tuple_t*)in, n, out, stride, nbits,
                                              kmin, kmax, ss, sc, flags, st[0]);
    }
    int part_sampled(const void* in, uint64_t n, void* out, uint32_t nbits, int64_t kmin,
                     int64_t kmax, int packed, int64_t* ss, int64_t* sc, uint32_t* flags) {
        return smj_dev_partition_range_sampled(w(), (const tuple_t*)in, n, out, nbits, kmin,
                                               kmax, packed, ss, sc, flags, st[0]);
    }
    int part_shards(const void* in, uint64_t n, void* out, uint32_t nbits, int64_t kmin,
                    int64_t kmax, int packed, int64_t* ss, int64_t* sc, uint32_t* flags) {
        return smj_dev_partition_range_shards(w(), (const tuple_t*)in, n, out, nbits, kmin, kmax,
                                              packed, ss, sc, flags, st[0]);
    }
    void part_exact(const void* in, uint64_t n, void* out, uint32_t nbits, int64_t kmin,
                    int64_t kmax, int64_t* hist) {
        smj_dev_partition_range(w(), (const tuple_t*)in, n, (tuple_t*)out, nbits, kmin, kmax,
                                hist, st[0]);
    }
    int part_exact_packed(const void* in, uint64_t n, void* out, uint32_t nbits, int64_t kmin,
                          int64_t kmax, int64_t* hist, uint32_t* bad) {
        return smj_dev_partition_range_packed(w(), (const tuple_t*)in, n, (uint64_t*)out, nbits,
                                              kmin, kmax, hist, bad, st[0]);
    }
    void hist_tables(const int64_t* hist, uint32_t F, uint32_t K, int64_t* ss, int64_t* sc) {
        smj::hist_tables(hist, F, K, ss, sc, st[0]);
    }
    void xsend(const int64_t* ss, const int64_t* sc, const uint32_t* flags, uint32_t F,
               uint32_t K, uint32_t G, uint32_t U, int64_t* msg, int64_t* chunk) {
        smj::xsend(ss, sc, flags, F, K, G, U, msg, chunk, st[0]);
    }
    void xrecv(const int64_t* msg, const int64_t* chunk, uint32_t G, uint32_t rank,
               uint32_t mine, uint32_t K, uint32_t nb, uint64_t cap, int64_t* ts, int64_t* tc,
               int64_t* summary) {
        smj::xrecv(msg, chunk, G, rank, mine, K, nb, cap, ts, tc, summary, st[0]);
    }
    void join(int lay, void* R, uint64_t strideR, uint64_t nR, const int64_t* tsR,
              const int64_t* tcR, void* S, uint64_t strideS, uint64_t nS, const int64_t* tsS,
              const int64_t* tcS, uint32_t nseg, uint32_t lbits, int64_t klo, int64_t khi,
              int stage, void* sortedR, void* sortedS, unsigned long long* count) {
        const uint32_t sf = stage == 1 ? SMJ_SEG_STAGE_R : stage == 2 ? SMJ_SEG_STAGE_REST : 0u;
        if (lay == mg::kPlanes)
            smj_dev_join_segmented_planes(w(), R, strideR, nR, tsR, tcR, S, strideS, nS, tsS,
                                          tcS, nseg, lbits, klo, khi, sf, (tuple_t*)sortedR,
                                          (tuple_t*)sortedS, count, st[0]);
        else
            smj_dev_join_segmented_tables(w(), R, nR, tsR, tcR, S, nS, tsS, tcS, nseg, lbits,
                                          klo, khi, sf | (lay == mg::kWords ? SMJ_SEG_PACKED : 0u),
                                          (tuple_t*)sortedR, (tuple_t*)sortedS, count, st[0]);
    }
    bool key_range(const void* R, uint64_t nR, const void* S, uint64_t nS, int64_t* lo,
                   int64_t* hi) {
        const Tup* rels[2] = {(const Tup*)R, (const Tup*)S};
        const uint64_t ns[2] = {nR, nS};
        return smj::key_range(ws, rels, ns, 2, lo, hi, st[0]);
    }
};

// ---------------------------------------------------------------------------
// collectives: RCCL, one communicator per stream; or device copies
// ---------------------------------------------------------------------------
struct DevColl {
    bool rccl = true;
    ncclComm_t comm[2] = {nullptr, nullptr};
    DevOps* ops = nullptr;
    int me = 0;
    mg::CopyColl<DevOps> copy;

    void exchange(int sid, const std::vector<mg::Piece>& sends,
                  const std::vector<mg::Piece>& recvs) {
        if (!rccl) {
            copy.exchange(sid, sends, recvs);
            return;
        }
        // a rank's pieces to itself are a device copy (the k-th sent with the
        // k-th received); the others one group of sends and receives, issued
        // per peer in NEXT order as the pieces come
        std::vector<const mg::Piece*> self_s, self_r;
        SMJ_NCCL(ncclGroupStart());
        for (const mg::Piece& p : sends) {
            if (p.peer == me) self_s.push_back(&p);
            else if (p.bytes)
                SMJ_NCCL(ncclSend(p.ptr, p.bytes, ncclUint8, p.peer, comm[sid], ops->st[sid]));
        }
        for (const mg::Piece& p : recvs) {
            if (p.peer == me) self_r.push_back(&p);
            else if (p.bytes)
                SMJ_NCCL(ncclRecv(p.ptr, p.bytes, ncclUint8, p.peer, comm[sid], ops->st[sid]));
        }
        SMJ_NCCL(ncclGroupEnd());
        if (self_s.size() != self_r.size()) {
            fprintf(stderr, "[ERROR] smj mpsm: %zu pieces to self, %zu from self\n",
                    self_s.size(), self_r.size());
            abort();
        }
        for (size_t k = 0; k < self_s.size(); k++)
            ops->copy(self_r[k]->ptr, self_s[k]->ptr, self_s[k]->bytes, sid);
    }
    void allreduce_sum_u64(int sid, unsigned long long* p) {
        if (!rccl) {
            copy.allreduce_sum_u64(sid, p);
            return;
        }
        SMJ_NCCL(ncclAllReduce(p, p, 1, ncclUint64, ncclSum, comm[sid], ops->st[sid]));
    }
    // a host value over the ranks (0 sum, 1 min, 2 max): in one process
    // through the host group, across processes one 8-byte ncclAllReduce
    int64_t* red_dev = nullptr;
    int64_t* red_host = nullptr;
    int64_t reduce(int64_t v, int op) {
        if (!rccl) return copy.reduce(v, op);
        if (!red_dev) {
            red_dev = (int64_t*)ops->alloc(8);
            red_host = (int64_t*)ops->host_alloc(8);
        }
        *red_host = v;
        ops->to_dev(red_dev, red_host, 8, mg::kMain);
        SMJ_NCCL(ncclAllReduce(red_dev, red_dev, 1, ncclInt64,
                               op == 1 ? ncclMin : op == 2 ? ncclMax : ncclSum, comm[mg::kMain],
                               ops->st[mg::kMain]));
        ops->to_host(red_host, red_dev, 8, mg::kMain);
        ops->sync(mg::kMain);
        return *red_host;
    }
    void release() {
        if (red_dev) ops->release(red_dev);
        if (red_host) ops->host_release(red_host);
        red_dev = red_host = nullptr;
    }
};

typedef mg::Rank<DevOps, DevColl> DevRank;

// One rank's device state, kept across calls (streams, events, workspace and
// the rank's sticky exchange buffers).
struct RankCtx {
    DevOps ops;
    DevColl coll;
    DevRank rank;
    Workspace ws;
    void* inbuf[2] = {nullptr, nullptr};  // staged input slices
    size_t inbytes[2] = {0, 0};
    int device = 0;

    explicit RankCtx(int dev) : device(dev) {
        SMJ_CHECK(hipSetDevice(dev));
        for (int s = 0; s < 2; s++)
            SMJ_CHECK(hipStreamCreateWithFlags(&ops.st[s], hipStreamNonBlocking));
        for (auto& e : ops.ev) SMJ_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        for (auto& e : ops.tev) SMJ_CHECK(hipEventCreate(&e));
        ops.device = dev;
        ops.ws = &ws;
        coll.ops = &ops;
        rank.ops = &ops;
        rank.coll = &coll;
    }
    ~RankCtx() {
        (void)hipSetDevice(device);
        rank.release_all();
        coll.release();
        for (int r = 0; r < 2; r++)
            if (inbuf[r]) (void)hipFree(inbuf[r]);
        for (auto& e : ops.ev) (void)hipEventDestroy(e);
        for (auto& e : ops.tev) (void)hipEventDestroy(e);
        for (int s = 0; s < 2; s++) (void)hipStreamDestroy(ops.st[s]);
    }
};

// The process's ranks for one configuration (G ranks, RCCL or copies); a
// call with another configuration releases them first.  Calls are
// serialised: every call uses all of the configuration's devices.
struct Group {
    int G = 0;
    bool rccl = true;
    std::vector<std::unique_ptr<RankCtx>> ranks;
    std::vector<ncclComm_t> comms[2];
    std::unique_ptr<mg::HostGroup> host;

    ~Group() {
        for (auto& c : comms)
            for (ncclComm_t x : c)
                if (x) (void)ncclCommDestroy(x);
        ranks.clear();
    }
};

std::mutex g_mu;
std::unique_ptr<Group> g_group;

Group& group_for(int G, bool rccl) {
    if (g_group && g_group->G == G && g_group->rccl == rccl) return *g_group;
    g_group.reset();
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        fprintf(stderr, "[ERROR] smj: no HIP device visible; the MI355X library has no CPU "
                        "fallback.\n");
        abort();
    }
    if (rccl && G > ndev) {
        fprintf(stderr, "[ERROR] smj mpsm: %d RCCL ranks need %d devices (%d visible); "
                        "SMJ_MG_COPY runs ranks on shared devices\n", G, G, ndev);
        abort();
    }
    std::unique_ptr<Group> g(new Group());
    g->G = G;
    g->rccl = rccl;
    g->host.reset(new mg::HostGroup(G));
    for (int r = 0; r < G; r++) g->ranks.emplace_back(new RankCtx(r % ndev));
    if (rccl) {
        std::vector<int> devs((size_t)G);
        for (int r = 0; r < G; r++) devs[r] = r;
        for (int c = 0; c < 2; c++) {
            g->comms[c].assign((size_t)G, nullptr);
            SMJ_NCCL(ncclCommInitAll(g->comms[c].data(), G, devs.data()));
        }
    }
    for (int r = 0; r < G; r++) {
        RankCtx& rc = *g->ranks[r];
        rc.rank.me = r;
        rc.rank.G = G;
        rc.coll.rccl = rccl;
        rc.coll.me = r;
        if (rccl)
            for (int c = 0; c < 2; c++) rc.coll.comm[c] = g->comms[c][r];
        rc.coll.copy.grp = g->host.get();
        rc.coll.copy.ops = &rc.ops;
        rc.coll.copy.me = r;
    }
    g_group = std::move(g);
    return *g_group;
}

// device of a pointer (-1: host memory)
int ptr_device(const void* p) {
    if (!p) return -1;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    if (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged) return a.device;
    return -1;
}

// Rank r's slice [off, off + n) of a caller relation on the rank's device: in
// place when it already lies there, else copied (host -> device, or peer).
const void* stage_slice(RankCtx& rc, int rel, const Tup* base, uint64_t off, uint64_t n) {
    const Tup* p = base + off;
    if (n == 0) return p;
    if (ptr_device(base) == rc.device) return p;
    const size_t b = n * sizeof(Tup);
    if (rc.inbytes[rel] < b) {
        if (rc.inbuf[rel]) SMJ_CHECK(hipFree(rc.inbuf[rel]));
        SMJ_CHECK(hipMalloc(&rc.inbuf[rel], b));
        rc.inbytes[rel] = b;
    }
    SMJ_CHECK(hipMemcpyAsync(rc.inbuf[rel], p, b, hipMemcpyDefault, rc.ops.st[0]));
    return rc.inbuf[rel];
}

struct CallArgs {
    const Tup* R;
    uint64_t nR;
    const Tup* S;
    uint64_t nS;
    // smj_mgpu_join_slices: rank g's slices (R and S above unused)
    const Tup* const* Rs = nullptr;
    const uint64_t* nRs = nullptr;
    const Tup* const* Ss = nullptr;
    const uint64_t* nSs = nullptr;
    mg::Options opt;
    Tup* sortedR = nullptr;  // host or device destinations of the sorted shares
    Tup* sortedS = nullptr;
    int mat = 0;             // materialise into per-rank buffers
    result_t* res = nullptr;
};

struct CallOut {
    uint64_t total = 0;
    std::vector<uint64_t> nR, nS, local;
    mg::Stats stats;               // rank 0's
    std::vector<mg::Stats> ranks;  // every rank's
    double ms = 0;
};

// the last call's per-rank statistics (smj_mgpu_last_stats; under g_mu)
std::vector<mg::Stats> g_last_stats;
double g_last_ms = 0;

void fill_stats(const mg::Stats& x, double ms, smj_mgpu_stats* o) {
    o->layout = x.layout;
    o->pbits = x.pbits;
    o->attempts = x.attempts;
    o->replans = x.replans;
    o->sent_bytes = x.sent_B;
    o->recv_bytes = x.recv_B;
    o->key_min = x.kmin;
    o->key_max = x.kmax;
    o->ms = ms;
    o->partition_ms = x.part_ms;
    o->tables_ms = x.tables_ms;
    o->wait_ms = x.wait_ms;
    o->join_ms = x.join_ms;
    o->reduce_ms = x.reduce_ms;
    o->busy_ms = x.busy_ms;
    o->rows_ms = x.rows_ms;
}

// level-1 buckets per rank: 2^8 (the 1-GPU join's fan-out), more while a
// bucket would exceed the tile pass's kLocalBucketCap (the 1024M-per-rank
// join of BASELINE configs[4] on one GPU: 2^9)
uint32_t bucket_bits_for(uint64_t n_per_rank) {
    uint32_t b = 8;
    while (b < mg::kMaxPartBits && (n_per_rank >> b) > mg::kLocalBucketCap) b++;
    return b;
}

void run_call(Group& grp, CallArgs a, CallOut& out) {
    const int G = grp.G;
    uint64_t share = std::max(a.nR, a.nS) / (uint64_t)G;
    if (a.Rs)
        for (int r = 0; r < G; r++) share = std::max(share, std::max(a.nRs[r], a.nSs[r]));
    a.opt.bucket_bits = bucket_bits_for(share);
    out.nR.assign((size_t)G, 0);
    out.nS.assign((size_t)G, 0);
    out.local.assign((size_t)G, 0);
    std::vector<uint64_t> total((size_t)G, 0);
    // joincommon.c:127-139: thread i takes [i n / T, (i + 1) n / T), the last
    // one the rest
    const uint64_t perR = a.nR / G, perS = a.nS / G;
    struct timeval t0, t1;
    gettimeofday(&t0, NULL);
    mg::run_ranks(G, [&](int r) {
        RankCtx& rc = *grp.ranks[r];
        SMJ_CHECK(hipSetDevice(rc.device));
        uint64_t nr = r == G - 1 ? a.nR - perR * r : perR;
        uint64_t ns = r == G - 1 ? a.nS - perS * r : perS;
        const void *R, *S;
        if (a.Rs) {  // the rank's own slices (on its GPU: read in place)
            nr = a.nRs[r];
            ns = a.nSs[r];
            R = stage_slice(rc, 0, a.Rs[r], 0, nr);
            S = stage_slice(rc, 1, a.Ss[r], 0, ns);
        } else {
            R = stage_slice(rc, 0, a.R, perR * r, nr);
            S = stage_slice(rc, 1, a.S, perS * r, ns);
        }
        uint64_t onR = 0, onS = 0, loc = 0;
        total[r] = rc.rank.run(R, nr, S, ns, a.opt, &onR, &onS, &loc);
        out.nR[r] = onR;
        out.nS[r] = onS;
        out.local[r] = loc;
        // the sorted shares, concatenated in rank order (one contiguous key
        // range per rank, ascending)
        if (a.sortedR || a.sortedS) {
            grp.host->barrier();
            uint64_t oR = 0, oS = 0;
            for (int g = 0; g < r; g++) {
                oR += out.nR[g];
                oS += out.nS[g];
            }
            if (a.sortedR) rc.ops.copy(a.sortedR + oR, rc.rank.sorted[0], onR * sizeof(Tup), 0);
            if (a.sortedS) rc.ops.copy(a.sortedS + oS, rc.rank.sorted[1], onS * sizeof(Tup), 0);
            rc.ops.sync(0);
        }
        if (a.mat && a.res) {
            chainedtuplebuffer_t* cb = chainedtuplebuffer_init();
            materialize_append_on(&rc.ws, rc.ops.st[0], (const Tup*)rc.rank.sorted[0], onR,
                                  (const Tup*)rc.rank.sorted[1], onS, cb);
            a.res->resultlist[r].results = cb;
        }
    });
    gettimeofday(&t1, NULL);
    for (int r = 1; r < G; r++)
        if (total[r] != total[0]) {
            fprintf(stderr, "[ERROR] smj mpsm: ranks disagree on the count (%llu, %llu)\n",
                    (unsigned long long)total[0], (unsigned long long)total[r]);
            abort();
        }
    out.total = total[0];
    out.stats = grp.ranks[0]->rank.stats;
    out.ranks.clear();
    for (int r = 0; r < G; r++) out.ranks.push_back(grp.ranks[r]->rank.stats);
    out.ms = (t1.tv_sec - t0.tv_sec) * 1e3 + (t1.tv_usec - t0.tv_usec) * 1e-3;
    g_last_stats = out.ranks;
    g_last_ms = out.ms;
}

// the rank with the longest busy span (the reference prints thread 0's
// phases after a barrier; here the slowest GPU sets the step)
const mg::Stats& slowest(const CallOut& o) {
    size_t k = 0;
    for (size_t r = 1; r < o.ranks.size(); r++)
        if (o.ranks[r].busy_ms > o.ranks[k].busy_ms) k = r;
    return o.ranks[k];
}

}  // namespace

namespace smj {

// sortmergejoin_mpsm: NTHREADS ranks, at most one per visible GPU (the
// reference's T threads become T GPUs; a 1-GPU host runs one rank), RCCL
// collectives; the key range guessed as 1..|R| like sortmergejoin_multiway
// (the reference's radix shift assumes it, sortmergejoin_multiway.c:372-376)
// and verified by the exchange partition.
result_t* mpsm_api(relation_t* relR, relation_t* relS, joinconfig_t* joincfg, int mat) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        fprintf(stderr, "[ERROR] smj: no HIP device visible; the MI355X library has no CPU "
                        "fallback.\n");
        abort();
    }
    const int T = joincfg->NTHREADS > 0 ? joincfg->NTHREADS : 1;
    const int G = T < ndev ? T : ndev;
    std::lock_guard<std::mutex> lk(g_mu);
    int dev0 = 0;
    SMJ_CHECK(hipGetDevice(&dev0));
    Group& grp = group_for(G, true);
    CallArgs a;
    a.R = (const Tup*)relR->tuples;
    a.nR = relR->num_tuples;
    a.S = (const Tup*)relS->tuples;
    a.nS = relS->num_tuples;
    a.opt.guess_max = a.nR;
    a.mat = (mat < 0 ? materialize_on() : mat > 0) ? 1 : 0;
    result_t* res = (result_t*)malloc(sizeof(result_t));
    res->nthreads = T;
    res->resultlist = (threadresult_t*)calloc((size_t)T, sizeof(threadresult_t));
    a.res = res;
    CallOut o;
    run_call(grp, a, o);
    SMJ_CHECK(hipSetDevice(dev0));
    res->totalresults = (int64_t)o.total;
    for (int r = 0; r < G; r++) {
        res->resultlist[r].nresults = (int64_t)o.local[r];
        res->resultlist[r].threadid = (uint32_t)r;
    }
    if (!getenv("SMJ_QUIET")) {
        // the reference's stats lines (joincommon.c:176-196): cumulative
        // phase ends of the slowest rank, device nanoseconds (the reference
        // prints cycles): partitioning = the range partitions and their
        // tables, then the exchange (the main stream's wait for the rows:
        // sortmergejoin_multiway.c:463-556 gathers the co-partitions there),
        // then the local join (sort + merge-join count), then the all-reduce
        const mg::Stats& x = slowest(o);
        const double p = x.part_ms + x.tables_ms, xw = p + x.wait_ms, j = xw + x.join_ms;
        auto ns = [](double ms) { return (unsigned long long)(ms * 1e6); };
        fprintf(stdout, "Total, Partitioning, Sort, First-Merge, Merge, Join\n");
        fprintf(stdout, "%llu, %llu, %llu, %llu, %llu, %llu\n", ns(x.busy_ms), ns(p), ns(xw),
                ns(xw), ns(j), ns(x.busy_ms));
        fprintf(stdout, "[INFO ] mpsm: %d GPU%s, exchange in %s, 2^%u partitions, %d "
                        "attempts\n", G, G > 1 ? "s" : "", mg::layout_name(o.stats.layout),
                o.stats.pbits, o.stats.attempts);
        fprintf(stdout, "[INFO ] mpsm phases (ms, slowest rank): partition %.3f, tables %.3f, "
                        "exchange wait %.3f, local join %.3f, all-reduce %.3f, busy %.3f; "
                        "rows stream %.3f\n", x.part_ms, x.tables_ms, x.wait_ms, x.join_ms,
                x.reduce_ms, x.busy_ms, x.rows_ms);
        fprintf(stderr, "NUM-TUPLES = %lld TOTAL-TIME-USECS = %.4lf ", (long long)a.nS,
                o.ms * 1e3);
        fprintf(stderr, "TUPLES-PER-SECOND = %.4lf ", a.nS / (o.ms * 1e-3));
        fflush(stdout);
        fflush(stderr);
    }
    return res;
}

}  // namespace smj

extern "C" {

int64_t smj_mgpu_join(const tuple_t* R, uint64_t nR, const tuple_t* S, uint64_t nS, int nranks,
                      uint32_t flags, int64_t key_min, int64_t key_max, tuple_t* sortedR,
                      tuple_t* sortedS, uint64_t* rank_counts, smj_mgpu_stats* stats) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        fprintf(stderr, "[ERROR] smj: no HIP device visible; the MI355X library has no CPU "
                        "fallback.\n");
        abort();
    }
    const int G = nranks > 0 ? nranks : ndev;
    if (G > 64) {
        fprintf(stderr, "[ERROR] smj_mgpu_join: %d ranks (at most 64)\n", G);
        abort();
    }
    std::lock_guard<std::mutex> lk(g_mu);
    int dev0 = 0;
    SMJ_CHECK(hipGetDevice(&dev0));
    Group& grp = group_for(G, !(flags & SMJ_MG_COPY));
    CallArgs a;
    a.R = (const Tup*)R;
    a.nR = nR;
    a.S = (const Tup*)S;
    a.nS = nS;
    if (key_min <= key_max) {
        a.opt.kmin = key_min;
        a.opt.kmax = key_max;
    } else {
        a.opt.guess_max = nR;
    }
    a.opt.planes = !(flags & SMJ_MG_NOPLANES);
    a.opt.staged = !(flags & SMJ_MG_ONECALL);
    a.opt.sampled = (flags & SMJ_MG_SAMPLED) ? 1 : (flags & SMJ_MG_EXACT) ? 0 : -1;
    a.sortedR = (Tup*)sortedR;
    a.sortedS = (Tup*)sortedS;
    CallOut o;
    run_call(grp, a, o);
    SMJ_CHECK(hipSetDevice(dev0));
    if (rank_counts)
        for (int r = 0; r < G; r++) {
            rank_counts[2 * r] = o.nR[r];
            rank_counts[2 * r + 1] = o.nS[r];
        }
    if (stats) fill_stats(o.stats, o.ms, stats);
    return (int64_t)o.total;
}

int64_t smj_mgpu_join_slices(const tuple_t* const* R, const uint64_t* nR,
                             const tuple_t* const* S, const uint64_t* nS, int nranks,
                             uint32_t flags, int64_t key_min, int64_t key_max,
                             uint64_t* rank_counts, smj_mgpu_stats* stats) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        fprintf(stderr, "[ERROR] smj: no HIP device visible; the MI355X library has no CPU "
                        "fallback.\n");
        abort();
    }
    if (nranks < 1 || nranks > 64 || !R || !S || !nR || !nS) {
        fprintf(stderr, "[ERROR] smj_mgpu_join_slices: %d ranks (1..64) and four arrays\n",
                nranks);
        abort();
    }
    const int G = nranks;
    std::lock_guard<std::mutex> lk(g_mu);
    int dev0 = 0;
    SMJ_CHECK(hipGetDevice(&dev0));
    Group& grp = group_for(G, !(flags & SMJ_MG_COPY));
    CallArgs a;
    a.R = a.S = nullptr;
    a.nR = a.nS = 0;
    uint64_t totR = 0;
    for (int r = 0; r < G; r++) {
        a.nR += nR[r];
        a.nS += nS[r];
        totR += nR[r];
    }
    a.Rs = (const Tup* const*)R;
    a.nRs = nR;
    a.Ss = (const Tup* const*)S;
    a.nSs = nS;
    if (key_min <= key_max) {
        a.opt.kmin = key_min;
        a.opt.kmax = key_max;
    } else {
        a.opt.guess_max = totR;
    }
    a.opt.planes = !(flags & SMJ_MG_NOPLANES);
    a.opt.staged = !(flags & SMJ_MG_ONECALL);
    a.opt.sampled = (flags & SMJ_MG_SAMPLED) ? 1 : (flags & SMJ_MG_EXACT) ? 0 : -1;
    CallOut o;
    run_call(grp, a, o);
    SMJ_CHECK(hipSetDevice(dev0));
    if (rank_counts)
        for (int r = 0; r < G; r++) {
            rank_counts[2 * r] = o.nR[r];
            rank_counts[2 * r + 1] = o.nS[r];
        }
    if (stats) fill_stats(o.stats, o.ms, stats);
    return (int64_t)o.total;
}

smj_workspace* smj_mgpu_group_workspace(int rank) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_group || rank < 0 || rank >= g_group->G) return nullptr;
    return g_group->ranks[rank]->ops.w();
}

int smj_mgpu_last_stats(int rank, smj_mgpu_stats* out) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (rank < 0 || rank >= (int)g_last_stats.size() || !out) return -1;
    fill_stats(g_last_stats[rank], g_last_ms, out);
    return 0;
}

int smj_mgpu_last_sorted(int rank, tuple_t** sortedR, uint64_t* nR, tuple_t** sortedS,
                         uint64_t* nS) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_group || rank < 0 || rank >= g_group->G) return -1;
    DevRank& k = g_group->ranks[rank]->rank;
    uint64_t n[2] = {0, 0};
    k.sorted_sizes(&n[0], &n[1]);
    if (sortedR) *sortedR = (tuple_t*)k.sorted[0];
    if (sortedS) *sortedS = (tuple_t*)k.sorted[1];
    if (nR) *nR = n[0];
    if (nS) *nS = n[1];
    return 0;
}

void smj_mgpu_release(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_group.reset();
    g_last_stats.clear();
}

// ---- one rank of a multi-process group (one process per GPU: bench.py
// --gpus N under torch.distributed.run).  The two communicators come from one
// id: ncclCommInitRank, then ncclCommSplit for the row exchange's own.
struct smj_mgpu_comm {
    RankCtx* rc;
    ncclComm_t comm[2];
};

int smj_mgpu_unique_id(void* out, int cap) {
    if (cap < (int)sizeof(ncclUniqueId)) return -(int)sizeof(ncclUniqueId);
    ncclUniqueId id;
    SMJ_NCCL(ncclGetUniqueId(&id));
    memcpy(out, &id, sizeof(id));
    return (int)sizeof(id);
}

smj_mgpu_comm* smj_mgpu_comm_init(const void* id, int nranks, int rank) {
    if (nranks < 1 || rank < 0 || rank >= nranks) {
        fprintf(stderr, "[ERROR] smj_mgpu_comm_init: rank %d of %d\n", rank, nranks);
        abort();
    }
    int dev = 0;
    SMJ_CHECK(hipGetDevice(&dev));
    smj_mgpu_comm* c = new smj_mgpu_comm();
    c->rc = new RankCtx(dev);
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    SMJ_NCCL(ncclCommInitRank(&c->comm[0], nranks, uid, rank));
    SMJ_NCCL(ncclCommSplit(c->comm[0], 0, rank, &c->comm[1], NULL));
    RankCtx& rc = *c->rc;
    rc.rank.me = rank;
    rc.rank.G = nranks;
    rc.coll.rccl = true;
    rc.coll.me = rank;
    rc.coll.comm[0] = c->comm[0];
    rc.coll.comm[1] = c->comm[1];
    return c;
}

int64_t smj_mgpu_rank_join(smj_mgpu_comm* c, const tuple_t* R, uint64_t nR, const tuple_t* S,
                           uint64_t nS, uint32_t flags, int64_t key_min, int64_t key_max,
                           uint64_t guess_max, tuple_t** sortedR, uint64_t* nR_out,
                           tuple_t** sortedS, uint64_t* nS_out, smj_mgpu_stats* stats) {
    RankCtx& rc = *c->rc;
    int dev0 = 0;
    SMJ_CHECK(hipGetDevice(&dev0));
    SMJ_CHECK(hipSetDevice(rc.device));
    mg::Options o;
    if (key_min <= key_max) {
        o.kmin = key_min;
        o.kmax = key_max;
    } else {
        o.guess_max = guess_max;
    }
    o.planes = !(flags & SMJ_MG_NOPLANES);
    o.staged = !(flags & SMJ_MG_ONECALL);
    o.sampled = (flags & SMJ_MG_SAMPLED) ? 1 : (flags & SMJ_MG_EXACT) ? 0 : -1;
    // every rank must take the same level-1 width: from the largest share
    // (an 8-byte all-reduce)
    const uint64_t nmax = (uint64_t)rc.coll.reduce((int64_t)(nR > nS ? nR : nS), 2);
    o.bucket_bits = bucket_bits_for(nmax);
    struct timeval t0, t1;
    gettimeofday(&t0, NULL);
    const void* r = stage_slice(rc, 0, (const Tup*)R, 0, nR);
    const void* s = stage_slice(rc, 1, (const Tup*)S, 0, nS);
    uint64_t onR = 0, onS = 0, loc = 0;
    const uint64_t total = rc.rank.run(r, nR, s, nS, o, &onR, &onS, &loc);
    gettimeofday(&t1, NULL);
    if (sortedR) *sortedR = (tuple_t*)rc.rank.sorted[0];
    if (sortedS) *sortedS = (tuple_t*)rc.rank.sorted[1];
    if (nR_out) *nR_out = onR;
    if (nS_out) *nS_out = onS;
    if (stats)
        fill_stats(rc.rank.stats,
                   (t1.tv_sec - t0.tv_sec) * 1e3 + (t1.tv_usec - t0.tv_usec) * 1e-3, stats);
    SMJ_CHECK(hipSetDevice(dev0));
    return (int64_t)total;
}

void smj_mgpu_rank_sorted(smj_mgpu_comm* c, tuple_t* outR, tuple_t* outS) {
    RankCtx& rc = *c->rc;
    int dev0 = 0;
    SMJ_CHECK(hipGetDevice(&dev0));
    SMJ_CHECK(hipSetDevice(rc.device));
    uint64_t n[2] = {0, 0};
    rc.rank.sorted_sizes(&n[0], &n[1]);
    if (outR) rc.ops.copy(outR, rc.rank.sorted[0], n[0] * sizeof(Tup), mg::kMain);
    if (outS) rc.ops.copy(outS, rc.rank.sorted[1], n[1] * sizeof(Tup), mg::kMain);
    rc.ops.sync(mg::kMain);
    SMJ_CHECK(hipSetDevice(dev0));
}

smj_workspace* smj_mgpu_comm_workspace(smj_mgpu_comm* c) { return c->rc->ops.w(); }

void smj_mgpu_comm_destroy(smj_mgpu_comm* c) {
    if (!c) return;
    delete c->rc;
    for (int i = 1; i >= 0; i--) (void)ncclCommDestroy(c->comm[i]);
    delete c;
}

}  // extern "C"
