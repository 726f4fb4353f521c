// smj_internal.hpp -- host-side internal interfaces between the .hip units.
#pragma once
#include <sched.h>

#include <chrono>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include <hip/hip_ext.h>

#include "smj_common.hpp"

namespace smj {

constexpr uint32_t kNarrowDigitBits = 12;  // widest digit of a single pass
// widest level-2 digit (groups per bucket): k_preft stages 64 prefix rows of
// 2^kMaxD2 + 1 entries in LDS
constexpr uint32_t kMaxD2 = 10;

// reference partition digit (runtime mask/shift), see smj_common.hpp
typedef RefDigit Digit32;

// wave-uniform 32/64-bit values into SGPRs
__device__ __forceinline__ uint32_t uniform32(uint32_t x) {
    return __builtin_amdgcn_readfirstlane(x);
}
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
    return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32) |
           __builtin_amdgcn_readfirstlane((uint32_t)x);
}

// level-1 digit of a range plan held by value (in SGPRs)
struct PlanDigitV {
    RangePlan p;
    __device__ __forceinline__ uint32_t operator()(const Tup& t) const {
        return plan_d1(p, plan_rel(p, tup_key(t)));
    }
};

// level-1 digit of a device-resident range plan.  Kernels call load() once:
// the plan is read a single time instead of at every digit (the output
// stores may alias it, so the compiler would reload it).
struct PlanDigit1 {
    const RangePlan* plan;
    __device__ __forceinline__ PlanDigitV load() const {
        RangePlan q = *plan;
        PlanDigitV v;
        v.p.base = (int64_t)uniform64((uint64_t)q.base);
        v.p.span = uniform64(q.span);
        v.p.D1 = uniform32(q.D1);
        v.p.D2 = uniform32(q.D2);
        v.p.D3 = uniform32(q.D3);
        v.p.s1 = uniform32(q.s1);
        v.p.s2 = uniform32(q.s2);
        v.p.s3 = uniform32(q.s3);
        return v;
    }
};

// Grow-only named device scratch.  Reallocation frees the old buffer with
// hipFree (which synchronises), so it only happens on warm-up calls.
#ifndef SMJ_SPIN_WAIT
#define SMJ_SPIN_WAIT 1  // Workspace::wait_stream polls an event (0: a lab build's stream sync)
#endif
struct Workspace {
    // layouts this workspace's sorts and joins may not use
    // (smj_workspace_set_layouts, SMJ_LAYOUT_* in smj.h)
    uint32_t layouts_off = 0;
    // What the last joins and sorts of a few shapes (relation sizes) learnt
    // about their payloads (capi.hip device_bucket), least recently used
    // first out, so a caller alternating shapes on one workspace (sort R,
    // sort S, join R and S) keeps every shape's:
    //   mode_hint: the layout the last call reached after leaving the
    //     narrower ones for its payloads (-2: none), with a re-probe every
    //     16th call (calls);
    //   p32_fail: its payloads did not fit 32-bit words, so its calls start at
    //     the wider layouts (no re-probe: the 32-bit words are for relations
    //     with tiny payloads, e.g. the sort's).
    struct ShapeHint {
        uint64_t shape = ~0ull;
        int mode_hint = -2;
        uint32_t calls = 0;
        bool p32_fail = false;
        uint64_t used = 0;  // LRU clock
    };
    ShapeHint hints[8];
    uint64_t hint_clock = 0;
    ShapeHint& hint_for(uint64_t shape) {
        ShapeHint* victim = &hints[0];
        for (ShapeHint& h : hints) {
            if (h.shape == shape) {
                h.used = ++hint_clock;
                return h;
            }
            if (h.used < victim->used) victim = &h;
        }
        *victim = ShapeHint();
        victim->shape = shape;
        victim->used = ++hint_clock;
        return *victim;
    }
    int last_layout = -1;  // smj_workspace_last_layout (SMJ_LAYOUT_USED_*)
    std::map<std::string, std::pair<void*, size_t>> bufs;
    std::map<std::string, std::pair<void*, size_t>> pinned;
    // the k-way merge's run table as last uploaded, and where (a repeated
    // merge of the same runs skips the upload)
    std::vector<unsigned char> km_last;
    const void* km_last_dev = nullptr;
    hipEvent_t ev[8] = {};
    bool ev_init = false;
    float phase_ms[5] = {0, 0, 0, 0, 0};

    void* scratch(const char* name, size_t bytes) {
        if (bytes == 0) bytes = 16;
        auto it = bufs.find(name);
        if (it != bufs.end() && it->second.second >= bytes)
            return it->second.first;
        if (it != bufs.end()) SMJ_CHECK(hipFree(it->second.first));
        void* p = nullptr;
        size_t cap = bytes + bytes / 8;
        SMJ_CHECK(hipMalloc(&p, cap));
        bufs[name] = {p, cap};
        return p;
    }
    void* host_pinned(const char* name, size_t bytes) {
        if (bytes == 0) bytes = 16;
        auto it = pinned.find(name);
        if (it != pinned.end() && it->second.second >= bytes)
            return it->second.first;
        if (it != pinned.end()) SMJ_CHECK(hipHostFree(it->second.first));
        void* p = nullptr;
        SMJ_CHECK(hipHostMalloc(&p, bytes, hipHostMallocDefault));
        pinned[name] = {p, bytes};
        return p;
    }
    // Rings of pinned staging slots for host-built tables that are uploaded
    // stream-ordered before a launch: a slot is rewritten only after the copy
    // that used it kNRing uploads ago has finished (its event), so
    // consecutive launches never wait for the stream to drain.
    static constexpr uint32_t kNRing = 8;
    struct RingSlot {
        void* p = nullptr;
        size_t cap = 0;
        hipEvent_t ev = nullptr;
        bool used = false;
    };
    std::map<std::string, std::pair<std::vector<RingSlot>, uint32_t>> rings;
    void* ring_acquire(const char* name, size_t bytes, uint32_t* slot) {
        auto& r = rings[name];
        if (r.first.empty()) r.first.resize(kNRing);
        const uint32_t i = r.second++ % kNRing;
        RingSlot& s = r.first[i];
        if (s.used) SMJ_CHECK(hipEventSynchronize(s.ev));
        if (s.cap < bytes) {
            if (s.p) SMJ_CHECK(hipHostFree(s.p));
            SMJ_CHECK(hipHostMalloc(&s.p, bytes ? bytes : 16, hipHostMallocDefault));
            s.cap = bytes;
        }
        if (!s.ev) SMJ_CHECK(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming));
        *slot = i;
        return s.p;
    }
    // after the hipMemcpyAsync that reads the slot
    void ring_release(const char* name, uint32_t slot, hipStream_t st) {
        RingSlot& s = rings[name].first[slot];
        SMJ_CHECK(hipEventRecord(s.ev, st));
        s.used = true;
    }
    // The host's wait for a stream (the per-call synchronisation that reads
    // the status flags): an event behind the stream's work, polled with
    // hipEventQuery (busy wait) instead of hipStreamSynchronize's blocking
    // wait, which wakes the thread several microseconds after the work ends.
    hipEvent_t wait_ev = nullptr;
    void wait_stream(hipStream_t st) {
#if SMJ_SPIN_WAIT
        if (!wait_ev) SMJ_CHECK(hipEventCreateWithFlags(&wait_ev, hipEventDisableTiming));
        SMJ_CHECK(hipEventRecord(wait_ev, st));
        // spin for a bounded time (the short waits of a join step end in a
        // few microseconds); past it, yield the core and then block, so long
        // sorts and merges do not hold a host core at 100 %
        hipError_t e;
        const auto t0 = std::chrono::steady_clock::now();
        while ((e = hipEventQuery(wait_ev)) == hipErrorNotReady) {
            const auto dt = std::chrono::steady_clock::now() - t0;
            if (dt > std::chrono::microseconds(200)) {
                e = hipEventSynchronize(wait_ev);
                break;
            }
            if (dt > std::chrono::microseconds(50)) sched_yield();
        }
        SMJ_CHECK(e);
#else
        SMJ_CHECK(hipStreamSynchronize(st));
#endif
    }
    void events() {
        if (!ev_init) {
            for (auto& e : ev) SMJ_CHECK(hipEventCreate(&e));
            ev_init = true;
        }
    }

    // per-kernel event trace (bench.py's roofline needs each kernel's own
    // duration over the timed region); off unless smj_trace_enable()
    struct TraceRec {
        const char* name;
        hipEvent_t a, b;
    };
    bool trace_on = false;
    std::string trace_only;  // non-empty: trace this kernel name alone
    std::vector<TraceRec> trace;
    size_t trace_n = 0;
    bool traced(const char* name) const {
        return trace_on && (trace_only.empty() || trace_only == name);
    }
    int trace_begin(const char* name, hipStream_t st) {
        if (!traced(name)) return -1;
        if (trace_n == trace.size()) {
            TraceRec r;
            SMJ_CHECK(hipEventCreate(&r.a));
            SMJ_CHECK(hipEventCreate(&r.b));
            trace.push_back(r);
        }
        trace[trace_n].name = name;
        SMJ_CHECK(hipEventRecord(trace[trace_n].a, st));
        return (int)trace_n++;
    }
    void trace_end(int idx, hipStream_t st) {
        if (idx >= 0) SMJ_CHECK(hipEventRecord(trace[idx].b, st));
    }
    // a trace record whose events the runtime stamps at the kernel's own start
    // and end (hipExtLaunchKernelGGL): no event-record gap around short kernels
    bool trace_ext(const char* name, hipEvent_t* a, hipEvent_t* b) {
        if (!traced(name)) return false;
        if (trace_n == trace.size()) {
            TraceRec r;
            SMJ_CHECK(hipEventCreate(&r.a));
            SMJ_CHECK(hipEventCreate(&r.b));
            trace.push_back(r);
        }
        trace[trace_n].name = name;
        *a = trace[trace_n].a;
        *b = trace[trace_n].b;
        trace_n++;
        return true;
    }

    ~Workspace() {
        for (auto& r : trace) {
            (void)hipEventDestroy(r.a);
            (void)hipEventDestroy(r.b);
        }
        for (auto& kv : bufs) (void)hipFree(kv.second.first);
        for (auto& kv : pinned) (void)hipHostFree(kv.second.first);
        if (ev_init)
            for (auto& e : ev) (void)hipEventDestroy(e);
    }
};

struct TraceScope {
    Workspace* ws;
    hipStream_t st;
    int idx;
    TraceScope(Workspace* w, const char* name, hipStream_t s)
        : ws(w), st(s), idx(w ? w->trace_begin(name, s) : -1) {}
    ~TraceScope() {
        if (ws) ws->trace_end(idx, st);
    }
};

// One traced kernel launch: with tracing on, the trace events are stamped by
// the launch itself (kernel-exact, like the profiler's kernel trace).
template <typename... KArgs, typename... Args>
inline void traced_launch(Workspace* ws, const char* name, void (*kernel)(KArgs...),
                          dim3 grid, dim3 block, uint32_t shmem, hipStream_t st,
                          Args... args) {
    hipEvent_t a, b;
    if (ws && ws->trace_ext(name, &a, &b))
        hipExtLaunchKernelGGL(kernel, grid, block, shmem, st, a, b, 0u, (KArgs)args...);
    else
        hipLaunchKernelGGL(kernel, grid, block, shmem, st, (KArgs)args...);
}

// ---- refgen.hip : the reference's rand()-driven generators, bit-exact
uint32_t glibc_rand_at(uint32_t seed, uint64_t k);  // the k-th rand() after srand(seed)
void gen_nonunique_ref(Workspace* ws, Tup* out, uint64_t n, uint64_t first, uint64_t total,
                       int64_t maxid, uint32_t seed, uint64_t skip, hipStream_t st);
void gen_zipf_ref(Workspace* ws, Tup* out, uint64_t n, uint64_t first, uint64_t maxid,
                  double theta, uint32_t seed, uint64_t skip, hipStream_t st);

// ---- exchange.hip : the multi-GPU exchange's tables
void xsend(const int64_t* start, const int64_t* cnt, const unsigned int* flags, uint32_t F,
           uint32_t K, uint32_t G, uint32_t U, int64_t* msg, int64_t* chunk, hipStream_t st);
void xrecv(const int64_t* msg, const int64_t* chunk, uint32_t G, uint32_t rank, uint32_t mine,
           uint32_t K, uint32_t nb, uint64_t cap, int64_t* tstart, int64_t* tcnt,
           int64_t* summary, hipStream_t st);
// exact partition (hist) -> start/cnt tables of K shards, shard 0 used (F <= 1024)
void hist_tables(const int64_t* hist, uint32_t F, uint32_t K, int64_t* start, int64_t* cnt,
                 hipStream_t st);

// ---- partition.hip
void stable_partition(Workspace* ws, const Tup* in, uint64_t n, Tup* out,
                      const Digit32& dig, uint32_t dbits, int padded,
                      int64_t* hist_out, int64_t* off_out, hipStream_t st);
void plan_partition(Workspace* ws, const Tup* in, uint64_t n, Tup* out,
                    const RangePlan* plan_dev, uint32_t dbits,
                    uint64_t* starts_dev, int64_t* hist_out, hipStream_t st);
#ifdef KEY_8B
void plan_partition_packed(Workspace* ws, const Tup* in, uint64_t n, uint64_t* out,
                           const RangePlan* plan_dev, const RangePlan& pack_plan,
                           uint32_t dbits, uint64_t* starts_dev, int64_t* hist_out,
                           unsigned int* pack_bad, hipStream_t st);
#endif
// sampled level-1 partition (join): regions with slack, no histogram pass
uint64_t sampled_capacity(uint64_t n, uint32_t dbits);
// every partition is kShards segments: seg_start/seg_cnt[d * kShards + q]
#ifndef SMJ_SHARDS
#define SMJ_SHARDS 8
#endif
constexpr uint32_t kShards = SMJ_SHARDS;
// Sampled level-1 partition of nrel (1 or 2) relations in shared launches.
// out[r] holds sampled_capacity() elements: tuples, or (packed, 16-byte tuples
// only) LayPacked words for host_plan.  When `bad` is given, *bad is OR-ed
// with kBadPayload (a payload does not pack) and kBadRange (a key lies
// outside host_plan): packed words need both, tuples are range-checked when
// the plan was guessed.  `sample` = nrel * 2^dbits counters, zeroed by the
// caller (k_join_begin).
void sampled_partition(Workspace* ws, int nrel, const Tup* const* in, const uint64_t* n,
                       void* const* out, const RangePlan* plan_dev, uint32_t dbits,
                       unsigned int* sample, uint64_t* const* starts_dev,
                       int64_t* const* hist_out, uint64_t* const* seg_start,
                       int64_t* const* seg_cnt, unsigned int* flag_dev, hipStream_t st,
                       const RangePlan* host_plan = nullptr, bool packed = false,
                       unsigned int* bad = nullptr, uint64_t p48_stride = 0,
                       bool p32 = false, bool exact = false, bool p96 = false);
void hist_memcpy(Workspace* ws, const Tup* in, uint64_t n, Tup* out,
                 uint32_t dbits, hipStream_t st);
// lane order of LDS atomic returns (k_scatter_swp's ranks): violations, 0 expected
uint64_t lds_order_selfcheck(Workspace* ws, hipStream_t st);

// ---- bucketsort.hip : MSD bucket sort (+ fused merge-join count)
extern const uint32_t kGroupTarget;  // expected tuples per group of the plan
extern const uint32_t kTileTuples;   // bucket-size unit of the plan (8192)
extern const uint32_t kGroupD3Max;   // widest level-3 digit of the group pass
struct BucketSortArgs {
    // level-1 partitioned relation(s): bucket b occupies
    // [bstart[b], bstart[b] + bcount[b]) of `part`.
    const void* part[2];        // tuples, or LayPacked words when `packed`
    const uint64_t* bstart[2];  // device, nbuckets
    const int64_t* bcount[2];   // device, nbuckets
    // optional (sampled partition): bucket b = kShards segments
    // [seg_start[b*kShards+q], + seg_cnt[...]) inside its region
    const uint64_t* seg_start[2] = {nullptr, nullptr};
    const int64_t* seg_cnt[2] = {nullptr, nullptr};
    uint32_t nseg = kShards;    // segments per bucket (the exchange: one per source GPU)
    void* tmp[2];               // same size as part (tile-local pass output)
    Tup* out[2];                // sorted output, bucket b at ostart[b]
    uint64_t n[2];
    int nrel;                   // 1 = sort only, 2 = R and S + join count
    uint32_t nbuckets;          // 1 << D1
    const RangePlan* plan_dev;
    unsigned long long* count_dev;  // join count (nrel == 2), accumulated
    const unsigned int* part_flag = nullptr;  // sampled partition overflowed?
    // the plan, when the host computed it (key-range hints): with a sampled
    // partition the bucket pass then runs without a mid-pipeline host sync
    const RangePlan* host_plan = nullptr;
    bool packed = false;            // part/tmp hold LayPacked words (host_plan's)
    // part/tmp hold LayP48 words (packed too): two planes of pstride[r]
    // elements each (lo uint32, then hi uint16)
    bool p48 = false;
    uint64_t pstride[2] = {0, 0};
    bool p32 = false;  // part/tmp hold LayP32 words (packed too, one plane)
    bool p96 = false;  // part/tmp hold LayP96 elements (two planes of pstride[r])
    // optional 4-word block zeroed by the caller: [0] = part_flag, [1] =
    // pack_bad, [2] = the skew queue length (read back in one copy)
    unsigned int* status = nullptr;
    const unsigned int* pack_bad = nullptr;  // set by the partition: not packable
    // host copy of status words [0] and [1] after a false return (why the
    // attempt was void: overflow, kBadPayload / kBadRange)
    uint32_t* status_out = nullptr;
    // the 32-bit digit fast path of the tile and group passes (keys outside
    // the plan range only in the first and the last bucket); the segmented
    // join turns it off for tuples (a caller's key outside its range could sit
    // in the last non-empty bucket instead)
    bool digit_fast = true;
    // which stages run (bucket_sort_nosync; segmented joins): bit r = the
    // tile stage (tile numbering, tile pass, prefix table) of relation r,
    // bit 2 = the group pass and the one synchronisation.  A later call runs
    // the stages an earlier one left out, with the same arguments: the
    // multi-GPU join sorts R's tiles while S's rows are still in flight.
    uint32_t stage = 7;
    hipEvent_t ev_tile = nullptr;   // optional phase markers
    hipEvent_t ev_bucket = nullptr;
    hipEvent_t ev_ovf = nullptr;
};
// Runs the tile pass and the group pass; handles overflowing groups (skew)
// with the merge-sort fallback.  Synchronises `st` twice: once for the bucket
// counts (launch sizes) and once for the overflow count.
// Returns false (and does nothing) when a->part_flag reports an overflowed
// sampled partition: the caller repeats the exact partition.
bool bucket_sort(Workspace* ws, const BucketSortArgs& a, hipStream_t st);

// plan selection from a device sample (writes plan_dev)
// (D2 is the size-preferred level-2 width, D2cap the widest the plan may use
// to make the last digit exact)
void plan_from_sample(Workspace* ws, const Tup* const* rels,
                      const uint64_t* ns, int nrel, uint32_t D1, uint32_t D2,
                      uint32_t D2cap, int64_t hint_min, int64_t hint_max,
                      RangePlan* plan_dev, hipStream_t st);

// ---- mergesort.hip : general segmented merge sort + merge path kernels
void segmented_sort(Workspace* ws, Tup* data, const uint64_t* seg_off_host,
                    const uint64_t* seg_len_host, uint32_t nseg, hipStream_t st);
void merge2(Workspace* ws, const Tup* a, uint64_t na, const Tup* b, uint64_t nb, Tup* out,
            hipStream_t st);
void merge_join_count(const Tup* r, uint64_t nr, const Tup* s, uint64_t ns,
                      unsigned long long* count_dev, hipStream_t st);
// k independent merge-join counts (host arrays), one launch
void merge_join_count_batch(Workspace* ws, const Tup* const* r, const uint64_t* nr,
                            const Tup* const* s, const uint64_t* ns, uint32_t k,
                            unsigned long long* count_dev, hipStream_t st);
void multiway_merge(Workspace* ws, const Tup* const* runs_host,
                    const uint64_t* lens_host, uint32_t k, Tup* out,
                    hipStream_t st);
// the 2-way merge-path tree only (the m-pass join's multi-pass merging)
void multiway_merge_tree(Workspace* ws, const Tup* const* runs_host,
                         const uint64_t* lens_host, uint32_t k, Tup* out,
                         hipStream_t st);

// ---- materialize.hip : merge-join output tuples (sorted R and S)
// Writes the first min(total, out_cap) output tuples and returns the total
// (synchronises `st` once, for the launch size of the write pass).
uint64_t materialize(Workspace* ws, const Tup* R, uint64_t nR, const Tup* S,
                     uint64_t nS, Tup* out, uint64_t out_cap, hipStream_t st);

// ---- datagen.hip
void gen_pk(Tup* out, uint64_t n, uint64_t first, uint64_t total,
            uint64_t seed, hipStream_t st);
void gen_fk(Tup* out, uint64_t n, uint64_t first, uint64_t total,
            uint64_t maxid, uint64_t seed, hipStream_t st);
void gen_zipf(Workspace* ws, Tup* out, uint64_t n, uint64_t first,
              uint64_t maxid, double theta, uint64_t seed, hipStream_t st);

}  // namespace smj
