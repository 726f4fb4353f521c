#include <atomic>
// capi.hip -- the C ABI of libsmj_hip[_k8].so (declared in include/smj.h).
//
// Reference-named entry points keep the reference's signatures, pointer-swap
// conventions and output layout; host pointers are staged through HBM, device
// pointers are used in place.  Nothing in here computes on the CPU: every
// sort, partition, merge and join runs in the HIP kernels of this library, and
// a missing/failed device aborts (fail-fast like the reference).
#include <math.h>
#include <string.h>
#include <sys/time.h>

#include <algorithm>
#include <vector>

#include "../../include/smj.h"
#include "smj_common.hpp"
#include "smj_internal.hpp"

__global__ void k_setplan(smj::RangePlan* p, smj::RangePlan v) { *p = v; }

// start of a join attempt: the plan (when known on the host), the count, the
// 4-word status block (BucketSortArgs::status) and the sampled partition's
// sample counters (nzero words, every attempt) in one launch
__global__ void __launch_bounds__(256)
k_join_begin(smj::RangePlan* p, smj::RangePlan v, int set_plan, unsigned long long* count,
             unsigned int* status, unsigned int* zero, uint32_t nzero) {
    if (threadIdx.x == 0) {
        if (set_plan) *p = v;
        *count = 0;
    }
    if (threadIdx.x < 4) status[threadIdx.x] = 0;
    for (uint32_t i = threadIdx.x; i < nzero; i += 256) zero[i] = 0;
}

// is_sorted_helper's scan (joincommon.c:397-500) in parallel: the first
// position whose key is below its predecessor's (the predecessor of item 0 is
// the key 0 the reference starts from) and the first whose key equals it
__global__ void __launch_bounds__(256)
k_sorted_scan(const smj::Tup* __restrict__ t, uint64_t n, unsigned long long* first) {
    const uint64_t G = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += G) {
        const int64_t k = smj::tup_key(smj::ld_g(t + i));
        const int64_t prev = i ? smj::tup_key(smj::ld_g(t + i - 1)) : 0;
        if (k < prev) atomicMin(&first[0], (unsigned long long)i);
        else if (k == prev) atomicMin(&first[1], (unsigned long long)i);
    }
}

namespace smj {
void gen_pk_nopayload(Tup* out, uint64_t n, uint64_t first, uint64_t total,
                      uint64_t seed, hipStream_t st);
// mgpu.hip: the multi-GPU join behind sortmergejoin_mpsm (mat: -1 = the
// process switch, else this call's materialisation)
result_t* mpsm_api(relation_t* relR, relation_t* relS, joinconfig_t* joincfg, int mat);
}

using namespace smj;

static_assert(sizeof(tuple_t) == sizeof(Tup), "tuple_t / device tuple mismatch");

// ---------------------------------------------------------------------------
// per-thread device context (the reference's L1 functions are called
// concurrently from T pthreads on disjoint data, SURVEY.md §8(b) Threading)
// ---------------------------------------------------------------------------
struct Ctx {
    hipStream_t st = nullptr;
    Workspace ws;
    int device = -1;
};

static Ctx& ctx() {
    thread_local Ctx* c = nullptr;
    if (!c) {
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
            fprintf(stderr,
                    "[ERROR] smj: no HIP device visible; the MI355X library has "
                    "no CPU fallback.\n");
            abort();
        }
        c = new Ctx();
        SMJ_CHECK(hipGetDevice(&c->device));
        SMJ_CHECK(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
    }
    return *c;
}


static bool is_device_ptr(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t a;
    hipError_t e = hipPointerGetAttributes(&a, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();  // clear
        return false;
    }
    return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

// Device view of a caller buffer: either the pointer itself or a staged copy.
struct DevBuf {
    Tup* d = nullptr;
    void* host = nullptr;
    bool staged = false;
};

static DevBuf dev_in(const void* p, uint64_t ntup, const char* slot,
                     bool copy_in) {
    DevBuf b;
    if (is_device_ptr(p)) {
        b.d = (Tup*)p;
        return b;
    }
    Ctx& c = ctx();
    b.d = (Tup*)c.ws.scratch(slot, (ntup ? ntup : 1) * sizeof(Tup));
    b.host = (void*)p;
    b.staged = true;
    if (copy_in && ntup)
        SMJ_CHECK(hipMemcpyAsync(b.d, p, ntup * sizeof(Tup),
                                 hipMemcpyHostToDevice, c.st));
    return b;
}

static void dev_out(const DevBuf& b, uint64_t ntup) {
    if (!b.staged || ntup == 0) return;
    SMJ_CHECK(hipMemcpyAsync(b.host, b.d, ntup * sizeof(Tup),
                             hipMemcpyDeviceToHost, ctx().st));
}

static void sync() { SMJ_CHECK(hipStreamSynchronize(ctx().st)); }

// ---------------------------------------------------------------------------
// device pipelines
// ---------------------------------------------------------------------------
static uint32_t ceil_log2(uint64_t x) {
    uint32_t b = 0;
    while (b < 63 && (1ull << b) < x) b++;
    return b;
}

// level widths: D1 (partition fan-out) and D2 (tile-pass fan-out = groups per
// bucket) so that the expected group is kGroupTarget tuples (3/4 of what the
// group pass holds in LDS); the plan may widen D2 up to D2cap to make the last
// digit the exact key
// `tile`: the elements of a tile-pass tile of the layout the buckets will
// hold (kTileTuples for 8-byte elements: words, 48-bit words, 8-byte tuples;
// half of it for 16-byte tuples in their own layout)
static void choose_levels(uint64_t n, uint32_t want_d1, uint32_t* D1,
                          uint32_t* D2, uint32_t* D2cap, uint32_t tile = kTileTuples) {
    const uint64_t target = kGroupTarget;
    uint32_t B = n > target ? ceil_log2((n + target - 1) / target) : 0;
    // level 1: 256 partitions by default, more when a bucket would exceed
    // ~192 tiles of the tile pass (the group pass takes up to 256 per bucket):
    // N1024 keeps 2^10 partitions, within the sampled scatter's LDS carries.
    // 128M x 128M, interleaved A/B on one box (tools/ab_fanout.sh): 256
    // partitions 3.57 / 3.09 ms (16 / 8 B) against 3.63 / 3.16 ms with 512 --
    // longer scatter streams and tile-pass runs, a slightly slower group pass
    uint32_t d1 = want_d1 ? want_d1 : 8;
    const uint64_t bucket_cap = 192ull * tile;
    while (d1 < kNarrowDigitBits && (n >> d1) > bucket_cap) d1++;
    if (d1 > B) d1 = B;
    if (d1 > kNarrowDigitBits) d1 = kNarrowDigitBits;
    uint32_t d2 = B > d1 ? B - d1 : 0;
    if (d2 > kMaxD2) d2 = kMaxD2;
    *D1 = d1;
    *D2 = d2;
    // the plan may add up to two level-2 bits to make the last digit exact
    *D2cap = d2 + 2 < kMaxD2 ? d2 + 2 : (d2 > kMaxD2 ? d2 : kMaxD2);
}

// level-1 partition of sorts and joins: sampled regions (no histogram pass)
// unless the workspace's layout policy turns them off (smj_workspace_set_layouts)
static bool use_sampled(const Workspace* ws) { return !(ws->layouts_off & SMJ_LAYOUT_NO_SAMPLED); }

// exact key range [min, max] of the relations (one read pass); min > max
// when they are empty.  16-byte non-temporal loads over one contiguous chunk
// per workgroup, two register tiles of KR_U alternating (the scalar 8-byte
// loads of the first version reached 3.0 TB/s on 2^27 x 8 B, the grid-stride
// 16-byte form 5.3 TB/s), one pair of atomics per workgroup.
typedef unsigned long long KrVec __attribute__((ext_vector_type(2)));
constexpr int KR_U = 8;
constexpr int KR_THREADS = 512;

__device__ __forceinline__ void kr_acc(uint64_t u, uint64_t& lo, uint64_t& hi) {
    lo = u < lo ? u : lo;
    hi = u > hi ? u : hi;
}

__device__ __forceinline__ void kr_vec(const KrVec& v, uint64_t& lo, uint64_t& hi) {
#ifdef KEY_8B
    kr_acc(key_u((int64_t)v.y), lo, hi);  // Tup {payload, key}
#else
    kr_acc(key_u(tup_key((Tup)v.x)), lo, hi);
    kr_acc(key_u(tup_key((Tup)v.y)), lo, hi);
#endif
}

// One contiguous chunk of 16-byte vectors per workgroup, two register tiles
// alternating (the next tile's loads fly while this one is reduced): the
// stable histogram's pattern (k_hist_v), which streams at ~6.5 TB/s.
__device__ __forceinline__ void kr_chunk(const KrVec* __restrict__ v, uint64_t nv,
                                         uint64_t& lo, uint64_t& hi) {
    const uint64_t per = (nv + gridDim.x - 1) / gridDim.x;
    const uint64_t beg = (uint64_t)blockIdx.x * per;
    const uint64_t end = beg + per < nv ? beg + per : nv;
    constexpr int TILE = KR_THREADS * KR_U;
    KrVec a[KR_U], b[KR_U];
    auto load = [&](KrVec (&x)[KR_U], uint64_t base) {
#pragma unroll
        for (int u = 0; u < KR_U; u++) {
            const uint64_t i = base + (uint64_t)u * KR_THREADS + threadIdx.x;
            x[u] = __builtin_nontemporal_load(v + (i < end ? i : end - 1));
        }
    };
    auto reduce = [&](const KrVec (&x)[KR_U], uint64_t base) {
#pragma unroll
        for (int u = 0; u < KR_U; u++)
            if (base + (uint64_t)u * KR_THREADS + threadIdx.x < end) kr_vec(x[u], lo, hi);
    };
    if (beg >= end) return;
    load(a, beg);
    for (uint64_t base = beg; base < end;) {
        load(b, base + TILE);
        reduce(a, base);
        if ((base += TILE) >= end) break;
        load(a, base + TILE);
        reduce(b, base);
        base += TILE;
    }
}

__global__ void __launch_bounds__(KR_THREADS)
k_keyrange(const Tup* __restrict__ r0, uint64_t n0, const Tup* __restrict__ r1, uint64_t n1,
           unsigned long long* __restrict__ mm) {
    __shared__ unsigned long long sl[KR_THREADS / 64], sh[KR_THREADS / 64];
    uint64_t lo = ~0ull, hi = 0;  // key_u order
    const uint64_t gt = (uint64_t)blockIdx.x * KR_THREADS + threadIdx.x;
    const uint64_t G = (uint64_t)gridDim.x * KR_THREADS;
    for (int rel = 0; rel < 2; rel++) {
        const Tup* p = rel ? r1 : r0;
        const uint64_t n = rel ? n1 : n0;
        if (!p || n == 0) continue;
        if (((uintptr_t)p & 15) == 0) {
            const uint64_t nv = n * sizeof(Tup) / 16;
            kr_chunk(reinterpret_cast<const KrVec*>(p), nv, lo, hi);
            // 8-byte tuples: an odd last one
            if (gt == 0 && nv * 16 / sizeof(Tup) < n) kr_acc(key_u(tup_key(p[n - 1])), lo, hi);
        } else {
            for (uint64_t i = gt; i < n; i += G) kr_acc(key_u(tup_key(p[i])), lo, hi);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t a = __shfl_xor(lo, o, 64), c = __shfl_xor(hi, o, 64);
        lo = a < lo ? a : lo;
        hi = c > hi ? c : hi;
    }
    if (lane_id() == 0) {
        sl[threadIdx.x >> 6] = lo;
        sh[threadIdx.x >> 6] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < KR_THREADS / 64; w++) {
            lo = sl[w] < lo ? sl[w] : lo;
            hi = sh[w] > hi ? sh[w] : hi;
        }
        atomicMin(&mm[0], (unsigned long long)lo);
        atomicMax(&mm[1], (unsigned long long)hi);
    }
}

namespace smj {
bool key_range(Workspace* ws, const Tup* const* rels, const uint64_t* ns, int nrel,
               int64_t* lo, int64_t* hi, hipStream_t st) {
    unsigned long long* mm = (unsigned long long*)ws->scratch("keyrange", 16);
    unsigned long long* h = (unsigned long long*)ws->host_pinned("keyrange_h", 16);
    const unsigned long long init[2] = {~0ull, 0ull};
    SMJ_CHECK(hipMemcpyAsync(mm, init, 16, hipMemcpyHostToDevice, st));
    const uint64_t n = ns[0] + (nrel > 1 ? ns[1] : 0);
    // one workgroup per CU, a contiguous chunk each (fewer for small inputs)
    uint64_t g = (n * sizeof(Tup) / 16 + KR_THREADS * KR_U - 1) / (KR_THREADS * KR_U);
    if (g > 256) g = 256;
    if (g == 0) g = 1;
    hipLaunchKernelGGL(k_keyrange, dim3((uint32_t)g), dim3(KR_THREADS), 0, st, rels[0], ns[0],
                       nrel > 1 ? rels[1] : (const Tup*)nullptr, nrel > 1 ? ns[1] : 0, mm);
    SMJ_CHECK(hipMemcpyAsync(h, mm, 16, hipMemcpyDeviceToHost, st));
    SMJ_CHECK(hipStreamSynchronize(st));
    if (h[0] > h[1]) return false;
    *lo = (int64_t)(h[0] ^ 0x8000000000000000ull);
    *hi = (int64_t)(h[1] ^ 0x8000000000000000ull);
    return true;
}
}  // namespace smj

// 16-byte sorts and joins carry packed words through the intermediate passes
// when the plan allows it (LayPacked) ...
static bool use_packing(const Workspace* ws) { return !(ws->layouts_off & SMJ_LAYOUT_NO_PACKED); }

// ... and 48-bit words in two planes first (LayP48) when every payload fits
// 48 - s1 bits
static bool use_p48(const Workspace* ws) { return !(ws->layouts_off & SMJ_LAYOUT_NO_P48); }

// ... and 32-bit words before those (LayP32) where the payloads are tiny
static bool use_p32(const Workspace* ws) { return !(ws->layouts_off & SMJ_LAYOUT_NO_P32); }

// ... and, where no packed word holds the payloads, 12-byte elements (LayP96:
// the payload and a 32-bit key offset) instead of the 16-byte tuples
static bool use_p96(const Workspace* ws) { return !(ws->layouts_off & SMJ_LAYOUT_NO_P96); }

// Sort of one relation (nrel 1) or sort + merge-join count of two (nrel 2):
// range plan -> sampled level-1 partition -> tile pass -> group pass.  The
// plan must be known on the host (no mid-pipeline synchronisation, and 16-byte
// tuples travel as packed words).  It comes from
//   - the caller's key-range hint (hint_min <= hint_max), else
//   - the relation size (size_guess > 0): keys 1..size_guess, the reference's
//     own assumption (its partitioning_phase derives the radix shift from
//     |R| * T, src/joins/sortmergejoin_multiway.c:372-376).  The level-1
//     scatter, which reads every key anyway, verifies it (kBadRange); a key
//     outside sends the call back to the exact plan below, else
//   - one exact min/max pass (key_range: one read and a host round trip).
// Keys outside a hinted plan are legal: they clamp to the end digits.
static void device_bucket(Workspace* ws, const Tup* const* rels, const uint64_t* ns,
                          int nrel, Tup* const* outs, uint32_t fanout_bits,
                          int64_t hint_min, int64_t hint_max, uint64_t size_guess,
                          unsigned long long* count_dev, hipStream_t st) {
    static const char* nm[2][6] = {{"bk_part0", "bk_st0", "bk_h0", "bk_sgs0", "bk_sgc0", ""},
                                   {"bk_part1", "bk_st1", "bk_h1", "bk_sgs1", "bk_sgc1", ""}};
    ws->events();
    SMJ_CHECK(hipEventRecord(ws->ev[0], st));
    const uint64_t nmax = nrel > 1 && ns[1] > ns[0] ? ns[1] : ns[0];
    uint32_t D1, D2, D2cap;
    choose_levels(nmax, fanout_bits, &D1, &D2, &D2cap);
    RangePlan* plan = (RangePlan*)ws->scratch("plan", sizeof(RangePlan));
    uint32_t nb = 1u << D1;
    const bool sampled = use_sampled(ws) && D1 <= 10;  // LDS carries up to 1024
    bool plan_on_host = hint_min <= hint_max;
    // a guessed plan is verified by the sampled scatter only
    bool guessed = false;
    const bool sample_plan = (ws->layouts_off & SMJ_LAYOUT_SAMPLE_PLAN) != 0;
    if (!plan_on_host && size_guess > 0 && sampled && !sample_plan) {
        hint_min = 1;
        hint_max = (int64_t)(size_guess < (uint64_t)INT64_MAX ? size_guess : INT64_MAX);
        plan_on_host = guessed = true;
    }
    if (!plan_on_host && !sample_plan)
        plan_on_host = key_range(ws, rels, ns, nrel, &hint_min, &hint_max, st);
    RangePlan hplan = make_plan(hint_min, hint_max, D1, D2, D2cap, kGroupD3Max);
    if (!plan_on_host)
        plan_from_sample(ws, rels, ns, nrel, D1, D2, D2cap, hint_min, hint_max, plan, st);
#ifdef KEY_8B
    bool can_pack = sampled && plan_on_host && use_packing(ws) && LayPacked::usable(hplan);
#else
    const bool can_pack = false;
#endif
    Tup* part[2] = {nullptr, nullptr};
    uint64_t* bst[2] = {nullptr, nullptr};
    int64_t* bh[2] = {nullptr, nullptr};
    uint64_t* sgs[2] = {nullptr, nullptr};
    int64_t* sgc[2] = {nullptr, nullptr};
    unsigned int* sample = nullptr;
    auto alloc = [&]() {
        for (int r = 0; r < nrel; r++) {
            const uint64_t cap = sampled ? sampled_capacity(ns[r], D1) : (ns[r] ? ns[r] : 1);
            part[r] = (Tup*)ws->scratch(nm[r][0], cap * sizeof(Tup));
            bst[r] = (uint64_t*)ws->scratch(nm[r][1], nb * 8);
            bh[r] = (int64_t*)ws->scratch(nm[r][2], nb * 8);
            sgs[r] = (uint64_t*)ws->scratch(nm[r][3], (size_t)nb * kShards * 8);
            sgc[r] = (int64_t*)ws->scratch(nm[r][4], (size_t)nb * kShards * 8);
        }
        // the sampled partition's counters: zeroed by k_join_begin on every
        // attempt (never assumed zero from an earlier call)
        sample = (unsigned int*)ws->scratch("sp_sample", (size_t)nrel * nb * 4);
    };
    alloc();
    // [0] region overflow, [1] bad tuple (kBadPayload | kBadRange), [2] skew
    // queue length
    unsigned int* status = (unsigned int*)ws->scratch("join_status", 16);
    // 16-byte tuples in their own layout hold tiles of kTileTuples / 2: when
    // an attempt falls back to them, the level widths are chosen again for
    // that tile (a bucket within the group pass's 256 tiles)
    bool tuple_levels = sizeof(Tup) != 16;
    auto tuple_plan = [&]() {
        if (tuple_levels) return;
        tuple_levels = true;
        uint32_t d1, d2, d2c;
        choose_levels(nmax, fanout_bits, &d1, &d2, &d2c, kTileTuples / 2);
        if (d1 == D1 || (sampled && d1 > 10)) return;  // the sampled scatter's carries
        D1 = d1;
        D2 = d2;
        D2cap = d2c;
        nb = 1u << D1;
        hplan = make_plan(hint_min, hint_max, D1, D2, D2cap, kGroupD3Max);
        if (!plan_on_host)
            plan_from_sample(ws, rels, ns, nrel, D1, D2, D2cap, hint_min, hint_max, plan, st);
        alloc();
    };
    unsigned long long* cnt = count_dev
        ? count_dev : (unsigned long long*)ws->scratch("sort_cnt", 8);
    // attempts: sampled + 48-bit words (-1), sampled + packed words (0),
    // sampled tuples (1), exact tuples (2); a later one runs only when the one
    // before reported a region overflow or an unpackable tuple (its tile and
    // group passes then did nothing or are discarded: the count restarts from
    // 0).  A payload too wide for 48 bits but not for 64 goes from -1 to 0.  A
    // guessed plan that a key falls outside of is replaced by the exact one
    // and the attempts restart.  The 48-bit scatter's carries (128 bytes a
    // partition) fit LDS up to 512 partitions.
    // (8-byte tuples have no 64-bit packed words: the 48-bit ones, else
    // tuples; the same conditions as packing, checked here)
    // A 48-bit word keeps 48 - s1 payload bits.  Payloads are taken to lie
    // within the key span (the row ids of a PK relation, as in the
    // benchmark): where they would not, the 48-bit attempt would fail on them
    // and partition a second time, so the join starts with 64-bit words (the
    // 1024M x 1024M join: 2^9 partitions leave 27 payload bits).
    const bool p48_fits = hplan.s1 >= 1 && hplan.s1 <= 32 && hplan.span < (1ull << (48 - hplan.s1));
    const uint64_t shape = ((uint64_t)nrel << 62) ^ ns[0] ^ (nrel > 1 ? ns[1] << 31 : 0);
    Workspace::ShapeHint& H = ws->hint_for(shape);
    // 48-bit words, whatever their payloads
    auto p48_ok = [&]() {
#ifdef KEY_8B
        return can_pack && use_p48(ws) && nb <= 512;
#else
        return sampled && plan_on_host && use_packing(ws) && use_p48(ws) &&
               LayP48::usable(hplan) && nb <= 512;
#endif
    };
    // 32-bit words (mode -2) are tried first: nothing tells the payloads'
    // width beforehand, and a shape whose payloads did not fit does not try
    // them again (Workspace::ShapeHint::p32_fail)
    auto first_mode = [&]() {
        if (sampled && plan_on_host && use_packing(ws) && use_p32(ws) &&
            LayP32::usable(hplan) && !H.p32_fail)
            return -2;
        if (p48_ok() && p48_fits) return -1;
        return can_pack ? 0 : (sampled ? 1 : 2);
    };
    // The layout hint of the workspace: when the last call of the same shape
    // had to leave the narrower layouts because of its payloads (too wide for
    // 48-bit words, or for packed words at all), start at the layout it
    // reached -- its partition would only be repeated -- and re-probe from the
    // top every 16th call.  Data-dependent like the fallback it skips; the
    // results are the same in every layout.
    bool hinted = false;
    auto hinted_mode = [&](int m) {
        hinted = false;
        if (H.mode_hint <= m || ++H.calls % 16 == 0) return m;
        const int h = H.mode_hint == 0 ? (can_pack ? 0 : (sampled ? 1 : 2))
                                         : (sampled ? 1 : 2);
        hinted = h > m;
        return h > m ? h : m;
    };
    // the sampled tuples' attempt (mode 1) on 16-byte tuples: 12-byte
    // elements where the plan spans at most 2^32 keys (LayP96)
    auto p96_ok = [&]() {
#ifdef KEY_8B
        // (16-element segments: the scatter's carries fit LDS up to 512
        // partitions, as for the 48-bit words)
        return sampled && plan_on_host && use_p96(ws) && LayP96::usable(hplan) &&
               nb <= (LayP96::Pack::kStoreBytes < 8 ? 512u : 1024u);
#else
        return false;
#endif
    };
    int mode = hinted_mode(first_mode());
    const bool started_hinted = hinted;
    int payload_fb = -2;  // the mode a payload flag sent this call to
    while (mode <= 2) {
        if (mode >= 1) tuple_plan();
        const bool p32 = mode == -2;
        const bool p48 = mode == -1;
        const bool packed = mode <= 0;
        const bool p96 = mode == 1 && p96_ok();
        // the status word the tile and group passes exit on (sampled modes)
        const bool check = packed || p96 || (guessed && mode == 1);
        hipLaunchKernelGGL(k_join_begin, dim3(1), dim3(256), 0, st, plan, hplan,
                           plan_on_host ? 1 : 0, cnt, status, sample,
                           mode < 2 ? (uint32_t)nrel * nb : 0u);
        // LayP48's plane stride: the partition buffer's capacity in elements,
        // rounded to 32 (the hi plane starts 16-byte aligned); the buffer
        // holds 16 bytes an element, the planes take 6
        uint64_t pstride[2] = {0, 0};
        for (int r = 0; r < nrel && (p48 || p96); r++)
            pstride[r] = (sampled_capacity(ns[r], D1) + 31) & ~31ull;
        if (mode < 2) {
            void* outs_v[2] = {part[0], part[nrel > 1 ? 1 : 0]};
            if ((p48 || p96) && nrel > 1 && pstride[0] != pstride[1]) {
                // one stride per launch: the two relations take turns.  Both
                // calls use relation 0's region scratch (cursor, cap_end):
                // correct because they run in order on the one stream `st`
                for (int r = 0; r < nrel; r++) {
                    const Tup* rr1[1] = {rels[r]};
                    const uint64_t nn1[1] = {ns[r]};
                    void* oo1[1] = {part[r]};
                    uint64_t* bs1[1] = {bst[r]};
                    int64_t* bh1[1] = {bh[r]};
                    uint64_t* sgs1[1] = {sgs[r]};
                    int64_t* sgc1[1] = {sgc[r]};
                    sampled_partition(ws, 1, rr1, nn1, oo1, plan, D1, sample + (size_t)r * nb,
                                      bs1, bh1, sgs1, sgc1, status, st, &hplan, true,
                                      status + 1, pstride[r], false, false, p96);
                }
            } else {
                sampled_partition(ws, nrel, rels, ns, outs_v, plan, D1, sample, bst, bh, sgs,
                                  sgc, status, st, plan_on_host ? &hplan : nullptr,
                                  packed || p96, check ? status + 1 : nullptr, pstride[0], p32,
                                  false, p96);
            }
        } else {
            for (int r = 0; r < nrel; r++)
                plan_partition(ws, rels[r], ns[r], part[r], plan, D1, bst[r], bh[r], st);
        }
        SMJ_CHECK(hipEventRecord(ws->ev[1], st));
        BucketSortArgs a;
        for (int r = 0; r < 2; r++) {
            a.part[r] = part[r];
            a.bstart[r] = bst[r];
            a.bcount[r] = bh[r];
            a.tmp[r] = part[r];
            a.out[r] = r < nrel ? outs[r] : nullptr;
            a.n[r] = r < nrel ? ns[r] : 0;
            if (mode < 2) {
                a.seg_start[r] = sgs[r];
                a.seg_cnt[r] = sgc[r];
            }
        }
        a.nrel = nrel;
        a.nbuckets = nb;
        a.plan_dev = plan;
        a.count_dev = nrel == 2 ? count_dev : nullptr;
        a.ev_tile = nullptr;
        a.ev_bucket = ws->ev[2];
        a.ev_ovf = ws->ev[3];
        a.host_plan = plan_on_host ? &hplan : nullptr;
        a.packed = packed;
        a.p48 = p48;
        a.p32 = p32;
        a.p96 = p96;
        a.pstride[0] = pstride[0];
        a.pstride[1] = pstride[1];
        a.pack_bad = check ? status + 1 : nullptr;
        a.status = status;
        if (mode < 2) a.part_flag = status;
        uint32_t why[2] = {0, 0};
        a.status_out = why;
        if (bucket_sort(ws, a, st)) break;
        if (mode == -2 && !(guessed && (why[1] & kBadRange))) {
            // payloads too wide for 32 bits: the narrowest wider words that
            // hold them; anything else (overflow, a key outside the plan) as
            // from 64-bit words
            const bool pay = !why[0] && !(why[1] & kBadRange);
            if (pay && (why[1] & (kBadPayload | kBadPayload48 | kBadPayload32)))
                H.p32_fail = true;
            if (pay && !(why[1] & (kBadPayload | kBadPayload48)) && p48_ok())
                mode = -1;
            else if (pay && !(why[1] & kBadPayload) && can_pack)
                mode = 0;
            else
                mode = 1;
            continue;
        }
        if (mode == -1 && !(guessed && (why[1] & kBadRange))) {
            // payloads too wide for 48 bits only: 64-bit words; anything else
            // (overflow, unpackable) as from 64-bit words
            mode = (why[1] & kBadPayload48) && !(why[1] & kBadPayload) && !why[0] && can_pack
                ? 0 : 1;
            if (!why[0] && (why[1] & (kBadPayload | kBadPayload48)) && !(why[1] & kBadRange))
                payload_fb = mode;
            continue;
        }
        if (guessed && (why[1] & kBadRange)) {
            // a key outside 1..size_guess: the exact plan, attempts from the top
            guessed = false;
            plan_on_host = key_range(ws, rels, ns, nrel, &hint_min, &hint_max, st);
            hplan = make_plan(hint_min, hint_max, D1, D2, D2cap, kGroupD3Max);
            if (!plan_on_host)  // empty relations never report a bad key
                plan_from_sample(ws, rels, ns, nrel, D1, D2, D2cap, hint_min, hint_max, plan,
                                 st);
#ifdef KEY_8B
            can_pack = sampled && plan_on_host && use_packing(ws) && LayPacked::usable(hplan);
#endif
            mode = hinted_mode(first_mode());
            continue;
        }
        if (mode == 0 && !why[0] && (why[1] & kBadPayload) && !(why[1] & kBadRange))
            payload_fb = 1;
        mode++;
    }
    ws->last_layout = mode == -2 ? SMJ_LAYOUT_USED_P32 : mode == -1 ? SMJ_LAYOUT_USED_P48
                    : mode == 0 ? SMJ_LAYOUT_USED_WORDS
                    : mode == 1 && p96_ok() ? SMJ_LAYOUT_USED_P96 : SMJ_LAYOUT_USED_TUPLES;
    if (payload_fb >= 0)
        H.mode_hint = payload_fb;
    else if (!started_hinted)
        H.mode_hint = -2;  // the narrow layouts held (or failed for other reasons)
    SMJ_CHECK(hipEventRecord(ws->ev[4], st));
}

// avxsort_tuples and friends: the plan is guessed from the size (keys 1..n,
// the shape of create_relation_pk) and verified, like the join's
static void device_sort(Workspace* ws, const Tup* in, uint64_t n, Tup* out,
                        hipStream_t st) {
    if (n == 0) return;
    const Tup* rels[1] = {in};
    uint64_t ns[1] = {n};
    Tup* outs[1] = {out};
    device_bucket(ws, rels, ns, 1, outs, 0, 1, 0, n, nullptr, st);
}

static void device_join(Workspace* ws, const Tup* R, uint64_t nR, const Tup* S,
                        uint64_t nS, Tup* sortedR, Tup* sortedS,
                        uint32_t fanout_bits, int64_t hint_min,
                        int64_t hint_max, unsigned long long* count_dev,
                        hipStream_t st, uint64_t size_guess = 0) {
    const Tup* rels[2] = {R, S};
    uint64_t ns[2] = {nR, nS};
    Tup* outs[2] = {sortedR, sortedS};
    device_bucket(ws, rels, ns, 2, outs, fanout_bits, hint_min, hint_max, size_guess,
                  count_dev, st);
}

// ---------------------------------------------------------------------------
// partitioning (reference src/partition/partition.c:301-436)
// ---------------------------------------------------------------------------
static void partition_common(relation_t** parts, relation_t* input,
                             relation_t* output, uint32_t nbits,
                             uint32_t shiftbits, int padded) {
    Ctx& c = ctx();
    const uint64_t n = input->num_tuples;
    const uint32_t fan = 1u << nbits;
    const uint32_t mask = (uint32_t)(((1ull << nbits) - 1) << shiftbits);
    DevBuf in = dev_in(input->tuples, n, "api_in", true);
    // output extent: n plus at most one cache line of padding per partition
    const uint64_t cap = n + (padded ? (uint64_t)fan * TUPLESPERCACHELINE : 0);
    DevBuf out = dev_in(output->tuples, cap, "api_out", false);
    int64_t* hist = (int64_t*)c.ws.scratch("api_hist", fan * 8);
    int64_t* off = (int64_t*)c.ws.scratch("api_off", fan * 8);
    Digit32 dig{mask, shiftbits};
    stable_partition(&c.ws, in.d, n, out.d, dig, nbits, padded, hist, off, c.st);
    std::vector<int64_t> hh(fan), ho(fan);
    SMJ_CHECK(hipMemcpyAsync(hh.data(), hist, fan * 8, hipMemcpyDeviceToHost, c.st));
    SMJ_CHECK(hipMemcpyAsync(ho.data(), off, fan * 8, hipMemcpyDeviceToHost, c.st));
    sync();
    const uint64_t extent = fan ? (uint64_t)(ho[fan - 1] + hh[fan - 1]) : 0;
    // the reference never writes the padding between padded partitions
    // (partition.c:183-206): keep the caller's bytes there when staging back
    std::vector<tuple_t> gaps;
    if (out.staged && padded) {
        for (uint32_t i = 0; i + 1 < fan; i++)
            for (int64_t j = ho[i] + hh[i]; j < ho[i + 1]; j++)
                gaps.push_back(output->tuples[j]);
    }
    dev_out(out, extent);
    sync();
    if (!gaps.empty()) {
        size_t k = 0;
        for (uint32_t i = 0; i + 1 < fan; i++)
            for (int64_t j = ho[i] + hh[i]; j < ho[i + 1]; j++)
                output->tuples[j] = gaps[k++];
    }
    for (uint32_t i = 0; i < fan; i++) {
        parts[i]->tuples = output->tuples + ho[i];
        parts[i]->num_tuples = (uint64_t)hh[i];
    }
}

extern "C" {

void partition_relation(relation_t** partitions, relation_t* input,
                        relation_t* output, int radixbits, int shiftbits) {
    partition_common(partitions, input, output, (uint32_t)radixbits,
                     (uint32_t)shiftbits, 0);
}

void partition_relation_optimized(relation_t** partitions, relation_t* input,
                                  relation_t* output, uint32_t nbits,
                                  uint32_t shiftbits) {
    partition_common(partitions, input, output, nbits, shiftbits, 1);
}

void partition_relation_optimized_V2(relation_t** partitions,
                                     relation_t* input, relation_t* output,
                                     uint32_t nbits, uint32_t shiftbits) {
    partition_common(partitions, input, output, nbits, shiftbits, 1);
}

void histogram_memcpy_bench(relation_t** partitions, relation_t* input,
                            relation_t* output, uint32_t nbits) {
    (void)partitions;
    Ctx& c = ctx();
    const uint64_t n = input->num_tuples;
    DevBuf in = dev_in(input->tuples, n, "api_in", true);
    DevBuf out = dev_in(output->tuples, n, "api_out", false);
    hist_memcpy(&c.ws, in.d, n, out.d, nbits, c.st);
    dev_out(out, n);
    sync();
}

// partition.c:93-149 (declared partition.h:38-43): the naive stable radix
// cluster on bits [R, R + D) of key - 1 (partition.c:29), partitions back to
// back, no padding.  The reference INCREMENTS the caller's int32 hist
// (:111-113) and places partition i at the prefix sum of that hist (:116-122),
// so counts already in hist shift the starts; this keeps that: a zero hist
// (every reference caller) scatters straight into outRel, a non-zero one
// scatters into scratch and moves each partition to its shifted start.
void radix_cluster(relation_t* outRel, relation_t* inRel, int32_t* hist, int R, int D) {
    Ctx& c = ctx();
    const uint64_t n = inRel->num_tuples;
    const uint32_t fan = 1u << D;
    const uint32_t mask = (uint32_t)((((1ull << D) - 1) << R) & 0xffffffffull);
    DevBuf in = dev_in(inRel->tuples, n, "api_in", true);
    bool zero = true;
    for (uint32_t i = 0; i < fan; i++) zero = zero && hist[i] == 0;
    int64_t* dh = (int64_t*)c.ws.scratch("api_hist", fan * 8);
    int64_t* doff = (int64_t*)c.ws.scratch("api_off", fan * 8);
    const Digit32 dig{mask, (uint32_t)R};
    std::vector<int64_t> hh(fan), ho(fan);
    if (zero) {
        DevBuf out = dev_in(outRel->tuples, n, "api_out", false);
        stable_partition(&c.ws, in.d, n, out.d, dig, (uint32_t)D, 0, dh, doff, c.st);
        SMJ_CHECK(hipMemcpyAsync(hh.data(), dh, fan * 8, hipMemcpyDeviceToHost, c.st));
        dev_out(out, n);
        sync();
    } else {
        Tup* tmp = (Tup*)c.ws.scratch("api_rc", (n ? n : 1) * sizeof(Tup));
        stable_partition(&c.ws, in.d, n, tmp, dig, (uint32_t)D, 0, dh, doff, c.st);
        SMJ_CHECK(hipMemcpyAsync(hh.data(), dh, fan * 8, hipMemcpyDeviceToHost, c.st));
        SMJ_CHECK(hipMemcpyAsync(ho.data(), doff, fan * 8, hipMemcpyDeviceToHost, c.st));
        sync();
        const bool dev = is_device_ptr(outRel->tuples);
        uint32_t dst = 0;  // partition.c:116-122, offsets from the incremented hist
        for (uint32_t i = 0; i < fan; i++) {
            if (hh[i])
                SMJ_CHECK(hipMemcpyAsync(outRel->tuples + dst, tmp + ho[i],
                                         (size_t)hh[i] * sizeof(Tup),
                                         dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                                         c.st));
            dst += (uint32_t)(hist[i] + (int32_t)hh[i]);
        }
        sync();
    }
    for (uint32_t i = 0; i < fan; i++) hist[i] += (int32_t)hh[i];
}

// ---------------------------------------------------------------------------
// sorting (reference src/avxsort/avxsort.c:212-250, avxsort_multiway.c,
// src/scalarsort/scalarsort.c)
// ---------------------------------------------------------------------------
static void sort_tuples_into(const void* inp, void* outp, uint64_t n) {
    Ctx& c = ctx();
    DevBuf in = dev_in(inp, n, "api_in", true);
    DevBuf out = dev_in(outp, n, "api_out", false);
    device_sort(&c.ws, in.d, n, out.d, c.st);
    dev_out(out, n);
    sync();
}

void avxsort_tuples(tuple_t** inputptr, tuple_t** outputptr, uint64_t nitems) {
    if (nitems == 0) return;
    sort_tuples_into(*inputptr, *outputptr, nitems);
    // sorted items are in *outputptr; *inputptr stays the other buffer
}

void avxsortmultiway_tuples(tuple_t** inputptr, tuple_t** outputptr,
                            uint64_t nitems) {
    if (nitems == 0) return;
    sort_tuples_into(*inputptr, *outputptr, nitems);
}

void scalarsort_tuples(tuple_t** inputptr, tuple_t** outputptr,
                       uint64_t nitems) {
    // reference sorts in place, then swaps (scalarsort.c:41-50)
    tuple_t* in = *inputptr;
    tuple_t* out = *outputptr;
    if (nitems) sort_tuples_into(in, in, nitems);
    *inputptr = out;
    *outputptr = in;
}
}  // extern "C"

// ---- int64 / int32 item sorts: items viewed as tuples with key = value
// The AVX int64 entry points order their items as IEEE doubles (the
// networks' _mm256_min_pd/_max_pd, reference src/avxsort/avxcommon.h:79-190):
// sign-magnitude order for every non-NaN pattern, which this fork's (key, ptr)
// carriers rely on (SetKeyInt, avxcommon.h:205-213).  fp64_ord maps a pattern
// to a signed int64 of that order and is its own inverse; the scalar twins
// keep plain int64 order (std::sort, src/scalarsort/scalarsort.c:23-30).
__device__ __forceinline__ int64_t fp64_ord(int64_t x) {
    return x ^ ((x >> 63) & INT64_MAX);
}
__global__ void k_fp64_ord(const int64_t* __restrict__ a, int64_t* __restrict__ b,
                           uint64_t n) {
    const uint64_t s = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += s)
        b[i] = fp64_ord(a[i]);
}

__global__ void k_expand_i64(const int64_t* __restrict__ a, Tup* __restrict__ t,
                             uint64_t n, bool fp64) {
    const uint64_t s = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += s) {
#ifdef KEY_8B
        Tup x;
        x.key = fp64 ? fp64_ord(a[i]) : a[i];
        x.payload = 0;
        t[i] = x;
#else
        t[i] = (uint64_t)(fp64 ? fp64_ord(a[i]) : a[i]);
#endif
    }
}
__global__ void k_compact_i64(const Tup* __restrict__ t, int64_t* __restrict__ a,
                              uint64_t n, bool fp64) {
    const uint64_t s = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += s) {
#ifdef KEY_8B
        a[i] = fp64 ? fp64_ord(t[i].key) : t[i].key;
#else
        a[i] = fp64 ? fp64_ord((int64_t)t[i]) : (int64_t)t[i];
#endif
    }
}
__global__ void k_expand_i32(const int32_t* __restrict__ a, Tup* __restrict__ t,
                             uint64_t n) {
    const uint64_t s = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += s) {
#ifdef KEY_8B
        Tup x;
        x.key = a[i];
        x.payload = 0;
        t[i] = x;
#else
        t[i] = (uint64_t)(uint32_t)a[i] << 32;
#endif
    }
}
__global__ void k_compact_i32(const Tup* __restrict__ t, int32_t* __restrict__ a,
                              uint64_t n) {
    const uint64_t s = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += s)
        a[i] = (int32_t)tup_key(t[i]);
}

static uint32_t grid_n(uint64_t n) {
    uint64_t b = (n + 255) / 256;
    return (uint32_t)(b < 4096 ? (b ? b : 1) : 4096);
}

// inregister_sort_keyval32 (src/avxsort/avxsort_core.h:1213-1274): one
// lane per column of a 16-item block, {x[j], x[j+4], x[j+8], x[j+12]} through
// the reference's 4x4 odd-even network of VMINPD / VMAXPD, written as row j
// (the network's output after its 4x4 transpose).  VMINPD(a, b) = a < b ? a
// : b and VMAXPD(a, b) = a > b ? a : b as IEEE doubles -- an unordered pair (a
// NaN) or two zeros give the second operand -- compared on the bit patterns
// in integer arithmetic (sign-magnitude), so denormals and NaNs behave
// exactly as on the AVX unit.
__device__ __forceinline__ bool fp64_lt_bits(uint64_t a, uint64_t b) {
    const uint64_t ma = a & 0x7fffffffffffffffull, mb = b & 0x7fffffffffffffffull;
    if (ma > 0x7ff0000000000000ull || mb > 0x7ff0000000000000ull) return false;
    if ((ma | mb) == 0) return false;
    const int64_t ka = (int64_t)a < 0 ? -(int64_t)ma : (int64_t)ma;
    const int64_t kb = (int64_t)b < 0 ? -(int64_t)mb : (int64_t)mb;
    return ka < kb;
}

__global__ void __launch_bounds__(256)
k_inreg4x4(const uint64_t* __restrict__ in, uint64_t* __restrict__ out, uint64_t nblocks) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nblocks * 4) return;
    const uint64_t b = i >> 2;
    const uint32_t j = (uint32_t)(i & 3);
    const uint64_t* x = in + 16 * b;
    auto mn = [](uint64_t p, uint64_t q) { return fp64_lt_bits(p, q) ? p : q; };
    auto mx = [](uint64_t p, uint64_t q) { return fp64_lt_bits(q, p) ? p : q; };
    const uint64_t a = x[j], bb = x[4 + j], c = x[8 + j], d = x[12 + j];
    const uint64_t a1 = mn(a, bb), b1 = mx(a, bb), c1 = mn(c, d), d1 = mx(c, d);
    const uint64_t b2 = mn(b1, d1), d2 = mx(b1, d1);
    const uint64_t a2 = mn(a1, c1), c2 = mx(a1, c1);
    const uint64_t b3 = mn(b2, c2), c3 = mx(b2, c2);
    uint64_t* o = out + 16 * b + 4 * j;
    o[0] = a2;
    o[1] = b3;
    o[2] = c3;
    o[3] = d2;
}

static void sort_int64_into(const int64_t* inp, int64_t* outp, uint64_t n, bool fp64) {
    if (n == 0) return;
    Ctx& c = ctx();
    const bool din = is_device_ptr(inp), dout = is_device_ptr(outp);
#ifndef KEY_8B
    if (!fp64) {
        sort_tuples_into(inp, outp, n);  // an 8-byte tuple is an int64 word
        return;
    }
    // map to int64 order, sort the words as tuples, map back
    int64_t* t = (int64_t*)c.ws.scratch("api_i64_t", n * 8);
    int64_t* u = (int64_t*)c.ws.scratch("api_i64_u", n * 8);
    const int64_t* src = inp;
    if (!din) {
        SMJ_CHECK(hipMemcpyAsync(t, inp, n * 8, hipMemcpyHostToDevice, c.st));
        src = t;
    }
    hipLaunchKernelGGL(k_fp64_ord, dim3(grid_n(n)), dim3(256), 0, c.st, src, t, n);
    device_sort(&c.ws, (const Tup*)t, n, (Tup*)u, c.st);
    int64_t* dst = dout ? outp : t;
    hipLaunchKernelGGL(k_fp64_ord, dim3(grid_n(n)), dim3(256), 0, c.st, u, dst, n);
    if (!dout) SMJ_CHECK(hipMemcpyAsync(outp, t, n * 8, hipMemcpyDeviceToHost, c.st));
    sync();
#else
    int64_t* di = (int64_t*)inp;
    int64_t* dout_p = outp;
    if (!din) {
        di = (int64_t*)c.ws.scratch("api_i64_in", n * 8);
        SMJ_CHECK(hipMemcpyAsync(di, inp, n * 8, hipMemcpyHostToDevice, c.st));
    }
    if (!dout) dout_p = (int64_t*)c.ws.scratch("api_i64_out", n * 8);
    Tup* t = (Tup*)c.ws.scratch("api_i64_t", n * sizeof(Tup));
    Tup* u = (Tup*)c.ws.scratch("api_i64_u", n * sizeof(Tup));
    hipLaunchKernelGGL(k_expand_i64, dim3(grid_n(n)), dim3(256), 0, c.st, di, t, n, fp64);
    device_sort(&c.ws, t, n, u, c.st);
    hipLaunchKernelGGL(k_compact_i64, dim3(grid_n(n)), dim3(256), 0, c.st, u, dout_p, n, fp64);
    if (!dout)
        SMJ_CHECK(hipMemcpyAsync(outp, dout_p, n * 8, hipMemcpyDeviceToHost, c.st));
    sync();
#endif
}

static void sort_int32_into(const int32_t* inp, int32_t* outp, uint64_t n) {
    if (n == 0) return;
    Ctx& c = ctx();
    const bool din = is_device_ptr(inp), dout = is_device_ptr(outp);
    int32_t* di = (int32_t*)inp;
    int32_t* dout_p = outp;
    if (!din) {
        di = (int32_t*)c.ws.scratch("api_i32_in", n * 4);
        SMJ_CHECK(hipMemcpyAsync(di, inp, n * 4, hipMemcpyHostToDevice, c.st));
    }
    if (!dout) dout_p = (int32_t*)c.ws.scratch("api_i32_out", n * 4);
    Tup* t = (Tup*)c.ws.scratch("api_i32_t", n * sizeof(Tup));
    Tup* u = (Tup*)c.ws.scratch("api_i32_u", n * sizeof(Tup));
    hipLaunchKernelGGL(k_expand_i32, dim3(grid_n(n)), dim3(256), 0, c.st, di, t, n);
    device_sort(&c.ws, t, n, u, c.st);
    hipLaunchKernelGGL(k_compact_i32, dim3(grid_n(n)), dim3(256), 0, c.st, u, dout_p, n);
    if (!dout)
        SMJ_CHECK(hipMemcpyAsync(outp, dout_p, n * 4, hipMemcpyDeviceToHost, c.st));
    sync();
}

extern "C" {

void smj_inregister_sort_keyval32(const int64_t* items, int64_t* output, uint64_t nblocks) {
    if (nblocks == 0) return;
    Ctx& c = ctx();
    const uint64_t ntup = nblocks * 128 / sizeof(Tup);
    DevBuf in = dev_in(items, ntup, "api_ir_in", true);
    DevBuf out = dev_in(output, ntup, "api_ir_out", false);
    const uint64_t lanes = nblocks * 4;
    hipLaunchKernelGGL(k_inreg4x4, dim3((uint32_t)((lanes + 255) / 256)), dim3(256), 0, c.st,
                       (const uint64_t*)in.d, (uint64_t*)out.d, nblocks);
    SMJ_CHECK(hipGetLastError());
    dev_out(out, ntup);
    sync();
}

void avxsort_int64(int64_t** inputptr, int64_t** outputptr, uint64_t nitems) {
    sort_int64_into(*inputptr, *outputptr, nitems, true);
}
void avxsortmultiway_int64(int64_t** inputptr, int64_t** outputptr,
                           uint64_t nitems) {
    sort_int64_into(*inputptr, *outputptr, nitems, true);
}
void avxsort_int32(int32_t** inputptr, int32_t** outputptr, uint64_t nitems) {
    sort_int32_into(*inputptr, *outputptr, nitems);
}
void scalarsort_int64(int64_t** inputptr, int64_t** outputptr, uint64_t nitems) {
    int64_t* in = *inputptr;
    int64_t* out = *outputptr;
    sort_int64_into(in, in, nitems, false);
    *inputptr = out;
    *outputptr = in;
}
void scalarsort_int32(int32_t** inputptr, int32_t** outputptr, uint64_t nitems) {
    int32_t* in = *inputptr;
    int32_t* out = *outputptr;
    sort_int32_into(in, in, nitems);
    *inputptr = out;
    *outputptr = in;
}

// ---------------------------------------------------------------------------
// merging (reference src/merge/merge.c:27-235, avx_multiwaymerge.c:199-338,
// scalar_multiwaymerge.c)
// ---------------------------------------------------------------------------
static uint64_t merge_tuples_common(const void* A, const void* B, void* O,
                                   uint64_t la, uint64_t lb) {
    Ctx& c = ctx();
    DevBuf a = dev_in(A, la, "api_ma", true);
    DevBuf b = dev_in(B, lb, "api_mb", true);
    DevBuf o = dev_in(O, la + lb, "api_mo", false);
    merge2(&c.ws, a.d, la, b.d, lb, o.d, c.st);
    dev_out(o, la + lb);
    sync();
    return la + lb;
}

uint64_t avx_merge_tuples(tuple_t* const inA, tuple_t* const inB,
                          tuple_t* const outp, const uint64_t lenA,
                          const uint64_t lenB) {
    return merge_tuples_common(inA, inB, outp, lenA, lenB);
}
uint64_t scalar_merge_tuples(tuple_t* const inA, tuple_t* const inB,
                             tuple_t* const outp, const uint64_t lenA,
                             const uint64_t lenB) {
    return merge_tuples_common(inA, inB, outp, lenA, lenB);
}

static uint64_t merge_int64_common(const int64_t* A, const int64_t* B, int64_t* O,
                                   uint64_t la, uint64_t lb, bool fp64) {
#ifndef KEY_8B
    if (!fp64) return merge_tuples_common(A, B, O, la, lb);
#endif
    // stage, map to int64 order (or widen to 16-byte tuples), merge, map back
    Ctx& c = ctx();
    const uint64_t n = la + lb;
    if (n == 0) return 0;
    int64_t* da = (int64_t*)c.ws.scratch("api_mi_a", (la ? la : 1) * 8);
    int64_t* db = (int64_t*)c.ws.scratch("api_mi_b", (lb ? lb : 1) * 8);
    int64_t* dn = (int64_t*)c.ws.scratch("api_mi_o", n * 8);
    if (la) SMJ_CHECK(hipMemcpyAsync(da, A, la * 8, hipMemcpyDefault, c.st));
    if (lb) SMJ_CHECK(hipMemcpyAsync(db, B, lb * 8, hipMemcpyDefault, c.st));
#ifndef KEY_8B
    if (la) hipLaunchKernelGGL(k_fp64_ord, dim3(grid_n(la)), dim3(256), 0, c.st, da, da, la);
    if (lb) hipLaunchKernelGGL(k_fp64_ord, dim3(grid_n(lb)), dim3(256), 0, c.st, db, db, lb);
    merge2(&c.ws, (const Tup*)da, la, (const Tup*)db, lb, (Tup*)dn, c.st);
    hipLaunchKernelGGL(k_fp64_ord, dim3(grid_n(n)), dim3(256), 0, c.st, dn, dn, n);
#else
    Tup* ta = (Tup*)c.ws.scratch("api_mi_ta", (la ? la : 1) * sizeof(Tup));
    Tup* tb = (Tup*)c.ws.scratch("api_mi_tb", (lb ? lb : 1) * sizeof(Tup));
    Tup* to = (Tup*)c.ws.scratch("api_mi_to", n * sizeof(Tup));
    if (la) hipLaunchKernelGGL(k_expand_i64, dim3(grid_n(la)), dim3(256), 0, c.st, da, ta, la, fp64);
    if (lb) hipLaunchKernelGGL(k_expand_i64, dim3(grid_n(lb)), dim3(256), 0, c.st, db, tb, lb, fp64);
    merge2(&c.ws, ta, la, tb, lb, to, c.st);
    hipLaunchKernelGGL(k_compact_i64, dim3(grid_n(n)), dim3(256), 0, c.st, to, dn, n, fp64);
#endif
    SMJ_CHECK(hipMemcpyAsync(O, dn, n * 8, hipMemcpyDefault, c.st));
    sync();
    return n;
}

uint64_t avx_merge_int64(int64_t* const inA, int64_t* const inB,
                         int64_t* const outp, const uint64_t lenA,
                         const uint64_t lenB) {
    return merge_int64_common(inA, inB, outp, lenA, lenB, true);
}
uint64_t scalar_merge_int64(int64_t* const inA, int64_t* const inB,
                            int64_t* const outp, const uint64_t lenA,
                            const uint64_t lenB) {
    return merge_int64_common(inA, inB, outp, lenA, lenB, false);
}

static uint64_t multiway_common(tuple_t* output, relation_t** parts,
                                uint32_t nparts) {
    Ctx& c = ctx();
    std::vector<const Tup*> runs(nparts);
    std::vector<uint64_t> lens(nparts);
    uint64_t total = 0;
    for (uint32_t i = 0; i < nparts; i++) total += parts[i]->num_tuples;
    // stage host runs into one packed device buffer
    bool all_dev = is_device_ptr(output);
    for (uint32_t i = 0; i < nparts && all_dev; i++)
        if (parts[i]->num_tuples && !is_device_ptr(parts[i]->tuples)) all_dev = false;
    Tup* packed = nullptr;
    if (!all_dev) packed = (Tup*)c.ws.scratch("api_mw_in", (total ? total : 1) * sizeof(Tup));
    uint64_t o = 0;
    for (uint32_t i = 0; i < nparts; i++) {
        lens[i] = parts[i]->num_tuples;
        if (all_dev) {
            runs[i] = (const Tup*)parts[i]->tuples;
        } else {
            runs[i] = packed + o;
            if (lens[i])
                SMJ_CHECK(hipMemcpyAsync(packed + o, parts[i]->tuples,
                                         lens[i] * sizeof(Tup), hipMemcpyDefault,
                                         c.st));
            o += lens[i];
        }
    }
    Tup* out = all_dev ? (Tup*)output
                       : (Tup*)c.ws.scratch("api_mw_out", (total ? total : 1) * sizeof(Tup));
    multiway_merge(&c.ws, runs.data(), lens.data(), nparts, out, c.st);
    if (!all_dev && total)
        SMJ_CHECK(hipMemcpyAsync(output, out, total * sizeof(Tup),
                                 hipMemcpyDeviceToHost, c.st));
    sync();
    // the reference consumes its inputs (avx_multiwaymerge.c:268-272)
    for (uint32_t i = 0; i < nparts; i++) {
        parts[i]->tuples += parts[i]->num_tuples;
        parts[i]->num_tuples = 0;
    }
    return total;
}

uint64_t avx_multiway_merge(tuple_t* output, relation_t** parts,
                            uint32_t nparts, tuple_t* fifobuffer,
                            uint32_t bufntuples) {
    (void)fifobuffer;
    (void)bufntuples;
    return multiway_common(output, parts, nparts);
}
uint64_t scalar_multiway_merge(tuple_t* output, relation_t** parts,
                               uint32_t nparts, tuple_t* fifobuffer,
                               uint32_t bufntuples) {
    (void)fifobuffer;
    (void)bufntuples;
    return multiway_common(output, parts, nparts);
}
uint64_t scalar_multiway_merge_modulo(tuple_t* output, relation_t** parts,
                                      uint32_t nparts, tuple_t* fifobuffer,
                                      uint32_t bufntuples) {
    (void)fifobuffer;
    (void)bufntuples;
    return multiway_common(output, parts, nparts);
}
uint64_t scalar_multiway_merge_bitand(tuple_t* output, relation_t** parts,
                                      uint32_t nparts, tuple_t* fifobuffer,
                                      uint32_t bufntuples) {
    (void)fifobuffer;
    (void)bufntuples;
    return multiway_common(output, parts, nparts);
}

// ---------------------------------------------------------------------------
// joins (reference src/joins/joincommon.c:239-312,
// src/joins/sortmergejoin_multiway.c:50-61)
// ---------------------------------------------------------------------------
// ---- materialised output (JOIN_MATERIALIZE; smj.h documents the buffer)
chainedtuplebuffer_t* chainedtuplebuffer_init(void) {
    return (chainedtuplebuffer_t*)calloc(1, sizeof(chainedtuplebuffer_t));
}

void chainedtuplebuffer_free(chainedtuplebuffer_t* cb) {
    if (!cb) return;
    free(cb->tuples);
    free(cb);
}

uint64_t chainedtuplebuffer_tuples(chainedtuplebuffer_t* cb) { return cb ? cb->numtuples : 0; }

// room for k more tuples at the end; returns where they go
static tuple_t* cb_reserve(chainedtuplebuffer_t* cb, uint64_t k) {
    if (cb->numtuples + k > cb->capacity) {
        uint64_t cap = cb->capacity ? cb->capacity : 1024;
        while (cap < cb->numtuples + k) cap *= 2;
        tuple_t* t = (tuple_t*)realloc(cb->tuples, cap * sizeof(tuple_t));
        if (!t) {
            fprintf(stderr, "[ERROR] smj: cannot grow the result buffer to %llu tuples\n",
                    (unsigned long long)cap);
            abort();
        }
        cb->tuples = t;
        cb->capacity = cap;
    }
    tuple_t* at = cb->tuples + cb->numtuples;
    cb->numtuples += k;
    return at;
}

tuple_t* cb_next_writepos(chainedtuplebuffer_t* cb) { return cb_reserve(cb, 1); }

// the matches of sorted device runs R and S, appended to cb (two device
// passes: the count sizes the device buffer, the second writes it)
}  // extern "C"
namespace smj {
uint64_t materialize_append_on(Workspace* wsp, hipStream_t st, const Tup* r, uint64_t nR,
                               const Tup* s, uint64_t nS, chainedtuplebuffer_t* cb) {
    smj_workspace* ws = (smj_workspace*)wsp;
    const uint64_t total = smj_dev_materialize(ws, (const tuple_t*)r, nR, (const tuple_t*)s,
                                               nS, nullptr, 0, st);
    if (total == 0) return 0;
    Tup* o = (Tup*)wsp->scratch("api_mat", total * sizeof(Tup));
    const uint64_t got = smj_dev_materialize(ws, (const tuple_t*)r, nR, (const tuple_t*)s, nS,
                                             (tuple_t*)o, total, st);
    if (got != total) {
        fprintf(stderr, "[ERROR] smj: materialisation count changed (%llu, %llu)\n",
                (unsigned long long)total, (unsigned long long)got);
        abort();
    }
    tuple_t* dst = cb_reserve(cb, total);
    SMJ_CHECK(hipMemcpyAsync(dst, o, total * sizeof(Tup), hipMemcpyDeviceToHost, st));
    SMJ_CHECK(hipStreamSynchronize(st));
    return total;
}
}  // namespace smj
extern "C" {

static uint64_t materialize_append(const Tup* r, uint64_t nR, const Tup* s, uint64_t nS,
                                   chainedtuplebuffer_t* cb) {
    Ctx& c = ctx();
    return materialize_append_on(&c.ws, c.st, r, nR, s, nS, cb);
}

// Process-wide, like the reference's compile-time -DJOIN_MATERIALIZE that it
// stands for: every join of the process sees the last value set (atomic, so
// concurrent callers read a whole value; callers that need different modes
// at once must not share a process).  -1: not decided yet (SMJ_MATERIALIZE).
static std::atomic<int> g_materialize{-1};

void smj_set_materialize(int on) { g_materialize.store(on ? 1 : 0); }

}  // extern "C"
namespace smj {
bool materialize_on() {
    int v = g_materialize.load();
    if (v < 0) {
        const char* e = getenv("SMJ_MATERIALIZE");
        int want = (e && atoi(e) != 0) ? 1 : 0;
        g_materialize.compare_exchange_strong(v, want);
        v = g_materialize.load();
    }
    return v > 0;
}
}  // namespace smj
extern "C" {

// decimal of a signed 32-bit value into p; returns the end
static char* put_i32(char* p, int32_t v) {
    char tmp[12];
    int k = 0;
    uint32_t u = v < 0 ? 0u - (uint32_t)v : (uint32_t)v;
    do {
        tmp[k++] = (char)('0' + u % 10);
        u /= 10;
    } while (u);
    if (v < 0) *p++ = '-';
    while (k) *p++ = tmp[--k];
    return p;
}

void write_result_relation(result_t* result, const char* filename) {
    if (!result) return;
    FILE* fp = fopen(filename, "a");
    if (!fp) {
        perror("write_result_relation");
        return;
    }
    fprintf(fp, "#KEY, VAL\n");
    const int T = result->nthreads > 0 ? result->nthreads : 1;
    std::vector<char> buf(1 << 20);
    for (int i = 0; i < T && result->resultlist; i++) {
        chainedtuplebuffer_t* cb = (chainedtuplebuffer_t*)result->resultlist[i].results;
        if (!cb) continue;
        char* p = buf.data();
        for (uint64_t j = 0; j < cb->numtuples; j++) {
            if (p - buf.data() > (ptrdiff_t)buf.size() - 32) {
                fwrite(buf.data(), 1, p - buf.data(), fp);
                p = buf.data();
            }
            // generator.c:210 prints key and payload with %d
            p = put_i32(p, (int32_t)cb->tuples[j].key);
            *p++ = ' ';
            p = put_i32(p, (int32_t)cb->tuples[j].payload);
            *p++ = '\n';
        }
        fwrite(buf.data(), 1, p - buf.data(), fp);
    }
    fclose(fp);
}

uint64_t merge_join(tuple_t* rtuples, tuple_t* stuples, const uint64_t numR,
                    const uint64_t numS, void* output) {
    Ctx& c = ctx();
    DevBuf r = dev_in(rtuples, numR, "api_jr", true);
    DevBuf s = dev_in(stuples, numS, "api_js", true);
    if (output)  // JOIN_MATERIALIZE: output is the caller's chainedtuplebuffer_t
        return materialize_append(r.d, numR, s.d, numS, (chainedtuplebuffer_t*)output);
    unsigned long long* cnt =
        (unsigned long long*)c.ws.scratch("api_cnt", sizeof(unsigned long long));
    SMJ_CHECK(hipMemsetAsync(cnt, 0, 8, c.st));
    merge_join_count(r.d, numR, s.d, numS, cnt, c.st);
    unsigned long long* hc = (unsigned long long*)c.ws.host_pinned("mj_cnt_h", 8);
    SMJ_CHECK(hipMemcpyAsync(hc, cnt, 8, hipMemcpyDeviceToHost, c.st));
    sync();
    return *hc;
}

uint64_t merge_join_interpolation(tuple_t* rtuples, tuple_t* stuples,
                                  const uint64_t numR, const uint64_t numS,
                                  void* output) {
    // the interpolation search only picks the CPU scan's start; the device
    // merge-path count needs none
    return merge_join(rtuples, stuples, numR, numS, output);
}

// joincommon.c:397-500 (declared joincommon.h:99-100): 1 when the keys of the
// `nitems` tuples at `items` never decrease, starting from key 0.  The 8-byte
// build (no KEY_8B) prints the reference's warning at the first equal key
// before any decrease and its error line at the first decrease; the KEY_8B
// build prints nothing.  The scan runs on the device (k_sorted_scan).
int is_sorted_helper(int64_t* items, uint64_t nitems) {
    if (nitems == 0) return 1;
    Ctx& c = ctx();
    DevBuf t = dev_in(items, nitems, "api_chk", true);
    unsigned long long* first = (unsigned long long*)c.ws.scratch("api_chk_first", 16);
    const unsigned long long init[2] = {~0ull, ~0ull};
    unsigned long long* h = (unsigned long long*)c.ws.host_pinned("api_chk_h", 16);
    memcpy(h, init, 16);
    SMJ_CHECK(hipMemcpyAsync(first, h, 16, hipMemcpyHostToDevice, c.st));
    uint64_t g = (nitems + 255) / 256;
    if (g > 2048) g = 2048;
    hipLaunchKernelGGL(k_sorted_scan, dim3((uint32_t)g), dim3(256), 0, c.st, t.d, nitems, first);
    SMJ_CHECK(hipGetLastError());
    SMJ_CHECK(hipMemcpyAsync(h, first, 16, hipMemcpyDeviceToHost, c.st));
    sync();
    const unsigned long long bad = h[0], eq = h[1];
#ifndef KEY_8B
    // the key at position i and its predecessor's (0 before item 0)
    auto key_at = [&](unsigned long long i) -> int32_t {
        Tup v;
        SMJ_CHECK(hipMemcpy(&v, t.d + i, sizeof(Tup), hipMemcpyDeviceToHost));
        return (int32_t)tup_key(v);
    };
    if (eq != ~0ull && eq < bad)
        printf("[WARN ] Equal items, still ok... item[%d].key=%d is equal to item[%d].key=%d\n",
               (int)eq, key_at(eq), (int)(eq - 1), key_at(eq));
    if (bad != ~0ull)
        printf("[ERROR] item[%d].key=%d is less than item[%d].key=%d\n", (int)bad, key_at(bad),
               (int)(bad - 1), bad ? key_at(bad - 1) : 0);
    fflush(stdout);
#endif
    return bad == ~0ull ? 1 : 0;
}

// joincommon.c:503-515 (declared joincommon.h:101-103)
void check_sorted(int64_t* R, int64_t* S, uint64_t nR, uint64_t nS, int my_tid) {
    if (is_sorted_helper(R, nR))
        printf("%d-thread -> R is sorted, size = %d\n", my_tid, (int)nR);
    else
        printf("%d-thread -> R is NOT sorted, size = %d\n", my_tid, (int)nR);
    if (is_sorted_helper(S, nS))
        printf("%d-thread -> S is sorted, size = %d\n", my_tid, (int)nS);
    else
        printf("%d-thread -> S is NOT sorted, size = %d\n", my_tid, (int)nS);
    fflush(stdout);
}

// joincommon.c:29-212.  The orchestration of the reference's T join threads,
// kept for drivers that bring their own join thread (tputbench.c:124-144).
// The CPU mapping (src/util/cpu_mapping.c) is the driver's: when the driver
// links it, thread i is pinned to get_cpu_id(i) and marked active in its NUMA
// region as joincommon.c:118-126 does (the driver's threads look themselves
// up there); the weak references resolve to nothing otherwise.  The chunk
// sizes are computed in 64 bits before they land in arg_t's int32 fields.
extern "C" int get_cpu_id(int thread_id) __attribute__((weak));
extern "C" void numa_thread_mark_active(int phytid) __attribute__((weak));
static void* host_alloc64(size_t bytes) {
    void* p = nullptr;
    if (posix_memalign(&p, CACHE_LINE_SIZE, bytes ? bytes : CACHE_LINE_SIZE)) {
        perror("[ERROR] smj: posix_memalign");
        exit(EXIT_FAILURE);
    }
    return p;
}

result_t* sortmergejoin_initrun(relation_t* relR, relation_t* relS,
                                joinconfig_t* joincfg,
                                void* (*jointhread)(void*)) {
    const int T = joincfg->NTHREADS;
    const int F = joincfg->PARTFANOUT;
    if (T <= 0) {
        fprintf(stdout, "[ERROR] NTHREADS must be positive.\n");
        return 0;
    }
    const uint64_t nR = relR->num_tuples, nS = relS->num_tuples;
    const size_t pad = RELATION_PADDING(T, F);
    tuple_t* tmpPR = (tuple_t*)host_alloc64(nR * sizeof(tuple_t) + pad);
    tuple_t* tmpPS = (tuple_t*)host_alloc64(nS * sizeof(tuple_t) + pad);
    tuple_t* tmpSR = (tuple_t*)host_alloc64(nR * sizeof(tuple_t) + pad);
    tuple_t* tmpSS = (tuple_t*)host_alloc64(nS * sizeof(tuple_t) + pad);
    relationpair_t** chunks = (relationpair_t**)calloc(T, sizeof(relationpair_t*));
    uint32_t** histR = (uint32_t**)calloc(T, sizeof(uint32_t*));
    // indexed by the driver's NUMA region id (< T, or 0 without libnuma)
    tuple_t** shared = (tuple_t**)calloc(T < 64 ? 64 : T, sizeof(tuple_t*));
    arg_t* args = (arg_t*)host_alloc64(sizeof(arg_t) * T);
    memset(args, 0, sizeof(arg_t) * T);
    std::vector<pthread_t> tid(T);
    pthread_barrier_t barrier;
    if (pthread_barrier_init(&barrier, NULL, T) != 0) {
        printf("[ERROR] Couldn't create the barrier\n");
        exit(EXIT_FAILURE);
    }
    pthread_attr_t attr;
    pthread_attr_init(&attr);
    size_t stack = 0;
    pthread_attr_getstacksize(&attr, &stack);
    const size_t kStack = 32u << 20;  // joincommon.c:26 REQUIRED_STACK_SIZE
    if (stack < kStack && pthread_attr_setstacksize(&attr, kStack)) {
        perror("[ERROR] pthread stack size could not be set!");
        exit(0);
    }
    const uint64_t perR = nR / T, perS = nS / T;
    const uint64_t cpad = CACHELINEPADDING(F);
    result_t* res = (result_t*)malloc(sizeof(result_t));
    res->resultlist = (threadresult_t*)calloc(T, sizeof(threadresult_t));
    for (int i = 0; i < T; i++) {
        arg_t& a = args[i];
        a.relR = relR->tuples + i * perR;
        a.relS = relS->tuples + i * perS;
        a.tmp_partR = tmpPR + i * (perR + cpad);
        a.tmp_partS = tmpPS + i * (perS + cpad);
        a.tmp_sortR = tmpSR + i * perR;
        a.tmp_sortS = tmpSS + i * perS;
        a.numR = (int32_t)(i == T - 1 ? nR - i * perR : perR);
        a.numS = (int32_t)(i == T - 1 ? nS - i * perS : perS);
        a.my_tid = i;
        a.nthreads = T;
        a.joincfg = joincfg;
        a.barrier = &barrier;
        a.threadrelchunks = chunks;
        a.sharedmergebuffer = shared;
        a.histR = histR;
        a.tmpRglobal = tmpPR;
        a.totalR = nR;
        if (get_cpu_id) {
            const int cpu = get_cpu_id(i);
            if (numa_thread_mark_active) numa_thread_mark_active(cpu);
            cpu_set_t set;
            CPU_ZERO(&set);
            CPU_SET(cpu, &set);
            pthread_attr_setaffinity_np(&attr, sizeof(cpu_set_t), &set);
        }
#ifdef JOIN_MATERIALIZE
        a.threadresult = &res->resultlist[i];
#endif
        const int rv = pthread_create(&tid[i], &attr, jointhread, (void*)&a);
        if (rv) {
            printf("[ERROR] return code from pthread_create() is %d\n", rv);
            exit(-1);
        }
    }
    int64_t total = 0;
    for (int i = 0; i < T; i++) {
        pthread_join(tid[i], NULL);
        total += args[i].result;
        res->resultlist[i].nresults = args[i].result;
    }
    res->totalresults = total;
    res->nthreads = T;
    // joincommon.c:176-199, the same lines from args[0]'s timers
    const arg_t& a0 = args[0];
    fprintf(stdout, "Total, Partitioning, Sort, First-Merge, Merge, Join\n");
    fprintf(stdout, "%llu, %llu, %llu, %llu, %llu, %llu\n",
            (unsigned long long)a0.join, (unsigned long long)a0.part,
            (unsigned long long)a0.sort, (unsigned long long)a0.mergedelta,
            (unsigned long long)a0.merge, (unsigned long long)a0.join);
    fprintf(stdout, "Perstage: ");
    fflush(stdout);
    fprintf(stderr, "%llu, %llu, %llu, %llu, %llu, ", (unsigned long long)a0.part,
            (unsigned long long)(a0.sort - a0.part),
            (unsigned long long)(a0.mergedelta - a0.sort),
            (unsigned long long)(a0.merge - a0.mergedelta),
            (unsigned long long)(a0.join - a0.merge));
    fflush(stderr);
    fprintf(stdout, "\n");
    print_timing(nS, &args[0].start, &args[0].end, stderr);
    const bool owned = args[0].tmp_partR != 0;
    free(chunks);
    free(shared);
    free(histR);
    free(args);
    if (owned) {
        free(tmpPR);
        free(tmpPS);
        free(tmpSR);
        free(tmpSS);
    }
    pthread_attr_destroy(&attr);
    pthread_barrier_destroy(&barrier);
    return res;
}

// mat: the materialisation of this call (1 / 0), or -1 for the process
// default (smj_set_materialize / SMJ_MATERIALIZE)
static result_t* join_api(relation_t* relR, relation_t* relS,
                          joinconfig_t* joincfg, const char* name, int mat = -1) {
    if ((joincfg->NTHREADS & (joincfg->NTHREADS - 1)) != 0) {
        fprintf(stdout, "[ERROR] %s sort-merge join runs with a power of 2 "
                        "#threads.\n", name);
        return 0;
    }
    Ctx& c = ctx();
    struct timeval t0, t1;
    gettimeofday(&t0, NULL);
    const uint64_t nR = relR->num_tuples, nS = relS->num_tuples;
    DevBuf r = dev_in(relR->tuples, nR, "api_jr", true);
    DevBuf s = dev_in(relS->tuples, nS, "api_js", true);
    Tup* sR = (Tup*)c.ws.scratch("api_sortedR", (nR ? nR : 1) * sizeof(Tup));
    Tup* sS = (Tup*)c.ws.scratch("api_sortedS", (nS ? nS : 1) * sizeof(Tup));
    unsigned long long* cnt =
        (unsigned long long*)c.ws.scratch("api_cnt", sizeof(unsigned long long));
    uint32_t fb = 0;
    if (joincfg->PARTFANOUT > 0) fb = ceil_log2((uint64_t)joincfg->PARTFANOUT);
    // the reference fan-out (128 by default) only sizes the level-1 pass here;
    // choose_levels raises it as the relation size needs
    if (fb < 8) fb = 8;
    // no key-range hint: the plan is guessed from |R| as the reference does
    // (keys 1..|R|) and verified by the level-1 scatter
    device_join(&c.ws, r.d, nR, s.d, nS, sR, sS, fb, 1, 0, cnt, c.st, nR);
    // the count comes back through pinned memory (a pageable destination
    // would stage the copy)
    unsigned long long* hc = (unsigned long long*)c.ws.host_pinned("api_cnt_h", 8);
    SMJ_CHECK(hipMemcpyAsync(hc, cnt, 8, hipMemcpyDeviceToHost, c.st));
    sync();
    const unsigned long long h = *hc;
    gettimeofday(&t1, NULL);
    result_t* res = (result_t*)malloc(sizeof(result_t));
    res->totalresults = (int64_t)h;
    res->nthreads = joincfg->NTHREADS;
    res->resultlist =
        (threadresult_t*)calloc(joincfg->NTHREADS > 0 ? joincfg->NTHREADS : 1,
                                sizeof(threadresult_t));
    res->resultlist[0].nresults = (int64_t)h;
    if (mat < 0 ? materialize_on() : mat > 0) {
        chainedtuplebuffer_t* cb = chainedtuplebuffer_init();
        materialize_append(sR, nR, sS, nS, cb);
        res->resultlist[0].results = cb;
    }
    if (!getenv("SMJ_QUIET")) {
        float ms[5];
        smj_join_phase_ms((smj_workspace*)&c.ws, ms);
        // same shape as the reference's stats lines (joincommon.c:176-196);
        // phase values are device nanoseconds instead of TSC cycles
        fprintf(stdout, "Total, Partitioning, Sort, First-Merge, Merge, Join\n");
        fprintf(stdout, "%llu, %llu, %llu, %llu, %llu, %llu\n",
                (unsigned long long)(ms[4] * 1e6), (unsigned long long)(ms[0] * 1e6),
                (unsigned long long)((ms[0] + ms[1]) * 1e6),
                (unsigned long long)((ms[0] + ms[1]) * 1e6),
                (unsigned long long)((ms[0] + ms[1]) * 1e6),
                (unsigned long long)(ms[4] * 1e6));
        double us = (t1.tv_sec - t0.tv_sec) * 1e6 + (t1.tv_usec - t0.tv_usec);
        fprintf(stderr, "NUM-TUPLES = %lld TOTAL-TIME-USECS = %.4lf ",
                (long long)nS, us);
        fprintf(stderr, "TUPLES-PER-SECOND = %.4lf ", nS / (us / 1e6));
        fflush(stdout);
        fflush(stderr);
    }
    return res;
}

result_t* sortmergejoin_multiway(relation_t* relR, relation_t* relS,
                                 joinconfig_t* joincfg) {
    return join_api(relR, relS, joincfg, "m-way");
}

// sortmergejoin_mpsm.c:38-45 is a stub in the reference; SURVEY.md §2 row 9
// and BASELINE configs[4] make it the multi-GPU join: NTHREADS ranks, one per
// visible GPU (mgpu.hip)
result_t* sortmergejoin_mpsm(relation_t* relR, relation_t* relS,
                             joinconfig_t* joincfg) {
    return mpsm_api(relR, relS, joincfg, -1);
}

void print_timing(uint64_t numtuples, struct timeval* start, struct timeval* end,
                  FILE* out) {
    const double us = (double)((end->tv_sec * 1000000L + end->tv_usec) -
                               (start->tv_sec * 1000000L + start->tv_usec));
    fprintf(out, "NUM-TUPLES = %lld TOTAL-TIME-USECS = %.4lf ", (long long)numtuples, us);
    fprintf(out, "TUPLES-PER-SECOND = ");
    fflush(out);
    fprintf(out, "%.4lf ", numtuples / (us / 1000000L));
    fflush(out);
}

// m-pass (src/joins/sortmergejoin_multipass.c:51-736) in the reference's
// phases, for its T = NTHREADS threads (each a chunk of n / T tuples, the
// last one the rest, joincommon.c), on the device:
//   mpass_partitioning_phase (:295-335)  every chunk radix-partitioned into
//       F = PARTFANOUT partitions on the key bits above
//       shift = ceil(log2(chunk * T)) - log2(F) - 1 (:323-328; the digit of
//       partition.c:29, ((key - 1) & mask) >> shift);
//   mpass_sorting_phase (:337-409)      every (chunk, partition) run sorted on
//       its own (segmented sort: LDS block sorts, then 2-way merge passes);
//   mpass_firstnumamerge_phase (:411-619) thread t owns partitions
//       [t F / T, (t + 1) F / T); their runs from the T chunks are merged
//       pairwise (chunks 2i, 2i + 1 of one partition), then
//   mpass_fullmultipassmerge_phase (:621-708) thread t's runs are merged pass
//       by pass with 2-way merges into one sorted relation per thread (both
//       phases: the merge-path tree over the runs in that order);
//   mpass_mergejoin_phase (:711-736)    one merge-join scan per thread, the
//       counts summed.
// Unlike m-way (one multi-way merge, fused here into the bucket sort) every
// merge pass reads and writes both relations once more.
static result_t* multipass_api(relation_t* relR, relation_t* relS, joinconfig_t* joincfg,
                               int mat) {
    if ((joincfg->NTHREADS & (joincfg->NTHREADS - 1)) != 0) {
        fprintf(stdout, "[ERROR] m-pass sort-merge join runs with a power of 2 "
                        "#threads.\n");
        return 0;
    }
    Ctx& c = ctx();
    struct timeval t0, t1;
    gettimeofday(&t0, NULL);
    const uint64_t nR = relR->num_tuples, nS = relS->num_tuples;
    DevBuf r = dev_in(relR->tuples, nR, "api_jr", true);
    DevBuf s = dev_in(relS->tuples, nS, "api_js", true);
    Tup* sR = (Tup*)c.ws.scratch("api_sortedR", (nR ? nR : 1) * sizeof(Tup));
    Tup* sS = (Tup*)c.ws.scratch("api_sortedS", (nS ? nS : 1) * sizeof(Tup));
    unsigned long long* cnt =
        (unsigned long long*)c.ws.scratch("api_cnt", sizeof(unsigned long long));
    const uint32_t T = joincfg->NTHREADS > 0 ? (uint32_t)joincfg->NTHREADS : 1;
    const uint32_t fan = joincfg->PARTFANOUT > 1 ? (uint32_t)joincfg->PARTFANOUT : 2;
    const uint32_t D = ceil_log2(fan);
    // partitions per thread: the reference needs PARTFANOUT >= NTHREADS
    const uint32_t F = (1u << D) >= T ? (1u << D) : T;
    const uint32_t bits = ceil_log2(F);
    int64_t* hist = (int64_t*)c.ws.scratch("mp_hist", (size_t)T * F * 8);
    int64_t* off = (int64_t*)c.ws.scratch("mp_off", (size_t)T * F * 8);
    const DevBuf* rels[2] = {&r, &s};
    Tup* sorted[2] = {sR, sS};
    const uint64_t ns[2] = {nR, nS};
    static const char* pn[2] = {"mp_partR", "mp_partS"};
    // per relation and thread: the thread's merged relation in sorted[q]
    std::vector<uint64_t> toff[2], tlen[2];
    for (int q = 0; q < 2; q++) {
        toff[q].assign(T, 0);
        tlen[q].assign(T, 0);
        if (ns[q] == 0) continue;
        Tup* part = (Tup*)c.ws.scratch(pn[q], ns[q] * sizeof(Tup));
        const uint64_t chunk = ns[q] / T;
        std::vector<uint64_t> c0(T), cl(T);
        for (uint32_t t = 0; t < T; t++) {
            c0[t] = t * chunk;
            cl[t] = t + 1 == T ? ns[q] - c0[t] : chunk;
            if (!cl[t]) continue;
            // the reference's shift from its thread's chunk of R, for R and S
            // alike (:323-328)
            const uint64_t rchunk = t + 1 == T ? nR - (uint64_t)t * (nR / T) : nR / T;
            const int64_t sh = rchunk ? (int64_t)ceil(log2((double)(rchunk * T))) - (int64_t)bits - 1
                                      : 0;
            // the reference's uint32_t mask (partition.c:100): the digit bits
            // above bit 31 drop out, so the digit stays below F for any shift
            const uint32_t shift = sh > 0 ? (uint32_t)(sh < 63 ? sh : 63) : 0u;
            const uint32_t mask =
                shift < 32 ? (uint32_t)((((1ull << bits) - 1) << shift) & 0xffffffffull) : 0u;
            const Digit32 dig{mask, shift};
            stable_partition(&c.ws, rels[q]->d + c0[t], cl[t], part + c0[t], dig, bits, 0,
                             hist + (size_t)t * F, off + (size_t)t * F, c.st);
        }
        std::vector<int64_t> hh((size_t)T * F, 0), ho((size_t)T * F, 0);
        for (uint32_t t = 0; t < T; t++) {
            if (!cl[t]) continue;
            SMJ_CHECK(hipMemcpyAsync(hh.data() + (size_t)t * F, hist + (size_t)t * F, F * 8,
                                     hipMemcpyDeviceToHost, c.st));
            SMJ_CHECK(hipMemcpyAsync(ho.data() + (size_t)t * F, off + (size_t)t * F, F * 8,
                                     hipMemcpyDeviceToHost, c.st));
        }
        sync();
        std::vector<uint64_t> so((size_t)T * F), sl((size_t)T * F);
        for (uint32_t t = 0; t < T; t++)
            for (uint32_t j = 0; j < F; j++) {
                so[(size_t)t * F + j] = c0[t] + (uint64_t)ho[(size_t)t * F + j];
                sl[(size_t)t * F + j] = (uint64_t)hh[(size_t)t * F + j];
            }
        segmented_sort(&c.ws, part, so.data(), sl.data(), T * F, c.st);
        const uint32_t per = F / T;
        uint64_t o = 0;
        for (uint32_t t = 0; t < T; t++) {
            std::vector<const Tup*> runs;
            std::vector<uint64_t> lens;
            for (uint32_t j = t * per; j < (t + 1) * per; j++)
                for (uint32_t i = 0; i < T; i++) {
                    runs.push_back(part + so[(size_t)i * F + j]);
                    lens.push_back(sl[(size_t)i * F + j]);
                }
            uint64_t tot = 0;
            for (uint64_t x : lens) tot += x;
            toff[q][t] = o;
            tlen[q][t] = tot;
            if (tot) multiway_merge_tree(&c.ws, runs.data(), lens.data(), (uint32_t)runs.size(),
                                         sorted[q] + o, c.st);
            o += tot;
        }
    }
    // one counter per thread (the reference's per-thread result lists)
    unsigned long long* tcnt =
        (unsigned long long*)c.ws.scratch("mp_cnt", (size_t)T * sizeof(unsigned long long));
    SMJ_CHECK(hipMemsetAsync(tcnt, 0, (size_t)T * 8, c.st));
    for (uint32_t t = 0; t < T; t++)
        merge_join_count(sR + toff[0][t], tlen[0][t], sS + toff[1][t], tlen[1][t], tcnt + t,
                         c.st);
    std::vector<unsigned long long> h(T, 0);
    SMJ_CHECK(hipMemcpyAsync(h.data(), tcnt, (size_t)T * 8, hipMemcpyDeviceToHost, c.st));
    sync();
    (void)cnt;
    gettimeofday(&t1, NULL);
    result_t* res = (result_t*)malloc(sizeof(result_t));
    res->totalresults = 0;
    res->nthreads = joincfg->NTHREADS;
    res->resultlist = (threadresult_t*)calloc(T, sizeof(threadresult_t));
    for (uint32_t t = 0; t < T; t++) {
        res->totalresults += (int64_t)h[t];
        res->resultlist[t].nresults = (int64_t)h[t];
        res->resultlist[t].threadid = t;
        if (mat < 0 ? materialize_on() : mat > 0) {
            // the thread's own sorted relations (its partitions), R-major
            chainedtuplebuffer_t* cb = chainedtuplebuffer_init();
            materialize_append(sR + toff[0][t], tlen[0][t], sS + toff[1][t], tlen[1][t], cb);
            res->resultlist[t].results = cb;
        }
    }
    if (!getenv("SMJ_QUIET")) {
        double us = (t1.tv_sec - t0.tv_sec) * 1e6 + (t1.tv_usec - t0.tv_usec);
        fprintf(stderr, "NUM-TUPLES = %lld TOTAL-TIME-USECS = %.4lf ", (long long)nS, us);
        fprintf(stderr, "TUPLES-PER-SECOND = %.4lf ", nS / (us / 1e6));
        fflush(stderr);
    }
    return res;
}

result_t* sortmergejoin_multipass(relation_t* relR, relation_t* relS,
                                  joinconfig_t* joincfg) {
    return multipass_api(relR, relS, joincfg, -1);
}

result_t* smj_join(relation_t* relR, relation_t* relS, joinconfig_t* joincfg, int algo,
                   int materialize) {
    const int mat = materialize < 0 ? -1 : (materialize ? 1 : 0);
    switch (algo) {
        case 0: return join_api(relR, relS, joincfg, "m-way", mat);
        case 1: return multipass_api(relR, relS, joincfg, mat);
        case 2: return mpsm_api(relR, relS, joincfg, mat);
        default:
            fprintf(stderr, "[ERROR] smj_join: unknown algorithm %d\n", algo);
            return 0;
    }
}

// ---------------------------------------------------------------------------
// device-resident API
// ---------------------------------------------------------------------------
int smj_tuple_bytes(void) { return (int)sizeof(Tup); }

const char* smj_device_name(void) {
    static char name[256] = {0};
    if (!name[0]) {
        Ctx& c = ctx();
        hipDeviceProp_t p;
        SMJ_CHECK(hipGetDeviceProperties(&p, c.device));
        snprintf(name, sizeof(name), "%s (%s)", p.name, p.gcnArchName);
    }
    return name;
}

smj_workspace* smj_workspace_create(void) {
    ctx();
    return (smj_workspace*)new Workspace();
}
void smj_workspace_destroy(smj_workspace* ws) { delete (Workspace*)ws; }

void smj_workspace_set_layouts(smj_workspace* ws, uint32_t off) {
    ((Workspace*)(ws ? ws : smj_context_workspace()))->layouts_off = off;
}

int smj_workspace_last_layout(smj_workspace* ws) {
    return ((Workspace*)(ws ? ws : smj_context_workspace()))->last_layout;
}

void smj_dev_partition(smj_workspace* ws, const tuple_t* in, uint64_t n,
                       tuple_t* out, uint32_t nbits, uint32_t shiftbits,
                       int padded, int64_t* hist_out, int64_t* off_out,
                       smj_stream_t stream) {
    const uint32_t mask = (uint32_t)(((1ull << nbits) - 1) << shiftbits);
    Digit32 dig{mask, shiftbits};
    stable_partition((Workspace*)ws, (const Tup*)in, n, (Tup*)out, dig, nbits,
                     padded, hist_out, off_out, (hipStream_t)stream);
}

void smj_dev_sort(smj_workspace* ws, const tuple_t* in, uint64_t n,
                  tuple_t* out, smj_stream_t stream) {
    device_sort((Workspace*)ws, (const Tup*)in, n, (Tup*)out,
                (hipStream_t)stream);
}

void smj_dev_merge2(const tuple_t* a, uint64_t na, const tuple_t* b,
                    uint64_t nb, tuple_t* out, smj_stream_t stream) {
    merge2(&ctx().ws, (const Tup*)a, na, (const Tup*)b, nb, (Tup*)out, (hipStream_t)stream);
}

void smj_dev_multiway_merge_host(smj_workspace* ws, const tuple_t* const* runs,
                                 const uint64_t* lens, uint32_t k,
                                 tuple_t* out, smj_stream_t stream) {
    multiway_merge((Workspace*)ws, (const Tup* const*)runs, lens, k, (Tup*)out,
                   (hipStream_t)stream);
}

void smj_dev_merge_join_count(const tuple_t* r, uint64_t nr, const tuple_t* s,
                              uint64_t ns, unsigned long long* count_dev,
                              smj_stream_t stream) {
    merge_join_count((const Tup*)r, nr, (const Tup*)s, ns, count_dev,
                     (hipStream_t)stream);
}

uint64_t smj_dev_materialize(smj_workspace* ws, const tuple_t* sortedR, uint64_t nR,
                             const tuple_t* sortedS, uint64_t nS, tuple_t* out,
                             uint64_t out_cap, smj_stream_t stream) {
    return materialize((Workspace*)ws, (const Tup*)sortedR, nR, (const Tup*)sortedS,
                       nS, (Tup*)out, out_cap, (hipStream_t)stream);
}

void smj_dev_join(smj_workspace* ws, const tuple_t* R, uint64_t nR,
                  const tuple_t* S, uint64_t nS, tuple_t* sortedR,
                  tuple_t* sortedS, uint32_t fanout_bits, int64_t key_min,
                  int64_t key_max, unsigned long long* count_dev,
                  smj_stream_t stream) {
    device_join((Workspace*)ws, (const Tup*)R, nR, (const Tup*)S, nS,
                (Tup*)sortedR, (Tup*)sortedS, fanout_bits, key_min, key_max,
                count_dev, (hipStream_t)stream);
}

// Segment tables of an exchanged relation: the receive buffer holds, for
// every source s in order, that source's partitions 0..nb-1 back to back
// (cnt[s * nb + b] tuples each).  Bucket b = the nseg segments
// seg_start/seg_cnt[b * nseg + s]; bucket starts are 0 (offsets absolute).
__global__ void __launch_bounds__(256)
k_seg_tables(const int64_t* __restrict__ cnt, uint32_t nseg, uint32_t nb,
             uint64_t* __restrict__ seg_start, int64_t* __restrict__ seg_cnt,
             int64_t* __restrict__ bcount, uint64_t* __restrict__ bstart) {
    __shared__ uint32_t scr[5];
    __shared__ unsigned long long base;
    if (threadIdx.x == 0) base = 0;
    for (uint32_t b = threadIdx.x; b < nb; b += 256) {
        bcount[b] = 0;
        bstart[b] = 0;
    }
    __syncthreads();
    for (uint32_t s = 0; s < nseg; s++) {
        for (uint32_t b0 = 0; b0 < nb; b0 += 256) {
            const uint32_t b = b0 + threadIdx.x;
            const int64_t c = b < nb ? cnt[(size_t)s * nb + b] : 0;
            uint32_t tot;  // a source sends < 2^32 tuples (checked by the host)
            const uint32_t ex = block_exclusive_scan((uint32_t)c, scr, &tot);
            if (b < nb) {
                seg_start[(size_t)b * nseg + s] = base + ex;
                seg_cnt[(size_t)b * nseg + s] = c;
                bcount[b] += c;
            }
            __syncthreads();
            if (threadIdx.x == 0) base += tot;
            __syncthreads();
        }
    }
}

// Bucket totals of explicit segment tables (bucket-major, nseg per bucket);
// bucket starts are 0 (segment offsets are absolute).  blockIdx.x = relation.
__global__ void __launch_bounds__(256)
k_seg_totals(const int64_t* __restrict__ cnt0, const int64_t* __restrict__ cnt1,
             uint32_t nseg, uint32_t nb, int64_t* __restrict__ bcount0,
             int64_t* __restrict__ bcount1, uint64_t* __restrict__ bstart0,
             uint64_t* __restrict__ bstart1) {
    const int64_t* cnt = blockIdx.x ? cnt1 : cnt0;
    int64_t* bcount = blockIdx.x ? bcount1 : bcount0;
    uint64_t* bstart = blockIdx.x ? bstart1 : bstart0;
    for (uint32_t b = threadIdx.x; b < nb; b += 256) {
        int64_t t = 0;
        for (uint32_t j = 0; j < nseg; j++) t += cnt[(size_t)b * nseg + j];
        bcount[b] = t;
        bstart[b] = 0;
    }
}

// The local join of the exchanged relations from their segment tables
// (seg_start / seg_cnt [b * nseg + j], element offsets into R / S): the
// buckets are the exchanged partitions, so the join starts at its tile pass.
static void join_segmented_core(Workspace* ws, void* R, uint64_t nR, void* S, uint64_t nS,
                                uint64_t* const* ss, int64_t* const* sc, uint32_t nseg,
                                uint32_t bucket_bits, int64_t key_lo, int64_t key_hi,
                                uint32_t flags, tuple_t* sortedR, tuple_t* sortedS,
                                unsigned long long* count_dev, hipStream_t st,
                                const uint64_t* pstride = nullptr) {
    if (!(flags & SMJ_SEG_STAGE_R))  // the count belongs to the group pass's call
        SMJ_CHECK(hipMemsetAsync(count_dev, 0, sizeof(unsigned long long), st));
    uint32_t D1, D2, D2cap;
    choose_levels(nR > nS ? nR : nS, bucket_bits, &D1, &D2, &D2cap);
    // the buckets are the exchanged partitions: level 1 is fixed
    const uint32_t tot_bits = D1 + D2;
    D1 = bucket_bits;
    D2 = tot_bits > D1 ? tot_bits - D1 : 0;
    if (D2 > kMaxD2) D2 = kMaxD2;
    D2cap = D2 + 2 < kMaxD2 ? D2 + 2 : (D2 > kMaxD2 ? D2 : kMaxD2);
    RangePlan hplan = make_plan(key_lo, key_hi, D1, D2, D2cap, kGroupD3Max);
    const bool p48 = pstride != nullptr;  // 48-bit words in two planes (LayP48)
    const bool packed = (flags & SMJ_SEG_PACKED) != 0 || p48;
    if (p48 && !LayP48::usable(hplan)) {
        fprintf(stderr, "[ERROR] smj_dev_join_segmented_planes: 48-bit words need "
                "1 <= s1 <= 32 (s1 = %u)\n", hplan.s1);
        abort();
    }
#ifdef KEY_8B
    if (packed && !p48 && !LayPacked::usable(hplan)) {
        fprintf(stderr, "[ERROR] smj_dev_join_segmented: packed words need 1 <= s1 <= 32 "
                "(s1 = %u)\n", hplan.s1);
        abort();
    }
#else
    if (packed && !p48) {
        fprintf(stderr, "[ERROR] smj_dev_join_segmented: packed words are a 16-byte-tuple "
                "layout\n");
        abort();
    }
#endif
    RangePlan* plan = (RangePlan*)ws->scratch("plan", sizeof(RangePlan));
    hipLaunchKernelGGL(k_setplan, dim3(1), dim3(1), 0, st, plan, hplan);
    const uint32_t nb = 1u << D1;
    void* rel[2] = {R, S};
    static const char* nm[2][2] = {{"xs_bcR", "xs_bsR"}, {"xs_bcS", "xs_bsS"}};
    int64_t* bc[2];
    uint64_t* bs[2];
    for (int r = 0; r < 2; r++) {
        bc[r] = (int64_t*)ws->scratch(nm[r][0], (size_t)nb * 8);
        bs[r] = (uint64_t*)ws->scratch(nm[r][1], (size_t)nb * 8);
    }
    hipLaunchKernelGGL(k_seg_totals, dim3(2), dim3(256), 0, st, sc[0], sc[1], nseg, nb, bc[0],
                       bc[1], bs[0], bs[1]);
    BucketSortArgs a;
    for (int r = 0; r < 2; r++) {
        a.part[r] = rel[r];
        a.tmp[r] = rel[r];  // the tile pass works in place in the receive buffer
        a.bstart[r] = bs[r];
        a.bcount[r] = bc[r];
        a.seg_start[r] = ss[r];
        a.seg_cnt[r] = sc[r];
    }
    a.nseg = nseg;
    a.out[0] = (Tup*)sortedR;
    a.out[1] = (Tup*)sortedS;
    a.n[0] = nR;
    a.n[1] = nS;
    a.nrel = 2;
    a.nbuckets = nb;
    a.plan_dev = plan;
    a.count_dev = count_dev;
    unsigned int* flag = (unsigned int*)ws->scratch("xs_flag", 4);
    SMJ_CHECK(hipMemsetAsync(flag, 0, 4, st));
    a.part_flag = flag;  // never set: the buckets are exact
    a.host_plan = &hplan;
    a.packed = packed;  // checked packable before the exchange: no pack_bad here
    a.digit_fast = packed;  // packed words never lie outside the plan
    a.p48 = p48;
    for (int r = 0; r < 2 && p48; r++) a.pstride[r] = pstride[r];
    if ((flags & SMJ_SEG_STAGE_R) && (flags & SMJ_SEG_STAGE_REST)) {
        fprintf(stderr, "[ERROR] smj_dev_join_segmented: SMJ_SEG_STAGE_R and _REST are two "
                "calls\n");
        abort();
    }
    if (flags & SMJ_SEG_STAGE_R) a.stage = 1;          // R's tile stage only
    else if (flags & SMJ_SEG_STAGE_REST) a.stage = 6;  // S's tile stage + group pass
    if (!bucket_sort(ws, a, st)) {
        fprintf(stderr, "[ERROR] smj_dev_join_segmented: unexpected partition flag\n");
        abort();
    }
}

static void check_segmented(const char* fn, uint32_t nseg, uint32_t bucket_bits, uint64_t nR,
                            uint64_t nS) {
    if (nseg == 0 || bucket_bits > 10 || nR >= (1ull << 32) || nS >= (1ull << 32)) {
        fprintf(stderr, "[ERROR] %s: nseg %u, bucket_bits %u (<= 10), nR %llu, nS %llu "
                "(< 2^32)\n", fn, nseg, bucket_bits, (unsigned long long)nR,
                (unsigned long long)nS);
        abort();
    }
}

void smj_dev_join_segmented(smj_workspace* wsp, void* R, uint64_t nR,
                            const int64_t* segR, void* S, uint64_t nS,
                            const int64_t* segS, uint32_t nseg, uint32_t bucket_bits,
                            int64_t key_lo, int64_t key_hi, uint32_t flags,
                            tuple_t* sortedR, tuple_t* sortedS,
                            unsigned long long* count_dev, smj_stream_t stream) {
    Workspace* ws = (Workspace*)wsp;
    hipStream_t st = (hipStream_t)stream;
    check_segmented("smj_dev_join_segmented", nseg, bucket_bits, nR, nS);
    const uint32_t nb = 1u << bucket_bits;
    const int64_t* seg[2] = {segR, segS};
    static const char* nm[2][4] = {{"xs_startR", "xs_cntR", "xs_bcR", "xs_bsR"},
                                   {"xs_startS", "xs_cntS", "xs_bcS", "xs_bsS"}};
    uint64_t* ss[2];
    int64_t* sc[2];
    for (int r = 0; r < 2; r++) {
        ss[r] = (uint64_t*)ws->scratch(nm[r][0], (size_t)nb * nseg * 8);
        sc[r] = (int64_t*)ws->scratch(nm[r][1], (size_t)nb * nseg * 8);
        int64_t* bc = (int64_t*)ws->scratch(nm[r][2], (size_t)nb * 8);
        uint64_t* bs = (uint64_t*)ws->scratch(nm[r][3], (size_t)nb * 8);
        hipLaunchKernelGGL(k_seg_tables, dim3(1), dim3(256), 0, st, seg[r], nseg, nb,
                           ss[r], sc[r], bc, bs);
    }
    join_segmented_core(ws, R, nR, S, nS, ss, sc, nseg, bucket_bits, key_lo, key_hi, flags,
                        sortedR, sortedS, count_dev, st);
}

void smj_dev_join_segmented_tables(smj_workspace* wsp, void* R, uint64_t nR,
                                   const int64_t* startR, const int64_t* cntR, void* S,
                                   uint64_t nS, const int64_t* startS, const int64_t* cntS,
                                   uint32_t nseg, uint32_t bucket_bits, int64_t key_lo,
                                   int64_t key_hi, uint32_t flags, tuple_t* sortedR,
                                   tuple_t* sortedS, unsigned long long* count_dev,
                                   smj_stream_t stream) {
    check_segmented("smj_dev_join_segmented_tables", nseg, bucket_bits, nR, nS);
    uint64_t* ss[2] = {(uint64_t*)startR, (uint64_t*)startS};
    int64_t* sc[2] = {(int64_t*)cntR, (int64_t*)cntS};
    join_segmented_core((Workspace*)wsp, R, nR, S, nS, ss, sc, nseg, bucket_bits, key_lo,
                        key_hi, flags, sortedR, sortedS, count_dev, (hipStream_t)stream);
}

void smj_dev_join_segmented_planes(smj_workspace* wsp, void* R, uint64_t strideR, uint64_t nR,
                                   const int64_t* startR, const int64_t* cntR, void* S,
                                   uint64_t strideS, uint64_t nS, const int64_t* startS,
                                   const int64_t* cntS, uint32_t nseg, uint32_t bucket_bits,
                                   int64_t key_lo, int64_t key_hi, uint32_t flags,
                                   tuple_t* sortedR, tuple_t* sortedS,
                                   unsigned long long* count_dev, smj_stream_t stream) {
    check_segmented("smj_dev_join_segmented_planes", nseg, bucket_bits, nR, nS);
    if ((flags & SMJ_SEG_PACKED) || strideR % 32 || strideS % 32 || strideR < nR ||
        strideS < nS) {
        fprintf(stderr, "[ERROR] smj_dev_join_segmented_planes: flags %u (stages only), "
                "strides %llu / %llu (multiples of 32, >= nR %llu / nS %llu)\n", flags,
                (unsigned long long)strideR, (unsigned long long)strideS,
                (unsigned long long)nR, (unsigned long long)nS);
        abort();
    }
    uint64_t* ss[2] = {(uint64_t*)startR, (uint64_t*)startS};
    int64_t* sc[2] = {(int64_t*)cntR, (int64_t*)cntS};
    const uint64_t pst[2] = {strideR, strideS};
    join_segmented_core((Workspace*)wsp, R, nR, S, nS, ss, sc, nseg, bucket_bits, key_lo,
                        key_hi, flags, sortedR, sortedS, count_dev, (hipStream_t)stream, pst);
}

void smj_join_phase_ms(smj_workspace* wsp, float* ms5) {
    Workspace* ws = (Workspace*)wsp;
    for (int i = 0; i < 5; i++) ms5[i] = 0.f;
    if (!ws->ev_init) return;
    SMJ_CHECK(hipEventSynchronize(ws->ev[4]));
    float a = 0, b = 0, cc = 0, d = 0;
    SMJ_CHECK(hipEventElapsedTime(&a, ws->ev[0], ws->ev[1]));
    SMJ_CHECK(hipEventElapsedTime(&b, ws->ev[1], ws->ev[2]));
    SMJ_CHECK(hipEventElapsedTime(&cc, ws->ev[2], ws->ev[3]));
    SMJ_CHECK(hipEventElapsedTime(&d, ws->ev[3], ws->ev[4]));
    ms5[0] = a;
    ms5[1] = b;
    ms5[2] = cc;
    ms5[3] = d;
    ms5[4] = a + b + cc + d;
}

void smj_dev_gen_pk(tuple_t* out, uint64_t n, uint64_t first, uint64_t total,
                    uint64_t seed, int with_payload, smj_stream_t stream) {
    if (with_payload)
        gen_pk((Tup*)out, n, first, total, seed, (hipStream_t)stream);
    else
        gen_pk_nopayload((Tup*)out, n, first, total, seed, (hipStream_t)stream);
}

void smj_dev_gen_fk(tuple_t* out, uint64_t n, uint64_t first, uint64_t total,
                    uint64_t maxid, uint64_t seed, smj_stream_t stream) {
    gen_fk((Tup*)out, n, first, total, maxid, seed, (hipStream_t)stream);
}

void smj_dev_gen_zipf(smj_workspace* ws, tuple_t* out, uint64_t n,
                      uint64_t first, uint64_t maxid, double theta,
                      uint64_t seed, smj_stream_t stream) {
    gen_zipf((Workspace*)ws, (Tup*)out, n, first, maxid, theta, seed,
             (hipStream_t)stream);
}

void smj_dev_gen_nonunique(smj_workspace* ws, tuple_t* out, uint64_t n, uint64_t first,
                           uint64_t total, int64_t maxid, uint32_t seed, uint64_t skip,
                           smj_stream_t stream) {
    gen_nonunique_ref((Workspace*)ws, (Tup*)out, n, first, total, maxid, seed, skip,
                      (hipStream_t)stream);
}

void smj_dev_gen_zipf_ref(smj_workspace* ws, tuple_t* out, uint64_t n, uint64_t first,
                          uint64_t maxid, double theta, uint32_t seed, uint64_t skip,
                          smj_stream_t stream) {
    gen_zipf_ref((Workspace*)ws, (Tup*)out, n, first, maxid, theta, seed, skip,
                 (hipStream_t)stream);
}

uint32_t smj_glibc_rand(uint32_t seed, uint64_t k) { return glibc_rand_at(seed, k); }

void smj_dev_synchronize(smj_stream_t stream) {
    SMJ_CHECK(hipStreamSynchronize((hipStream_t)stream));
}

void smj_dev_partition_range(smj_workspace* wsp, const tuple_t* in, uint64_t n,
                             tuple_t* out, uint32_t nbits, int64_t key_min,
                             int64_t key_max, int64_t* hist_out,
                             smj_stream_t stream) {
    Workspace* ws = (Workspace*)wsp;
    hipStream_t st = (hipStream_t)stream;
    RangePlan* plan = (RangePlan*)ws->scratch("range_plan", sizeof(RangePlan));
    RangePlan h = make_plan(key_min, key_max, nbits, 0, 0, 0);
    hipLaunchKernelGGL(k_setplan, dim3(1), dim3(1), 0, st, plan, h);
    uint64_t* starts = (uint64_t*)ws->scratch("range_starts", (1u << nbits) * 8);
    plan_partition(ws, (const Tup*)in, n, (Tup*)out, plan, nbits, starts,
                   hist_out, st);
}

int smj_dev_partition_range_packed(smj_workspace* wsp, const tuple_t* in, uint64_t n,
                                   uint64_t* out, uint32_t nbits, int64_t key_min,
                                   int64_t key_max, int64_t* hist_out,
                                   unsigned int* bad_flag, smj_stream_t stream) {
#ifdef KEY_8B
    Workspace* ws = (Workspace*)wsp;
    hipStream_t st = (hipStream_t)stream;
    RangePlan h = make_plan(key_min, key_max, nbits, 0, 0, 0);
    if (!LayPacked::usable(h)) return 0;
    RangePlan* plan = (RangePlan*)ws->scratch("range_plan", sizeof(RangePlan));
    hipLaunchKernelGGL(k_setplan, dim3(1), dim3(1), 0, st, plan, h);
    uint64_t* starts = (uint64_t*)ws->scratch("range_starts", (1u << nbits) * 8);
    plan_partition_packed(ws, (const Tup*)in, n, out, plan, h, nbits, starts, hist_out,
                          bad_flag, st);
    return 1;
#else
    (void)wsp; (void)in; (void)n; (void)out; (void)nbits; (void)key_min; (void)key_max;
    (void)hist_out; (void)bad_flag; (void)stream;
    return 0;
#endif
}

uint64_t smj_sampled_capacity(uint64_t n, uint32_t nbits) { return sampled_capacity(n, nbits); }

uint32_t smj_sampled_shards(void) { return kShards; }

void smj_dev_xsend(const int64_t* start, const int64_t* cnt, const unsigned int* flags, uint32_t F,
                   uint32_t K, uint32_t world, uint32_t used, int64_t* msg, int64_t* chunk,
                   smj_stream_t stream) {
    if (used == 0) used = F;
    if (F > 1024 || world == 0 || world > 1024 || world > F || used > F) {
        fprintf(stderr, "[ERROR] smj_dev_xsend: F %u, world %u, used %u (1 <= world <= F <= "
                        "1024, used <= F)\n", F, world, used);
        abort();
    }
    xsend(start, cnt, flags, F, K, world, used, msg, chunk, (hipStream_t)stream);
}

void smj_dev_xrecv(const int64_t* msg, const int64_t* chunk, uint32_t world, uint32_t rank,
                   uint32_t mine, uint32_t K, uint32_t nbuckets, uint64_t cap, int64_t* tstart,
                   int64_t* tcnt, int64_t* summary, smj_stream_t stream) {
    if (world == 0 || world > 1024 || rank >= world || mine > nbuckets) {
        fprintf(stderr, "[ERROR] smj_dev_xrecv: world %u, rank %u, mine %u, nbuckets %u\n",
                world, rank, mine, nbuckets);
        abort();
    }
    xrecv(msg, chunk, world, rank, mine, K, nbuckets, cap, tstart, tcnt, summary,
          (hipStream_t)stream);
}

int smj_dev_partition_range_sampled(smj_workspace* wsp, const tuple_t* in, uint64_t n,
                                    void* out, uint32_t nbits, int64_t key_min,
                                    int64_t key_max, int packed, int64_t* seg_start_out,
                                    int64_t* seg_cnt_out, unsigned int* flags,
                                    smj_stream_t stream) {
    Workspace* ws = (Workspace*)wsp;
    hipStream_t st = (hipStream_t)stream;
    if (nbits > 10 || n >= (1ull << 32)) return 0;  // LDS carries: up to 1024 partitions
    RangePlan h = make_plan(key_min, key_max, nbits, 0, 0, 0);
#ifdef KEY_8B
    if (packed && !LayPacked::usable(h)) return 0;
#else
    if (packed) return 0;
#endif
    const uint32_t nbins = 1u << nbits;
    RangePlan* plan = (RangePlan*)ws->scratch("xp_plan", sizeof(RangePlan));
    hipLaunchKernelGGL(k_setplan, dim3(1), dim3(1), 0, st, plan, h);
    unsigned int* sample = (unsigned int*)ws->scratch("xp_sample", (size_t)nbins * 4);
    SMJ_CHECK(hipMemsetAsync(sample, 0, (size_t)nbins * 4, st));
    SMJ_CHECK(hipMemsetAsync(flags, 0, 8, st));
    uint64_t* starts = (uint64_t*)ws->scratch("xp_starts", (size_t)nbins * 8);
    int64_t* hist = (int64_t*)ws->scratch("xp_hist", (size_t)nbins * 8);
    const Tup* rels[1] = {(const Tup*)in};
    const uint64_t ns[1] = {n};
    void* outs[1] = {out};
    uint64_t* st_[1] = {starts};
    int64_t* h_[1] = {hist};
    uint64_t* ss[1] = {(uint64_t*)seg_start_out};
    int64_t* sc[1] = {seg_cnt_out};
    sampled_partition(ws, 1, rels, ns, outs, plan, nbits, sample, st_, h_, ss, sc, flags, st,
                      &h, packed != 0, packed ? flags + 1 : nullptr);
    return 1;
}

int smj_dev_partition_range_shards(smj_workspace* wsp, const tuple_t* in, uint64_t n,
                                   void* out, uint32_t nbits, int64_t key_min, int64_t key_max,
                                   int packed, int64_t* seg_start_out, int64_t* seg_cnt_out,
                                   unsigned int* flags, smj_stream_t stream) {
    Workspace* ws = (Workspace*)wsp;
    hipStream_t st = (hipStream_t)stream;
    if (nbits > 10 || n >= (1ull << 32)) return 0;  // the scatter's LDS carries
    RangePlan h = make_plan(key_min, key_max, nbits, 0, 0, 0);
#ifdef KEY_8B
    if (packed && !LayPacked::usable(h)) return 0;
#else
    if (packed) return 0;
#endif
    const uint32_t nbins = 1u << nbits;
    RangePlan* plan = (RangePlan*)ws->scratch("xp_plan", sizeof(RangePlan));
    hipLaunchKernelGGL(k_setplan, dim3(1), dim3(1), 0, st, plan, h);
    // exact (partition, shard) counts instead of a sample
    unsigned int* counts =
        (unsigned int*)ws->scratch("xp_shard_counts", (size_t)nbins * kShards * 4);
    SMJ_CHECK(hipMemsetAsync(counts, 0, (size_t)nbins * kShards * 4, st));
    SMJ_CHECK(hipMemsetAsync(flags, 0, 8, st));
    uint64_t* starts = (uint64_t*)ws->scratch("xp_starts", (size_t)nbins * 8);
    int64_t* hist = (int64_t*)ws->scratch("xp_hist", (size_t)nbins * 8);
    const Tup* rels[1] = {(const Tup*)in};
    const uint64_t ns[1] = {n};
    void* outs[1] = {out};
    uint64_t* st_[1] = {starts};
    int64_t* h_[1] = {hist};
    uint64_t* ss[1] = {(uint64_t*)seg_start_out};
    int64_t* sc[1] = {seg_cnt_out};
    sampled_partition(ws, 1, rels, ns, outs, plan, nbits, counts, st_, h_, ss, sc, flags, st,
                      &h, packed != 0, packed ? flags + 1 : nullptr, 0, false, true);
    return 1;
}

int smj_dev_partition_range_planes(smj_workspace* wsp, const tuple_t* in, uint64_t n,
                                   void* out, uint64_t stride, uint32_t nbits,
                                   int64_t key_min, int64_t key_max, int64_t* seg_start_out,
                                   int64_t* seg_cnt_out, unsigned int* flags,
                                   smj_stream_t stream) {
    Workspace* ws = (Workspace*)wsp;
    hipStream_t st = (hipStream_t)stream;
    // the scatter's LDS carries hold 2^10 partitions of 48-bit words with its
    // 16-byte segments (round 6; 2^9 was the limit of 64-byte segments)
    if (nbits > 10 || n >= (1ull << 32)) return 0;
    RangePlan h = make_plan(key_min, key_max, nbits, 0, 0, 0);
    if (!LayP48::usable(h)) return 0;
    if (stride % 32 || stride < sampled_capacity(n, nbits)) {
        fprintf(stderr, "[ERROR] smj_dev_partition_range_planes: stride %llu (a multiple of "
                "32, >= smj_sampled_capacity = %llu)\n", (unsigned long long)stride,
                (unsigned long long)sampled_capacity(n, nbits));
        abort();
    }
    const uint32_t nbins = 1u << nbits;
    RangePlan* plan = (RangePlan*)ws->scratch("xp_plan", sizeof(RangePlan));
    hipLaunchKernelGGL(k_setplan, dim3(1), dim3(1), 0, st, plan, h);
    unsigned int* sample = (unsigned int*)ws->scratch("xp_sample", (size_t)nbins * 4);
    SMJ_CHECK(hipMemsetAsync(sample, 0, (size_t)nbins * 4, st));
    SMJ_CHECK(hipMemsetAsync(flags, 0, 8, st));
    uint64_t* starts = (uint64_t*)ws->scratch("xp_starts", (size_t)nbins * 8);
    int64_t* hist = (int64_t*)ws->scratch("xp_hist", (size_t)nbins * 8);
    const Tup* rels[1] = {(const Tup*)in};
    const uint64_t ns[1] = {n};
    void* outs[1] = {out};
    uint64_t* st_[1] = {starts};
    int64_t* h_[1] = {hist};
    uint64_t* ss[1] = {(uint64_t*)seg_start_out};
    int64_t* sc[1] = {seg_cnt_out};
    sampled_partition(ws, 1, rels, ns, outs, plan, nbits, sample, st_, h_, ss, sc, flags, st,
                      &h, true, flags + 1, stride);
    return 1;
}

uint64_t smj_selfcheck_lds_order(smj_workspace* ws, smj_stream_t stream) {
    return lds_order_selfcheck((Workspace*)ws, (hipStream_t)stream);
}

smj_workspace* smj_context_workspace(void) { return (smj_workspace*)&ctx().ws; }

void smj_trace_enable(smj_workspace* wsp, int on) {
    ((Workspace*)wsp)->trace_on = on != 0;
}

void smj_trace_reset(smj_workspace* wsp) { ((Workspace*)wsp)->trace_n = 0; }

void smj_trace_only(smj_workspace* wsp, const char* name) {
    ((Workspace*)wsp)->trace_only = name ? name : "";
}

// Aggregate the traced kernels by name: returns the number of names written;
// names are '\n'-separated in `names` (capacity `cap` bytes).
int smj_trace_read(smj_workspace* wsp, char* names, int cap, float* ms_sum,
                   int* launches, int max) {
    Workspace* ws = (Workspace*)wsp;
    if (ws->trace_n == 0) return 0;
    SMJ_CHECK(hipEventSynchronize(ws->trace[ws->trace_n - 1].b));
    std::vector<std::string> nm;
    std::vector<float> ms;
    std::vector<int> cnt;
    for (size_t i = 0; i < ws->trace_n; i++) {
        float t = 0;
        SMJ_CHECK(hipEventElapsedTime(&t, ws->trace[i].a, ws->trace[i].b));
        size_t k = 0;
        while (k < nm.size() && nm[k] != ws->trace[i].name) k++;
        if (k == nm.size()) {
            nm.push_back(ws->trace[i].name);
            ms.push_back(0);
            cnt.push_back(0);
        }
        ms[k] += t;
        cnt[k]++;
    }
    int w = 0, pos = 0;
    for (size_t k = 0; k < nm.size() && w < max; k++, w++) {
        int l = (int)nm[k].size();
        if (pos + l + 1 >= cap) break;
        memcpy(names + pos, nm[k].data(), l);
        names[pos + l] = '\n';
        pos += l + 1;
        ms_sum[w] = ms[k];
        launches[w] = cnt[k];
    }
    if (pos < cap) names[pos] = 0;
    return w;
}

}  // extern "C"
