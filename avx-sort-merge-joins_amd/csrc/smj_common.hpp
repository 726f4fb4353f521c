// smj_common.hpp -- shared device/host definitions for the MI355X sort-merge
// join kernels (gfx950, wave64).
//
// Tuple width is fixed per build (KEY_8B -> 16-byte tuples), mirroring the
// reference's compile-time switch (src/types.h:23-29).  On the device a tuple
// is handled as one machine word:
//   8-byte  tuple -> uint64_t  (payload in bits 0..31, key in bits 32..63)
//   16-byte tuple -> Tup16     {int64 payload; int64 key}
// Sort order (the parity contract):
//   8-byte : signed int64 order of the packed word  (what avxsort produces,
//            src/avxsort/avxcommon.h:79-190, inside the generators' domain)
//   16-byte: (key, payload) lexicographic, both signed
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define SMJ_CHECK(call)                                                        \
    do {                                                                       \
        hipError_t e_ = (call);                                                \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "[ERROR] smj: %s failed at %s:%d: %s\n", #call,    \
                    __FILE__, __LINE__, hipGetErrorString(e_));                \
            abort();                                                           \
        }                                                                      \
    } while (0)

#include <mutex>
#include <set>
#include <utility>

namespace smj {

// hipFuncSetAttribute(kernel, MaxDynamicSharedMemorySize, bytes) once per
// (device, kernel): the attribute is held per device, and the in-process
// multi-GPU join (mgpu.hip) launches from one host thread per device at once.
// The attribute is set under the lock, so no thread launches before it holds.
inline void set_lds_attr(const void* kernel, int bytes) {
    static std::mutex mu;
    static std::set<std::pair<int, const void*>> done;
    int dev = 0;
    SMJ_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    if (!done.insert({dev, kernel}).second) return;
    SMJ_CHECK(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
}

#ifdef KEY_8B
struct __attribute__((aligned(16))) Tup {
    int64_t payload;
    int64_t key;
};
#else
typedef uint64_t Tup;
#endif

constexpr int kTupBytes = sizeof(Tup);

// Streaming accesses of the tuple passes (each byte read once, written once):
// optionally with the non-temporal cache policy.
#ifndef SMJ_NT_STORES
#define SMJ_NT_STORES 1
#endif
#ifndef SMJ_NT_LOADS
#define SMJ_NT_LOADS 0
#endif
#ifdef KEY_8B
typedef long long TupVec __attribute__((ext_vector_type(2)));
#endif
__device__ __forceinline__ void st_stream(Tup* p, const Tup& v) {
#if SMJ_NT_STORES
#ifdef KEY_8B
    TupVec x = {v.payload, v.key};
    __builtin_nontemporal_store(x, reinterpret_cast<TupVec*>(p));
#else
    __builtin_nontemporal_store(v, p);
#endif
#else
    *p = v;
#endif
}
__device__ __forceinline__ Tup ld_stream(const Tup* p) {
#if SMJ_NT_LOADS
#ifdef KEY_8B
    const TupVec x = __builtin_nontemporal_load(reinterpret_cast<const TupVec*>(p));
    Tup t;
    t.payload = x.x;
    t.key = x.y;
    return t;
#else
    return __builtin_nontemporal_load(p);
#endif
#else
    return *p;
#endif
}

// streaming store of an intermediate element (tuple or packed word)
__device__ __forceinline__ void st_w(uint64_t* p, uint64_t v) {
#if SMJ_NT_STORES
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}
#ifdef KEY_8B
__device__ __forceinline__ void st_w(Tup* p, const Tup& v) { st_stream(p, v); }
#endif

// non-temporal load regardless of SMJ_NT_LOADS: gathers of once-read tuples
// that must not push the small per-group tables out of L2
__device__ __forceinline__ Tup ld_nt(const Tup* p) {
#ifdef KEY_8B
    const TupVec x = __builtin_nontemporal_load(reinterpret_cast<const TupVec*>(p));
    Tup t;
    t.payload = x.x;
    t.key = x.y;
    return t;
#else
    return __builtin_nontemporal_load(p);
#endif
}

// Load through a pointer the compiler cannot prove global (read from LDS or
// from a table in device memory): left alone it becomes a flat load, which
// also counts against lgkmcnt, so every later LDS wait waits for it too and
// gathers lose their overlap.  The cast keeps it a global_load.
typedef const __attribute__((address_space(1))) uint64_t* GlobalU64Ptr;
__device__ __forceinline__ Tup ld_g(const Tup* p) {
#ifdef KEY_8B
    typedef const __attribute__((address_space(1))) TupVec* GV;
    const TupVec x = *(GV)p;
    Tup t;
    t.payload = x.x;
    t.key = x.y;
    return t;
#else
    return *(GlobalU64Ptr)p;
#endif
}

__device__ __forceinline__ void st_g(Tup* p, const Tup& v) {
#ifdef KEY_8B
    typedef __attribute__((address_space(1))) TupVec* GV;
    TupVec x = {v.payload, v.key};
    *(GV)p = x;
#else
    *(__attribute__((address_space(1))) uint64_t*)p = v;
#endif
}

__host__ __device__ __forceinline__ int64_t tup_key(const Tup& t) {
#ifdef KEY_8B
    return t.key;
#else
    return (int64_t)(int32_t)(uint32_t)(t >> 32);
#endif
}

// strict weak order == total order on the tuple's bytes (see header)
__host__ __device__ __forceinline__ bool tup_less(const Tup& a, const Tup& b) {
#ifdef KEY_8B
    return (a.key < b.key) || (a.key == b.key && a.payload < b.payload);
#else
    return (int64_t)a < (int64_t)b;
#endif
}

// c ? a : b field by field: a ternary on the 16-byte struct can become a
// select between the addresses of two stack copies (scratch memory)
__host__ __device__ __forceinline__ Tup tup_sel(bool c, const Tup& a, const Tup& b) {
#ifdef KEY_8B
    Tup r;
    r.payload = c ? a.payload : b.payload;
    r.key = c ? a.key : b.key;
    return r;
#else
    return c ? a : b;
#endif
}

__host__ __device__ __forceinline__ bool tup_eq(const Tup& a, const Tup& b) {
#ifdef KEY_8B
    return a.key == b.key && a.payload == b.payload;
#else
    return a == b;
#endif
}

__host__ __device__ __forceinline__ Tup tup_max_sentinel() {
#ifdef KEY_8B
    Tup t;
    t.payload = INT64_MAX;
    t.key = INT64_MAX;
    return t;
#else
    return (uint64_t)INT64_MAX;
#endif
}

// order-preserving map of a signed key to unsigned
__host__ __device__ __forceinline__ uint64_t key_u(int64_t k) {
    return (uint64_t)k ^ 0x8000000000000000ull;
}

// ---------------------------------------------------------------------------
// Partition digit of the reference API (src/partition/partition.c:29):
//   ((key - 1) & (((1<<D)-1) << R)) >> R    with a 32-bit mask
// ---------------------------------------------------------------------------
struct RefDigit {
    uint32_t mask;
    uint32_t shift;
    __host__ __device__ __forceinline__ RefDigit load() const { return *this; }
    __device__ __forceinline__ uint32_t operator()(const Tup& t) const {
        uint64_t km1 = (uint64_t)(tup_key(t) - 1);
        return (uint32_t)((km1 & (uint64_t)mask) >> shift);
    }
};

// ---------------------------------------------------------------------------
// Range plan: monotone (order preserving) multi-level MSD digits over the key
// range [base, base + 2^L).  Keys outside the range clamp to the first/last
// digit, so every level stays monotone in the key whatever the estimate.
//   rel(k) = clamp(key_u(k) - key_u(base), 0, 2^L - 1)
//   level-1 digit  d1 = rel >> s1                       (fanout 2^D1)
//   level-2 digit  d2 = (rel >> s2) - (d1 << D2)        (2^D2 per bucket)
//   level-3 digit  d3 = (rel >> s3) - ((d1<<D2|d2) << D3)
// ---------------------------------------------------------------------------
// bits of a partition's "bad tuple" flag (status word 1 of a join)
constexpr uint32_t kBadPayload = 1;  // a payload does not fit a packed word
constexpr uint32_t kBadRange = 2;    // a key lies outside the plan range
constexpr uint32_t kBadPayload48 = 4;  // ... fits a 64-bit word, not a 48-bit one
constexpr uint32_t kBadPayload32 = 8;  // ... fits a 48-bit word, not a 32-bit one

struct RangePlan {
    int64_t base;     // smallest key of the range
    uint64_t span;    // 2^L - 1 (all-ones of width L), L <= 64
    uint32_t D1, D2, D3;
    uint32_t s1, s2, s3;
};

__host__ __device__ __forceinline__ uint64_t plan_rel(const RangePlan& p,
                                                      int64_t k) {
    uint64_t ku = key_u(k), bu = key_u(p.base);
    if (ku < bu) return 0;
    uint64_t r = ku - bu;
    return r > p.span ? p.span : r;
}

__host__ __device__ __forceinline__ uint32_t plan_d1(const RangePlan& p,
                                                     uint64_t rel) {
    uint64_t d = rel >> p.s1;
    uint64_t lim = (1ull << p.D1) - 1;
    return (uint32_t)(d > lim ? lim : d);
}

// level-2 digit of `rel` inside bucket d1
// ---------------------------------------------------------------------------
// Element layouts of the intermediate passes (tile pass, group pass, skew
// kernels).  LayTup: the tuples themselves.  LayPacked (16-byte tuples): the
// level-1 partition packs every tuple into ONE 64-bit word
//     w = (rel mod 2^s1) << pb  |  payload          (pb = 64 - s1)
// where rel = key_u(key) - key_u(base) is the key's offset in the plan range
// and the bucket (rel >> s1) is implied by where the word sits.  Within a
// bucket the unsigned order of w is the (key, payload) order, so the passes
// sort words; the group pass unpacks when it writes the sorted tuples.  It
// applies when every key lies in the plan range and every payload in
// [0, 2^pb) -- the partition flags anything else and the join reruns on
// tuples.  Halves the bytes of the two intermediate passes.
// ---------------------------------------------------------------------------
struct LayTup {
    typedef Tup W;
    static constexpr bool packed = false;
    // element views of an intermediate buffer (base, plane stride): plain
    // pointers for the one-array layouts
    typedef const W* CView;
    typedef W* View;
    __device__ static __forceinline__ CView cview(const void* b, uint64_t) {
        return static_cast<const W*>(b);
    }
    __device__ static __forceinline__ View view(void* b, uint64_t) { return static_cast<W*>(b); }
    __device__ static __forceinline__ uint64_t rel(const RangePlan& P, const W& w, uint32_t) {
        return plan_rel(P, tup_key(w));
    }
    __device__ static __forceinline__ bool clamped(const RangePlan& P, const W& w) {
        const uint64_t ku = key_u(tup_key(w)), bu = key_u(P.base);
        return ku < bu || ku - bu > P.span;
    }
    __device__ static __forceinline__ bool less(const W& a, const W& b) { return tup_less(a, b); }
    __device__ static __forceinline__ Tup unpack(const RangePlan&, const W& w, uint32_t) {
        return w;
    }
    // Digit `sh`/`mask` of an element whose key lies inside the plan range
    // (no clamping: every group but the first and the last): the low 32 bits
    // of rel = key - base are exact modulo 2^32, so 32-bit arithmetic gives
    // bits [sh, sh + width) when sh + width <= 32 (fast_ok).
    __device__ static __forceinline__ uint32_t digit_fast(const W& w, uint32_t base_lo,
                                                          uint32_t, uint32_t sh, uint32_t mask) {
        return (((uint32_t)tup_key(w) - base_lo) >> sh) & mask;
    }
    __host__ static bool fast_ok(const RangePlan& P, uint32_t sh, uint32_t width) {
        return sh + width <= 32;
    }
    // digit_fast and unpack with their plan values read once (per group) into
    // registers: the group pass's per-element code then reads no argument
    // memory (bucketsort.hip sort_two)
    struct FastDigit {
        uint32_t base_lo, sh, mask;
        __device__ FastDigit(const RangePlan& P, uint32_t s, uint32_t width)
            : base_lo((uint32_t)P.base), sh(s), mask((1u << width) - 1) {}
        __device__ __forceinline__ uint32_t operator()(const W& w) const {
            return (((uint32_t)tup_key(w) - base_lo) >> sh) & mask;
        }
    };
    struct Unpack {
        __device__ Unpack(const RangePlan&, uint32_t) {}
        __device__ __forceinline__ Tup operator()(const W& w) const { return w; }
    };
    // equal keys: the elements are identical iff these values are
    __device__ static __forceinline__ uint64_t same_key_id(const W& w) {
#ifdef KEY_8B
        return (uint64_t)w.payload;
#else
        return w;
#endif
    }
};

#ifdef KEY_8B
struct LayPacked {
    typedef uint64_t W;
    static constexpr bool packed = true;
    typedef const W* CView;
    typedef W* View;
    __device__ static __forceinline__ CView cview(const void* b, uint64_t) {
        return static_cast<const W*>(b);
    }
    __device__ static __forceinline__ View view(void* b, uint64_t) { return static_cast<W*>(b); }
    __device__ static __forceinline__ uint64_t rel(const RangePlan& P, const W& w, uint32_t b) {
        return ((uint64_t)b << P.s1) | (w >> (64 - P.s1));
    }
    __device__ static __forceinline__ bool clamped(const RangePlan&, const W&) { return false; }
    __device__ static __forceinline__ bool less(const W& a, const W& b) { return a < b; }
    __device__ static __forceinline__ uint64_t same_key_id(const W& w) { return w; }
    // bits [sh, sh + width) of rel (sh + width <= s1, inside the word)
    __device__ static __forceinline__ uint32_t digit_fast(const W& w, uint32_t, uint32_t s1,
                                                          uint32_t sh, uint32_t mask) {
        return (uint32_t)(w >> (64 - s1 + sh)) & mask;
    }
    __host__ static bool fast_ok(const RangePlan& P, uint32_t sh, uint32_t width) {
        return sh + width <= P.s1;
    }
    __device__ static __forceinline__ Tup unpack(const RangePlan& P, const W& w, uint32_t b) {
        Tup t;
        t.payload = (int64_t)(w & (~0ull >> P.s1));
        t.key = (int64_t)((key_u(P.base) + rel(P, w, b)) ^ 0x8000000000000000ull);
        return t;
    }
    struct FastDigit {  // digit_fast with the plan read once (LayTup::FastDigit)
        uint32_t tsh, mask;
        __device__ FastDigit(const RangePlan& P, uint32_t s, uint32_t width)
            : tsh(64 - P.s1 + s), mask((1u << width) - 1) {}
        __device__ __forceinline__ uint32_t operator()(const W& w) const {
            return (uint32_t)(w >> tsh) & mask;
        }
    };
    struct Unpack {  // unpack of bucket b's words, the plan read once
        uint64_t kbu, pmask;
        uint32_t sh;
        __device__ Unpack(const RangePlan& P, uint32_t b)
            : kbu(key_u(P.base) + ((uint64_t)b << P.s1)), pmask(~0ull >> P.s1), sh(64 - P.s1) {}
        __device__ __forceinline__ Tup operator()(const W& w) const {
            Tup t;
            t.payload = (int64_t)(w & pmask);
            t.key = (int64_t)((kbu + (w >> sh)) ^ 0x8000000000000000ull);
            return t;
        }
    };
    // the level-1 partition's packing of tuple t into bucket rel >> s1;
    // `bad` gets kBadPayload when the payload lies outside [0, 2^pb) and
    // kBadRange when the key lies outside the plan (t cannot be packed)
    struct Pack {
        typedef uint64_t OutT;
        uint64_t bu, span;
        uint32_t s1;
        __device__ __forceinline__ uint64_t operator()(const Tup& t, uint32_t& bad) const {
            const uint64_t ku = key_u(t.key);
            const uint64_t r = ku - bu;
            const uint32_t pb = 64 - s1;
            bad |= (ku < bu || r > span) ? kBadRange : 0u;
            bad |= ((uint64_t)t.payload >> pb) != 0 ? kBadPayload : 0u;
            return ((r & ((1ull << s1) - 1)) << pb) | (uint64_t)t.payload;
        }
        static constexpr uint32_t kStoreBytes = 8;  // bytes of one element in a plane
        __device__ static __forceinline__ void store(void* out, uint64_t, uint64_t i,
                                                     uint64_t x) {
            static_cast<uint64_t*>(out)[i] = x;
        }
        static constexpr bool kPairs = false;  // store2: LayP48's two-plane pairs only
        template <class X>
        __device__ static __forceinline__ void store2(void*, uint64_t, uint64_t, const X&,
                                                      const X&) {}
    };
    // packing applies to plans whose level-1 buckets span 2^1 .. 2^32 keys
    __host__ static bool usable(const RangePlan& P) { return P.s1 >= 1 && P.s1 <= 32; }
};
#endif

#ifndef SMJ_P96_SEGB
#define SMJ_P96_SEGB 8  // LayP96::Pack::kStoreBytes
#endif
#ifdef KEY_8B
// ---------------------------------------------------------------------------
// LayP96 (round 6, 16-byte tuples whose payloads no packed word holds): the
// full 64-bit payload and the key's offset in the plan range,
//     rel = key_u(key) - key_u(base)      (< 2^32: plans spanning <= 2^32 keys)
// stored as two planes of one buffer: pay = int64[stride], then rel =
// uint32[stride].  12 bytes an element instead of the 16 of the tuple: the
// level-1 scatter writes, the tile pass reads and writes and the group pass
// reads a quarter fewer bytes.  In registers and LDS an element is a packed
// 12-byte P96W (three dwords) ordered like (key, payload): a group-pass
// workgroup's buffer is then 30 KB instead of 41, and three fit a CU instead
// of two (round 6: the join 4.70 -> 4.33 ms, the group pass 1.81 -> 1.56 ms,
// profiles/r06_lab/p12_ab.txt).  The group pass writes the full tuples.  A
// key outside the plan is flagged kBadRange by the partition (the join then
// takes the 16-byte tuples).
// ---------------------------------------------------------------------------
struct __attribute__((packed, aligned(4))) P96W {
    int64_t pay;
    uint32_t rel;
};
static_assert(sizeof(P96W) == 12, "12-byte element");
typedef const __attribute__((address_space(1))) int64_t* G64c;
typedef __attribute__((address_space(1))) int64_t* G64;
typedef const __attribute__((address_space(1))) uint32_t* G32c96;
typedef __attribute__((address_space(1))) uint32_t* G32w96;
struct P96CView {
    G64c pay;
    G32c96 rel;
    __device__ __forceinline__ P96W operator[](uint64_t i) const {
        P96W w;
        w.pay = pay[i];
        w.rel = rel[i];
        return w;
    }
    __device__ __forceinline__ P96CView operator+(uint64_t k) const {
        return P96CView{pay + k, rel + k};
    }
};
struct P96View {
    G64 pay;
    G32w96 rel;
    __device__ __forceinline__ P96View operator+(uint64_t k) const {
        return P96View{pay + k, rel + k};
    }
};
__device__ __forceinline__ void st_w(const P96View& p, const P96W& w) {
#if SMJ_NT_STORES
    __builtin_nontemporal_store(w.pay, (int64_t*)p.pay);
    __builtin_nontemporal_store(w.rel, (uint32_t*)p.rel);
#else
    p.pay[0] = w.pay;
    p.rel[0] = w.rel;
#endif
}

struct LayP96 {
    typedef P96W W;
    static constexpr bool packed = true;
    typedef P96CView CView;
    typedef P96View View;
    __device__ static __forceinline__ CView cview(const void* b, uint64_t stride) {
        const int64_t* pay = static_cast<const int64_t*>(b);
        return CView{(G64c)pay, (G32c96)(const uint32_t*)(pay + stride)};
    }
    __device__ static __forceinline__ View view(void* b, uint64_t stride) {
        int64_t* pay = static_cast<int64_t*>(b);
        return View{(G64)pay, (G32w96)(uint32_t*)(pay + stride)};
    }
    __device__ static __forceinline__ uint64_t rel(const RangePlan&, const W& w, uint32_t) {
        return w.rel;
    }
    __device__ static __forceinline__ bool clamped(const RangePlan&, const W&) { return false; }
    __device__ static __forceinline__ bool less(const W& a, const W& b) {
        return a.rel < b.rel || (a.rel == b.rel && a.pay < b.pay);
    }
    __device__ static __forceinline__ uint64_t same_key_id(const W& w) {
        return (uint64_t)w.pay;
    }
    // bits [sh, sh + width) of rel (sh + width <= 32)
    __device__ static __forceinline__ uint32_t digit_fast(const W& w, uint32_t, uint32_t,
                                                          uint32_t sh, uint32_t mask) {
        return (w.rel >> sh) & mask;
    }
    __host__ static bool fast_ok(const RangePlan&, uint32_t sh, uint32_t width) {
        return sh + width <= 32;
    }
    __device__ static __forceinline__ Tup unpack(const RangePlan& P, const W& w, uint32_t) {
        Tup t;
        t.payload = w.pay;
        t.key = (int64_t)((key_u(P.base) + w.rel) ^ 0x8000000000000000ull);
        return t;
    }
    struct FastDigit {
        uint32_t sh, mask;
        __device__ FastDigit(const RangePlan&, uint32_t s, uint32_t width)
            : sh(s), mask((1u << width) - 1) {}
        __device__ __forceinline__ uint32_t operator()(const W& w) const {
            return (w.rel >> sh) & mask;
        }
    };
    struct Unpack {
        uint64_t kbu;
        __device__ Unpack(const RangePlan& P, uint32_t) : kbu(key_u(P.base)) {}
        __device__ __forceinline__ Tup operator()(const W& w) const {
            Tup t;
            t.payload = w.pay;
            t.key = (int64_t)((kbu + w.rel) ^ 0x8000000000000000ull);
            return t;
        }
    };
    // the level-1 partition's element of tuple t: kBadRange when the key
    // lies outside the plan (its offset would not be exact)
    struct Pack {
        typedef P96W OutT;
        uint64_t bu, span;
        __device__ __forceinline__ P96W operator()(const Tup& t, uint32_t& bad) const {
            const uint64_t ku = key_u(t.key);
            const uint64_t r = ku - bu;
            bad |= (ku < bu || r > span) ? kBadRange : 0u;
            P96W w;
            w.pay = t.payload;
            w.rel = (uint32_t)r;
            return w;
        }
        // the plane whose 64 bytes make a segment: 8, the payload plane (8
        // elements); 4, the offset plane (16)
        static constexpr uint32_t kStoreBytes = SMJ_P96_SEGB;
        __device__ static __forceinline__ void store(void* out, uint64_t stride, uint64_t i,
                                                     const P96W& x) {
            int64_t* pay = static_cast<int64_t*>(out);
            ((G64)pay)[i] = x.pay;
            ((G32w96)(uint32_t*)(pay + stride))[i] = x.rel;
        }
        // elements i and i + 1 (i even): one 16-byte and one 8-byte store
        static constexpr bool kPairs = true;
        __device__ static __forceinline__ void store2(void* out, uint64_t stride, uint64_t i,
                                                      const P96W& x0, const P96W& x1) {
            typedef long long L2 __attribute__((ext_vector_type(2)));
            typedef uint32_t U2 __attribute__((ext_vector_type(2)));
            int64_t* pay = static_cast<int64_t*>(out);
            L2 p = {x0.pay, x1.pay};
            U2 r = {x0.rel, x1.rel};
            *(__attribute__((address_space(1))) L2*)(pay + i) = p;
            *(__attribute__((address_space(1))) U2*)((uint32_t*)(pay + stride) + i) = r;
        }
    };
    // plans whose range spans at most 2^32 keys (rel fits 32 bits)
    __host__ static bool usable(const RangePlan& P) { return P.span < (1ull << 32); }
};
#endif

// ---------------------------------------------------------------------------
// LayP48 (round 4, both tuple widths): the packed word of LayPacked cut to
// 48 bits,
//     w = (rel mod 2^s1) << (48 - s1)  |  payload          (payload < 2^(48-s1))
// (8-byte tuples: the payload as the unsigned 32-bit value their order uses)
// and stored as two planes of one buffer: lo = w mod 2^32 (uint32[stride])
// then hi = w >> 32 (uint16[stride]), element i at lo[i] and hi[i].  6 bytes
// an element instead of 8: the level-1 scatter writes, the tile pass reads and
// writes and the group pass reads a quarter fewer bytes.  In registers and in
// LDS an element is still a uint64_t, ordered like the (key, payload) order.
// The partition flags kBadPayload48 when a payload needs more than 48 - s1
// bits; the join then reruns with 64-bit words (LayPacked).
// ---------------------------------------------------------------------------
typedef const __attribute__((address_space(1))) uint32_t* G32c;
typedef const __attribute__((address_space(1))) uint16_t* G16c;
typedef __attribute__((address_space(1))) uint32_t* G32;
typedef __attribute__((address_space(1))) uint16_t* G16;

struct P48CView {
    G32c lo;
    G16c hi;
    __device__ __forceinline__ uint64_t operator[](uint64_t i) const {
        return (uint64_t)lo[i] | ((uint64_t)hi[i] << 32);
    }
    __device__ __forceinline__ P48CView operator+(uint64_t k) const {
        return P48CView{lo + k, hi + k};
    }
};

struct P48View {
    G32 lo;
    G16 hi;
    __device__ __forceinline__ uint64_t operator[](uint64_t i) const {
        return (uint64_t)lo[i] | ((uint64_t)hi[i] << 32);
    }
    __device__ __forceinline__ P48View operator+(uint64_t k) const {
        return P48View{lo + k, hi + k};
    }
};

// streaming store of element 0 of a view (the plane counterpart of st_w)
__device__ __forceinline__ void st_w(const P48View& p, uint64_t v) {
#if SMJ_NT_STORES
    __builtin_nontemporal_store((uint32_t)v, p.lo);
    __builtin_nontemporal_store((uint16_t)(v >> 32), p.hi);
#else
    p.lo[0] = (uint32_t)v;
    p.hi[0] = (uint16_t)(v >> 32);
#endif
}

struct LayP48 {
    typedef uint64_t W;
    static constexpr bool packed = true;
    typedef P48CView CView;
    typedef P48View View;
    __device__ static __forceinline__ CView cview(const void* b, uint64_t stride) {
        const uint32_t* lo = static_cast<const uint32_t*>(b);
        return CView{(G32c)lo, (G16c)(const uint16_t*)(lo + stride)};
    }
    __device__ static __forceinline__ View view(void* b, uint64_t stride) {
        uint32_t* lo = static_cast<uint32_t*>(b);
        return View{(G32)lo, (G16)(uint16_t*)(lo + stride)};
    }
    __device__ static __forceinline__ uint64_t rel(const RangePlan& P, const W& w, uint32_t b) {
        return ((uint64_t)b << P.s1) | (w >> (48 - P.s1));
    }
    __device__ static __forceinline__ bool clamped(const RangePlan&, const W&) { return false; }
    __device__ static __forceinline__ bool less(const W& a, const W& b) { return a < b; }
    __device__ static __forceinline__ uint64_t same_key_id(const W& w) { return w; }
    __device__ static __forceinline__ uint32_t digit_fast(const W& w, uint32_t, uint32_t s1,
                                                          uint32_t sh, uint32_t mask) {
        return (uint32_t)(w >> (48 - s1 + sh)) & mask;
    }
    __host__ static bool fast_ok(const RangePlan& P, uint32_t sh, uint32_t width) {
        return sh + width <= P.s1;
    }
    __device__ static __forceinline__ Tup unpack(const RangePlan& P, const W& w, uint32_t b) {
        const uint64_t pay = w & (~0ull >> (16 + P.s1));
        const int64_t key = (int64_t)((key_u(P.base) + rel(P, w, b)) ^ 0x8000000000000000ull);
#ifdef KEY_8B
        Tup t;
        t.payload = (int64_t)pay;
        t.key = key;
        return t;
#else
        return ((uint64_t)(uint32_t)key << 32) | pay;
#endif
    }
    struct FastDigit {  // digit_fast with the plan read once (LayTup::FastDigit)
        uint32_t tsh, mask;
        __device__ FastDigit(const RangePlan& P, uint32_t s, uint32_t width)
            : tsh(48 - P.s1 + s), mask((1u << width) - 1) {}
        __device__ __forceinline__ uint32_t operator()(const W& w) const {
            return (uint32_t)(w >> tsh) & mask;
        }
    };
    // unpack of bucket b's words, the plan read once: key = base + b 2^s1 +
    // (w >> (48 - s1)) (the low s1 bits of the offset and the bucket's bits
    // do not overlap, so + is |); 8-byte tuples need the low 32 bits only
    struct Unpack {
        uint64_t kbu, pmask;
        uint32_t sh;
        __device__ Unpack(const RangePlan& P, uint32_t b)
            : kbu(key_u(P.base) + ((uint64_t)b << P.s1)), pmask(~0ull >> (16 + P.s1)),
              sh(48 - P.s1) {}
        __device__ __forceinline__ Tup operator()(const W& w) const {
#ifdef KEY_8B
            Tup t;
            t.payload = (int64_t)(w & pmask);
            t.key = (int64_t)((kbu + (w >> sh)) ^ 0x8000000000000000ull);
            return t;
#else
            const uint32_t key = (uint32_t)kbu + (uint32_t)(w >> sh);
            return ((uint64_t)key << 32) | (uint32_t)(w & pmask);
#endif
        }
    };
    struct Pack {
        typedef uint64_t OutT;
        uint64_t bu, span;
        uint32_t s1;
        __device__ __forceinline__ uint64_t operator()(const Tup& t, uint32_t& bad) const {
            const uint64_t ku = key_u(tup_key(t));
            const uint64_t r = ku - bu;
            const uint32_t pb = 48 - s1;
#ifdef KEY_8B
            const uint64_t pay = (uint64_t)t.payload;
#else
            const uint64_t pay = (uint32_t)t;  // unsigned, as the 8-byte order takes it
#endif
            bad |= (ku < bu || r > span) ? kBadRange : 0u;
            bad |= (pay >> (64 - s1)) != 0 ? kBadPayload : 0u;
            bad |= (pay >> pb) != 0 ? kBadPayload48 : 0u;
            return ((r & ((1ull << s1) - 1)) << pb) | (pay & ((1ull << pb) - 1));
        }
        // the lo plane sets the segment: 16 elements = 64 bytes (hi: 32 bytes)
        static constexpr uint32_t kStoreBytes = 4;
        __device__ static __forceinline__ void store(void* out, uint64_t stride, uint64_t i,
                                                     uint64_t x) {
            uint32_t* lo = static_cast<uint32_t*>(out);
            ((G32)lo)[i] = (uint32_t)x;
            ((G16)(uint16_t*)(lo + stride))[i] = (uint16_t)(x >> 32);
        }
        // elements i and i + 1 (i even) with one store per plane: 8 + 4
        // bytes a lane instead of 4 + 2 (half the store instructions)
        static constexpr bool kPairs = true;
        __device__ static __forceinline__ void store2(void* out, uint64_t stride, uint64_t i,
                                                      uint64_t x0, uint64_t x1) {
            typedef uint32_t U2 __attribute__((ext_vector_type(2)));
            typedef uint16_t H2 __attribute__((ext_vector_type(2)));
            uint32_t* lo = static_cast<uint32_t*>(out);
            const U2 l = {(uint32_t)x0, (uint32_t)x1};
            const H2 h = {(uint16_t)(x0 >> 32), (uint16_t)(x1 >> 32)};
            *(__attribute__((address_space(1))) U2*)(lo + i) = l;
            *(__attribute__((address_space(1))) H2*)((uint16_t*)(lo + stride) + i) = h;
        }
    };
    __host__ static bool usable(const RangePlan& P) { return P.s1 >= 1 && P.s1 <= 32; }
};

// LayP32 (round 5, both tuple widths): the packed word cut to 32 bits, one
// plane, W = uint32_t in registers and LDS as well:
//     w = (rel mod 2^s1) << (32 - s1)  |  payload        (payload < 2^(32 - s1))
// It holds where the payloads are tiny -- the sort benchmark's relation
// (create_relation_pk: keys 1..N, payload 0, BASELINE configs[1]) -- and
// moves 4 bytes an element through the intermediate passes instead of 6; its
// tiles hold 32768 elements.  The partition flags kBadPayload32 when a
// payload needs more bits (with kBadPayload48 / kBadPayload as for the wider
// words), and the call reruns in the next wider layout.
// views of a LayP32 buffer: global pointers (loads through them stay
// global_load), elements read by value
struct P32CView {
    G32c p;
    __device__ __forceinline__ uint32_t operator[](uint64_t i) const { return p[i]; }
    __device__ __forceinline__ P32CView operator+(uint64_t k) const { return P32CView{p + k}; }
};
struct P32View {
    G32 p;
    __device__ __forceinline__ uint32_t operator[](uint64_t i) const { return p[i]; }
    __device__ __forceinline__ P32View operator+(uint64_t k) const { return P32View{p + k}; }
};
__device__ __forceinline__ void st_w(const P32View& v, uint32_t x) {
#if SMJ_NT_STORES
    __builtin_nontemporal_store(x, v.p);
#else
    v.p[0] = x;
#endif
}

struct LayP32 {
    typedef uint32_t W;
    static constexpr bool packed = true;
    typedef P32CView CView;
    typedef P32View View;
    __device__ static __forceinline__ CView cview(const void* b, uint64_t) {
        return CView{(G32c) static_cast<const uint32_t*>(b)};
    }
    __device__ static __forceinline__ View view(void* b, uint64_t) {
        return View{(G32) static_cast<uint32_t*>(b)};
    }
    __device__ static __forceinline__ uint64_t rel(const RangePlan& P, const W& w, uint32_t b) {
        return ((uint64_t)b << P.s1) | (uint64_t)(w >> (32 - P.s1));
    }
    __device__ static __forceinline__ bool clamped(const RangePlan&, const W&) { return false; }
    __device__ static __forceinline__ bool less(const W& a, const W& b) { return a < b; }
    __device__ static __forceinline__ uint64_t same_key_id(const W& w) { return w; }
    __device__ static __forceinline__ uint32_t digit_fast(const W& w, uint32_t, uint32_t s1,
                                                          uint32_t sh, uint32_t mask) {
        return (w >> (32 - s1 + sh)) & mask;
    }
    __host__ static bool fast_ok(const RangePlan& P, uint32_t sh, uint32_t width) {
        return sh + width <= P.s1;
    }
    __device__ static __forceinline__ Tup unpack(const RangePlan& P, const W& w, uint32_t b) {
        const uint32_t pay = w & (0xffffffffu >> P.s1);
        const int64_t key = (int64_t)((key_u(P.base) + rel(P, w, b)) ^ 0x8000000000000000ull);
#ifdef KEY_8B
        Tup t;
        t.payload = (int64_t)pay;
        t.key = key;
        return t;
#else
        return ((uint64_t)(uint32_t)key << 32) | pay;
#endif
    }
    struct FastDigit {
        uint32_t tsh, mask;
        __device__ FastDigit(const RangePlan& P, uint32_t s, uint32_t width)
            : tsh(32 - P.s1 + s), mask((1u << width) - 1) {}
        __device__ __forceinline__ uint32_t operator()(const W& w) const {
            return (w >> tsh) & mask;
        }
    };
    struct Unpack {
        uint64_t kbu;
        uint32_t pmask, sh;
        __device__ Unpack(const RangePlan& P, uint32_t b)
            : kbu(key_u(P.base) + ((uint64_t)b << P.s1)), pmask(0xffffffffu >> P.s1),
              sh(32 - P.s1) {}
        __device__ __forceinline__ Tup operator()(const W& w) const {
#ifdef KEY_8B
            Tup t;
            t.payload = (int64_t)(w & pmask);
            t.key = (int64_t)((kbu + (w >> sh)) ^ 0x8000000000000000ull);
            return t;
#else
            const uint32_t key = (uint32_t)kbu + (w >> sh);
            return ((uint64_t)key << 32) | (w & pmask);
#endif
        }
    };
    struct Pack {
        typedef uint32_t OutT;
        uint64_t bu, span;
        uint32_t s1;
        __device__ __forceinline__ uint32_t operator()(const Tup& t, uint32_t& bad) const {
            const uint64_t ku = key_u(tup_key(t));
            const uint64_t r = ku - bu;
#ifdef KEY_8B
            const uint64_t pay = (uint64_t)t.payload;
#else
            const uint64_t pay = (uint32_t)t;  // unsigned, as the 8-byte order takes it
#endif
            bad |= (ku < bu || r > span) ? kBadRange : 0u;
            bad |= (pay >> (64 - s1)) != 0 ? kBadPayload : 0u;
            bad |= (pay >> (48 - s1)) != 0 ? kBadPayload48 : 0u;
            bad |= (pay >> (32 - s1)) != 0 ? kBadPayload32 : 0u;
            return ((uint32_t)r << (32 - s1)) | ((uint32_t)pay & (0xffffffffu >> s1));
        }
        static constexpr uint32_t kStoreBytes = 4;
        __device__ static __forceinline__ void store(void* out, uint64_t, uint64_t i, uint32_t x) {
#if SMJ_NT_STORES
            __builtin_nontemporal_store(x, (G32) static_cast<uint32_t*>(out) + i);
#else
            ((G32) static_cast<uint32_t*>(out))[i] = x;
#endif
        }
        // a whole 16-byte segment (i a multiple of 4) with one store
#ifndef SMJ_P32_QUADS
#define SMJ_P32_QUADS 1
#endif
        static constexpr bool kQuads = SMJ_P32_QUADS;
        __device__ static __forceinline__ void store4(void* out, uint64_t, uint64_t i,
                                                      const uint32_t (&x)[4]) {
            typedef uint32_t U4 __attribute__((ext_vector_type(4)));
            const U4 v = {x[0], x[1], x[2], x[3]};
            __attribute__((address_space(1))) U4* p =
                (__attribute__((address_space(1))) U4*)(static_cast<uint32_t*>(out) + i);
#if SMJ_NT_STORES
            __builtin_nontemporal_store(v, p);
#else
            *p = v;
#endif
        }
        // elements i and i + 1 (i even) with one 8-byte store
        static constexpr bool kPairs = true;
        __device__ static __forceinline__ void store2(void* out, uint64_t, uint64_t i, uint32_t x0,
                                                      uint32_t x1) {
            typedef uint32_t U2 __attribute__((ext_vector_type(2)));
            const U2 v = {x0, x1};
            __attribute__((address_space(1))) U2* p =
                (__attribute__((address_space(1))) U2*)(static_cast<uint32_t*>(out) + i);
#if SMJ_NT_STORES
            __builtin_nontemporal_store(v, p);
#else
            *p = v;
#endif
        }
    };
    // s1 key bits and at least one payload bit
    __host__ static bool usable(const RangePlan& P) { return P.s1 >= 1 && P.s1 <= 31; }
};

// LayP40 (round 5): the tile pass's output of 48-bit words.  Inside one
// group (bucket b, level-2 digit g) the word's top D2 bits are g, so the tile
// pass stores only the low 48 - D2 <= 40 bits: the lo plane in place, bits
// 32..39 in a byte plane of their own (the 16-bit plane of the input is still
// being read by other tiles), 5 bytes an element instead of 6.  A view made
// for one group (with_group) ORs g back in on every load, so the group pass
// and the skew kernels see LayP48's words and use LayP48's arithmetic.  The
// plane "stride" of this layout is the byte offset from the lo plane to the
// byte plane (any buffer; the offset wraps modulo 2^64).  Applies when D2 >= 8.
typedef const __attribute__((address_space(1))) uint8_t* G8c;
typedef __attribute__((address_space(1))) uint8_t* G8;
struct P40CView {
    G32c lo;
    G8c hi;
    uint64_t gbits;  // the group's digit, in place (0 before with_group)
    __device__ __forceinline__ uint64_t operator[](uint64_t i) const {
        return (uint64_t)lo[i] | ((uint64_t)hi[i] << 32) | gbits;
    }
    __device__ __forceinline__ P40CView operator+(uint64_t k) const {
        return P40CView{lo + k, hi + k, gbits};
    }
};
struct P40View {
    G32 lo;
    G8 hi;
    __device__ __forceinline__ P40View operator+(uint64_t k) const { return P40View{lo + k, hi + k}; }
};
__device__ __forceinline__ void st_w(const P40View& p, uint64_t v) {
#if SMJ_NT_STORES
    __builtin_nontemporal_store((uint32_t)v, p.lo);
    __builtin_nontemporal_store((uint8_t)(v >> 32), p.hi);
#else
    p.lo[0] = (uint32_t)v;
    p.hi[0] = (uint8_t)(v >> 32);
#endif
}
struct LayP40 : LayP48 {
    typedef P40CView CView;
    typedef P40View View;
    __device__ static __forceinline__ CView cview(const void* b, uint64_t hoff) {
        return CView{(G32c) static_cast<const uint32_t*>(b),
                     (G8c)(static_cast<const uint8_t*>(b) + hoff), 0ull};
    }
    __device__ static __forceinline__ View view(void* b, uint64_t hoff) {
        return View{(G32) static_cast<uint32_t*>(b), (G8)(static_cast<uint8_t*>(b) + hoff)};
    }
    __host__ static bool holds(const RangePlan& P) { return P.D2 >= 8; }
};
// a view of group g's elements: LayP40 restores the digit; the other layouts'
// views are complete already
template <class V>
__device__ __forceinline__ V with_group(const V& v, uint32_t, const RangePlan&) {
    return v;
}
__device__ __forceinline__ P40CView with_group(const P40CView& v, uint32_t g, const RangePlan& P) {
    return P40CView{v.lo, v.hi, (uint64_t)g << (48 - P.D2)};
}

// identity "packing" of the plain layout
struct PackNone {
    typedef Tup OutT;
    __device__ __forceinline__ Tup operator()(const Tup& t, uint32_t&) const { return t; }
    static constexpr uint32_t kStoreBytes = sizeof(Tup);
    __device__ static __forceinline__ void store(void* out, uint64_t, uint64_t i, const Tup& x) {
        static_cast<Tup*>(out)[i] = x;
    }
    static constexpr bool kPairs = false;  // store2: LayP48's two-plane pairs only
    template <class X>
    __device__ static __forceinline__ void store2(void*, uint64_t, uint64_t, const X&,
                              const X&) {}
};

// the plain layout with a range check: kBadRange when the key lies outside
// [bu, bu + span] (key_u order).  A plan guessed from the relation size (the
// reference's own assumption, keys <= |R|) is verified this way in the pass
// that reads every key anyway; bu = 0, span = ~0 checks nothing.
struct PackRange {
    typedef Tup OutT;
    uint64_t bu, span;
    __device__ __forceinline__ Tup operator()(const Tup& t, uint32_t& bad) const {
        const uint64_t ku = key_u(tup_key(t));
        bad |= (ku < bu || ku - bu > span) ? kBadRange : 0u;
        return t;
    }
    static constexpr uint32_t kStoreBytes = sizeof(Tup);
    __device__ static __forceinline__ void store(void* out, uint64_t, uint64_t i, const Tup& x) {
        static_cast<Tup*>(out)[i] = x;
    }
    static constexpr bool kPairs = false;  // store2: LayP48's two-plane pairs only
    template <class X>
    __device__ static __forceinline__ void store2(void*, uint64_t, uint64_t, const X&,
                              const X&) {}
};

__host__ __device__ __forceinline__ uint32_t plan_d2(const RangePlan& p,
                                                     uint64_t rel,
                                                     uint32_t d1) {
    uint64_t v = rel >> p.s2;
    uint64_t lo = (uint64_t)d1 << p.D2;
    uint64_t lim = (1ull << p.D2) - 1;
    if (v < lo) return 0;
    v -= lo;
    return (uint32_t)(v > lim ? lim : v);
}

__host__ __device__ __forceinline__ uint32_t plan_d3(const RangePlan& p,
                                                     uint64_t rel,
                                                     uint32_t d12) {
    uint64_t v = rel >> p.s3;
    uint64_t lo = (uint64_t)d12 << p.D3;
    uint64_t lim = (1ull << p.D3) - 1;
    if (v < lo) return 0;
    v -= lo;
    return (uint32_t)(v > lim ? lim : v);
}

// Build a plan for key range [kmin, kmax]: D1 level-1 bits, D2 level-2 bits
// preferred by size, widened up to D2cap when that makes the last digit exact
// (s3 == 0 with D3 <= D3max).
__host__ __device__ inline RangePlan make_plan(int64_t kmin, int64_t kmax,
                                               uint32_t D1, uint32_t D2,
                                               uint32_t D2cap, uint32_t D3max) {
    RangePlan p;
    p.base = kmin;
    uint64_t width = (kmax >= kmin) ? (key_u(kmax) - key_u(kmin)) : 0;
    uint32_t L = 0;
    while (L < 64 && (width >> L) != 0) L++;
    p.span = (L >= 64) ? ~0ull : ((1ull << L) - 1);
    p.D1 = D1;
    p.s1 = L > D1 ? L - D1 : 0;
    p.D2 = D2 < p.s1 ? D2 : p.s1;  // never more level-2 bits than remain
    uint32_t s2 = p.s1 - p.D2;
    if (s2 > D3max && p.D2 < D2cap) {
        uint32_t extra = s2 - D3max;
        if (extra > D2cap - p.D2) extra = D2cap - p.D2;
        p.D2 += extra;
        s2 -= extra;
    }
    p.s2 = s2;
    p.D3 = s2 < D3max ? s2 : D3max;
    p.s3 = s2 - p.D3;
    return p;
}

// ---------------------------------------------------------------------------
// Wave / block helpers (wave64)
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ uint64_t lanemask_lt() {
    int l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// block-wide exclusive scan of one uint32 per thread (blockDim.x threads,
// multiple of 64). `scratch` >= blockDim.x/64 + 1 words of LDS.
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v,
                                                         uint32_t* scratch,
                                                         uint32_t* total) {
    const int lane = lane_id();
    const int wid = threadIdx.x >> 6;
    const int nw = blockDim.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) scratch[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int w = 0; w < nw; w++) {
            uint32_t t = scratch[w];
            scratch[w] = run;
            run += t;
        }
        scratch[nw] = run;
    }
    __syncthreads();
    uint32_t res = scratch[wid] + x - v;
    if (total) *total = scratch[nw];
    __syncthreads();
    return res;
}

__host__ __device__ __forceinline__ uint64_t align_tuples(uint64_t n) {
    const uint64_t tpl = 64 / sizeof(Tup);
    return (n + tpl - 1) & ~(tpl - 1);
}

}  // namespace smj
