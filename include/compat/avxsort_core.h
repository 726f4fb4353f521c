/*
 * avxsort_core.h -- drop-in for the reference header src/avxsort/avxsort_core.h
 * (sdecoder/AVX-sort-merge-joins) as tests/check_merge.c uses it.  In the
 * reference this header holds the AVX register kernels themselves: the bitonic
 * merge networks merge{4,8,16}_{eqlen,varlen}[_aligned] (avxsort_core.h:76-1100,
 * 1601-1750), the 4x4 in-register sort inregister_sort_keyval32
 * (avxsort_core.h:1213-1290, 1538-1600) and keycmp (avxsort_core.h:1400-1412).
 * On MI355X there are no host register kernels: each one is a library call on
 * the device.  inregister_sort_keyval32 is the reference's network itself
 * (smj_inregister_sort_keyval32, byte-identical).  The merges are the
 * library's device merge of the same int64 items in the same FP64 order
 * (avx_merge_int64): the same output; unlike the reference's _varlen
 * kernels they never write into their inputs (the reference flushes its last
 * register into consumed input slots, avxsort_core.h:461-475; INTEGRATION.md
 * documents the difference).  The reference header has no include
 * guard; this one has.  Host wrappers only; the declarations live in ../smj.h.
 */
#ifndef SMJ_COMPAT_AVXSORT_CORE_H
#define SMJ_COMPAT_AVXSORT_CORE_H
#ifndef SMJ_H
#define SMJ_COMPAT_HIDE_PRINT_TIMING
#endif
#include <stdint.h>
#include <string.h>
#include "../smj.h"

/* int64 three-way compare (avxsort_core.h:1400-1412) */
static inline int keycmp(const void * k1, const void * k2)
{
    const int64_t a = *(const int64_t *)k1, b = *(const int64_t *)k2;
    return a < b ? -1 : (a > b ? 1 : 0);
}

/* two sorted lists of len items each -> 2 len items */
#define SMJ_COMPAT_MERGE_EQLEN(name)                                             \
    static inline void name(int64_t * const inpA, int64_t * const inpB,          \
                            int64_t * const out, const uint32_t len)             \
    {                                                                            \
        avx_merge_int64(inpA, inpB, out, len, len);                              \
    }
SMJ_COMPAT_MERGE_EQLEN(merge4_eqlen)
SMJ_COMPAT_MERGE_EQLEN(merge8_eqlen)
SMJ_COMPAT_MERGE_EQLEN(merge16_eqlen)
SMJ_COMPAT_MERGE_EQLEN(merge4_eqlen_aligned)
SMJ_COMPAT_MERGE_EQLEN(merge8_eqlen_aligned)
SMJ_COMPAT_MERGE_EQLEN(merge16_eqlen_aligned)
#undef SMJ_COMPAT_MERGE_EQLEN

/* sorted lists of lenA and lenB items -> lenA + lenB items */
#define SMJ_COMPAT_MERGE_VARLEN(name)                                            \
    static inline void name(int64_t * inpA, int64_t * inpB, int64_t * out,       \
                            const uint32_t lenA, const uint32_t lenB)            \
    {                                                                            \
        avx_merge_int64(inpA, inpB, out, lenA, lenB);                            \
    }
SMJ_COMPAT_MERGE_VARLEN(merge4_varlen)
SMJ_COMPAT_MERGE_VARLEN(merge8_varlen)
SMJ_COMPAT_MERGE_VARLEN(merge16_varlen)
SMJ_COMPAT_MERGE_VARLEN(merge4_varlen_aligned)
SMJ_COMPAT_MERGE_VARLEN(merge8_varlen_aligned)
SMJ_COMPAT_MERGE_VARLEN(merge16_varlen_aligned)
#undef SMJ_COMPAT_MERGE_VARLEN

/* 16 items -> four rows of four: row j = column j of the 4x4 input through
 * the reference's odd-even network (avxsort_core.h:1213-1274), byte-identical
 * (the device kernel behind smj_inregister_sort_keyval32) */
static inline void inregister_sort_keyval32(int64_t * items, int64_t * output)
{
    smj_inregister_sort_keyval32(items, output, 1);
}

static inline void inregister_sort_keyval32_aligned(int64_t * items, int64_t * output)
{
    inregister_sort_keyval32(items, output);
}

#endif /* SMJ_COMPAT_AVXSORT_CORE_H */
