/*
 * avxsort.h -- drop-in for the reference header src/avxsort/avxsort.h:35-57
 * (sdecoder/AVX-sort-merge-joins).  Same file name and include guard, so a
 * reference driver that includes "avxsort.h" compiles unchanged against
 * libsmj_hip.so (8-byte tuples) or libsmj_hip_k8.so (-DKEY_8B, 16-byte tuples).
 * Provides: avxsort_tuples, avxsort_int64, avxsort_int32.  The declarations live in ../smj.h.
 */
#ifndef AVXSORT_H
#define AVXSORT_H
#ifndef SMJ_H
#define SMJ_COMPAT_HIDE_PRINT_TIMING
#endif
#include "../smj.h"
#endif /* AVXSORT_H */
