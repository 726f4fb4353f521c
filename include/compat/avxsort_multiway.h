/*
 * avxsort_multiway.h -- drop-in for the reference header src/avxsort/avxsort_multiway.h:35-55
 * (sdecoder/AVX-sort-merge-joins).  Same file name and include guard, so a
 * reference driver that includes "avxsort_multiway.h" compiles unchanged against
 * libsmj_hip.so (8-byte tuples) or libsmj_hip_k8.so (-DKEY_8B, 16-byte tuples).
 * Provides: avxsortmultiway_tuples, avxsortmultiway_int64.  The declarations live in ../smj.h.
 */
#ifndef AVXSORT_MULTIWAYMERGE_H_
#define AVXSORT_MULTIWAYMERGE_H_
#ifndef SMJ_H
#define SMJ_COMPAT_HIDE_PRINT_TIMING
#endif
#include "../smj.h"
#endif /* AVXSORT_MULTIWAYMERGE_H_ */
