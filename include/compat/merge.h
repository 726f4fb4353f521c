/*
 * merge.h -- drop-in for the reference header src/merge/merge.h:35-97
 * (sdecoder/AVX-sort-merge-joins).  Same file name and include guard, so a
 * reference driver that includes "merge.h" compiles unchanged against
 * libsmj_hip.so (8-byte tuples) or libsmj_hip_k8.so (-DKEY_8B, 16-byte tuples).
 * Provides: avx_merge_tuples/_int64, scalar_merge_tuples/_int64.  The declarations live in ../smj.h.
 */
#ifndef MERGE_H
#define MERGE_H
#ifndef SMJ_H
#define SMJ_COMPAT_HIDE_PRINT_TIMING
#endif
#include "../smj.h"
#endif /* MERGE_H */
