/*
 * scalarsort.h -- drop-in for the reference header src/scalarsort/scalarsort.h:31-51
 * (sdecoder/AVX-sort-merge-joins).  Same file name and include guard, so a
 * reference driver that includes "scalarsort.h" compiles unchanged against
 * libsmj_hip.so (8-byte tuples) or libsmj_hip_k8.so (-DKEY_8B, 16-byte tuples).
 * Provides: scalarsort_tuples, scalarsort_int64, scalarsort_int32.  The declarations live in ../smj.h.
 */
#ifndef SCALARSORT_H
#define SCALARSORT_H
#ifndef SMJ_H
#define SMJ_COMPAT_HIDE_PRINT_TIMING
#endif
#include "../smj.h"
#endif /* SCALARSORT_H */
