/*
 * scalar_multiwaymerge.h -- drop-in for the reference header src/merge/scalar_multiwaymerge.h:31-78
 * (sdecoder/AVX-sort-merge-joins).  Same file name and include guard, so a
 * reference driver that includes "scalar_multiwaymerge.h" compiles unchanged against
 * libsmj_hip.so (8-byte tuples) or libsmj_hip_k8.so (-DKEY_8B, 16-byte tuples).
 * Provides: scalar_multiway_merge[_modulo|_bitand].  The declarations live in ../smj.h.
 */
#ifndef SCALARMULTIWAYMERGE_H
#define SCALARMULTIWAYMERGE_H
#ifndef SMJ_H
#define SMJ_COMPAT_HIDE_PRINT_TIMING
#endif
#include "../smj.h"
#endif /* SCALARMULTIWAYMERGE_H */
