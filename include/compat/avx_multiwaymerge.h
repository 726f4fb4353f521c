/*
 * avx_multiwaymerge.h -- drop-in for the reference header src/merge/avx_multiwaymerge.h:33-38
 * (sdecoder/AVX-sort-merge-joins).  Same file name and include guard, so a
 * reference driver that includes "avx_multiwaymerge.h" compiles unchanged against
 * libsmj_hip.so (8-byte tuples) or libsmj_hip_k8.so (-DKEY_8B, 16-byte tuples).
 * Provides: avx_multiway_merge.  The declarations live in ../smj.h.
 */
#ifndef AVXMULTIWAYMERGE_H
#define AVXMULTIWAYMERGE_H
#ifndef SMJ_H
#define SMJ_COMPAT_HIDE_PRINT_TIMING
#endif
#include "../smj.h"
#endif /* AVXMULTIWAYMERGE_H */
