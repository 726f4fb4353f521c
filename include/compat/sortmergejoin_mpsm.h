/*
 * sortmergejoin_mpsm.h -- drop-in for the reference header src/joins/sortmergejoin_mpsm.h:32-33
 * (sdecoder/AVX-sort-merge-joins).  Same file name and include guard, so a
 * reference driver that includes "sortmergejoin_mpsm.h" compiles unchanged against
 * libsmj_hip.so (8-byte tuples) or libsmj_hip_k8.so (-DKEY_8B, 16-byte tuples).
 * Provides: sortmergejoin_mpsm.  The declarations live in ../smj.h.
 */
#ifndef SORTMERGEJOIN_MPSM_H
#define SORTMERGEJOIN_MPSM_H
#ifndef SMJ_H
#define SMJ_COMPAT_HIDE_PRINT_TIMING
#endif
#include "../smj.h"
#endif /* SORTMERGEJOIN_MPSM_H */
