/*
 * sortmergejoin_multipass.h -- drop-in for the reference header
 * src/joins/sortmergejoin_multipass.h:39-40 (sdecoder/AVX-sort-merge-joins).
 * Same file name and include guard, so a reference driver that includes
 * "sortmergejoin_multipass.h" compiles unchanged against libsmj_hip.so (8-byte
 * tuples) or libsmj_hip_k8.so (-DKEY_8B, 16-byte tuples).
 * Provides: sortmergejoin_multipass.  The declarations live in ../smj.h.
 */
#ifndef SORTMERGEJOIN_MULTIPASS_H_
#define SORTMERGEJOIN_MULTIPASS_H_
#ifndef SMJ_H
#define SMJ_COMPAT_HIDE_PRINT_TIMING
#endif
#include "../smj.h"
#endif /* SORTMERGEJOIN_MULTIPASS_H_ */
