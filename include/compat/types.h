/*
 * types.h -- drop-in for the reference header src/types.h:11-98
 * (sdecoder/AVX-sort-merge-joins).  ../smj.h defines these under the
 * reference's own include guard (TYPES_H), so this file and the reference's
 * types.h are interchangeable in one translation unit.
 * Provides: tuple_t, relation_t, result_t, threadresult_t, joinconfig_t (KEY_8B selects 16-byte tuples).
 */
#ifndef SMJ_H
#define SMJ_COMPAT_HIDE_PRINT_TIMING
#endif
#include "../smj.h"
