/*
 * params.h -- drop-in for the reference header src/params.h:12-80
 * (sdecoder/AVX-sort-merge-joins).  ../smj.h defines these under the
 * reference's own include guard (PARAMS_H_), so this file and the reference's
 * params.h are interchangeable in one translation unit.
 * Provides: NRADIXBITS_DEFAULT, CACHELINEPADDING, RELATION_PADDING, ALIGN_NUMTUPLES, ....
 */
#ifndef SMJ_H
#define SMJ_COMPAT_HIDE_PRINT_TIMING
#endif
#include "../smj.h"
