/*
 * joincommon.h -- drop-in for the hot-path part of the reference header
 * src/joins/joincommon.h:78-80 (sdecoder/AVX-sort-merge-joins): merge_join.
 * The reference's pthread scaffolding (arg_t, sortmergejoin_initrun,
 * print_timing) drives CPU threads and has no counterpart here: the joins in
 * ../smj.h own their device work.
 */
#ifndef JOINCOMMON_H_
#define JOINCOMMON_H_
#include "../smj.h"
#ifdef SMJ_COMPAT_HIDE_PRINT_TIMING
/* joincommon.h:64-66 (smj.h was included first by another compat header) */
void print_timing(uint64_t numtuples, struct timeval * start,
                  struct timeval * end, FILE * out);
#endif
#endif /* JOINCOMMON_H_ */
