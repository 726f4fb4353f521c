/*
 * joincommon.h -- drop-in for the reference header src/joins/joincommon.h
 * (sdecoder/AVX-sort-merge-joins): merge_join (:78-80),
 * merge_join_interpolation (:92-95), sortmergejoin_initrun (:59-61),
 * print_timing (:64-66),
 * is_sorted_helper / check_sorted (:99-103), and the thread scaffolding arg_t / relationpair_t
 * (:105-155), all declared in ../smj.h.  DEBUGMSG keeps the reference's
 * macro (:46-54) for drivers that use it.
 */
#ifndef JOINCOMMON_H_
#define JOINCOMMON_H_
#include "../smj.h"
#ifdef SMJ_COMPAT_HIDE_PRINT_TIMING
/* joincommon.h:64-66 (smj.h was included first by another compat header) */
void print_timing(uint64_t numtuples, struct timeval * start,
                  struct timeval * end, FILE * out);
#endif
#ifndef DEBUGMSG
#ifdef DEBUG
#define DEBUGMSG(COND, MSG, ...)                                         \
    if (COND) {                                                          \
        fprintf(stdout, "[DEBUG @ %s:%d] " MSG, __FILE__, __LINE__,      \
                ##__VA_ARGS__);                                          \
    }
#else
#define DEBUGMSG(COND, MSG, ...)
#endif
#endif
#endif /* JOINCOMMON_H_ */
