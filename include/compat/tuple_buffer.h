/*
 * tuple_buffer.h -- drop-in for the header the reference includes when built
 * with JOIN_MATERIALIZE (src/joins/joincommon.c:22-24, src/main.c:340-342)
 * but does not ship.  chainedtuplebuffer_t, chainedtuplebuffer_init/_free/
 * _tuples and cb_next_writepos are this library's definitions, declared in
 * ../smj.h together with write_result_relation (main.c:612).
 */
#ifndef SMJ_COMPAT_TUPLE_BUFFER_H
#define SMJ_COMPAT_TUPLE_BUFFER_H
#include "../smj.h"
/* Only a JOIN_MATERIALIZE build includes this header: such a program wants
 * the join entry points to hand back their output, so including it turns the
 * library's materialisation on when the program loads. */
static void __attribute__((constructor, used)) smj_compat_materialize_on(void) {
    smj_set_materialize(1);
}
#endif /* SMJ_COMPAT_TUPLE_BUFFER_H */
