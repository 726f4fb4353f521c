/*
 * check.h -- a minimal, header-only stand-in for the parts of the Check unit
 * test framework (libcheck 0.9) that the reference's tests/check_*.c use, so
 * those test sources compile unchanged against the MI355X library
 * (oracle/build_dropin.sh).  Test infrastructure only; it runs every test in
 * the calling process (no fork), prints one line per test and reports the
 * number of failures like srunner_ntests_failed().
 */
#ifndef SMJ_COMPAT_CHECK_H
#define SMJ_COMPAT_CHECK_H

#include <setjmp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum print_output { CK_SILENT, CK_MINIMAL, CK_NORMAL, CK_VERBOSE };
enum fork_status { CK_FORK_GETENV, CK_FORK, CK_NOFORK };

typedef void (*ck_test_fn)(void);

typedef struct {
    const char *name;
    ck_test_fn fn;
} ck_test;

typedef struct TCase {
    const char *name;
    ck_test tests[64];
    int n;
} TCase;

typedef struct Suite {
    const char *name;
    TCase *tc[32];
    int n;
} Suite;

typedef struct SRunner {
    Suite *s;
    int failed;
} SRunner;

static jmp_buf ck_jmp;
static int ck_failed_now;

#define START_TEST(name) static void name(void)
#define END_TEST

static inline void ck_fail_at(const char *file, int line, const char *msg) {
    fprintf(stderr, "%s:%d: check failed: %s\n", file, line, msg);
    ck_failed_now = 1;
    longjmp(ck_jmp, 1);
}

#define ck_assert_msg(expr, ...)                                               \
    do {                                                                       \
        if (!(expr)) {                                                         \
            char ck_buf_[512];                                                 \
            snprintf(ck_buf_, sizeof(ck_buf_), __VA_ARGS__);                   \
            ck_fail_at(__FILE__, __LINE__, ck_buf_);                           \
        }                                                                      \
    } while (0)
#define ck_assert(expr) ck_assert_msg(expr, "%s", #expr)
#define ck_assert_int_eq(X, Y)                                                 \
    ck_assert_msg((long long)(X) == (long long)(Y), "%s == %s (%lld != %lld)", \
                  #X, #Y, (long long)(X), (long long)(Y))
#define ck_assert_int_ne(X, Y)                                                 \
    ck_assert_msg((long long)(X) != (long long)(Y), "%s != %s", #X, #Y)
#define fail_unless(expr, ...) ck_assert_msg(expr, __VA_ARGS__)
#define fail_if(expr, ...) ck_assert_msg(!(expr), __VA_ARGS__)

static inline Suite *suite_create(const char *name) {
    Suite *s = (Suite *)calloc(1, sizeof(Suite));
    s->name = name;
    return s;
}
static inline TCase *tcase_create(const char *name) {
    TCase *t = (TCase *)calloc(1, sizeof(TCase));
    t->name = name;
    return t;
}
#define tcase_add_test(tc, fn) tcase_add_test_named((tc), (fn), #fn)
static inline void tcase_add_test_named(TCase *tc, ck_test_fn fn, const char *name) {
    if (tc->n < 64) {
        tc->tests[tc->n].fn = fn;
        tc->tests[tc->n].name = name;
        tc->n++;
    }
}
static inline void tcase_set_timeout(TCase *tc, double t) { (void)tc; (void)t; }
static inline void suite_add_tcase(Suite *s, TCase *tc) {
    if (s->n < 32) s->tc[s->n++] = tc;
}
static inline SRunner *srunner_create(Suite *s) {
    SRunner *r = (SRunner *)calloc(1, sizeof(SRunner));
    r->s = s;
    return r;
}
static inline void srunner_set_fork_status(SRunner *r, enum fork_status f) {
    (void)r; (void)f;
}
static inline void srunner_run_all(SRunner *r, enum print_output p) {
    (void)p;
    int total = 0;
    for (int i = 0; i < r->s->n; i++) {
        TCase *tc = r->s->tc[i];
        for (int j = 0; j < tc->n; j++) {
            ck_failed_now = 0;
            if (setjmp(ck_jmp) == 0) tc->tests[j].fn();
            total++;
            if (ck_failed_now) r->failed++;
            printf("CHECK %s:%s:%s: %s\n", r->s->name, tc->name, tc->tests[j].name,
                   ck_failed_now ? "FAIL" : "PASS");
            fflush(stdout);
        }
    }
    printf("CHECK %s: %d%%: Checks: %d, Failures: %d\n", r->s->name,
           total ? 100 * (total - r->failed) / total : 100, total, r->failed);
}
static inline int srunner_ntests_failed(SRunner *r) { return r->failed; }
static inline void srunner_free(SRunner *r) { free(r); }

#endif /* SMJ_COMPAT_CHECK_H */
