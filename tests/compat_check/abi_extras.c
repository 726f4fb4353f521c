/*
 * abi_extras.c -- a C caller of three reference-header functions, compiled
 * against include/compat/ and linked with libsmj_hip[_k8].so like the
 * reference's own drivers (tests/test_abi.py builds and links it on the CPU,
 * tests/test_gpu_abi.py runs it on the GPU):
 *
 *   radix_cluster     partition.h:38-43   (partition.c:93-149)
 *   is_sorted_helper  joincommon.h:99-100 (joincommon.c:397-500)
 *   check_sorted      joincommon.h:101-103 (joincommon.c:503-515)
 *
 * The expected values are computed here on the host by the plain loops the
 * reference runs; the program prints "ABI-EXTRAS OK" when every one matches
 * and exits non-zero at the first mismatch.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "types.h"
#include "partition.h"
#include "joincommon.h"

#define FAIL(...)                                   \
    do {                                            \
        fprintf(stderr, "ABI-EXTRAS FAIL: ");       \
        fprintf(stderr, __VA_ARGS__);               \
        fprintf(stderr, "\n");                      \
        exit(1);                                    \
    } while (0)

static uint32_t digit(intkey_t k, int R, int D) {
    uint32_t M = (uint32_t)((((1ull << D) - 1) << R) & 0xffffffffull);
    return (uint32_t)((uint64_t)(k - 1) & M) >> R;
}

/* radix_cluster against the reference's two loops, for a given start hist */
static void check_cluster(const tuple_t* in, uint32_t n, int R, int D, const int32_t* h0) {
    const uint32_t fan = 1u << D;
    int32_t* hist = (int32_t*)malloc(fan * sizeof(int32_t));
    int32_t* want_h = (int32_t*)malloc(fan * sizeof(int32_t));
    uint32_t* dst = (uint32_t*)malloc(fan * sizeof(uint32_t));
    uint64_t extra = 0;
    for (uint32_t i = 0; i < fan; i++) {
        hist[i] = want_h[i] = h0 ? h0[i] : 0;
        extra += (uint64_t)hist[i];
    }
    tuple_t* want = (tuple_t*)calloc(n + extra + 1, sizeof(tuple_t));
    tuple_t* got = (tuple_t*)calloc(n + extra + 1, sizeof(tuple_t));
    for (uint32_t i = 0; i < n; i++) want_h[digit(in[i].key, R, D)]++;
    uint32_t off = 0;
    for (uint32_t i = 0; i < fan; i++) {
        dst[i] = off;
        off += want_h[i];
    }
    for (uint32_t i = 0; i < n; i++) want[dst[digit(in[i].key, R, D)]++] = in[i];

    relation_t rin = {(tuple_t*)in, n}, rout = {got, n};
    radix_cluster(&rout, &rin, hist, R, D);
    for (uint32_t i = 0; i < fan; i++)
        if (hist[i] != want_h[i]) FAIL("radix_cluster R=%d D=%d hist[%u] %d != %d", R, D, i,
                                       hist[i], want_h[i]);
    /* every partition's tuples in input order at the reference's offsets */
    for (uint32_t i = 0; i < fan; i++) {
        const uint32_t end = dst[i], cnt = (uint32_t)(want_h[i] - (h0 ? h0[i] : 0));
        if (cnt && memcmp(got + end - cnt, want + end - cnt, cnt * sizeof(tuple_t)))
            FAIL("radix_cluster R=%d D=%d partition %u differs", R, D, i);
    }
    free(hist);
    free(want_h);
    free(dst);
    free(want);
    free(got);
}

int main(void) {
    const uint32_t n = 100003;
    tuple_t* t = (tuple_t*)malloc(n * sizeof(tuple_t));
    /* keys 1..n in a multiplicative permutation, payload = position */
    for (uint32_t i = 0; i < n; i++) {
        t[i].key = (intkey_t)(((uint64_t)i * 40503u) % n + 1);
        t[i].payload = (value_t)i;
    }
    check_cluster(t, n, 0, 7, NULL);
    check_cluster(t, n, 3, 10, NULL);
    check_cluster(t, n, 9, 4, NULL);
    {
        int32_t h0[16];
        for (int i = 0; i < 16; i++) h0[i] = (i * 7) % 5;  /* a caller hist not zeroed */
        check_cluster(t, n, 2, 4, h0);
    }
    /* is_sorted_helper: keys never decreasing from 0 */
    tuple_t* s = (tuple_t*)malloc(n * sizeof(tuple_t));
    for (uint32_t i = 0; i < n; i++) {
        s[i].key = (intkey_t)(i / 3 + 1);
        s[i].payload = (value_t)i;
    }
    if (is_sorted_helper((int64_t*)s, n) != 1) FAIL("sorted run reported unsorted");
    s[n / 2].key = 0;
    if (is_sorted_helper((int64_t*)s, n) != 0) FAIL("a decrease at %u not found", n / 2);
    s[n / 2].key = s[n / 2 - 1].key;
    if (is_sorted_helper((int64_t*)s, n) != 1) FAIL("an equal key reported unsorted");
    s[0].key = -5; /* below the reference's start key 0 */
    if (is_sorted_helper((int64_t*)s, n) != 0) FAIL("negative first key accepted");
    if (is_sorted_helper((int64_t*)s, 0) != 1) FAIL("empty input reported unsorted");
    s[0].key = 1;
    check_sorted((int64_t*)s, (int64_t*)t, n, n, 3);
    printf("ABI-EXTRAS OK\n");
    free(s);
    free(t);
    return 0;
}
