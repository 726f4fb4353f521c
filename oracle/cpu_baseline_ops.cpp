// cpu_baseline_ops.cpp -- times the REFERENCE's single-core partition and sort
// (compiled from /root/reference/src by oracle/build_ref.sh into
// oracle/_ref/) on the host, for bench.py --op partition / --op sort.  Not
// part of the product.
//
// usage: cpu_baseline_ops partition N BITS SHIFT
//        cpu_baseline_ops sort N
//        cpu_baseline_ops merge RUNLEN FANIN  (bench_multiwaymerge: FANIN sorted
//        runs as generate_rand_ordered_tuples makes them, tests/testutil.c:
//        266-287, merged by avx_multiway_merge / scalar_multiway_merge for
//        16-byte tuples, with a 4 MiB FIFO buffer)
// Inputs follow the reference benches: create_relation_pk after
// seed_generator(12345) (src/bench/partitioningbench.c:105-108,
// src/bench/sortbench.c:103-106).  The timed call is
// partition_relation_optimized (partitioningbench.c:165-173, WHATTODO 1) or
// avxsort_tuples (sortbench.c:154; 16-byte tuples: scalarsort_tuples, the
// reference forces the scalar path for KEY_8B, src/main.c:871-877).
// Prints one line "SMJ_CPU_OPS {json}" on stdout.
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

#include "avx_multiwaymerge.h"
#include "avxsort.h"
#include "scalar_multiwaymerge.h"
#include "generator.h"
#include "params.h"
#include "partition.h"
#include "scalarsort.h"
#include "types.h"

static double now() {
    struct timeval t;
    gettimeofday(&t, NULL);
    return t.tv_sec + t.tv_usec * 1e-6;
}

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s partition N BITS SHIFT | sort N\n", argv[0]);
        return 2;
    }
    if (!strcmp(argv[1], "merge")) {
        const int64_t runlen = atoll(argv[2]);
        const int fanin = argc > 3 ? atoi(argv[3]) : 64;
        srand(12345);
        relation_t* runs = (relation_t*)malloc(sizeof(relation_t) * fanin);
        relation_t** ptrs = (relation_t**)malloc(sizeof(relation_t*) * fanin);
        const intkey_t maxint = ~(1 << 31) - 100;
        for (int r = 0; r < fanin; r++) {
            tuple_t* a = (tuple_t*)aligned_alloc(64, ((runlen * sizeof(tuple_t) + 63) / 64) * 64);
            intkey_t k = 1 + rand() % 100;
            for (int64_t j = 0; j < runlen; j++) {
                a[j].key = k;
                a[j].payload = 0;
                if (k < maxint) k += rand() % 100;
            }
            runs[r].tuples = a;
            runs[r].num_tuples = runlen;
            ptrs[r] = &runs[r];
        }
        const int64_t n = runlen * fanin;
        tuple_t* out = (tuple_t*)aligned_alloc(64, ((n * sizeof(tuple_t) + 63) / 64) * 64);
        const uint32_t bufbytes = 4u << 20;
        tuple_t* fifo = (tuple_t*)aligned_alloc(64, bufbytes);
        const double t0 = now();
#ifdef KEY_8B
        const uint64_t m = scalar_multiway_merge(out, ptrs, fanin, fifo, bufbytes / sizeof(tuple_t));
#else
        const uint64_t m = avx_multiway_merge(out, ptrs, fanin, fifo, bufbytes / sizeof(tuple_t));
#endif
        const double sec = now() - t0;
        int ok = m == (uint64_t)n;
        for (int64_t i = 1; i < n && ok; i++) ok = out[i - 1].key <= out[i].key;
        printf("SMJ_CPU_OPS {\"op\": \"merge\", \"seconds\": %.6f, \"n\": %" PRId64
               ", \"tuple_bytes\": %d, \"ok\": %d}\n",
               sec, n, (int)sizeof(tuple_t), ok);
        return 0;
    }
    const int64_t n = atoll(argv[2]);
    relation_t rel;
    rel.tuples = (tuple_t*)aligned_alloc(64, ((n * sizeof(tuple_t) + 63) / 64) * 64);
    seed_generator(12345);
    create_relation_pk(&rel, n);
    double sec = 0;
    int ok = 1;
    if (!strcmp(argv[1], "partition")) {
        const int bits = argc > 3 ? atoi(argv[3]) : 10;
        const int shift = argc > 4 ? atoi(argv[4]) : 0;
        const int fan = 1 << bits;
        relation_t out;
        out.tuples = (tuple_t*)aligned_alloc(64, ((n * sizeof(tuple_t) + fan * 64 + 63) / 64) * 64);
        out.num_tuples = n;
        relation_t** parts = (relation_t**)malloc(sizeof(relation_t*) * fan);
        for (int i = 0; i < fan; i++) parts[i] = (relation_t*)malloc(sizeof(relation_t));
        const double t0 = now();
        partition_relation_optimized(parts, &rel, &out, bits, shift);
        sec = now() - t0;
        uint64_t tot = 0;
        for (int i = 0; i < fan; i++) tot += parts[i]->num_tuples;
        ok = tot == (uint64_t)n;
    } else {
        tuple_t* outbuf = (tuple_t*)aligned_alloc(64, ((n * sizeof(tuple_t) + 63) / 64) * 64);
        tuple_t* in = rel.tuples;
        tuple_t* out = outbuf;
        const double t0 = now();
#ifdef KEY_8B
        scalarsort_tuples(&in, &out, n);
#else
        avxsort_tuples(&in, &out, n);
#endif
        sec = now() - t0;
        for (int64_t i = 1; i < n && ok; i++) ok = out[i - 1].key <= out[i].key;
    }
    printf("SMJ_CPU_OPS {\"op\": \"%s\", \"seconds\": %.6f, \"n\": %" PRId64
           ", \"tuple_bytes\": %d, \"ok\": %d}\n",
           argv[1], sec, n, (int)sizeof(tuple_t), ok);
    return 0;
}
