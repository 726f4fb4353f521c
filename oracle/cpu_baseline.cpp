// cpu_baseline.cpp -- times the REFERENCE m-way join (compiled from
// /root/reference/src by oracle/build_ref.sh into oracle/_ref/) on the host
// cores, for bench.py's cpu_baseline leg.  Not part of the product.
//
// usage: cpu_baseline NR NS NTHREADS [FANOUT [SKEW]]
// Inputs follow the reference driver (src/main.c:502-583): R = PK keys
// 1..NR with payload 5+i (parallel_create_relation), S = uniform FK over
// 1..NR, or with SKEW > 0 the driver's --skew input, create_relation_zipf
// (main.c:572-575).  Prints one line "SMJ_CPU_BASELINE {json}" on stdout at
// the end.
#include <stdio.h>
#include <stdlib.h>
#include <sys/time.h>
#include <unistd.h>

#include "cpu_mapping.h"
#include "generator.h"
#include "params.h"
#include "numa_shuffle.h"
#include "sortmergejoin_multiway.h"

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s NR NS NTHREADS [FANOUT]\n", argv[0]);
        return 2;
    }
    const int64_t nR = atoll(argv[1]), nS = atoll(argv[2]);
    const int nthr = atoi(argv[3]);
    const int fan = argc > 4 ? atoi(argv[4]) : 128;
    const double skew = argc > 5 ? atof(argv[5]) : 0.0;
    cpu_mapping_init();
    joinconfig_t cfg;
    cfg.NTHREADS = nthr;
    cfg.PARTFANOUT = fan;
#ifdef KEY_8B
    cfg.SCALARSORT = 1;  // the reference forces scalar for 16-byte tuples
    cfg.SCALARMERGE = 1; // (src/main.c:871-877)
#else
    cfg.SCALARSORT = 0;
    cfg.SCALARMERGE = 0;
#endif
    cfg.MWAYMERGEBUFFERSIZE = 20 * 1024 * 1024;
    cfg.NUMASTRATEGY = NEXT;
    numa_shuffle_init(cfg.NUMASTRATEGY, cfg.NTHREADS);
    const size_t pad = RELATION_PADDING(nthr, fan);
    relation_t R, S;
    R.tuples = (tuple_t*)aligned_alloc(64, ((nR * sizeof(tuple_t) + pad + 63) / 64) * 64);
    S.tuples = (tuple_t*)aligned_alloc(64, ((nS * sizeof(tuple_t) + pad + 63) / 64) * 64);
    seed_generator(12345);
    parallel_create_relation(&R, nR, nthr, nR);
    seed_generator(54321);
    if (skew > 0)
        create_relation_zipf(&S, nS, nR, skew);
    else
        parallel_create_relation(&S, nS, nthr, nR);
    struct timeval t0, t1;
    gettimeofday(&t0, NULL);
    result_t* res = sortmergejoin_multiway(&R, &S, &cfg);
    gettimeofday(&t1, NULL);
    const double sec = (t1.tv_sec - t0.tv_sec) + (t1.tv_usec - t0.tv_usec) * 1e-6;
    fflush(stderr);
    printf("\nSMJ_CPU_BASELINE {\"seconds\": %.6f, \"count\": %lld, "
           "\"threads\": %d, \"tuple_bytes\": %d, \"nR\": %lld, \"nS\": %lld}\n",
           sec, res ? (long long)res->totalresults : -1LL, nthr,
           (int)sizeof(tuple_t), (long long)nR, (long long)nS);
    fflush(stdout);
    return 0;
}
