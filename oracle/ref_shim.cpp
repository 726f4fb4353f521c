// ref_shim.cpp -- extern "C" entry points onto the REFERENCE implementation
// compiled from /root/reference/src by oracle/build_ref.sh (test
// infrastructure only: it generates tests/golden/ and times the CPU baseline).
// The reference is C compiled as C++, so its own symbols are C++-mangled;
// these thin wrappers give ctypes a stable C name for each one.
#include <stdlib.h>
#include <string.h>

#include "avx_multiwaymerge.h"
#include "avxsort.h"
#include "avxsort_multiway.h"
#include "cpu_mapping.h"
#include "generator.h"
#include "joincommon.h"
#include "merge.h"
#include "numa_shuffle.h"
#include "partition.h"
#include "scalar_multiwaymerge.h"
#include "scalarsort.h"
#include "sortmergejoin_multiway.h"

extern "C" {

int ref_tuple_bytes(void) { return (int)sizeof(tuple_t); }

void ref_seed(unsigned int s) { seed_generator(s); }

int ref_create_relation_pk(tuple_t* t, int64_t n) {
    relation_t r;
    r.tuples = t;
    r.num_tuples = 0;
    return create_relation_pk(&r, n);
}

int ref_create_relation_nonunique(tuple_t* t, int64_t n, int64_t maxid) {
    relation_t r;
    r.tuples = t;
    r.num_tuples = 0;
    return create_relation_nonunique(&r, n, maxid);
}

int ref_create_relation_fk(tuple_t* t, int64_t n, int64_t maxid) {
    relation_t r;
    r.tuples = t;
    r.num_tuples = 0;
    return create_relation_fk(&r, n, maxid);
}

int ref_create_relation_zipf(tuple_t* t, int64_t n, int64_t maxid,
                             double theta) {
    relation_t r;
    r.tuples = t;
    r.num_tuples = 0;
    return create_relation_zipf(&r, n, maxid, theta);
}

// variant 0: partition_relation, 1: _optimized, 2: _optimized_V2
void ref_partition(tuple_t* in, int64_t n, tuple_t* out, int nbits, int shift,
                   int variant, int64_t* cnt, int64_t* off) {
    const int fan = 1 << nbits;
    relation_t rin, rout;
    rin.tuples = in;
    rin.num_tuples = n;
    rout.tuples = out;
    rout.num_tuples = n;
    relation_t* parts = (relation_t*)malloc(fan * sizeof(relation_t));
    relation_t** pp = (relation_t**)malloc(fan * sizeof(relation_t*));
    for (int i = 0; i < fan; i++) pp[i] = parts + i;
    if (variant == 0)
        partition_relation(pp, &rin, &rout, nbits, shift);
    else if (variant == 1)
        partition_relation_optimized(pp, &rin, &rout, nbits, shift);
    else
        partition_relation_optimized_V2(pp, &rin, &rout, nbits, shift);
    for (int i = 0; i < fan; i++) {
        cnt[i] = (int64_t)pp[i]->num_tuples;
        off[i] = (int64_t)(pp[i]->tuples - out);
    }
    free(pp);
    free(parts);
}

// sorted result copied to `result` (follows the pointer-swap convention)
void ref_avxsort_tuples(tuple_t* in, tuple_t* out, uint64_t n,
                        tuple_t* result) {
    tuple_t* a = in;
    tuple_t* b = out;
    avxsort_tuples(&a, &b, n);
    memcpy(result, b, n * sizeof(tuple_t));
}

void ref_avxsort_int64(int64_t* in, int64_t* out, uint64_t n,
                       int64_t* result) {
    int64_t* a = in;
    int64_t* b = out;
    avxsort_int64(&a, &b, n);
    memcpy(result, b, n * sizeof(int64_t));
}

void ref_avxsortmultiway_tuples(tuple_t* in, tuple_t* out, uint64_t n,
                                tuple_t* result) {
    tuple_t* a = in;
    tuple_t* b = out;
    avxsortmultiway_tuples(&a, &b, n);
    memcpy(result, b, n * sizeof(tuple_t));
}

void ref_scalarsort_tuples(tuple_t* in, tuple_t* out, uint64_t n,
                           tuple_t* result) {
    tuple_t* a = in;
    tuple_t* b = out;
    scalarsort_tuples(&a, &b, n);
    memcpy(result, b, n * sizeof(tuple_t));
}

uint64_t ref_avx_merge_tuples(tuple_t* A, tuple_t* B, tuple_t* out,
                              uint64_t la, uint64_t lb) {
    return avx_merge_tuples(A, B, out, la, lb);
}

uint64_t ref_avx_merge_int64(int64_t* A, int64_t* B, int64_t* out,
                             uint64_t la, uint64_t lb) {
    return avx_merge_int64(A, B, out, la, lb);
}

uint64_t ref_scalar_merge_tuples(tuple_t* A, tuple_t* B, tuple_t* out,
                                 uint64_t la, uint64_t lb) {
    return scalar_merge_tuples(A, B, out, la, lb);
}

// runs are copied (the reference clobbers its inputs)
uint64_t ref_multiway_merge(tuple_t* out, tuple_t* const* runs,
                            const uint64_t* lens, uint32_t k,
                            uint32_t bufbytes, int scalar) {
    relation_t* rels = (relation_t*)malloc(k * sizeof(relation_t));
    relation_t** pp = (relation_t**)malloc(k * sizeof(relation_t*));
    for (uint32_t i = 0; i < k; i++) {
        rels[i].tuples = (tuple_t*)malloc((lens[i] + 64) * sizeof(tuple_t));
        memcpy(rels[i].tuples, runs[i], lens[i] * sizeof(tuple_t));
        rels[i].num_tuples = lens[i];
        pp[i] = rels + i;
    }
    tuple_t* base[4096];
    for (uint32_t i = 0; i < k && i < 4096; i++) base[i] = rels[i].tuples;
    tuple_t* fifo = (tuple_t*)aligned_alloc(64, bufbytes);
    const uint32_t bufn = bufbytes / sizeof(tuple_t);
    uint64_t r = scalar ? scalar_multiway_merge(out, pp, k, fifo, bufn)
                        : avx_multiway_merge(out, pp, k, fifo, bufn);
    free(fifo);
    for (uint32_t i = 0; i < k && i < 4096; i++) free(base[i]);
    free(pp);
    free(rels);
    return r;
}

uint64_t ref_merge_join(tuple_t* R, tuple_t* S, uint64_t nR, uint64_t nS) {
    return merge_join(R, S, nR, nS, NULL);
}

// sortmergejoin_multiway on copies of R and S (the join clobbers inputs);
// returns the match count
int64_t ref_sortmergejoin_multiway(tuple_t* R, uint64_t nR, tuple_t* S,
                                   uint64_t nS, int nthreads, int fanout,
                                   int scalar) {
    static int mapped = 0;
    if (!mapped) {
        cpu_mapping_init();
        mapped = 1;
    }
    joinconfig_t cfg;
    cfg.NTHREADS = nthreads;
    cfg.PARTFANOUT = fanout;
    cfg.SCALARSORT = scalar;
    cfg.SCALARMERGE = scalar;
    cfg.MWAYMERGEBUFFERSIZE = 20 * 1024 * 1024;
    cfg.NUMASTRATEGY = NEXT;
    numa_shuffle_init(cfg.NUMASTRATEGY, cfg.NTHREADS);
    const size_t pad = RELATION_PADDING(nthreads, fanout);
    relation_t r, s;
    r.tuples = (tuple_t*)aligned_alloc(64, ((nR * sizeof(tuple_t) + pad + 63) / 64) * 64);
    s.tuples = (tuple_t*)aligned_alloc(64, ((nS * sizeof(tuple_t) + pad + 63) / 64) * 64);
    memcpy(r.tuples, R, nR * sizeof(tuple_t));
    memcpy(s.tuples, S, nS * sizeof(tuple_t));
    r.num_tuples = nR;
    s.num_tuples = nS;
    result_t* res = sortmergejoin_multiway(&r, &s, &cfg);
    int64_t cnt = res ? res->totalresults : -1;
    if (res) {
        free(res->resultlist);
        free(res);
    }
    free(r.tuples);
    free(s.tuples);
    return cnt;
}

}  // extern "C"
