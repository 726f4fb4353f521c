/*
 * smj.h -- C ABI of the MI355X sort-merge-join library (libsmj_hip*.so).
 *
 * This header is the drop-in boundary for the m-way sort-merge-join hot path of
 * sdecoder/AVX-sort-merge-joins.  Every entry point below keeps the name,
 * argument meaning, pointer-swap conventions and data layout of the reference
 * function it replaces (cited as reference-path:line), so the reference's own
 * drivers (bench_sort, bench_partitioning, bench_multiwaymerge, tputbench,
 * sortmergejoins) and check_* tests compile against include/compat/ and link
 * against this library instead of the AVX objects.
 *
 * Tuple width is a compile-time choice, exactly like the reference
 * (configure --enable-key8B -> -DKEY_8B, src/types.h:23-29):
 *   default : 8-byte tuples  {int32 payload; int32 key}  -> libsmj_hip.so
 *   KEY_8B  : 16-byte tuples {int64 payload; int64 key}  -> libsmj_hip_k8.so
 *
 * Pointers handed to the reference-named functions may be host memory (the
 * library stages them through HBM and writes results back to the same host
 * addresses/layout) or device memory from hipMalloc (work stays in HBM, no
 * copies).  The smj_dev_* functions are the asynchronous device-resident form
 * used by bench.py: device pointers only, explicit HIP stream, no host sync.
 *
 * Order of the sorted output (the parity contract):
 *   8-byte tuples : ascending signed-int64 order of the packed word
 *                   (key << 32 | (uint32)payload) == what the AVX path yields
 *                   for keys in the generators' domain (src/avxsort/avxcommon.h).
 *   16-byte tuples: ascending (key, payload), both signed int64 == the
 *                   reference scalar path (key-only std::sort,
 *                   src/scalarsort/scalarsort.c:41-50) with equal-key runs
 *                   canonicalised by payload.
 *
 * Errors: like the reference (no error codes), a HIP failure prints a message
 * and aborts; the library never falls back to a CPU implementation.
 */
#ifndef SMJ_H
#define SMJ_H

#include <stdint.h>
#include <stddef.h>
#include <stdio.h>
#include <inttypes.h>
#include <sys/time.h>
#include <pthread.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------ */
/* Data ABI (reference src/types.h:22-98). Layout is byte-identical, and the */
/* include guard is the reference's own (TYPES_H), so this header and the    */
/* reference's types.h can both be included in one translation unit.        */
/* ------------------------------------------------------------------------ */
#ifndef TYPES_H
#define TYPES_H
#ifdef KEY_8B
typedef int64_t intkey_t;   /* 16-byte tuples */
typedef int64_t value_t;
#else
typedef int32_t intkey_t;   /* 8-byte tuples (reference default) */
typedef int32_t value_t;
#endif

typedef struct tuple_t        tuple_t;
typedef struct relation_t     relation_t;
typedef struct result_t       result_t;
typedef struct threadresult_t threadresult_t;
typedef struct joinconfig_t   joinconfig_t;

/* payload first, then key: the reference packs an 8-byte tuple into one
 * little-endian word whose high half is the key (src/types.h:51-54). */
struct tuple_t {
    value_t  payload;
    intkey_t key;
};

struct relation_t {
    tuple_t * tuples;
    uint64_t  num_tuples;
};

struct threadresult_t {
    int64_t  nresults;
    void *   results;
    uint32_t threadid;
};

struct result_t {
    int64_t          totalresults;
    threadresult_t * resultlist;
    int              nthreads;
};

enum numa_strategy_t { RANDOM, RING, NEXT };

struct joinconfig_t {
    int NTHREADS;
    int PARTFANOUT;
    int SCALARSORT;
    int SCALARMERGE;
    int MWAYMERGEBUFFERSIZE;
    enum numa_strategy_t NUMASTRATEGY;
};
#endif /* TYPES_H */

/* ------------------------------------------------------------------------ */
/* Compile-time parameters (reference src/params.h:17-72, guard PARAMS_H_).  */
/* ------------------------------------------------------------------------ */
#ifndef PARAMS_H_
#define PARAMS_H_
#ifndef NRADIXBITS_DEFAULT
#define NRADIXBITS_DEFAULT 7
#endif
#ifndef PARTFANOUT_DEFAULT
#define PARTFANOUT_DEFAULT (1 << NRADIXBITS_DEFAULT)
#endif
#ifndef CACHE_LINE_SIZE
#define CACHE_LINE_SIZE 64
#endif
#ifndef L2_CACHE_SIZE
#define L2_CACHE_SIZE (256 * 1024)
#endif
#ifndef L3_CACHE_SIZE
#define L3_CACHE_SIZE (20 * 1024 * 1024)
#endif
/* one cache line of padding per partition (params.h:47) */
#ifndef CACHELINEPADDING
#define CACHELINEPADDING(FANOUT) ((FANOUT) * CACHE_LINE_SIZE / sizeof(tuple_t))
#endif
/* tail padding callers allocate behind R, S and temporaries (params.h:56) */
#ifndef RELATION_PADDING
#define RELATION_PADDING(NTHR, FANOUT) \
    ((NTHR) * CACHELINEPADDING(FANOUT) * sizeof(tuple_t))
#endif
#ifndef MWAY_MERGE_BUFFER_SIZE_DEFAULT
#define MWAY_MERGE_BUFFER_SIZE_DEFAULT L3_CACHE_SIZE
#endif
#define TUPLESPERCACHELINE (CACHE_LINE_SIZE / sizeof(tuple_t))
#define ALIGN_NUMTUPLES(N) \
    (((N) + TUPLESPERCACHELINE - 1) & ~(TUPLESPERCACHELINE - 1))
#endif /* PARAMS_H_ */

/* ------------------------------------------------------------------------ */
/* Radix partitioning (reference src/partition/partition.h:57-120).          */
/* Partition index of a tuple: ((key - 1) & (((1<<nbits)-1) << shift))      */
/*   >> shift (partition.c:29). Output is a stable scatter.                  */
/* ------------------------------------------------------------------------ */

/* partition.c:301-327 -- naive stable layout, partitions back to back. */
void partition_relation(relation_t ** partitions, relation_t * input,
                        relation_t * output, int radixbits, int shiftbits);

/* partition.c:329-354 -- stable scatter, every partition starts on a 64-byte
 * boundary (offsets advance by ALIGN_NUMTUPLES(count)). */
void partition_relation_optimized(relation_t ** partitions, relation_t * input,
                                  relation_t * output, uint32_t nbits,
                                  uint32_t shiftbits);

/* partition.c:356-385 -- same output as the optimized variant. */
void partition_relation_optimized_V2(relation_t ** partitions,
                                     relation_t * input, relation_t * output,
                                     uint32_t nbits, uint32_t shiftbits);

/* partition.c:422-436 -- histogram pass + plain copy (bandwidth probe). */
void histogram_memcpy_bench(relation_t ** partitions, relation_t * input,
                            relation_t * output, uint32_t nbits);

/* partition.h:38-43 (defined partition.c:93-149) -- the naive stable radix
 * cluster on bits [R, R + D) of key - 1 into outRel->tuples, partitions back
 * to back (no padding).  Like the reference it ADDS each partition's count to
 * hist[0 .. 2^D) and starts partition i at the prefix sum of the updated hist,
 * so the caller zeroes hist first for the usual layout. */
void radix_cluster(relation_t * outRel, relation_t * inRel, int32_t * hist,
                   int R, int D);

/* ------------------------------------------------------------------------ */
/* Sorting (reference src/avxsort/avxsort.h:35-57,                           */
/* src/avxsort/avxsort_multiway.h:35-55, src/scalarsort/scalarsort.h).       */
/* Result convention (avxsort.c:117-118,224-225): on return *outputptr       */
/* points at the sorted items, *inputptr at the other buffer; both buffers   */
/* may be clobbered.                                                         */
/* ------------------------------------------------------------------------ */
void avxsort_tuples(tuple_t ** inputptr, tuple_t ** outputptr, uint64_t nitems);
void avxsort_int64(int64_t ** inputptr, int64_t ** outputptr, uint64_t nitems);
/* avxsort.c:247-250 is an empty stub in the reference; here it sorts. */
void avxsort_int32(int32_t ** inputptr, int32_t ** outputptr, uint64_t nitems);
void avxsortmultiway_tuples(tuple_t ** inputptr, tuple_t ** outputptr,
                            uint64_t nitems);
void avxsortmultiway_int64(int64_t ** inputptr, int64_t ** outputptr,
                           uint64_t nitems);
/* scalarsort.c:41-50 sorts in place and swaps the pointers. */
void scalarsort_tuples(tuple_t ** inputptr, tuple_t ** outputptr,
                       uint64_t nitems);
void scalarsort_int64(int64_t ** inputptr, int64_t ** outputptr,
                      uint64_t nitems);
void scalarsort_int32(int32_t ** inputptr, int32_t ** outputptr,
                      uint64_t nitems);

/* The reference's in-register kernel inregister_sort_keyval32
 * (src/avxsort/avxsort_core.h:1213-1274, the compat header
 * include/compat/avxsort_core.h maps that name here), on nblocks consecutive
 * blocks of 16 int64 items: output row j of a block (items 4j..4j+3) is the
 * column {x[j], x[j+4], x[j+8], x[j+12]} after the reference's 4x4 odd-even
 * network of VMINPD/VMAXPD on the items as IEEE doubles, byte-identical to
 * the AVX kernel (NaNs and signed zeros included).  Runs on the device. */
void smj_inregister_sort_keyval32(const int64_t * items, int64_t * output,
                                  uint64_t nblocks);

/* ------------------------------------------------------------------------ */
/* Merging (reference src/merge/merge.h:35-97, avx_multiwaymerge.h:33-38,    */
/* scalar_multiwaymerge.h:31-78). Return value = tuples written.             */
/* ------------------------------------------------------------------------ */
uint64_t avx_merge_tuples(tuple_t * const inA, tuple_t * const inB,
                          tuple_t * const outp, const uint64_t lenA,
                          const uint64_t lenB);
uint64_t avx_merge_int64(int64_t * const inA, int64_t * const inB,
                         int64_t * const outp, const uint64_t lenA,
                         const uint64_t lenB);
uint64_t scalar_merge_tuples(tuple_t * const inA, tuple_t * const inB,
                             tuple_t * const outp, const uint64_t lenA,
                             const uint64_t lenB);
uint64_t scalar_merge_int64(int64_t * const inA, int64_t * const inB,
                            int64_t * const outp, const uint64_t lenA,
                            const uint64_t lenB);

/* avx_multiwaymerge.c:199-338. `fifobuffer`/`bufntuples` are accepted for
 * ABI compatibility; the GPU merge stages run heads in LDS instead of an
 * L3-resident FIFO tree. On return every parts[i] has been consumed:
 * parts[i]->tuples advanced by its count and parts[i]->num_tuples == 0,
 * as the reference leaves them (avx_multiwaymerge.c:268-272). */
uint64_t avx_multiway_merge(tuple_t * output, relation_t ** parts,
                            uint32_t nparts, tuple_t * fifobuffer,
                            uint32_t bufntuples);
uint64_t scalar_multiway_merge(tuple_t * output, relation_t ** parts,
                               uint32_t nparts, tuple_t * fifobuffer,
                               uint32_t bufntuples);
uint64_t scalar_multiway_merge_modulo(tuple_t * output, relation_t ** parts,
                                      uint32_t nparts, tuple_t * fifobuffer,
                                      uint32_t bufntuples);
uint64_t scalar_multiway_merge_bitand(tuple_t * output, relation_t ** parts,
                                      uint32_t nparts, tuple_t * fifobuffer,
                                      uint32_t bufntuples);

/* ------------------------------------------------------------------------ */
/* Joins (reference src/joins/joincommon.h:78-80,                            */
/* src/joins/sortmergejoin_multiway.h:37-38, sortmergejoin_mpsm.h).          */
/* ------------------------------------------------------------------------ */

/* Materialised join output (the reference's JOIN_MATERIALIZE build,
 * joincommon.c:256-289, sortmergejoin_multiway.c:565-598, main.c:609-626).
 * The reference takes chainedtuplebuffer_t and its functions from
 * tuple_buffer.h, which is not in its tree, so this is the library's own
 * definition of that interface: one growable host array holding one
 * <S.key, S.payload> tuple per match, in merge_join's R-major order (per key,
 * the S run repeated |R_k| times, keys ascending).  A pointer returned by
 * cb_next_writepos stays valid until the next write. */
#ifndef SMJ_TUPLE_BUFFER
#define SMJ_TUPLE_BUFFER
typedef struct chainedtuplebuffer_t {
    tuple_t * tuples;
    uint64_t  numtuples;
    uint64_t  capacity;
} chainedtuplebuffer_t;
chainedtuplebuffer_t * chainedtuplebuffer_init(void);
/* NULL is a no-op (main.c:621-626 frees every thread's list) */
void chainedtuplebuffer_free(chainedtuplebuffer_t * cb);
uint64_t chainedtuplebuffer_tuples(chainedtuplebuffer_t * cb);
tuple_t * cb_next_writepos(chainedtuplebuffer_t * cb);
#endif /* SMJ_TUPLE_BUFFER */

/* joincommon.c:239-312: number of (r, s) pairs with equal key between two
 * sorted runs, duplicates on both sides included.  A non-NULL `output` is a
 * chainedtuplebuffer_t that receives the matches appended (JOIN_MATERIALIZE);
 * they are produced on the device (smj_dev_materialize) and copied back. */
uint64_t merge_join(tuple_t * rtuples, tuple_t * stuples, const uint64_t numR,
                    const uint64_t numS, void * output);

/* Materialisation switch of the join entry points (the reference decides it
 * at compile time with -DJOIN_MATERIALIZE; the library cannot see the
 * caller's flags): on, sortmergejoin_multiway / _multipass / _mpsm hand the
 * whole output in result->resultlist[0].results as a chainedtuplebuffer_t
 * (the other threads' lists stay NULL; m-pass fills one list per thread, as
 * its threads own disjoint partitions).  Default: the environment variable
 * SMJ_MATERIALIZE (unset = off).  The switch is process-wide, like the
 * compile-time flag it stands for: every reference-named join in the
 * process sees the last value set (an atomic).  Callers that need a mode per
 * call use smj_join below instead. */
void smj_set_materialize(int on);

/* The reference's three join algorithms with the materialisation chosen per
 * call (library extension; the reference fixes it per build): algo 0 =
 * sortmergejoin_multiway, 1 = sortmergejoin_multipass, 2 =
 * sortmergejoin_mpsm; materialize 1 / 0 overrides the process switch for this
 * call only, -1 follows it.  Returns what the named function returns (NULL
 * for an unknown algo). */
result_t * smj_join(relation_t * relR, relation_t * relS, joinconfig_t * joincfg,
                    int algo, int materialize);

/* main.c:609-614 (PERSIST_RELATIONS + JOIN_MATERIALIZE): append the
 * materialised result to `filename` in the text format of write_relation
 * (src/datagen/generator.c:200-213): a "#KEY, VAL" line, then "key payload"
 * per tuple, both printed with %d as the reference does (for 16-byte tuples
 * that is the low 32 bits of each field, what its int64 arguments print as
 * on x86-64).  The reference calls this function but never defines it. */
void write_result_relation(result_t * result, const char * filename);

/* joincommon.c:214-227: the drivers' timing line ("NUM-TUPLES = ...
 * TOTAL-TIME-USECS = ... TUPLES-PER-SECOND = ..."), host-side.  Declared in
 * the reference only by joincommon.h (some drivers define their own
 * print_timing), so the compat headers other than joincommon.h hide it. */
#ifndef SMJ_COMPAT_HIDE_PRINT_TIMING
void print_timing(uint64_t numtuples, struct timeval * start,
                  struct timeval * end, FILE * out);
#endif

/* joincommon.h:99-100 (defined joincommon.c:397-500): 1 when the keys of
 * the `nitems` tuples at `items` (a tuple_t array passed as int64_t*) never
 * decrease, starting from key 0, else 0.  Without KEY_8B it prints the
 * reference's "[WARN ] Equal items" line at the first repeated key before any
 * decrease and its "[ERROR]" line at the first decrease; with KEY_8B it
 * prints nothing.  The scan runs on the device. */
int is_sorted_helper(int64_t * items, uint64_t nitems);

/* joincommon.h:101-103 (defined joincommon.c:503-515): prints whether R and
 * S are sorted ("%d-thread -> R is sorted, size = %d"). */
void check_sorted(int64_t * R, int64_t * S, uint64_t nR, uint64_t nS, int my_tid);

/* joincommon.c (not in joincommon.h's prose): merge_join with an
 * interpolation search for the start; same count as merge_join. */
uint64_t merge_join_interpolation(tuple_t * rtuples, tuple_t * stuples,
                                  const uint64_t numR, const uint64_t numS,
                                  void * output);

/* The thread scaffolding of the reference joins (joincommon.h:40-44,
 * 105-155), layout-identical so that drivers with their own join thread
 * (tputbench.c:124-144) run unchanged on sortmergejoin_initrun below. */
#ifndef SMJ_ARG_T
#define SMJ_ARG_T
typedef struct arg_t arg_t;
typedef struct relationpair_t relationpair_t;
struct arg_t {
    tuple_t *  relR;
    tuple_t *  relS;
    tuple_t *  tmp_partR;   /* partitioning output, per thread */
    tuple_t *  tmp_partS;
    tuple_t *  tmp_sortR;   /* sorting output, per thread */
    tuple_t *  tmp_sortS;
    int32_t numR;
    int32_t numS;
    int32_t my_tid;
    int     nthreads;
    joinconfig_t * joincfg;
    pthread_barrier_t * barrier;
    int64_t result;
    relationpair_t ** threadrelchunks;
    tuple_t ** sharedmergebuffer;
    uint32_t ** histR;      /* mpsm-specific */
    tuple_t * tmpRglobal;
    uint64_t totalR;
#ifdef JOIN_MATERIALIZE
    threadresult_t * threadresult;
#endif
    struct timeval start, end;
    uint64_t part, sort, mergedelta, merge, join;
} __attribute__((aligned(CACHE_LINE_SIZE)));
struct relationpair_t {
    relation_t R;
    relation_t S;
};
#endif /* SMJ_ARG_T */

/* joincommon.c:29-212: allocates the per-thread temporaries (partition and
 * sort outputs, RELATION_PADDING behind each), slices R and S into T
 * contiguous chunks, runs `jointhread` on T pthreads sharing one barrier,
 * sums args[i].result into a malloc'd result_t and prints the stats lines
 * from args[0]'s timers.  The join thread's own calls (partition, sort,
 * merge, merge_join) are this library's device entry points.  Host-side
 * orchestration only: no tuple is touched here. */
result_t * sortmergejoin_initrun(relation_t * relR, relation_t * relS,
                                 joinconfig_t * joincfg,
                                 void * (*jointhread)(void *));

/* sortmergejoin_multiway.c:50-61: m-way sort-merge join. Returns a malloc'd
 * result_t (caller frees resultlist and the struct, main.c:629-632) whose
 * totalresults is the match count; NULL for a non-power-of-2 NTHREADS as the
 * reference does. NTHREADS only selects the reference-visible partition
 * fan-out checks: the whole join runs on the current HIP device. */
result_t * sortmergejoin_multiway(relation_t * relR, relation_t * relS,
                                  joinconfig_t * joincfg);

/* sortmergejoin_multipass.c:51-736 (m-pass): sort R and S completely, then
 * one merge-join scan; same result contract as sortmergejoin_multiway. */
result_t * sortmergejoin_multipass(relation_t * relR, relation_t * relS,
                                   joinconfig_t * joincfg);

/* sortmergejoin_mpsm.c:38-45 is a stub that exits in the reference; SURVEY.md
 * §2 row 9 and BASELINE configs[4] make it the multi-GPU join, and here it is
 * that: G = min(NTHREADS, visible GPUs) ranks in this process, one host thread
 * and one GPU each (the reference's T threads, joincommon.c:118-165, on
 * contiguous chunks of R and S, :127-139).  Every rank range-partitions its
 * chunks on its GPU, the partitions go to their owner GPUs over RCCL (grouped
 * ncclSend/ncclRecv, peers in NEXT order, numa_shuffle.c:83; the co-partition
 * exchange of sortmergejoin_multiway.c:463-556), each GPU sorts and joins the
 * contiguous key range it owns, and the counts are all-reduced
 * (ncclAllReduce).  totalresults = the global count; resultlist[g].nresults
 * = rank g's; with materialisation resultlist[g].results holds rank g's
 * matches (ranks in key order).  Keys are planned as 1..|R| like the m-way
 * join and verified (a key outside -> the measured range). */
result_t * sortmergejoin_mpsm(relation_t * relR, relation_t * relS,
                              joinconfig_t * joincfg);

/* The multi-GPU join of sortmergejoin_mpsm with its outputs (library
 * extension).  nranks ranks (0 = one per visible GPU); R and S in host memory
 * or in device memory any rank's GPU can read; rank g takes the g-th chunk of
 * each (the last one the rest).  key_min <= key_max: the key range (keys
 * outside it are legal but unbalance the ranks); otherwise 1..nR, verified.
 * sortedR / sortedS (optional, nR / nS tuples, host or device): the sorted
 * relations, the ranks' shares concatenated in rank order -- each rank owns
 * one contiguous key range, so this is the globally sorted relation.
 * rank_counts (optional, 2 * nranks): the tuples of R and of S each rank
 * sorted.  Returns the number of matching pairs.  Device inputs are read on
 * the ranks' own streams with no ordering against any caller stream: the
 * caller finishes every write to R and S before the call. */
#define SMJ_MG_COPY     1u  /* collectives by device copies instead of RCCL:
                               ranks may share a GPU (rank g on device g mod
                               the visible count); every exchange synchronises */
#define SMJ_MG_NOPLANES 2u  /* no 48-bit planes: 64-bit words or tuples */
#define SMJ_MG_ONECALL  4u  /* the local join in one call (not staged) */
#define SMJ_MG_SAMPLED  8u  /* sampled exchange partitions (default: one rank) */
#define SMJ_MG_EXACT   16u  /* exact exchange partitions (default: > 1 rank) */
typedef struct smj_mgpu_stats {
    int      layout;      /* of the exchange: 0 tuples, 1 64-bit words, 2 48-bit planes */
    uint32_t pbits;       /* exchange partitions = 2^pbits */
    int      attempts;    /* exchange attempts of rank 0 (2 = none repeated) */
    int      replans;     /* the guessed key range replaced by the measured one */
    uint64_t sent_bytes;  /* rows rank 0 sent to other ranks */
    uint64_t recv_bytes;  /* ... and received */
    int64_t  key_min;     /* the global plan's range */
    int64_t  key_max;
    double   ms;          /* host wall time of the call */
    /* device phases of the call on the rank's streams (HIP events), ms.  The
     * first five are consecutive on the rank's main stream and add up to
     * busy_ms: the range partitions of R and S (every attempt); their table
     * messages (k_xsend, the table exchange, k_xrecv, the summary copy); the
     * main stream waiting (host decisions and the row exchange the local work
     * did not hide); the local join (tile pass, group pass and count, both
     * stages); the count's all-reduce.  rows_ms: the row exchange on the
     * rank's row stream, which overlaps them. */
    double   partition_ms;
    double   tables_ms;
    double   wait_ms;
    double   join_ms;
    double   reduce_ms;
    double   busy_ms;
    double   rows_ms;
} smj_mgpu_stats;
int64_t smj_mgpu_join(const tuple_t * R, uint64_t nR, const tuple_t * S, uint64_t nS,
                      int nranks, uint32_t flags, int64_t key_min, int64_t key_max,
                      tuple_t * sortedR, tuple_t * sortedS, uint64_t * rank_counts,
                      smj_mgpu_stats * stats);
/* The multi-GPU join over ranks whose slices already lie on their GPUs (the
 * layout of a relation sharded over the node's HBM): rank g reads R[g]
 * (nR[g] tuples) and S[g] (nS[g]), host memory or device memory of GPU g, and
 * runs on GPU g (SMJ_MG_COPY: g mod the visible count).  Otherwise as
 * smj_mgpu_join; the sorted shares stay on the ranks' GPUs
 * (smj_mgpu_last_sorted).  key_min <= key_max: the global key range;
 * otherwise keys 1..sum(nR), verified. */
int64_t smj_mgpu_join_slices(const tuple_t * const * R, const uint64_t * nR,
                             const tuple_t * const * S, const uint64_t * nS, int nranks,
                             uint32_t flags, int64_t key_min, int64_t key_max,
                             uint64_t * rank_counts, smj_mgpu_stats * stats);
/* Rank `rank`'s statistics of the last smj_mgpu_join / _slices call (its
 * phases; `ms` is the call's host time).  Returns 0, or -1 when there is no
 * such rank. */
int smj_mgpu_last_stats(int rank, smj_mgpu_stats * out);
/* Device pointers to rank `rank`'s sorted shares of the last smj_mgpu_join /
 * _slices call (on the rank's GPU, valid until the next call) and their
 * sizes.  Returns 0, or -1 when there is no such rank. */
int smj_mgpu_last_sorted(int rank, tuple_t ** sortedR, uint64_t * nR, tuple_t ** sortedS,
                         uint64_t * nS);
/* Rank `rank`'s workspace in the in-process group of the last smj_mgpu_join
 * / _slices call (its kernel trace: smj_trace_*), NULL when there is none. */
struct smj_workspace * smj_mgpu_group_workspace(int rank);
/* Frees the ranks' devices buffers, streams and communicators (kept across
 * calls of one configuration). */
void smj_mgpu_release(void);

/* The same join with one rank per PROCESS (one process per GPU, e.g. under
 * torch.distributed.run): rank 0 gets an id (smj_mgpu_unique_id: writes up to
 * `cap` bytes, returns their count, 128), every process passes it to
 * smj_mgpu_comm_init on its current device, then every rank calls
 * smj_mgpu_rank_join with its own slices of R and S (host, or device memory
 * of its GPU).  key_min <= key_max: the global key range, the same on every
 * rank; otherwise keys 1..guess_max (the global |R|), verified.  *sortedR /
 * *sortedS receive device pointers to the rank's sorted share (*nR_out /
 * *nS_out tuples, one contiguous key range, ranks in order), valid until the
 * next call on the communicator.  Returns the global match count on every
 * rank.  flags: SMJ_MG_NOPLANES / _ONECALL / _SAMPLED / _EXACT. */
typedef struct smj_mgpu_comm smj_mgpu_comm;
int smj_mgpu_unique_id(void * out, int cap);
smj_mgpu_comm * smj_mgpu_comm_init(const void * id, int nranks, int rank);
int64_t smj_mgpu_rank_join(smj_mgpu_comm * comm, const tuple_t * R, uint64_t nR,
                           const tuple_t * S, uint64_t nS, uint32_t flags,
                           int64_t key_min, int64_t key_max, uint64_t guess_max,
                           tuple_t ** sortedR, uint64_t * nR_out, tuple_t ** sortedS,
                           uint64_t * nS_out, smj_mgpu_stats * stats);
/* copies the rank's sorted shares of the last smj_mgpu_rank_join (host or
 * device destinations; NULL skips one) */
void smj_mgpu_rank_sorted(smj_mgpu_comm * comm, tuple_t * outR, tuple_t * outS);
/* the rank's workspace (its kernel trace: smj_trace_*) */
struct smj_workspace * smj_mgpu_comm_workspace(smj_mgpu_comm * comm);
void smj_mgpu_comm_destroy(smj_mgpu_comm * comm);

/* ------------------------------------------------------------------------ */
/* Device-resident asynchronous API (no reference counterpart: this is the   */
/* form a GPU-aware caller binds).  All pointers are device pointers,        */
/* `stream` is a hipStream_t (NULL = default stream).                        */
/* ------------------------------------------------------------------------ */
typedef void * smj_stream_t;

/* Tuple width this library was built for (8 or 16). */
int smj_tuple_bytes(void);
/* Name of the device the library initialised, for logs. */
const char * smj_device_name(void);

/* Opaque reusable scratch (device memory).  One per stream/thread: calls on
 * one workspace must be ordered on one stream (they share its scratch and
 * the group pass's argument slot). */
typedef struct smj_workspace smj_workspace;
smj_workspace * smj_workspace_create(void);
void smj_workspace_destroy(smj_workspace * ws);

/* Layouts the sorts and joins on `ws` may not use (NULL: the calling thread's
 * workspace behind the reference-named entry points).  Default 0: every
 * layout allowed, each taken where it applies; the results
 * are the same whichever layout runs.  For A/B measurements and tests. */
#define SMJ_LAYOUT_NO_P48      1u  /* no 48-bit words in two planes */
#define SMJ_LAYOUT_NO_PACKED   2u  /* no 64-bit packed words (16-byte tuples) */
#define SMJ_LAYOUT_NO_SAMPLED  4u  /* exact histogram + scatter level-1 partition */
#define SMJ_LAYOUT_SAMPLE_PLAN 8u  /* without a key-range hint: plan from a device
                                      sample instead of from the relation size */
#define SMJ_LAYOUT_NO_P32     16u  /* no 32-bit words (tiny payloads) */
#define SMJ_LAYOUT_NO_P96     32u  /* no 12-byte elements (payloads no packed word
                                      holds: 16-byte tuples instead) */
void smj_workspace_set_layouts(smj_workspace * ws, uint32_t off);
/* The intermediate layout the last device sort or join on `ws` (NULL: the
 * calling thread's workspace) finished in: tuples, 64-bit packed words,
 * 48-bit words in two planes, 32-bit words, 12-byte elements (the full
 * payload and a 32-bit key offset, in two planes); -1 before the first
 * call. */
#define SMJ_LAYOUT_USED_TUPLES 0
#define SMJ_LAYOUT_USED_WORDS  1
#define SMJ_LAYOUT_USED_P48    2
#define SMJ_LAYOUT_USED_P32    3
#define SMJ_LAYOUT_USED_P96    4
int smj_workspace_last_layout(smj_workspace * ws);

/* Stable radix partition, the device form of partition_relation*.
 * padded != 0 -> partition_relation_optimized layout.
 * hist_out / off_out (device, int64[1<<nbits]) receive per-partition counts
 * and start offsets in tuples. */
void smj_dev_partition(smj_workspace * ws, const tuple_t * in, uint64_t n,
                       tuple_t * out, uint32_t nbits, uint32_t shiftbits,
                       int padded, int64_t * hist_out, int64_t * off_out,
                       smj_stream_t stream);

/* Full sort of n tuples into `out` (may equal `in`). */
void smj_dev_sort(smj_workspace * ws, const tuple_t * in, uint64_t n,
                  tuple_t * out, smj_stream_t stream);

/* Merge two sorted runs. */
void smj_dev_merge2(const tuple_t * a, uint64_t na, const tuple_t * b,
                    uint64_t nb, tuple_t * out, smj_stream_t stream);

/* k-way merge of sorted device runs whose pointers/lengths are host arrays.
 * Stream-ordered: for 3..256 runs no host synchronisation (round 5; the
 * host arrays may be reused as soon as the call returns). */
void smj_dev_multiway_merge_host(smj_workspace * ws,
                                 const tuple_t * const * runs,
                                 const uint64_t * lens, uint32_t k,
                                 tuple_t * out, smj_stream_t stream);

/* Merge-join count of two sorted runs; result is ADDED to *count_dev. */
void smj_dev_merge_join_count(const tuple_t * r, uint64_t nr,
                              const tuple_t * s, uint64_t ns,
                              unsigned long long * count_dev,
                              smj_stream_t stream);

/* Materialised merge join of two sorted relations: the output of
 * merge_join built with JOIN_MATERIALIZE (src/joins/joincommon.c:256-289),
 * one <S.key, S.payload> tuple per match, R-major -- per key, the S run
 * repeated |R_k| times, keys ascending -- as one flat array (the reference's
 * chained buffer, tuple_buffer.h, is not in its tree).  Writes the first
 * min(total, out_cap) tuples to `out` (device) and returns the total number
 * of matches; out_cap = 0 only counts.  Synchronises `stream` once. */
uint64_t smj_dev_materialize(smj_workspace * ws, const tuple_t * sortedR,
                             uint64_t nR, const tuple_t * sortedS, uint64_t nS,
                             tuple_t * out, uint64_t out_cap, smj_stream_t stream);

/* The m-way join on one device.  R and S are left untouched; sortedR/sortedS
 * (n tuples each) receive the fully sorted relations; the match count is
 * written to *count_dev.  key_min <= key_max is an optional hint of the key
 * range (pass key_min > key_max to sample it on the device).  Asynchronous
 * except for one stream synchronisation that checks for skewed sub-buckets. */
void smj_dev_join(smj_workspace * ws, const tuple_t * R, uint64_t nR,
                  const tuple_t * S, uint64_t nS, tuple_t * sortedR,
                  tuple_t * sortedS, uint32_t fanout_bits, int64_t key_min,
                  int64_t key_max, unsigned long long * count_dev,
                  smj_stream_t stream);

/* Phase timings (ms) of the last smj_dev_join on this workspace, from HIP
 * events: [0]=partition [1]=tile pass [2]=bucket sort+join [3]=skew path
 * [4]=total. */
void smj_join_phase_ms(smj_workspace * ws, float * ms5);

/* Deterministic synthetic relations generated in HBM.
 * pk  : keys 1..total, each once (keyed bijection of the global index),
 *       payload 5 + global index (or 0 when with_payload == 0, as
 *       create_relation_pk leaves it);
 * fk  : keys perm(i) % maxid + 1 (uniform, |S| == maxid -> a permutation);
 * zipf: keys Zipf(theta) over 1..maxid, hot ranks spread by a bijection,
 *       payload 0.  `first` = global index of this shard's first tuple. */
void smj_dev_gen_pk(tuple_t * out, uint64_t n, uint64_t first, uint64_t total,
                    uint64_t seed, int with_payload, smj_stream_t stream);
void smj_dev_gen_fk(tuple_t * out, uint64_t n, uint64_t first, uint64_t total,
                    uint64_t maxid, uint64_t seed, smj_stream_t stream);
void smj_dev_gen_zipf(smj_workspace * ws, tuple_t * out, uint64_t n,
                      uint64_t first, uint64_t maxid, double theta,
                      uint64_t seed, smj_stream_t stream);

/* The reference's own rand()-driven generators, bit-exact (refgen.hip): the
 * relation create_relation_nonunique / create_relation_zipf would produce
 * after srand(seed) and `skip` earlier rand() calls (generator.c:220-231,
 * 490-505; genzipf.c:28-159, generator.c:517-534), shard [first, first + n) of
 * a relation of `total` tuples.  glibc rand()'s additive stream is jumped
 * ahead per shard (31 x 31 matrix powers); the Zipf alphabet and CDF table are
 * built on the host in the reference's order and cached per workspace.
 * nonunique: key = RAND_RANGE(maxid), payload = total - index, avoid_NaN;
 * zipf_ref : key = alphabet[CDF^-1(rand() / RAND_MAX)], payload 0
 *            (maxid < 2^32). */
void smj_dev_gen_nonunique(smj_workspace * ws, tuple_t * out, uint64_t n, uint64_t first,
                           uint64_t total, int64_t maxid, uint32_t seed, uint64_t skip,
                           smj_stream_t stream);
void smj_dev_gen_zipf_ref(smj_workspace * ws, tuple_t * out, uint64_t n, uint64_t first,
                          uint64_t maxid, double theta, uint32_t seed, uint64_t skip,
                          smj_stream_t stream);
/* The k-th rand() value after srand(seed) (k = 0 is the first call), by the
 * same jump-ahead, on the host (no device needed). */
uint32_t smj_glibc_rand(uint32_t seed, uint64_t k);

void smj_dev_synchronize(smj_stream_t stream);

/* Multi-GPU building block: stable partition of a device relation into
 * 2^nbits key ranges of [key_min, key_max] (monotone digits, unpadded), so a
 * caller can hand contiguous partition ranges to their owner GPU with one
 * all-to-all (bench.py does this over RCCL).  hist_out: device int64[2^nbits]. */
void smj_dev_partition_range(smj_workspace * ws, const tuple_t * in, uint64_t n,
                             tuple_t * out, uint32_t nbits, int64_t key_min,
                             int64_t key_max, int64_t * hist_out,
                             smj_stream_t stream);

/* Range partition of smj_dev_partition_range writing one 64-bit word per
 * tuple instead of the tuple (16-byte tuples only): word = (key offset inside
 * its partition, the low s1 bits) << (64 - s1) | payload, where partitions
 * cover 2^s1 keys.  Halves the bytes of the multi-GPU exchange.  Returns 0
 * (and launches nothing) when the layout does not apply -- the 8-byte
 * library, or partitions wider than 2^32 keys; otherwise 1, and *bad_flag is
 * OR-ed with 1 when some tuple cannot be packed (key outside [key_min,
 * key_max], payload outside [0, 2^(64 - s1))): the caller then partitions
 * the tuples instead. */
int smj_dev_partition_range_packed(smj_workspace * ws, const tuple_t * in, uint64_t n,
                                   uint64_t * out, uint32_t nbits, int64_t key_min,
                                   int64_t key_max, int64_t * hist_out,
                                   unsigned int * bad_flag, smj_stream_t stream);

/* Local join of one GPU's share after the exchange (multi-GPU join, no
 * reference counterpart: it replaces the per-thread multiway merge of the
 * reference's T>1 path, src/joins/sortmergejoin_multiway.c:463-556).  R and
 * S are the receive buffers: for every source GPU s in order, its range
 * partitions 0..2^bucket_bits-1 back to back, seg[s * 2^bucket_bits + b]
 * elements each (device int64).  Every partition b covers the keys
 * [key_lo + b * w, key_lo + (b + 1) * w) with 2^bucket_bits * w = 2^L, L the
 * bit length of key_hi - key_lo (any key_hi in [key_lo + 2^(L-1),
 * key_lo + 2^L - 1] gives the same plan), so the partitions are the level-1
 * buckets of the local sort: no local partition pass.  The elements are
 * tuples, or (flags & SMJ_SEG_PACKED) the words of
 * smj_dev_partition_range_packed for the same w.  R and S are used as
 * scratch (overwritten).  sortedR/sortedS receive the sorted relations as
 * tuples, count_dev the number of matching pairs. */
#define SMJ_SEG_PACKED 1u
/* Stages of one local join split over two calls with the same arguments
 * (the multi-GPU join overlaps them with the row exchange): a call with
 * SMJ_SEG_STAGE_R sorts only R's tiles (its tile pass: R must be complete,
 * S need not have arrived); the next call with SMJ_SEG_STAGE_REST sorts S's
 * tiles and runs the group pass and the count.  Neither flag: the whole join
 * in one call. */
#define SMJ_SEG_STAGE_R 2u
#define SMJ_SEG_STAGE_REST 4u
void smj_dev_join_segmented(smj_workspace * ws, void * R, uint64_t nR,
                            const int64_t * segR, void * S, uint64_t nS,
                            const int64_t * segS, uint32_t nseg,
                            uint32_t bucket_bits, int64_t key_lo, int64_t key_hi,
                            uint32_t flags, tuple_t * sortedR, tuple_t * sortedS,
                            unsigned long long * count_dev, smj_stream_t stream);

/* The local join of smj_dev_join_segmented from explicit segment tables:
 * bucket b (b < 2^bucket_bits) is the nseg segments startX/cntX[b * nseg + j]
 * (device int64, element offsets into X and element counts), so a receive
 * buffer may hold unused gaps between segments (the sampled exchange below).
 * nR / nS count the elements inside the segments. */
void smj_dev_join_segmented_tables(smj_workspace * ws, void * R, uint64_t nR,
                                   const int64_t * startR, const int64_t * cntR,
                                   void * S, uint64_t nS, const int64_t * startS,
                                   const int64_t * cntS, uint32_t nseg,
                                   uint32_t bucket_bits, int64_t key_lo, int64_t key_hi,
                                   uint32_t flags, tuple_t * sortedR, tuple_t * sortedS,
                                   unsigned long long * count_dev, smj_stream_t stream);

/* smj_dev_join_segmented_tables on 48-bit words in two planes (the layout
 * smj_dev_partition_range_planes writes): X's element i is
 * lo[i] | hi[i] << 32 with lo = (uint32_t *)X and hi = (uint16_t *)(lo +
 * strideX); strideX a multiple of 32 elements.  flags: the stage bits only.
 * Both tuple widths. */
void smj_dev_join_segmented_planes(smj_workspace * ws, void * R, uint64_t strideR,
                                   uint64_t nR, const int64_t * startR,
                                   const int64_t * cntR, void * S, uint64_t strideS,
                                   uint64_t nS, const int64_t * startS,
                                   const int64_t * cntS, uint32_t nseg,
                                   uint32_t bucket_bits, int64_t key_lo, int64_t key_hi,
                                   uint32_t flags, tuple_t * sortedR, tuple_t * sortedS,
                                   unsigned long long * count_dev, smj_stream_t stream);

/* Range partition of smj_dev_partition_range by the 1-GPU join's sampled
 * scatter (no histogram pass; packed words when `packed`).  Partition p is
 * smj_sampled_shards() consecutive regions, p's before p + 1's; region
 * i = p * shards + q holds seg_cnt[i] elements from element offset
 * seg_start[i] of `out` and is followed by unused slack, so `out` must hold
 * smj_sampled_capacity(n, nbits) elements (tuples, or 8-byte words).
 * flags (device uint32[2], zeroed here): [0] = 1 when a region overflowed
 * (the output is incomplete: use the exact partition), [1] = 1 when packed
 * and some tuple did not pack.  Returns 0 (nothing launched) when the form
 * does not apply: nbits > 10, n >= 2^32, or packed words unusable. */
int smj_dev_partition_range_sampled(smj_workspace * ws, const tuple_t * in, uint64_t n,
                                    void * out, uint32_t nbits, int64_t key_min,
                                    int64_t key_max, int packed, int64_t * seg_start,
                                    int64_t * seg_cnt, unsigned int * flags,
                                    smj_stream_t stream);
/* smj_dev_partition_range_sampled writing 48-bit words (both tuple widths,
 * the 1-GPU join's LayP48): w = (key - base) mod 2^s1 << (48 - s1) | payload,
 * s1 the partition width's bit count, payload as unsigned (8-byte tuples:
 * its 32 bits), stored as two planes of `out`: lo = w mod 2^32 at
 * (uint32_t *)out, hi = w >> 32 at (uint16_t *)((uint32_t *)out + stride);
 * stride >= smj_sampled_capacity(n, nbits), a multiple of 32.  flags[1]
 * gets 1 (payload wider than 64 - s1 bits), 2 (key outside the range) or 4
 * (payload wider than 48 - s1 bits), or-ed.  Returns 0 (nothing launched)
 * when the form does not apply: nbits > 10, n >= 2^32, or s1 outside 1..32. */
int smj_dev_partition_range_planes(smj_workspace * ws, const tuple_t * in, uint64_t n,
                                   void * out, uint64_t stride, uint32_t nbits,
                                   int64_t key_min, int64_t key_max, int64_t * seg_start,
                                   int64_t * seg_cnt, unsigned int * flags,
                                   smj_stream_t stream);
/* The same partition with exactly sized regions (round 6; the multi-GPU
 * exchange's form across ranks): one read pass counts every (partition,
 * shard), the regions are laid out back to back with no slack, so `out` needs
 * n elements and the partitions come out contiguous -- partition p is its
 * smj_sampled_shards() shard regions one after the other.  Tables and flags
 * as smj_dev_partition_range_sampled (the overflow flag stays 0).  Returns 0
 * when it does not apply (nbits > 10, n >= 2^32, packed words the plan does
 * not allow). */
int smj_dev_partition_range_shards(smj_workspace * ws, const tuple_t * in, uint64_t n,
                                   void * out, uint32_t nbits, int64_t key_min,
                                   int64_t key_max, int packed, int64_t * seg_start,
                                   int64_t * seg_cnt, unsigned int * flags,
                                   smj_stream_t stream);
uint64_t smj_sampled_capacity(uint64_t n, uint32_t nbits);
uint32_t smj_sampled_shards(void);

/* The multi-GPU exchange's tables (smj/dist.py; exchange.hip).  A rank's
 * range partition into F partitions of K shard regions (start/cnt: F x K
 * int64, exact partitions use shard 0; flags: uint32[2] = region overflow,
 * not packable, as smj_dev_partition_range_sampled writes them) goes to
 * `world` ranks: of the `used` partitions the plan's key range reaches
 * (0 = all F), partition p goes to rank p*world/used, and the partitions
 * from `used` on to the last rank (the ranks split the keys, not the
 * power-of-two partition space).
 * smj_dev_xsend writes the message to every rank g, rank after rank
 * ([chunk size, used elements, flags[1], flags[0], the owned regions'
 * offsets inside the chunk, their counts]: 4 + 2 K n_g int64 for n_g owned
 * partitions) and chunk[0..world) = chunk starts, chunk[world..2 world) =
 * chunk sizes.  smj_dev_xrecv takes the `world` messages received (each
 * 4 + 2 K mine int64) and writes the local join's segment tables (tstart,
 * tcnt: nbuckets x world*K, bucket-major; the rank's own chunk in place at
 * its chunk start, the others from element `cap` on, rank order) and
 * summary[4 world + 2] = chunk starts, chunk sizes (sends), receive sizes,
 * used elements received, the not-packable and overflow flags OR-ed over
 * the ranks. */
void smj_dev_xsend(const int64_t * start, const int64_t * cnt, const unsigned int * flags,
                   uint32_t F, uint32_t K, uint32_t world, uint32_t used, int64_t * msg,
                   int64_t * chunk, smj_stream_t stream);
void smj_dev_xrecv(const int64_t * msg, const int64_t * chunk, uint32_t world, uint32_t rank,
                   uint32_t mine, uint32_t K, uint32_t nbuckets, uint64_t cap,
                   int64_t * tstart, int64_t * tcnt, int64_t * summary, smj_stream_t stream);

/* Self-check of the hardware property behind the stable partition's ranks:
 * LDS atomic adds return their old values to the lanes of one instruction
 * that hit the same word in lane order (partition.hip, k_scatter_swp).
 * Returns the number of violations (0 expected; synchronises `stream`).  The
 * library runs it once per process before its first stable partition and
 * falls back to ballot ranks on a device without the property. */
uint64_t smj_selfcheck_lds_order(smj_workspace * ws, smj_stream_t stream);

/* The calling thread's workspace behind the reference-named entry points
 * (sortmergejoin_multiway, avxsort_tuples, ...): lets a caller trace their
 * kernels with smj_trace_* (bench.py --api). */
smj_workspace * smj_context_workspace(void);

/* Per-kernel HIP-event trace of the join pipeline (bench.py roofline). */
void smj_trace_enable(smj_workspace * ws, int on);
void smj_trace_reset(smj_workspace * ws);
/* Trace only the kernel `name` (NULL or "": every kernel): one event pair per
 * step instead of one per kernel in bench.py's timed loop. */
void smj_trace_only(smj_workspace * ws, const char * name);
int smj_trace_read(smj_workspace * ws, char * names, int cap, float * ms_sum,
                   int * launches, int max);

#ifdef __cplusplus
}
#endif
#endif /* SMJ_H */
