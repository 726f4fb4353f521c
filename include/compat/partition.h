/*
 * partition.h -- drop-in for the reference header src/partition/partition.h:57-120
 * (sdecoder/AVX-sort-merge-joins).  Same file name and include guard, so a
 * reference driver that includes "partition.h" compiles unchanged against
 * libsmj_hip.so (8-byte tuples) or libsmj_hip_k8.so (-DKEY_8B, 16-byte tuples).
 * Provides: partition_relation, partition_relation_optimized[_V2], histogram_memcpy_bench, radix_cluster (:38-43).  The declarations live in ../smj.h.
 */
#ifndef PARTITION_H
#define PARTITION_H
#ifndef SMJ_H
#define SMJ_COMPAT_HIDE_PRINT_TIMING
#endif
#include "../smj.h"
#endif /* PARTITION_H */
