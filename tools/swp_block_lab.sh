#!/bin/bash
# Lab (round 6): block-interleaved tile order of the stable scatter
# (SMJ_SWP_BLOCK_TILES) -- parity of one variant, then an interleaved A/B of
# bench_partitioning (2^27 x 8 B, 10 bits) over the variant builds.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/swpb; mkdir -p $O
SMJ_LIB_DIR=$PWD/avx-sort-merge-joins_amd/lib_b4 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "partition" > $O/pytest_b4.txt 2>&1 || { tail -30 $O/pytest_b4.txt; exit 1; }
tail -1 $O/pytest_b4.txt
LIBS="base:avx-sort-merge-joins_amd/lib b4:avx-sort-merge-joins_amd/lib_b4 b8:avx-sort-merge-joins_amd/lib_b8 b16:avx-sort-merge-joins_amd/lib_b16" CFGS="part8:--op,partition,--width,8" ROUNDS=3 TAG=swpb bash tools/ab.sh
