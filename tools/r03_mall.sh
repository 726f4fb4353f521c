#!/usr/bin/env bash
# Lab: what Infinity-Cache residency of the tile-pass output buys the group
# pass.  The lab library (make BUILD=build_lab LIBOUT=lib_flush
# EXTRA=-DSMJ_LAB_FLUSH=1) writes 1 GiB between the tile and the group pass;
# the group pass time with and without it, at sizes whose tile-pass output
# fits the 256 MiB cache (8 B: 4M, 8M; 16 B packed words: 4M, 8M) and one
# that does not (128M).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03_mall; mkdir -p $O
for n in 4000000 8000000 128000000; do
  for w in 8 16; do
    for v in lib lib_flush; do
      SMJ_LIB_DIR=avx-sort-merge-joins_amd/$v timeout -k 10 120 python3 bench.py --n $n --width $w --steps 20 --warmup 3 --no-cpu-baseline > $O/${v}_${n}_${w}.json 2> $O/${v}_${n}_${w}.err || { tail -3 $O/${v}_${n}_${w}.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/${v}_${n}_${w}.json')); print('$v n=$n w=$w', d['ms_per_step'], d['detail']['kernels_ms_per_step'])"
    done
  done
done
