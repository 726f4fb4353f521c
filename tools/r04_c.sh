#!/usr/bin/env bash
# Round 4 call c: the plane-layout copy probe, the multi-GPU path on one GPU
# (one-rank RCCL group), then more interleaved reps of the sort_two A/B on the
# 16-byte lines.  The first failure ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04_c
mkdir -p $O
timeout -k 10 120 build_lab/planelab > $O/planelab.txt 2>&1 || { cat $O/planelab.txt; exit 1; }
cat $O/planelab.txt
timeout -k 10 300 python3 bench.py --exchange-path --steps 10 --no-cpu-baseline > $O/xpath16.json 2> $O/xpath16.err || { tail -20 $O/xpath16.err; exit 1; }
head -c 400 $O/xpath16.json; echo
REPS="1 2 3" ALT=avx-sort-merge-joins_amd/lib_two0 OUT=$O bash tools/r04_ab.sh "--steps 10" "--dist zipf --steps 10"
