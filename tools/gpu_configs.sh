#!/usr/bin/env bash
# BASELINE.json configs[1..2] on one MI355X: bench_sort (2^27, device sort) and
# bench_partitioning (2^27, 10 bits, partition_relation_optimized layout)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/cfg}
mkdir -p "$OUT"
for w in 16 8; do
  timeout -k 10 120 python tools/microbench.py sort --n 134217728 --width $w --reps 5 > "$OUT/sort$w.json" 2>&1 || exit $?
  echo "sort w$w $(tail -1 $OUT/sort$w.json)"
  timeout -k 10 120 python tools/microbench.py partition --n 134217728 --bits 10 --width $w --reps 5 > "$OUT/part$w.json" 2>&1 || exit $?
  echo "partition w$w $(tail -1 $OUT/part$w.json)"
  timeout -k 10 120 python tools/microbench.py join --n 128000000 --width $w --reps 5 --nohint > "$OUT/joinnh$w.json" 2>&1 || exit $?
  echo "join-nohint w$w $(tail -1 $OUT/joinnh$w.json)"
done
