#!/usr/bin/env bash
# Round-2 starting point on one MI355X: the reference-API stable partitioner
# and the device sort at 2^27 (BASELINE configs 2 and 3), per-kernel times
# from the library trace and a rocprofv3 kernel-stats pass of the partition.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02_base
mkdir -p "$OUT"
N=134217728
for w in 8 16; do
  timeout -k 10 120 python tools/microbench.py partition --n $N --bits 10 --width $w >> "$OUT/micro.jsonl" 2>> "$OUT/micro.err" || exit $?
  timeout -k 10 120 python tools/microbench.py sort --n $N --width $w >> "$OUT/micro.jsonl" 2>> "$OUT/micro.err" || exit $?
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/part8" -o run -- python3 tools/microbench.py partition --n $N --bits 10 --width 8 > "$OUT/part8.log" 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/sort8" -o run -- python3 tools/microbench.py sort --n $N --width 8 > "$OUT/sort8.log" 2>&1 || exit $?
cat "$OUT/micro.jsonl"
