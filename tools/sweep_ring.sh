#!/usr/bin/env bash
# ring-size sweep of the 1-GPU join (16- and 8-byte tuples)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/ring}
mkdir -p "$OUT"
for w in 16 8; do
for mb in 0 16 32 64 128; do
  SMJ_RING_MB=$mb timeout -k 10 120 python tools/microbench.py join --n 128000000 --width $w --reps 5 > "$OUT/w${w}_mb$mb.json" 2>&1 || exit $?
  echo "w$w mb$mb $(tail -1 $OUT/w${w}_mb$mb.json)"
done
done
