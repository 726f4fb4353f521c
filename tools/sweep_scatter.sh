#!/usr/bin/env bash
# scatter ablations (timing only: results are wrong for modes 1/2) and tile variants
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/scat; mkdir -p $OUT
for w in 16 8; do
for cfg in "SMJ_SCATTER_MODE=0" "SMJ_SCATTER_MODE=1" "SMJ_SCATTER_MODE=2" "SMJ_PTU_VARIANT=1" "SMJ_PTU_VARIANT=0"; do
  env $cfg timeout -k 10 120 python tools/microbench.py join --n 128000000 --width $w --reps 5 > $OUT/x.json 2>&1 || exit $?
  echo "w$w $cfg $(tail -1 $OUT/x.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["kernels_ms"])')"
done; done
