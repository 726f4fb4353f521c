#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/d1; mkdir -p $OUT
for wc in 0 1; do for w in 16 8; do for bits in ${BITS:-7 8 9 10}; do
  SMJ_SCATTER_WC=$wc timeout -k 10 120 python tools/microbench.py join --n 128000000 --width $w --reps 3 --bits $bits > $OUT/x.json 2>&1 || exit $?
  echo "wc$wc w$w bits$bits $(tail -1 $OUT/x.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms"], d["count"], d["kernels_ms"])')"
done; done; done
