#!/usr/bin/env bash
# compare library variants built under build/v_*/lib (SMJ_LIB_DIR)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/var; mkdir -p $OUT
for v in default ${VARIANTS:-}; do for w in 16 8; do
  if [ $v = default ]; then unset SMJ_LIB_DIR; else export SMJ_LIB_DIR=$PWD/avx-sort-merge-joins_amd/build/$v/lib; fi
  timeout -k 10 120 python tools/microbench.py join --n 128000000 --width $w --reps 5 ${MB_ARGS:-} > $OUT/x.json 2>&1 || exit $?
  echo "$v w$w $(tail -1 $OUT/x.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms"], d["count"], d["kernels_ms"])')"
done; done
