#!/usr/bin/env bash
# 8-byte join: level-1 scatter items per thread (SMJ_SC_ITEMS8 builds under
# build_v*) x 16-byte pair loads (SMJ_SC_VEC), interleaved rounds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/scvec; mkdir -p $OUT
for r in 1 2 3; do
  for cfg in default:1 v12:0 v12:1 v14:0 v14:1; do
    v=${cfg%%:*}; vec=${cfg##*:}
    if [ $v = default ]; then unset SMJ_LIB_DIR; else export SMJ_LIB_DIR=$PWD/avx-sort-merge-joins_amd/build_$v/lib; fi
    SMJ_SC_VEC=$vec timeout -k 10 120 python tools/microbench.py join --n 128000000 --width 8 --reps 5 > $OUT/x.json 2>&1 || { tail -5 $OUT/x.json; exit 1; }
    echo "$v vec=$vec r$r $(tail -1 $OUT/x.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms"], d["count"], d["kernels_ms"])')"
  done
done
