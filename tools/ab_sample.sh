#!/usr/bin/env bash
# join level-1 sample histogram: workgroups per relation (SMJ_SAMPLE_WG
# builds: default 256, build_sw1024, build_sw128), interleaved, after the
# join GPU tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/sample; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -k "join or dist or golden" -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do for w in 16 8; do for v in default sw1024 sw128; do
  if [ $v = default ]; then unset SMJ_LIB_DIR; else export SMJ_LIB_DIR=$PWD/avx-sort-merge-joins_amd/build_$v/lib; fi
  timeout -k 10 120 python tools/microbench.py join --n 128000000 --width $w --reps 5 > $OUT/x.json 2>&1 || { tail -5 $OUT/x.json; exit 1; }
  echo "w$w $v r$r $(tail -1 $OUT/x.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms"], d["count"], d["kernels_ms"])')"
done; done; done
