#!/usr/bin/env bash
# sort: the key-range pass as chunked, pipelined 16-byte loads (default build)
# against the previous grid-stride form (build_old), interleaved, after the
# sort GPU tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/keyrange; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -k "sort or golden or fullsize or join" -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do for w in 8 16; do for v in default old; do
  if [ $v = default ]; then unset SMJ_LIB_DIR; else export SMJ_LIB_DIR=$PWD/avx-sort-merge-joins_amd/build_$v/lib; fi
  timeout -k 10 120 python bench.py --op sort --width $w --steps 10 --no-cpu-baseline > $OUT/s.json 2> $OUT/s.err || { tail -5 $OUT/s.err; exit 1; }
  echo "sort w$w $v r$r $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["result_ok"], d["detail"]["kernels_ms_per_step"])' $OUT/s.json)"
done; done; done
