#!/usr/bin/env bash
# Interleaved A/B of library builds on one box: every round runs every config
# on every build (SMJ_LIB_DIR), unprofiled, no CPU baseline; one summary line
# per run: ms/step and the per-kernel ms of the traced untimed steps.
# usage: LIBS="base:avx-sort-merge-joins_amd/lib_base new:avx-sort-merge-joins_amd/lib" \
#        CFGS="join8:--width,8 sort8:--op,sort,--width,8" ROUNDS=2 TAG=x bash tools/ab.sh
# (a build's tests: TESTS="tests/test_gpu_parity.py ..." run first on the last build)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-ab}
mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
  tail -1 $O/tests.txt
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for cfg in $CFGS; do
    name=${cfg%%:*}; args=${cfg#*:}
    for lb in $LIBS; do
      ln=${lb%%:*}; ld=${lb#*:}
      f=$O/${name}_${ln}_$r.json
      SMJ_LIB_DIR=$PWD/$ld timeout -k 10 300 python3 bench.py ${args//,/ } --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 > $f 2> $f.err || { echo "FAIL $name $ln"; tail -5 $f.err; exit 1; }
      python3 - "$f" "$name" "$ln" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = d["detail"]["kernels_ms_per_step"]
print(f"{sys.argv[2]:8s} {sys.argv[3]:6s} ms/step {d['ms_per_step']:.3f} ok {d['result_ok']} " +
      " ".join(f"{n}={v:.3f}" for n, v in k.items() if v > 0.02))
PY
    done
  done
done
