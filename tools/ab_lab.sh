#!/usr/bin/env bash
# Interleaved A/B of library builds: $VARIANTS (base = lib/, others =
# avx-sort-merge-joins_amd/lab/<v>, built with make BUILD=build_<v>
# LIBOUT=lab/<v> EXTRA=...) over $BENCH (';'-separated bench.py argument
# lists), $REPS rounds; optionally the GPU suite first ($TESTS).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-ab}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 ${PT_TIMEOUT:-600} python -u -m pytest $TESTS -m gpu ${K:+-k "$K"} -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -4 $O/pytest.log
  [ $rc = 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $rc; }
fi
dir() { [ "$1" = base ] && echo avx-sort-merge-joins_amd/lib || echo avx-sort-merge-joins_amd/lab/$1; }
IFS=';' read -ra BL <<< "${BENCH:---op sort --width 8 --steps 10 --no-cpu-baseline}"
for rep in $(seq ${REPS:-2}); do
for v in ${VARIANTS:-base}; do
  for b in "${BL[@]}"; do
    SMJ_LIB_DIR=$(dir $v) timeout -k 10 200 python3 bench.py $b > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b.json')); print('$v', '$b'.split('--no')[0], '|', d['ms_per_step'], 'ms', 'ok' if d.get('result_ok') else 'BAD', d['detail']['kernels_ms_per_step'])" | tee -a $O/lines.txt
  done
done
done
