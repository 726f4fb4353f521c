#!/usr/bin/env bash
# pytest subset ($TESTS, -k $K) then optional bench commands ($BENCH: ';'-separated
# bench.py argument lists), each under its own time limit; stops at the first failure.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-chk}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 ${PT_TIMEOUT:-900} python -u -m pytest $TESTS ${K:+-k "$K"} -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -4 $O/pytest.log
  [ $rc = 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $rc; }
fi
if [ -n "$BENCH" ]; then
  IFS=';' read -ra BL <<< "$BENCH"
  i=0
  for b in "${BL[@]}"; do
    i=$((i+1))
    timeout -k 10 300 python bench.py $b > $O/bench$i.json 2> $O/bench$i.err || { tail -5 $O/bench$i.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/bench$i.json')); r=d.get('roofline') or {}; print('$b', '|', d['ms_per_step'], 'ms', d['value'], d['unit'], 'ok' if d.get('result_ok') else 'BAD', '| kernels', d['detail']['kernels_ms_per_step'], '| frac', r.get('frac'), r.get('kernel'))"
  done
fi
