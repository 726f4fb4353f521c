# k_fused first light: smoke (small join, both widths) under a short limit,
# then the parity suite, then the bench lines.  Stops at the first failure.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
rc=$?; tail -3 $O/smoke.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_materialize.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $rc; }
for b in "--steps 10 --no-cpu-baseline" "--width 8 --steps 10 --no-cpu-baseline" "--op sort --width 8 --steps 10 --no-cpu-baseline" "--dist zipf --steps 5 --no-cpu-baseline"; do
  timeout -k 10 200 python3 bench.py $b > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); r=d.get('roofline') or {}; print('$b', '|', d['ms_per_step'], 'ms', d['value'], 'ok' if d.get('result_ok') else 'BAD', d['detail']['kernels_ms_per_step'], r.get('kernel'), r.get('frac'))"
done
