#!/usr/bin/env bash
# round-2 iteration: partition lab, materialisation + partition tests, partition bench lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r02a}
mkdir -p $O
if [ -n "$LAB" ]; then
  timeout -k 10 150 ./build_lab/pl2_8 > $O/lab8.txt 2>&1 || exit $?
  timeout -k 10 150 ./build_lab/pl2_16 > $O/lab16.txt 2>&1 || exit $?
  grep -v "check.*ok" $O/lab8.txt $O/lab16.txt
fi
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_materialize.py tests/test_dropin.py tests/test_gpu_parity.py tests/test_gpu_golden.py} ${K:+-k "$K"} -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log
[ $rc = 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -30; exit $rc; }
for w in 8 16; do
  timeout -k 10 300 python bench.py --op partition --width $w --no-cpu-baseline > $O/part$w.json 2> $O/part$w.err || exit $?
  python3 -c "import json; d=json.load(open('$O/part$w.json')); print('part w$w', d['ms_per_step'], d['detail']['kernels_ms_per_step'], d['detail']['alg_frac_2Nw'], d['result_ok'])"
done
