#!/usr/bin/env bash
# round-2 iteration: selected GPU tests, then bench lines given as
# op:width[:n[:extra bench args]] in $BENCHES (e.g. "sort:8 merge:8:2097152")
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r02b}
mkdir -p $O
if [ -n "${TESTS}" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS} ${K:+-k "$K"} -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -4 $O/pytest.log
  [ $rc = 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -30; exit $rc; }
fi
i=0
for b in ${BENCHES}; do
  IFS=: read -r op w n extra <<< "$b"
  i=$((i+1))
  f=$O/b${i}_${op}${w}
  timeout -k 10 300 python bench.py --op $op --width $w ${n:+--n $n} ${extra//,/ } --no-cpu-baseline > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
  python3 -c "import json; d=json.load(open('$f.json')); print('$b', d['ms_per_step'], d['detail'].get('kernels_ms_per_step'), d['roofline']['frac'], d.get('result_ok'))"
done
