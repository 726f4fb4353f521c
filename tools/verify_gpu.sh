#!/usr/bin/env bash
# GPU check of the tree: the whole GPU suite, smoke, then short bench lines
# (extra lines: LINES="name:args ..." ).  usage: TAG=x bash tools/verify_gpu.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-verify}
mkdir -p $O
if [ -z "${SKIP_SUITE:-}" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
  tail -2 $O/pytest_gpu.txt
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
fi
for cfg in ${LINES:-}; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 python3 bench.py ${args//,/ } --no-cpu-baseline > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -5 $O/$name.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); print('$name', d['ms_per_step'], d['value'], d['result_ok'], d['roofline']['name'] if d.get('roofline') else None, round(d['roofline']['frac'],3) if d.get('roofline') else None)"
done
