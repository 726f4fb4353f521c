#!/bin/bash
# Round-6 iteration check: the tests a change touches, then the lines it moves.
# usage: TESTS="..." LINES="name:args ..." bash tools/r06_iter.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-iter}
mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu $TESTS > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
  tail -1 $O/pytest.txt
fi
for cfg in ${LINES:-}; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 python3 bench.py ${args//,/ } --no-cpu-baseline > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -5 $O/$name.err; exit 1; }
  python3 - "$O/$name.json" "$name" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = d["detail"].get("kernels_ms_per_step") or d["detail"].get("kernels_ms_per_step_rank0") or {}
print(f"{sys.argv[2]:10s} ms/step {d['ms_per_step']:.3f} ok {d['result_ok']} " +
      " ".join(f"{n}={v:.3f}" for n, v in k.items() if v > 0.01))
PY
done
