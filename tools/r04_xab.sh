#!/usr/bin/env bash
# The multi-GPU path on one GPU (--exchange-path) against the 1-GPU join,
# interleaved on one box, unprofiled lines without the CPU baseline.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r04_xab}; mkdir -p $O
for rep in ${REPS:-1 2}; do
  for b in "--steps 10" "--exchange-path --steps 10" ${EXTRA_LINES:+"$EXTRA_LINES"}; do
    timeout -k 10 200 python3 bench.py $b --no-cpu-baseline > $O/b.json 2> $O/b.err || { echo "FAIL $b"; tail -5 $O/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b.json')); x=d['detail'].get('exchange') or {}; print('$rep', '$b', '|', d['ms_per_step'], 'ms', 'ok' if d.get('result_ok') else 'BAD', x.get('exchange_layout', ''), {k: v for k, v in d['detail']['kernels_ms_per_step'].items()})"
  done
done
