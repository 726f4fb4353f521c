#!/usr/bin/env bash
# Lab: k_fused schedule parameters (lag, groups per item), the cost of its sc1
# loads (plain-load build: not coherent, timing only) and the separate passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03_fusedlab; mkdir -p $O
for v in ${VARIANTS:-nofuse l8g8 l16g8 l8g16 l8g8p}; do
  for b in "--steps 10 --no-cpu-baseline" "--width 8 --steps 10 --no-cpu-baseline" "--op sort --width 8 --steps 10 --no-cpu-baseline"; do
    SMJ_LIB_DIR=avx-sort-merge-joins_amd/lab/$v timeout -k 10 200 python3 bench.py $b > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b.json')); print('$v', '$b'.split('--no')[0], '|', d['ms_per_step'], 'ms', 'ok' if d.get('result_ok') else 'BAD', d['detail']['kernels_ms_per_step'])"
  done
done
