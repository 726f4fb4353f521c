#!/usr/bin/env bash
# Lab: the join's level-1 scatter at two workgroups per CU (smaller tiles)
# against one (the default), 8- and 16-byte joins and the 8-byte sort.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03_sclab; mkdir -p $O
for rep in 1 2; do
for v in ${VARIANTS:-base sc2 sc2b}; do
  for b in "--steps 10 --no-cpu-baseline" "--width 8 --steps 10 --no-cpu-baseline" "--op sort --width 8 --steps 10 --no-cpu-baseline"; do
    SMJ_LIB_DIR=avx-sort-merge-joins_amd/lab/$v timeout -k 10 200 python3 bench.py $b > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b.json')); print('$v', '$b'.split('--no')[0], '|', d['ms_per_step'], 'ms', 'ok' if d.get('result_ok') else 'BAD', d['detail']['kernels_ms_per_step'])"
  done
done
done
