#!/usr/bin/env bash
# Lab: group-pass ablations and geometry (lab builds under
# avx-sort-merge-joins_amd/lab/<variant>: make BUILD=build_<v> LIBOUT=lab/<v> EXTRA=...):
#   abl1 no in-group sort, abl2 no equal-digit run fixing, abl3 no write-out,
#   t512 512-thread workgroups.  Bench lines interleaved, two rounds; results
#   of the ablations are wrong by construction (only their times matter).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r03_gslab}; mkdir -p $O
dir() { [ "$1" = base ] && echo avx-sort-merge-joins_amd/lib || echo avx-sort-merge-joins_amd/lab/$1; }
for rep in 1 2; do
for v in ${VARIANTS:-base abl1 abl2 abl3 t512}; do
  for b in "--steps 10 --no-cpu-baseline" "--width 8 --steps 10 --no-cpu-baseline" "--op sort --width 8 --steps 10 --no-cpu-baseline"; do
    SMJ_LIB_DIR=$(dir $v) timeout -k 10 200 python3 bench.py $b > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b.json')); print('$v', '$b'.split('--no')[0], '|', d['ms_per_step'], 'ms', 'ok' if d.get('result_ok') else 'BAD', d['detail']['kernels_ms_per_step'])" | tee -a $O/lines.txt
  done
done
done
