#!/usr/bin/env bash
# Lab (round 4): the join's level-1 scatter geometry with the 48-bit layout.
# Variant libraries lib_<v>/ (built with make BUILD=build_<v> LIBOUT=lib_<v>
# EXTRA=...) against lib/, interleaved, unprofiled lines without the CPU
# baseline; per line the step time and the per-kernel breakdown.
#   VARIANTS="s2 s3" REPS="1 2" tools/r04_sclab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r04_sclab}; mkdir -p $O
for rep in ${REPS:-1 2}; do
  # LINES: bench arguments, one line per config (default: the 16 B and 8 B
  # joins and the 8 B sort)
  while IFS= read -r b; do
    [ -z "$b" ] && continue
    for v in base ${VARIANTS:-s2 s3 s4}; do
      if [ $v = base ]; then unset SMJ_LIB_DIR; else export SMJ_LIB_DIR=avx-sort-merge-joins_amd/lib_$v; fi
      timeout -k 10 200 python3 bench.py $b --no-cpu-baseline < /dev/null > $O/b.json 2> $O/b.err || { echo "FAIL $v $b"; tail -5 $O/b.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/b.json')); print('$rep', '$v', '$b', '|', d['ms_per_step'], 'ms', 'ok' if d.get('result_ok') else 'BAD', {k: v for k, v in d['detail']['kernels_ms_per_step'].items()})"
    done
  done <<< "${LINES:-"--steps 10
--width 8 --steps 10
--op sort --width 8 --steps 10"}"
done
unset SMJ_LIB_DIR
