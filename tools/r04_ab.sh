#!/usr/bin/env bash
# Round 4 A/B on one box: the library in lib/ against an alternative build
# (SMJ_LIB_DIR=$ALT), interleaved, unprofiled bench lines without the CPU
# baseline.  usage: ALT=avx-sort-merge-joins_amd/lib_x OUT=gpurun_out/x tools/r04_ab.sh "args" ...
# Optionally runs the GPU suite first (SUITE=1).  The first failure ends it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r04_ab}
mkdir -p $O
if [ -n "${SUITE:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
  tail -1 $O/pytest_gpu.txt
fi
for rep in ${REPS:-1 2}; do
  for args in "$@"; do
    tag=$(echo "$args" | tr -c 'a-z0-9' '_')
    for side in new alt; do
      if [ $side = alt ]; then export SMJ_LIB_DIR=$ALT; else unset SMJ_LIB_DIR; fi
      timeout -k 10 200 python3 bench.py $args --no-cpu-baseline > $O/${tag}_${side}_$rep.json 2> $O/${tag}_${side}_$rep.err || { echo "FAIL $side $args"; tail -5 $O/${tag}_${side}_$rep.err; exit 1; }
      python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], sys.argv[3], sys.argv[4], d['ms_per_step'], d['result_ok'], {k:v for k,v in d['detail']['kernels_ms_per_step'].items()})" $O/${tag}_${side}_$rep.json "$rep" "$side" "$args"
    done
  done
done
unset SMJ_LIB_DIR
