#!/usr/bin/env bash
# Round 4 call d: the GPU suite, then the 48-bit plane layout A/B against
# 64-bit words (SMJ_P48=0), interleaved, unprofiled, and the plane copy probe.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r04_d}
mkdir -p $O
[ -n "${NOSUITE:-}" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
[ -n "${NOSUITE:-}" ] || tail -1 $O/pytest_gpu.txt
[ -n "${NOSUITE:-}" ] || timeout -k 10 120 build_lab/planelab > $O/planelab.txt 2>&1 || { cat $O/planelab.txt; exit 1; }
[ -n "${NOSUITE:-}" ] || cat $O/planelab.txt
DEFAULT_ARGS=$'--steps 10\n--dist zipf --steps 10\n--op sort --width 16 --steps 10'
for rep in 1 2; do
  while IFS= read -r args; do
    [ -z "$args" ] && continue
    tag=$(echo "$args" | tr -c 'a-z0-9' '_')
    for side in p48 p64; do
      if [ $side = p64 ]; then export SMJ_P48=0; else unset SMJ_P48; fi
      timeout -k 10 200 python3 bench.py $args --no-cpu-baseline > $O/${tag}_${side}_$rep.json 2> $O/${tag}_${side}_$rep.err < /dev/null || { echo "FAIL $side $args"; tail -5 $O/${tag}_${side}_$rep.err; exit 1; }
      python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], sys.argv[3], sys.argv[4], d['ms_per_step'], d['result_ok'], d['detail']['kernels_ms_per_step'])" $O/${tag}_${side}_$rep.json "$rep" "$side" "$args" < /dev/null
    done
  done <<< "${ARGS:-$DEFAULT_ARGS}"
done
unset SMJ_P48
