#!/usr/bin/env bash
# Full-size parity of the BASELINE single-GPU configs + the sort/partition
# bench lines with rocprofv3 kernel stats.  Stops at the first GPU failure.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${OUTDIR:-r02_ops}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_materialize.py tests/test_gpu_dist.py -x -v --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -5 "$OUT/pytest.log"
[ $rc = 0 ] || exit $rc
for w in 8 16; do
  timeout -k 10 300 python bench.py --op partition --width $w > "$OUT/part$w.json" 2> "$OUT/part$w.err" || exit $?
  timeout -k 10 300 python bench.py --op sort --width $w > "$OUT/sort$w.json" 2> "$OUT/sort$w.err" || exit $?
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_part16" -o run -- python3 bench.py --op partition --width 16 --no-cpu-baseline > "$OUT/trace_part16.log" 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_sort16" -o run -- python3 bench.py --op sort --width 16 --no-cpu-baseline > "$OUT/trace_sort16.log" 2>&1 || exit $?
cat "$OUT"/*.json
