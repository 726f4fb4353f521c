#!/usr/bin/env bash
# Round-2 artifacts after the merge changes: bench_multiwaymerge lines (64 x 65536
# with the reference's CPU baseline, 64 x 2M) and their rocprofv3 kernel stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02m
mkdir -p "$OUT"
timeout -k 10 300 python bench.py --op merge --width 8 > "$OUT/merge8.json" 2> "$OUT/merge8.err" || { tail -5 "$OUT/merge8.err"; exit 1; }
timeout -k 10 300 python bench.py --op merge --width 8 --n 2097152 --no-cpu-baseline > "$OUT/merge8_64x2M.json" 2> "$OUT/merge8_64x2M.err" || { tail -5 "$OUT/merge8_64x2M.err"; exit 1; }
head -c 300 "$OUT/merge8.json"; echo
for cfg in "merge8:" "merge8_64x2M:--n 2097152"; do
  name=${cfg%%:*}; extra=${cfg#*:}
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$name" -o run -- python3 bench.py --op merge --width 8 $extra --no-cpu-baseline > "$OUT/trace_$name.json" 2> "$OUT/trace_$name.log" || { echo "FAIL trace $name"; exit 1; }
  echo "traced $name"
done
