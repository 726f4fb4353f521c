#!/usr/bin/env bash
# Round-2 artifacts after the 8-byte scatter change: the 8 B join and 8 B sort
# bench lines (with the reference's CPU baselines), their rocprofv3 kernel stats
# and PMC traffic passes.  The first failure ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02g
mkdir -p "$OUT"
run() {  # name args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "FAIL $name"; tail -5 "$OUT/$name.err"; exit 1; }
  echo "$name $(head -c 200 $OUT/$name.json)"
}
prof() {  # key name args...
  local key=$1 name=$2; shift 2
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$name" -o run -- python3 bench.py "$@" --no-cpu-baseline > "$OUT/trace_$name.json" 2> "$OUT/trace_$name.log" || { echo "FAIL trace $name"; exit 1; }
  timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch_$name" -o run -- python3 bench.py "$@" --no-cpu-baseline > "$OUT/fetch_$name.log" 2>&1 || { echo "FAIL fetch $name"; exit 1; }
  timeout -k 10 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write_$name" -o run -- python3 bench.py "$@" --no-cpu-baseline > "$OUT/write_$name.log" 2>&1 || { echo "FAIL write $name"; exit 1; }
  python3 tools/make_traffic.py "$key" "$OUT/fetch_$name" "$OUT/write_$name" "$OUT/pmc_traffic.json" > /dev/null || exit 1
  echo "profiled $name"
}
run bench8 --steps 5 --warmup 2 --width 8
run sort8 --op sort --width 8
run bench16 --steps 5 --warmup 2 --no-cpu-baseline
prof n128000000_w8_uniform bench8 --steps 5 --warmup 2 --width 8
prof sort_n134217728_w8 sort8 --op sort --width 8
