#!/usr/bin/env bash
# Round-2 artifacts on one MI355X (no pytest: run separately), PHASE=runs
# (bench lines) or PHASE=prof (rocprofv3 traces and PMC passes): the bench
# lines (join 16/8 B, Zipf, and the sort / partition / merge ops with their
# CPU baselines), rocprofv3 --kernel-trace --stats of the same commands, and
# the PMC traffic passes (FETCH_SIZE and WRITE_SIZE in separate runs).  Every
# GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=${ROUND:-r02}
OUT=gpurun_out/$R
mkdir -p "$OUT"
B="--steps 5 --warmup 2"
run() {  # name args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "FAIL $name"; tail -5 "$OUT/$name.err"; exit 1; }
  echo "$name $(head -c 300 $OUT/$name.json)"
}
prof() {  # name args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$name" -o run -- python3 bench.py "$@" --no-cpu-baseline > "$OUT/trace_$name.log" 2>&1 || { echo "FAIL trace $name"; exit 1; }
  echo "traced $name"
}
pmc() {  # cfgkey name args...
  local key=$1 name=$2; shift 2
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch_$name" -o run -- python3 bench.py "$@" --no-cpu-baseline > "$OUT/fetch_$name.log" 2>&1 || { echo "FAIL fetch $name"; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write_$name" -o run -- python3 bench.py "$@" --no-cpu-baseline > "$OUT/write_$name.log" 2>&1 || { echo "FAIL write $name"; exit 1; }
  python3 tools/make_traffic.py "$key" "$OUT/fetch_$name" "$OUT/write_$name" "$OUT/pmc_traffic.json" > /dev/null || exit 1
  echo "pmc $name"
}
if [ "${PHASE:-runs}" = runs ]; then
run bench16 $B
run bench8 $B --width 8
run bench16_zipf $B --dist zipf --no-cpu-baseline
run part8 --op partition --width 8
run part16 --op partition --width 16 --no-cpu-baseline
run sort8 --op sort --width 8
run sort16 --op sort --width 16 --no-cpu-baseline
run merge8 --op merge --width 8
run merge8_64x2M --op merge --width 8 --n 2097152 --no-cpu-baseline
run bench16_exchange_path $B --exchange-path --no-cpu-baseline
run exchange_n1 --op exchange --no-cpu-baseline
run n1024_uniform --n-total 1024000000 --no-cpu-baseline
run n1024_zipf --n-total 1024000000 --dist zipf --no-cpu-baseline
else
prof bench16 $B
prof part8 --op partition --width 8
prof sort8 --op sort --width 8
prof merge8 --op merge --width 8 --n 2097152
pmc n128000000_w16_uniform bench16 $B
pmc n128000000_w8_uniform bench8 $B --width 8
pmc partition_n134217728_w8 part8 --op partition --width 8
pmc sort_n134217728_w8 sort8 --op sort --width 8
fi
