#!/usr/bin/env bash
# Round-2 closing check at HEAD: the whole GPU suite, smoke(), then the lines
# changed since the last artifacts (bench_partitioning 8 B with its CPU
# baseline, bench_sort 8 B, the default 16 B join) with rocprofv3 kernel stats
# and the partition's PMC traffic.  The first failure ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02h
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.txt"; [ $rc = 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -5 "$OUT/smoke.txt"; exit 1; }
tail -2 "$OUT/smoke.txt"
run() {  # name args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "FAIL $name"; tail -5 "$OUT/$name.err"; exit 1; }
  echo "$name $(head -c 160 $OUT/$name.json)"
}
run part8 --op partition --width 8
run sort8 --op sort --width 8
run bench16 --steps 5 --warmup 2
for cfg in "part8:--op partition --width 8" "sort8:--op sort --width 8"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$name" -o run -- python3 bench.py $args --no-cpu-baseline > "$OUT/trace_$name.json" 2> "$OUT/trace_$name.log" || { echo "FAIL trace $name"; exit 1; }
  echo "traced $name"
done
timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch_part8" -o run -- python3 bench.py --op partition --width 8 --no-cpu-baseline > "$OUT/fetch_part8.log" 2>&1 || { echo "FAIL fetch"; exit 1; }
timeout -k 10 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write_part8" -o run -- python3 bench.py --op partition --width 8 --no-cpu-baseline > "$OUT/write_part8.log" 2>&1 || { echo "FAIL write"; exit 1; }
python3 tools/make_traffic.py partition_n134217728_w8 "$OUT/fetch_part8" "$OUT/write_part8" "$OUT/pmc_traffic.json" > /dev/null || exit 1
echo "pmc part8"
