#!/usr/bin/env bash
# End-of-round check after the stable-partition work: the whole GPU suite,
# smoke(), then the bench_partitioning lines (8 B with the reference's CPU
# baseline, 16 B), their rocprofv3 kernel stats and PMC traffic passes.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02f
mkdir -p "$OUT"
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1
  rc=$?; tail -3 "$OUT/pytest_gpu.txt"; [ $rc = 0 ] || exit $rc
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -5 "$OUT/smoke.txt"; exit 1; }
  tail -2 "$OUT/smoke.txt"
fi
timeout -k 10 300 python bench.py --op partition --width 8 > "$OUT/part8.json" 2> "$OUT/part8.err" || { tail -5 "$OUT/part8.err"; exit 1; }
timeout -k 10 300 python bench.py --op partition --width 16 --no-cpu-baseline > "$OUT/part16.json" 2> "$OUT/part16.err" || { tail -5 "$OUT/part16.err"; exit 1; }
head -c 400 "$OUT/part8.json"; echo; head -c 300 "$OUT/part16.json"; echo
for w in 8 16; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_part$w" -o run -- python3 bench.py --op partition --width $w --no-cpu-baseline > "$OUT/trace_part$w.json" 2> "$OUT/trace_part$w.log" || { echo "FAIL trace $w"; exit 1; }
  timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch_part$w" -o run -- python3 bench.py --op partition --width $w --no-cpu-baseline > "$OUT/fetch_part$w.log" 2>&1 || { echo "FAIL fetch $w"; exit 1; }
  timeout -k 10 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write_part$w" -o run -- python3 bench.py --op partition --width $w --no-cpu-baseline > "$OUT/write_part$w.log" 2>&1 || { echo "FAIL write $w"; exit 1; }
  python3 tools/make_traffic.py "partition_n134217728_w$w" "$OUT/fetch_part$w" "$OUT/write_part$w" "$OUT/pmc_traffic.json" > /dev/null || exit 1
  echo "profiled part$w"
done
