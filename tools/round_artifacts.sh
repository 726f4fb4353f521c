#!/usr/bin/env bash
# Round artifacts on one MI355X: GPU parity tests, the bench lines, the
# rocprofv3 kernel-trace summary of the bench command and the PMC traffic
# passes (FETCH_SIZE and WRITE_SIZE in separate runs).  Stops at the first
# GPU failure.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=${ROUND:-r01}
OUT=gpurun_out/$R
mkdir -p "$OUT"
timeout -k 10 900 python -m pytest tests -m gpu -q > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"
case $rc in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit $rc;; esac
B="--steps 5 --warmup 2"
timeout -k 10 300 python bench.py $B > "$OUT/bench16.json" 2> "$OUT/bench16.err" || exit $?
timeout -k 10 300 python bench.py $B --width 8 --no-cpu-baseline > "$OUT/bench8.json" 2> "$OUT/bench8.err" || exit $?
timeout -k 10 300 python bench.py $B --dist zipf --no-cpu-baseline > "$OUT/bench16_zipf.json" 2> "$OUT/bench16_zipf.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace16" -o run -- python3 bench.py $B --no-cpu-baseline > "$OUT/trace16.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch16" -o run -- python3 bench.py $B --no-cpu-baseline > "$OUT/fetch16.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write16" -o run -- python3 bench.py $B --no-cpu-baseline > "$OUT/write16.log" 2>&1 || exit $?
python3 tools/make_traffic.py n128000000_w16_uniform "$OUT/fetch16" "$OUT/write16" "$OUT/pmc_traffic.json" > /dev/null || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch8" -o run -- python3 bench.py $B --width 8 --no-cpu-baseline > "$OUT/fetch8.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write8" -o run -- python3 bench.py $B --width 8 --no-cpu-baseline > "$OUT/write8.log" 2>&1 || exit $?
python3 tools/make_traffic.py n128000000_w8_uniform "$OUT/fetch8" "$OUT/write8" "$OUT/pmc_traffic.json" > /dev/null || exit $?
cat "$OUT/bench16.json"
