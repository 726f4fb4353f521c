#!/usr/bin/env bash
# One gpurun call: GPU parity tests, the 1-GPU bench (16- and 8-byte tuples)
# and a rocprofv3 kernel-trace summary of the bench.  Stops at the first GPU
# fault / abort / timeout (a plain test failure still lets the bench run).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
timeout -k 10 600 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest exit $rc" >> "$OUT/pytest_gpu.log"
case $rc in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit $rc;; esac
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > "$OUT/bench16.log" 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --width 8 --no-cpu-baseline > "$OUT/bench8.log" 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof16" -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof16.log" 2>&1
