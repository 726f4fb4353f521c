#!/usr/bin/env bash
# Round-3 closing artifacts, part A (joins): per config the unprofiled line
# (with the reference's CPU baseline), the line printed under rocprofv3
# --kernel-trace --stats with that run's kernel stats, FETCH_SIZE/WRITE_SIZE
# passes -> pmc_traffic.json, and tools/roofcheck.py's comparison.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03_final
bash tools/r03_lines.sh $O "join16:--steps 10 --warmup 2" "join8:--width 8 --steps 10 --warmup 2" "zipf16:--dist zipf --steps 10 --warmup 2" || exit 1
NO_PMC=1 CPU_ARGS=--no-cpu-baseline bash tools/r03_lines.sh $O/nopmc "api16:--api --steps 10 --warmup 2" "xpath16:--exchange-path --steps 10 --warmup 2" || exit 1
