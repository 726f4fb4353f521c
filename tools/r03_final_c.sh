#!/usr/bin/env bash
# Round-3 closing run at HEAD, one box: the GPU suite and smoke, then every
# BASELINE line (tools/r03_lines.sh: unprofiled line with the CPU baseline,
# the line under rocprofv3 with its kernel stats, FETCH/WRITE passes ->
# pmc_traffic.json, roofcheck), then the reference-named join and the
# multi-GPU path on one GPU without PMC passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03_fin
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -20 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
bash tools/r03_lines.sh $O "join16:--steps 10 --warmup 2" "join8:--width 8 --steps 10 --warmup 2" "zipf16:--dist zipf --steps 10 --warmup 2" "sort8:--op sort --width 8 --steps 10 --warmup 2" "part8:--op partition --width 8 --steps 10 --warmup 2" "merge8:--op merge --steps 20 --warmup 3" || exit 1
NO_PMC=1 CPU_ARGS=--no-cpu-baseline bash tools/r03_lines.sh $O/nopmc "api16:--api --steps 10 --warmup 2" "xpath16:--exchange-path --steps 10 --warmup 2" "join16:--steps 10 --warmup 2" || exit 1
