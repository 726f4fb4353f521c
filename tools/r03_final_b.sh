#!/usr/bin/env bash
# Round-3 closing artifacts, part B (bench_sort, bench_partitioning,
# bench_multiwaymerge), as part A.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03_final
[ -f $O/pmc_traffic.json ] && cp $O/pmc_traffic.json profiles/pmc_traffic.json
bash tools/r03_lines.sh $O/ops "sort8:--op sort --width 8 --steps 10 --warmup 2" "part8:--op partition --width 8 --steps 10 --warmup 2" "merge8:--op merge --steps 20 --warmup 3" || exit 1
# the reference-named entry point against smj_dev_join, back to back (twice)
NO_PMC=1 CPU_ARGS=--no-cpu-baseline bash tools/r03_lines.sh $O/api "join16a:--steps 10 --warmup 2" "api16a:--api --steps 10 --warmup 2" "join16b:--steps 10 --warmup 2" "api16b:--api --steps 10 --warmup 2" || exit 1
