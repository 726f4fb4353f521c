#!/usr/bin/env bash
# Round-5 second closing call: the op lines, the 16-byte payload layouts, the
# reference-named join, both multi-GPU paths on one GPU, and the SQ counters
# of the 8-byte join.  usage: bash tools/r05_part2.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O2=${O2:-gpurun_out/r05_fin2}
bash tools/lines.sh $O2 "sort8:--op sort --width 8 --steps 10 --warmup 2" "part8:--op partition --width 8 --steps 10 --warmup 2" "merge8:--op merge --steps 20 --warmup 3" "wide16:--payload wide48 --steps 10 --warmup 2" "full16:--payload full64 --steps 10 --warmup 2" || exit 1
NO_PMC=1 CPU_ARGS=--no-cpu-baseline bash tools/lines.sh $O2/nopmc "api16:--api --steps 10 --warmup 2" "xpath16:--exchange-path --steps 10 --warmup 2" "xpathc16:--exchange-path --impl c --steps 10 --warmup 2" "join16:--steps 10 --warmup 2" || exit 1
O=$O2/sq bash tools/sqprobe.sh --width 8 > $O2/sq_join8.txt 2>&1 || { tail -5 $O2/sq_join8.txt; exit 1; }
