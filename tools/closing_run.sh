#!/usr/bin/env bash
# A round's closing run at HEAD in three calls (each within gpurun's limit):
#   PART=1: the GPU suite and smoke, then the join lines (16 B, 8 B, Zipf);
#   PART=2: the op lines (sort, partition, merge), the 16-byte payload layouts
#           (64-bit words, 16-byte tuples), then without PMC passes the
#           reference-named join, both multi-GPU paths on one GPU (the
#           one-process-per-GPU C path and Python path, the in-process
#           threads path) and a second headline line, and the SQ counters of
#           the 8-byte join;
#   PART=3: BASELINE configs[4]'s size on one GPU (1024M x 1024M, uniform and
#           the reference's create_relation_zipf S).
# Each line: tools/lines.sh (unprofiled line with the CPU baseline, the line
# under rocprofv3 with its kernel stats, FETCH/WRITE passes ->
# pmc_traffic.json, roofcheck).  PART=2/3 start from the pmc_traffic.json in
# profiles/ (tools/collect.sh after PART=1).
# usage: R=r06 PART=1 bash tools/closing_run.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=${R:?round prefix}
O=${O:-gpurun_out/${R}_fin}
mkdir -p $O
case "${PART:-1}" in
1)
  if [ -z "${SKIP_SUITE:-}" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -20 $O/pytest_gpu.txt; exit 1; }
    tail -1 $O/pytest_gpu.txt
  fi
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
  bash tools/lines.sh $O ${LINES1:-"join16:--steps 10 --warmup 2" "join8:--width 8 --steps 10 --warmup 2" "zipf16:--dist zipf --steps 10 --warmup 2"} || exit 1
  ;;
2)
  O2=${O2:-gpurun_out/${R}_fin2}
  bash tools/lines.sh $O2 "sort8:--op sort --width 8 --steps 10 --warmup 2" "part8:--op partition --width 8 --steps 10 --warmup 2" "merge8:--op merge --steps 20 --warmup 3" "wide16:--payload wide48 --steps 10 --warmup 2" "full16:--payload full64 --steps 10 --warmup 2" || exit 1
  NO_PMC=1 CPU_ARGS=--no-cpu-baseline bash tools/lines.sh $O2/nopmc "api16:--api --steps 10 --warmup 2" "xpath16:--exchange-path --impl python --steps 10 --warmup 2" "xpathc16:--exchange-path --impl c --steps 10 --warmup 2" "threads16:--launch threads --steps 10 --warmup 2" "xdev16:--op exchange --steps 10 --warmup 2" "join16:--steps 10 --warmup 2" || exit 1
  O=$O2/sq bash tools/sqprobe.sh --width 8 > $O2/sq_join8.txt 2>&1 || { tail -5 $O2/sq_join8.txt; exit 1; }
  ;;
3)
  O3=${O3:-gpurun_out/${R}_fin3}
  NO_PMC=1 CPU_ARGS=--no-cpu-baseline bash tools/lines.sh $O3/n1024 "n1024u:--n 1024000000 --steps 3 --warmup 1" "n1024z:--n 1024000000 --dist zipf --zipf-gen reference --steps 3 --warmup 1" || exit 1
  ;;
esac
