#!/usr/bin/env bash
# partlab on the box: both widths, then counter passes on one variant
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/lab/${TAG:-x}
mkdir -p $O
timeout -k 10 120 ./build_lab/partlab8 > $O/p8.txt 2>&1 || exit $?
timeout -k 10 120 ./build_lab/partlab16 > $O/p16.txt 2>&1 || exit $?
if [ -n "$PMCV" ]; then
  i=0
  PMCG=${PMCG:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"}
  IFS=';' read -ra GL <<< "$PMCG"
  for grp in "${GL[@]}"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc$i -o run -- ./build_lab/partlab${PMCW:-8} 134217728 10 0 "$PMCV" > $O/pmc$i.log 2>&1 || exit $?
  done
fi
cat $O/p8.txt $O/p16.txt | grep -v "check.*ok"
