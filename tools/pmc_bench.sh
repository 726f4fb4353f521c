#!/usr/bin/env bash
# PMC passes (one rocprofv3 run per group, kernel trace only) on one bench.py
# command.  usage: TAG=x PMCG="A B;C D" ARGS="--width 8" bash tools/pmc_bench.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-pmc}
mkdir -p $O
PMCG=${PMCG:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY;FETCH_SIZE;WRITE_SIZE"}
IFS=';' read -ra GL <<< "$PMCG"
i=0
for grp in "${GL[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc$i -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $ARGS > $O/pmc$i.log 2>&1 || { tail -5 $O/pmc$i.log; exit 1; }
done
echo done
