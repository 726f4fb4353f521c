#!/usr/bin/env bash
# Kernel-trace + PMC passes (one counter group per rocprofv3 run, as the
# MI355X guide prescribes; never combined with --sys-trace etc.).
# usage: tools/profile.sh OUTDIR -- python tools/microbench.py join ...
set -euo pipefail
OUT="$1"; shift
[ "$1" = "--" ] && shift
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
T=${PROF_TIMEOUT:-240}
timeout -k 10 "$T" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- "$@" > "$OUT/trace.log" 2>&1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU" \
           "TCC_EA0_WRREQ TCC_EA0_WRREQ_64B TCC_EA0_RDREQ TCC_EA0_RDREQ_128B" \
           ${EXTRA_PMC:-}; do
    i=$((i+1))
    timeout -k 10 "$T" rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/pmc$i" -o run -- "$@" > "$OUT/pmc$i.log" 2>&1
done
python3 "$(dirname "$0")/parse_prof.py" "$OUT" > "$OUT/summary.txt"
cat "$OUT/summary.txt"
