#!/usr/bin/env bash
# SQ counters of the join's three passes (issue, wait and LDS behaviour), one
# rocprofv3 --pmc pass per counter set (at most 8 SQ counters a pass), then a
# per-launch table.  usage: tools/sqprobe.sh [bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${O:-gpurun_out/sq}; mkdir -p $O
ARGS=${*:---width 8}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P3="SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_ADDR_CONFLICT SQ_LDS_ATOMIC_RETURN SQ_INSTS_LDS_ATOMIC SQ_VMEM_TA_ADDR_FIFO_FULL SQ_WAVES"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/p$i -o run -- python3 bench.py $ARGS --steps 2 --warmup 1 --no-cpu-baseline > $O/p$i.log 2>&1 \
    || { echo "FAIL pass $i"; tail -5 $O/p$i.log; exit 1; }
done
python3 - $O $P1 $P2 $P3 <<'EOF'
import sys
sys.path.insert(0, "tools")
from make_traffic import per_launch
O, names = sys.argv[1], sys.argv[2:]
rows = {}
for i in (1, 2, 3):
    for c in names:
        for k, (v, n) in per_launch(f"{O}/p{i}", c).items():
            rows.setdefault(k, {})[c] = v
for k in ("k_scatter", "k_tilepass", "k_groupsort", "k_skew_small"):
    if k in rows:
        print(k)
        for c in names:
            if c in rows[k]:
                print(f"  {c:28s} {rows[k][c]:.4g}")
EOF
