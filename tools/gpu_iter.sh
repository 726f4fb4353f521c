#!/usr/bin/env bash
# iteration loop: GPU parity tests, join microbench (16/8 B), optional PMC pass
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_quick.sh || exit $?
if [ -n "${PMC:-}" ]; then
  PROF_TIMEOUT=200 bash tools/profile.sh gpurun_out/pmc_iter -- python3 tools/microbench.py join --n 128000000 --width 16 --reps 3 > /dev/null 2>&1 || exit $?
  python3 - <<'PY'
import json
d=json.load(open('gpurun_out/pmc_iter/summary.txt'))
for k,v in d.items():
    if v.get('total_ms',0) < 0.2: continue
    print(k[:36], 'us=%.0f'%v['avg_us'], 'R=%.2fGB W=%.2fGB'%(v.get('HBM_READ_B',0)/1e9, v.get('WRITE_SIZE',0)/1e9),
          'wait=%.2f'%(v.get('SQ_WAIT_ANY',0)/max(1,v.get('SQ_WAVE_CYCLES',1))), 'valu=%.3g'%v.get('SQ_INSTS_VALU',0),
          'lds=%.3g conf=%.3g'%(v.get('SQ_LDS_IDX_ACTIVE',0), v.get('SQ_LDS_BANK_CONFLICT',0)), 'waitlds=%.3g'%v.get('SQ_WAIT_INST_LDS',0))
PY
fi
