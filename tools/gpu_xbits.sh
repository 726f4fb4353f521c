#!/usr/bin/env bash
# exchange path on one GPU with the partition width of G GPUs (SMJ_XBITS)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/xb}
mkdir -p "$OUT"
for xb in ${XBITS:-9 10 11 12}; do
  SMJ_XBITS=$xb timeout -k 10 300 python bench.py --exchange-path --no-cpu-baseline > "$OUT/b$xb.json" 2> "$OUT/b$xb.err" || exit $?
  python3 -c "import json; d=json.loads(open('$OUT/b$xb.json').read().strip().splitlines()[-1]); print('xbits $xb', d['ms_per_step'], d['result_ok'], d['detail']['kernels_ms_per_step'])"
done
