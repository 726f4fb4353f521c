#!/usr/bin/env bash
# The multi-GPU code path on one GPU (bench.py --exchange-path: range
# partition, one-rank RCCL all-to-all, segmented local join): 16/8 B uniform
# and 16 B Zipf.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/x}
mkdir -p "$OUT"
for w in 16 8; do
  timeout -k 10 300 python bench.py --exchange-path --no-cpu-baseline --width $w > "$OUT/b$w.json" 2> "$OUT/b$w.err" || exit $?
done
timeout -k 10 300 python bench.py --exchange-path --no-cpu-baseline --dist zipf > "$OUT/bz.json" 2> "$OUT/bz.err" || exit $?
for f in b16 b8 bz; do
  python3 -c "import json; d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['value'], d['result_ok'], d['detail']['kernels_ms_per_step'])"
done
