#!/usr/bin/env bash
# Lab: XCD-aware group order in k_groupsort (the library's default) against
# the contiguous chunk per workgroup (lab/noxcd, -DSMJ_GS_XCD=0): bench lines
# interleaved, then one FETCH_SIZE pass per variant on the 8-byte join.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03_xcdlab; mkdir -p $O
dir() { [ "$1" = base ] && echo avx-sort-merge-joins_amd/lib || echo avx-sort-merge-joins_amd/lab/$1; }
for rep in 1 2; do
for v in ${VARIANTS:-base noxcd}; do
  for b in "--steps 10 --no-cpu-baseline" "--width 8 --steps 10 --no-cpu-baseline" "--op sort --width 8 --steps 10 --no-cpu-baseline"; do
    SMJ_LIB_DIR=$(dir $v) timeout -k 10 200 python3 bench.py $b > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b.json')); print('$v', '$b'.split('--no')[0], '|', d['ms_per_step'], 'ms', 'ok' if d.get('result_ok') else 'BAD', d['detail']['kernels_ms_per_step'])"
  done
done
done
for v in ${VARIANTS:-base noxcd}; do
  for w in 8 16; do
    SMJ_LIB_DIR=$(dir $v) timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_${v}_$w -o run -- python3 bench.py --width $w --steps 3 --warmup 1 --no-cpu-baseline > $O/fetch_${v}_$w.log 2>&1 || { echo "FAIL fetch $v"; exit 1; }
    python3 - $O/fetch_${v}_$w $v $w <<'EOF'
import sys
sys.path.insert(0, "tools")
from make_traffic import per_launch
f = per_launch(sys.argv[1], "FETCH_SIZE")
for k in ("k_groupsort", "k_tilepass", "k_scatter"):
    if k in f:
        print(sys.argv[2], "w" + sys.argv[3], k, "read_B(2xFETCH) %.3f GB" % (2 * f[k][0] * 1024 / 1e9), "launches", f[k][1])
EOF
  done
done
