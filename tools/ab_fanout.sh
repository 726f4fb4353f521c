#!/usr/bin/env bash
# A/B of the level-1 fan-out on one box, interleaved to cancel drift
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/ab_fanout; mkdir -p $O
for rep in 1 2 3; do for w in 16 8; do for fb in ${FBS:-9 8}; do
  timeout -k 10 200 python bench.py --fanout-bits $fb --width $w --steps 20 --warmup 3 --no-cpu-baseline > $O/x.json 2> $O/x.err || { tail -3 $O/x.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/x.json')); print('rep $rep w$w fb$fb', d['ms_per_step'], d['result_ok'], {k: round(v,3) for k,v in d['detail']['kernels_ms_per_step'].items()})"
done; done; done
