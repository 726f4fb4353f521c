#!/usr/bin/env bash
# Lab: the local join's shape at G = 4 with the 48-bit planes (2^9 exchange
# partitions -> 2^7 local buckets) against 64-bit words (2^10 -> 2^8), played
# by the 1-GPU join: --fanout-bits 7 / 8 with SMJ_P48=1 / 0, interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r04_fanlab}; mkdir -p $O
for rep in 1 2; do
  for w in 16 8; do
    for cfg in "1 7" "1 8" "0 8" "0 7"; do
      set -- $cfg
      SMJ_P48=$1 timeout -k 10 200 python3 bench.py --width $w --fanout-bits $2 --steps 10 --no-cpu-baseline < /dev/null > $O/b.json 2> $O/b.err || { echo "FAIL $cfg"; tail -5 $O/b.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/b.json')); print('$rep', 'w$w', 'p48=$1', 'fanout=$2', '|', d['ms_per_step'], 'ms', 'ok' if d.get('result_ok') else 'BAD', d['detail']['kernels_ms_per_step'])"
    done
  done
done
