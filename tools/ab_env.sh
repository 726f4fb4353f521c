#!/usr/bin/env bash
# Interleaved A/B of environment variants on one bench.py op:
#   OP=sort WIDTHS="8 16" ENVS="X=0 X=1" ROUNDS=2 bash tools/ab_env.sh
# ("-" as an env entry = no extra variable)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/ab_env}; mkdir -p "$OUT"
i=0
for r in $(seq 1 ${ROUNDS:-2}); do
  for e in ${ENVS:--}; do for w in ${WIDTHS:-8}; do
    i=$((i+1)); f="$OUT/${OP:-sort}_${i}.json"
    if [ "$e" = "-" ]; then ev=""; else ev="$e"; fi
    env $ev timeout -k 10 120 python bench.py --op ${OP:-sort} --width $w --steps ${STEPS:-10} \
      --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > "$f" 2> "${f%.json}.err" || exit $?
    echo "${OP:-sort} [$e] w$w r$r $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d.get("result_ok"), d["detail"].get("kernels_ms_per_step"))' "$f")"
  done; done
done
