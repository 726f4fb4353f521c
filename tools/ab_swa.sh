#!/usr/bin/env bash
# A/B of the stable partition's software pipelining (SMJ_SWA_PIPE: bit 0
# k_hist_p, bit 1 k_scatter_swp) on bench_partitioning (2^27, 10 bits), after
# the partition GPU tests; variants interleaved, ROUNDS rounds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/ab_swa}; mkdir -p "$OUT"
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "${PYTEST_K:-partition}" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
  tail -2 "$OUT/pytest.log"
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-0 1 2 3}; do for w in ${WIDTHS:-8 16}; do
    SMJ_SWA_PIPE=$v timeout -k 10 120 python bench.py --op partition --width $w --steps 10 \
      --warmup 3 --no-cpu-baseline > "$OUT/p_${v}_w${w}_r${r}.json" 2> "$OUT/p_${v}_w${w}_r${r}.err" || exit $?
    echo "pipe=$v w$w r$r $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["result_ok"], d["detail"]["kernels_ms_per_step"])' "$OUT/p_${v}_w${w}_r${r}.json")"
  done; done
done
