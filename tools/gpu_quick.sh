#!/usr/bin/env bash
# quick loop: GPU parity tests, then the join microbench (16 and 8 B tuples)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/quick}
mkdir -p "$OUT"
timeout -k 10 600 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"
case $rc in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit $rc;; esac
for w in 16 8; do
  timeout -k 10 120 python tools/microbench.py join --n 128000000 --width $w --reps 5 > "$OUT/join_w${w}.json" 2>&1 || exit $?
  echo "w$w $(tail -1 $OUT/join_w${w}.json)"
done
for w in ${ZIPF_WIDTHS:-16}; do
  timeout -k 10 120 python tools/microbench.py join --n 128000000 --width $w --reps 5 --dist zipf > "$OUT/join_w${w}_zipf.json" 2>&1 || exit $?
  echo "w$w zipf $(tail -1 $OUT/join_w${w}_zipf.json)"
done
