#!/usr/bin/env bash
# PMC pass over the 1-GPU join (16-byte tuples) and a D2D copy reference.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/pmc}
mkdir -p "$OUT"
timeout -k 10 120 python tools/microbench.py copy --n 128000000 --width 16 > "$OUT/copy16.json" 2>&1 || exit $?
PROF_TIMEOUT=200 bash tools/profile.sh "$OUT/join16" -- python3 tools/microbench.py join --n 128000000 --width 16 --reps 3
