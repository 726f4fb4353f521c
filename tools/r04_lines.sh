#!/usr/bin/env bash
# Lab: bench lines interleaved on one box, unprofiled, no CPU baseline.
# LINES: one line per config, "tag|ENV=value ...|bench args" (the env part
# may be empty); REPS rounds.  Per line the step time and kernel breakdown.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r04_lines}; mkdir -p $O
for rep in ${REPS:-1 2}; do
  while IFS='|' read -r tag envs args; do
    [ -z "$tag" ] && continue
    timeout -k 10 200 env $envs python3 bench.py $args --no-cpu-baseline < /dev/null > $O/b.json 2> $O/b.err || { echo "FAIL $tag"; tail -5 $O/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b.json')); print('$rep', '$tag', '|', d['ms_per_step'], 'ms', 'ok' if d.get('result_ok') else 'BAD', d['detail']['kernels_ms_per_step'])"
  done <<< "$LINES"
done
