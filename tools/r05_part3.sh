#!/usr/bin/env bash
# Round-5 third closing call: the merge line after the host-wait removal, and
# BASELINE configs[4]'s size on one GPU (1024M x 1024M; Zipf 0.75 from the
# reference's create_relation_zipf stream).  usage: bash tools/r05_part3.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O3=${O3:-gpurun_out/r05_fin5}
bash tools/lines.sh $O3 "merge8:--op merge --steps 20 --warmup 3" || exit 1
NO_PMC=1 CPU_ARGS=--no-cpu-baseline bash tools/lines.sh $O3/n1024 "n1024u:--n 1024000000 --steps 3 --warmup 1" "n1024z:--n 1024000000 --dist zipf --zipf-gen reference --steps 3 --warmup 1" || exit 1
