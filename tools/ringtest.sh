set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ring
for mb in 0 32 64 128 256; do for w in 16 8; do
SMJ_SAMPLED=0 SMJ_RING_MB=$mb timeout -k 10 120 python tools/microbench.py join --n 128000000 --width $w --reps 5 > gpurun_out/ring/x.json 2>&1 || exit $?
echo "mb$mb w$w $(tail -1 gpurun_out/ring/x.json)"
done; done
