set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in ${VARIANTS:-lib}; do
  for w in 8 16; do
    SMJ_LIB_DIR=$PWD/avx-sort-merge-joins_amd/$v timeout -k 10 120 python bench.py --width $w --no-cpu-baseline > /tmp/b.json 2>/tmp/b.err || { tail -3 /tmp/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('/tmp/b.json')); print('$v', $w, d['ms_per_step'], d['result_ok'], d['detail']['kernels_ms_per_step'])"
  done
done
