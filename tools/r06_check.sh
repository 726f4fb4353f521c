#!/bin/bash
# Round-6 GPU check: the multi-GPU C path's new entries (slices, phases),
# the full-size payload-layout parity, and the bench lines they feed.
# Usage (GPU box): bash tools/r06_check.sh <tag>
set -o pipefail
cd "$(dirname "$0")/.."
T=${1:-r06a}
O=gpurun_out/$T
mkdir -p $O
PY="python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu"
timeout -k 10 600 $PY tests/test_gpu_mgpu.py tests/test_gpu_dist.py tests/test_gpu_parity.py > $O/pytest_mgpu.txt 2>&1 &&
timeout -k 10 900 $PY tests/test_gpu_fullsize.py -k "payload_layouts or copy8_zipf" > $O/pytest_full.txt 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/join16.json 2> $O/join16.err &&
timeout -k 10 300 python bench.py --no-cpu-baseline --exchange-path --impl c > $O/xpathc16.json 2> $O/xpathc16.err &&
timeout -k 10 300 python bench.py --no-cpu-baseline --launch threads --gpus 1 > $O/threads1.json 2> $O/threads1.err &&
{ timeout -k 10 120 python bench.py --gpus 2 > $O/gpus2.json 2> $O/gpus2.err; echo "rc=$?" >> $O/gpus2.err; true; }
