#!/usr/bin/env bash
# Round 4, first GPU call: the whole GPU suite (new: the ABI extras, the
# full-size join at the benched plan and on the reference Zipf stream), then
# the headline line with the output check and the CPU baseline, and the
# bench_sort line.  The first failure ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04_a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread --durations 25 > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -3 $O/pytest_gpu.txt
timeout -k 10 400 python bench.py > $O/join16.json 2> $O/join16.err || { tail -20 $O/join16.err; exit 1; }
cat $O/join16.json
timeout -k 10 200 python bench.py --op sort --width 8 --no-cpu-baseline > $O/sort8.json 2> $O/sort8.err || { tail -20 $O/sort8.err; exit 1; }
cat $O/sort8.json
timeout -k 10 300 build_lab/scatterlab 27 > $O/scatterlab.txt 2>&1 || { tail -5 $O/scatterlab.txt; exit 1; }
cat $O/scatterlab.txt
