set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 200 python3 bench.py --exchange-path --steps 10 --no-cpu-baseline > $O/xp.json 2> $O/xp.err || { tail -5 $O/xp.err; exit 1; }
head -c 300 $O/xp.json; echo
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace_xp -o run -- python3 bench.py --exchange-path --steps 5 --no-cpu-baseline > $O/xp_traced.json 2> $O/xp_traced.err || { tail -5 $O/xp_traced.err; exit 1; }
python3 tools/timeline.py $O/trace_xp/run_kernel_trace.csv 4.5 $O/xp_timeline.csv | tail -45
bash tools/r03_mall.sh
