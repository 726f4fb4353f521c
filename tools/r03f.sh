set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_fullsize.py::test_distributed_join_n1024_one_rank -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $rc; }
for i in 1 2; do
timeout -k 10 200 python3 bench.py --exchange-path --steps 10 --no-cpu-baseline > $O/xp$i.json 2> $O/xp$i.err || { tail -5 $O/xp$i.err; exit 1; }
timeout -k 10 200 python3 bench.py --steps 10 --no-cpu-baseline > $O/j$i.json 2> $O/j$i.err || { tail -5 $O/j$i.err; exit 1; }
python3 -c "import json; a=json.load(open('$O/xp$i.json')); b=json.load(open('$O/j$i.json')); print('exchange-path', a['ms_per_step'], 'join', b['ms_per_step'], 'ratio', round(a['ms_per_step']/b['ms_per_step'],3))"
done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace_xp -o run -- python3 bench.py --exchange-path --steps 5 --no-cpu-baseline > $O/xp_traced.json 2> $O/xp_traced.err || { tail -5 $O/xp_traced.err; exit 1; }
python3 tools/timeline.py $O/trace_xp/run_kernel_trace.csv 4.5 $O/xp_timeline.csv | tail -42
