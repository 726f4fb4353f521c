set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_materialize.py tests/test_dropin.py "tests/test_gpu_parity.py::test_sortmergejoin_count" tests/test_gpu_golden.py tests/test_gpu_fullsize.py::test_distributed_join_n1024_one_rank "tests/test_gpu_parity.py::test_reference_generators_vs_oracle" -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace_xp -o run -- python3 bench.py --exchange-path --steps 5 --no-cpu-baseline > $O/xp.json 2> $O/xp.err || { tail -5 $O/xp.err; exit 1; }
python3 tools/timeline.py $(ls $O/trace_xp/*/run_kernel_trace.csv $O/trace_xp/run_kernel_trace.csv 2>/dev/null | head -1) 5 $O/xp_timeline.csv | tail -60
