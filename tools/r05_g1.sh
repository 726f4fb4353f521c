set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_mgpu.py tests/test_dropin.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/r05_mgpu_tests.txt 2>&1
rc=$?
tail -5 gpurun_out/r05_mgpu_tests.txt
exit $rc
