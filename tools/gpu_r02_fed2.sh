# Host-fed path after the split staging: parity tests, then host-API timings per piece count.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_host_path.py tests/test_gpu_threads.py tests/test_gpu_dist.py > gpurun_out/pytest_fed2.log 2>&1 || { tail -30 gpurun_out/pytest_fed2.log; exit 1; }
tail -1 gpurun_out/pytest_fed2.log
timeout -k 10 300 python3 tools/host_api_bench.py 20
