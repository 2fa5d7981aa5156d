# MSM parity then the 2^20 kernel timeline and a fork/no-fork A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_host_path.py tests/test_gpu_threads.py > gpurun_out/pytest_t2.log 2>&1 || { tail -30 gpurun_out/pytest_t2.log; exit 1; }
tail -1 gpurun_out/pytest_t2.log
timeout -k 10 200 python3 tools/msm_sweep_env.py 20 "SVGPU_SORT_FORK=1" "SVGPU_SORT_FORK=0" > gpurun_out/sweep_fork.log 2>&1 || { tail -20 gpurun_out/sweep_fork.log; exit 1; }
grep "2^" gpurun_out/sweep_fork.log
bash tools/gpu_r02_trace.sh
