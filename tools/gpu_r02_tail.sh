# MSM parity (all MSM files), then 2^20 A/B of the group-sum split and the lean event mode, and the
# GLV cut-over at 2^21.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_host_path.py tests/test_gpu_msm_config4.py tests/test_gpu_threads.py > gpurun_out/pytest_tail.log 2>&1 || { tail -30 gpurun_out/pytest_tail.log; exit 1; }
tail -1 gpurun_out/pytest_tail.log
: > gpurun_out/sweep_tail.log
SVGPU_MSM_STATS=1 timeout -k 10 200 python3 tools/msm_sweep_env.py 20 "SVGPU_GROUP_P=2" "SVGPU_GROUP_P=1" "SVGPU_GLV=0" >> gpurun_out/sweep_tail.log 2>&1 || { tail -20 gpurun_out/sweep_tail.log; exit 1; }
timeout -k 10 200 python3 tools/msm_sweep_env.py 20 "SVGPU_MSM_LEAN=0" "SVGPU_MSM_LEAN=1" >> gpurun_out/sweep_tail.log 2>&1 || { tail -20 gpurun_out/sweep_tail.log; exit 1; }
timeout -k 10 200 python3 tools/msm_sweep_env.py 21 "SVGPU_GLV=0" "SVGPU_GLV=1" >> gpurun_out/sweep_tail.log 2>&1 || { tail -20 gpurun_out/sweep_tail.log; exit 1; }
grep "2^" gpurun_out/sweep_tail.log
