# MSM parity, then GLV on/off at several sizes and the u32 sort entries A/B at 2^20 (each line checks
# every setting gives the same point).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_msm.py > gpurun_out/pytest_glv.log 2>&1 || { tail -30 gpurun_out/pytest_glv.log; exit 1; }
tail -1 gpurun_out/pytest_glv.log
: > gpurun_out/sweep_sizes.log
SVGPU_MSM_STATS=1 timeout -k 10 200 python3 tools/msm_sweep_env.py 20 "SVGPU_GLV=1" "SVGPU_GLV=1,SVGPU_SORT_E32=0" "SVGPU_GLV=0" "SVGPU_GLV=0,SVGPU_SORT_E32=0" >> gpurun_out/sweep_sizes.log 2>&1 || { tail -20 gpurun_out/sweep_sizes.log; exit 1; }
for lg in 14 16 18 22 24; do
  timeout -k 10 200 python3 tools/msm_sweep_env.py $lg "SVGPU_GLV=0" "SVGPU_GLV=1" >> gpurun_out/sweep_sizes.log 2>&1 || { tail -20 gpurun_out/sweep_sizes.log; exit 1; }
done
grep "2^" gpurun_out/sweep_sizes.log
