# MSM + Poseidon parity, then the 2^20 GLV / reduction-segment sweep and the Poseidon timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_poseidon.py > gpurun_out/pytest_glv.log 2>&1 || { tail -30 gpurun_out/pytest_glv.log; exit 1; }
tail -1 gpurun_out/pytest_glv.log
SVGPU_MSM_STATS=1 timeout -k 10 300 python3 tools/msm_sweep_env.py 20 "SVGPU_GLV=0" "SVGPU_GLV=1" "SVGPU_GLV=1,SVGPU_RED_LOG=2" > gpurun_out/sweep_glv.log 2>&1 || { tail -20 gpurun_out/sweep_glv.log; exit 1; }
cat gpurun_out/sweep_glv.log
timeout -k 10 200 python3 tools/poseidon_bench.py 2>&1 | tail -8
