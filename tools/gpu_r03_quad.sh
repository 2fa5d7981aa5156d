# Quad-split group sums (k_group_sum_q) vs the per-lane tree (k_group_sum): parity + timing.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_msm.py tests/test_gpu_host_path.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_quad.log 2>&1 || { tail -30 gpurun_out/pytest_quad.log; exit 1; }
tail -2 gpurun_out/pytest_quad.log
SVGPU_MSM_STATS=1 timeout -k 10 200 python3 tools/msm_sweep_env.py 20 'SVGPU_GROUP_QUAD=0' 'SVGPU_GROUP_QUAD=1' 'SVGPU_GROUP_QUAD=1,SVGPU_GROUP_P=1' 'SVGPU_GROUP_QUAD=1,SVGPU_GROUP_P=4' 'SVGPU_GROUP_QUAD=1,SVGPU_GROUP_P=3' > gpurun_out/quad_sweep.log 2>&1 || exit 1
cat gpurun_out/quad_sweep.log
