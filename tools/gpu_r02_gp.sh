# 2^20 group-sum split A/B (lean events).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SVGPU_MSM_STATS=1 timeout -k 10 200 python3 tools/msm_sweep_env.py 20 "SVGPU_GROUP_P=1" "SVGPU_GROUP_P=2" "SVGPU_GROUP_P=3" "SVGPU_GROUP_P=4" > gpurun_out/sweep_gp.log 2>&1 || { tail -20 gpurun_out/sweep_gp.log; exit 1; }
grep "2^" gpurun_out/sweep_gp.log
