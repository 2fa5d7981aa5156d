# 2^20 A/B (three rounds, lean events): beta-x table vs whole phi(P) records vs no GLV.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/sweep_phi2.log
for r in 1 2 3; do
SVGPU_MSM_LEAN=1 timeout -k 10 200 python3 tools/msm_sweep_env.py 20 "SVGPU_GLV_PHI64=0" "SVGPU_GLV_PHI64=1" "SVGPU_GLV=0" >> gpurun_out/sweep_phi2.log 2>&1 || { tail -20 gpurun_out/sweep_phi2.log; exit 1; }
done
grep "2^" gpurun_out/sweep_phi2.log
