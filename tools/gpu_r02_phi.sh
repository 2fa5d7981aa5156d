# GLV table layout and accumulate chunk A/B at 2^20 (lean events), parity of the variants included.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SVGPU_GLV_PHI64=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_msm.py -k "glv or edge or 1048576" > gpurun_out/pytest_phi.log 2>&1 || { tail -30 gpurun_out/pytest_phi.log; exit 1; }
tail -1 gpurun_out/pytest_phi.log
SVGPU_MSM_LEAN=1 timeout -k 10 300 python3 tools/msm_sweep_env.py 20 "SVGPU_GLV_PHI64=0" "SVGPU_GLV_PHI64=1" "SVGPU_ACC_K=32" "SVGPU_ACC_K=128" "SVGPU_GLV_PHI64=1,SVGPU_ACC_K=32" > gpurun_out/sweep_phi.log 2>&1 || { tail -20 gpurun_out/sweep_phi.log; exit 1; }
grep "2^" gpurun_out/sweep_phi.log
