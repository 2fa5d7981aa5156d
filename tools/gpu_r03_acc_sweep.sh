# k_accumulate efficiency vs piece size: device-resident MSMs at 2^18 / 2^19 / 2^20 with the
# 2^20 plan's window (c = 16, GLV) and several chunk lengths K (entries per thread).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
export SVGPU_MSM_STATS=1 SVGPU_GLV=1 SVGPU_WINDOW_BITS=16
timeout -k 10 200 python3 tools/msm_sweep_env.py 20 'SVGPU_ACC_K=64' 'SVGPU_ACC_K=32' 'SVGPU_ACC_K=128' > gpurun_out/acc_sweep20.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/msm_sweep_env.py 19 'SVGPU_ACC_K=32' 'SVGPU_ACC_K=16' 'SVGPU_ACC_K=64' 'SVGPU_ACC_K=128' > gpurun_out/acc_sweep19.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/msm_sweep_env.py 18 'SVGPU_ACC_K=16' 'SVGPU_ACC_K=8' 'SVGPU_ACC_K=32' 'SVGPU_ACC_K=64' 'SVGPU_ACC_K=128' > gpurun_out/acc_sweep18.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/msm_sweep_env.py 17 'SVGPU_ACC_K=8' 'SVGPU_ACC_K=16' 'SVGPU_ACC_K=32' 'SVGPU_ACC_K=64' > gpurun_out/acc_sweep17.log 2>&1 || exit 1
tail -n 8 gpurun_out/acc_sweep*.log
