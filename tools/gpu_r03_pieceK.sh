# Best accumulate chunk length K for host-fed piece sizes (device-resident MSMs of the piece sizes
# with the 2^20 plan's window: c = 16, GLV), accumulate + fixup times.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp SVGPU_MSM_STATS=1 SVGPU_GLV=1 SVGPU_WINDOW_BITS=16
mkdir -p gpurun_out
for n in 65536 131072 196608 262144 349525; do
  timeout -k 10 200 python3 tools/msm_sweep_env.py n=$n 'SVGPU_ACC_K=6' 'SVGPU_ACC_K=8' 'SVGPU_ACC_K=12' 'SVGPU_ACC_K=16' 'SVGPU_ACC_K=21' 'SVGPU_ACC_K=24' 'SVGPU_ACC_K=32' 'SVGPU_ACC_K=42' > gpurun_out/pieceK_$n.log 2>&1 || exit 1
done
tail -n 8 gpurun_out/pieceK_*.log
