# Round 6: re-sweep of the reduction segment length and the accumulate chunk after the accumulate changes
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/msm_sweep_env.py 20 '' 'SVGPU_RED_LOG=1' 'SVGPU_RED_LOG=3' 'SVGPU_ACC_K=48' 'SVGPU_ACC_K=96' 'SVGPU_ACC_K=128' > gpurun_out/r06g_sweep.log 2>&1
rc=$?; cat gpurun_out/r06g_sweep.log; exit $rc
