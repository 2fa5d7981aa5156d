# round 6: host-fed piece schedules re-swept after the faster accumulate; decider per-op ubench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06d
timeout -k 10 400 python3 tools/host_api_bench.py 20 "" "SVGPU_H2D_SPLIT=5,5,4,2" "SVGPU_H2D_SPLIT=6,5,4,1" "SVGPU_H2D_SPLIT=5,4,4,2,1" "SVGPU_H2D_SPLIT=6,5,3,2" "SVGPU_H2D_SPLIT=4,4,4,4" "SVGPU_H2D_SPLIT=6,5,5" "" "SVGPU_H2D_SPLIT=5,5,4,2" "SVGPU_H2D_SPLIT=6,5,4,1" > gpurun_out/r06d/host_sweep.log 2>&1 || { tail -20 gpurun_out/r06d/host_sweep.log; exit 1; }
cat gpurun_out/r06d/host_sweep.log | grep -v amdgpu.ids
timeout -k 10 120 ./tools/bin/ubench_wg > gpurun_out/r06d/ubench_wg.log 2>&1 || { tail -5 gpurun_out/r06d/ubench_wg.log; exit 1; }
cat gpurun_out/r06d/ubench_wg.log
