# sweep the running-sum segment length of the MSM bucket reduction (SVGPU_RED_LOG) at 2^20 and 2^24
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_msm.py -x -q --timeout 120 --timeout-method thread -k "random_sizes or window_bits or full_size" > gpurun_out/t.log 2>&1 || { tail -5 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for lg in 1 2 3 4 5; do
  SVGPU_RED_LOG=$lg timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-extras --steps 20 > gpurun_out/b$lg.log 2>&1 || { tail -3 gpurun_out/b$lg.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/b$lg.log').read().strip().splitlines()[-1]);print('logL=$lg', round(d['ms_per_step'],3), d['breakdown_ms'], round(d['config4_msm_2_24']['ms_per_msm'],2))"
done
