#!/bin/bash
# round 4: host-fed call with piece 0's scalars staged by the calling thread, the 29-bit table's
# beta x computed in its own form -- parity, the piece-schedule sweep, the 2^20 step
set -o pipefail
mkdir -p gpurun_out
T="tests/test_gpu_msm.py tests/test_gpu_host_path.py tests/test_gpu_threads.py"
timeout -k 10 400 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_fed.log 2>&1; rc=$?; tail -2 gpurun_out/r04_fed.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/host_api_bench.py 20 "" "SVGPU_H2D_SPLIT=5,5,4,2" "SVGPU_H2D_SPLIT=4,4,4,3,1" "SVGPU_H2D_SPLIT=5,4,4,3" "SVGPU_H2D_SPLIT=6,5,3,2" "SVGPU_H2D_SPLIT=5,5,5,1" "SVGPU_H2D_SPLIT=3,4,4,3,2" "" 2>&1 | grep -v amdgpu.ids || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --config4-log-n 0 --steps 40 > gpurun_out/r04_fed_b.$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r04_fed_b.$i.json'));print('step', round(d['ms_per_step'],4), d['breakdown_ms'])"
done
