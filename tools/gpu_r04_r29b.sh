#!/bin/bash
# round 4: r29w readers' conversion in 32-bit arithmetic -- MSM parity, step, and a K re-sweep at
# 4 waves/SIMD (SVGPU_ACC_K)
set -o pipefail
mkdir -p gpurun_out
T="tests/test_gpu_msm.py tests/test_gpu_host_path.py"
timeout -k 10 400 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_r29b_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04_r29b_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for k in 64 48 80; do
    SVGPU_ACC_K=$k timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --config4-log-n 0 --steps 40 > gpurun_out/r04_r29b_$k.$i.json 2>gpurun_out/r04_r29b_$k.$i.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/r04_r29b_$k.$i.json'));print('K=$k', round(d['ms_per_step'],4), d['breakdown_ms'])"
  done
done
