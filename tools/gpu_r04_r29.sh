#!/bin/bash
# round 4: k_accumulate's chain over 9 x 29-bit limbs (curve29.hpp, 125 VGPRs = 4 waves/SIMD, bucket
# sums stored as x R' words and converted by their readers) -- MSM parity (both chains), then A/B
# against the 32-bit chain (SVGPU_ACC_R29=0) on the bench's 2^20 step
set -o pipefail
mkdir -p gpurun_out
T="tests/test_gpu_msm.py tests/test_gpu_host_path.py tests/test_gpu_msm_config4.py"
timeout -k 10 500 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_r29_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04_r29_tests.log; [ $rc -ne 0 ] && exit $rc
SVGPU_ACC_R29=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_host_path.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_r32_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04_r32_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for v in 1 0; do
    SVGPU_ACC_R29=$v timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --config4-log-n 0 --steps 40 > gpurun_out/r04_r29_$v.$i.json 2>gpurun_out/r04_r29_$v.$i.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/r04_r29_$v.$i.json'));print('r29=$v', round(d['ms_per_step'],4), d['breakdown_ms'])"
  done
done
