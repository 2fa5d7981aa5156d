#!/bin/bash
# round 4: k_wsum_tree's running sums on the 29-bit chain (bucket sums read in their stored form) --
# MSM parity, then A/B against the previous library (abtmp/prev) on the 2^20 step
set -o pipefail
mkdir -p gpurun_out
T="tests/test_gpu_msm.py tests/test_gpu_host_path.py tests/test_gpu_msm_config4.py"
timeout -k 10 500 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_wsum29_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04_wsum29_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for v in new prev; do
    unset SVGPU_LIB
    [ $v = prev ] && export SVGPU_LIB=$PWD/abtmp/prev/libsvgpu.so
    timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --config4-log-n 0 --steps 40 > gpurun_out/r04_wsum29_$v.$i.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/r04_wsum29_$v.$i.json'));print('$v', round(d['ms_per_step'],4), d['breakdown_ms'])"
  done
done
