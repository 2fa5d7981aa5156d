#!/bin/bash
# round 4: window-split MSM pipeline -- parity, then A/B of SVGPU_MSM_SPLIT on bench.py's MSM line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_config4.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_split_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r04_split_tests.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for sp in 0 1; do
    SVGPU_MSM_SPLIT=$sp timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --config4-log-n 0 --steps 40 > gpurun_out/r04_split_$sp.$i.json 2>gpurun_out/r04_split_$sp.$i.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/r04_split_$sp.$i.json'));print('split=$sp', round(d['ms_per_step'],4), d['breakdown_ms'], round(d['int_mac']['kernel_frac'],3), d['roofline']['kernel_avg_ms'])"
  done
done
