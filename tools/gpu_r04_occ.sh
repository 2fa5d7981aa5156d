#!/bin/bash
# round 4: k_accumulate at 4 waves/SIMD (128 VGPRs, 11 spilled) vs the default 3 (146 VGPRs)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in default occ4; do
    if [ $v = occ4 ]; then export SVGPU_LIB=$PWD/abtmp/occ4/libsvgpu.so; else unset SVGPU_LIB; fi
    timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --config4-log-n 0 --steps 40 > gpurun_out/r04_occ_$v.$i.json 2>gpurun_out/r04_occ_$v.$i.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/r04_occ_$v.$i.json'));print('$v', round(d['ms_per_step'],4), d['breakdown_ms'], d.get('host_api',{}).get('msm_host_ms'))"
  done
done
