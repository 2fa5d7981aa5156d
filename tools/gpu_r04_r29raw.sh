#!/bin/bash
# round 4 probe: is k_accumulate's 29-bit chain held back by its segment-end conversions (run by the
# whole wave whenever one lane ends a segment)?  abtmp/raw stores the raw limbs instead (wrong sums,
# timing only) -- A/B against the converting default and the 32-bit chain
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in r29 raw r32; do
    unset SVGPU_LIB SVGPU_ACC_R29
    [ $v = raw ] && export SVGPU_LIB=$PWD/abtmp/raw/libsvgpu.so
    [ $v = r32 ] && export SVGPU_ACC_R29=0
    timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --config4-log-n 0 --steps 40 > gpurun_out/r04_raw_$v.$i.json 2>gpurun_out/r04_raw_$v.$i.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/r04_raw_$v.$i.json'));print('$v', round(d['ms_per_step'],4), d['breakdown_ms'])"
  done
done
