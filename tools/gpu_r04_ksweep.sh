#!/bin/bash
# round 4: k_accumulate chunk length K at 2^20 (146 VGPRs -> 3 waves/SIMD -> 768 resident 256-thread
# blocks; K = 64 launches 1024 blocks = 1.33 rounds)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for K in 64 86 88 96 112 128; do
    SVGPU_ACC_K=$K timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --config4-log-n 0 --steps 40 > gpurun_out/r04_k_$K.$i.json 2>gpurun_out/r04_k_$K.$i.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/r04_k_$K.$i.json'));print('K=$K', round(d['ms_per_step'],4), d['breakdown_ms'])"
  done
done
