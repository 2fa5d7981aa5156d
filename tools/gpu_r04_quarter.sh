#!/bin/bash
# round 4: is the host-fed quarter piece's accumulate (0.43-0.45 ms, fed trace r03) slow because of the
# piece size (occupancy) or because of the fed path (ADD mode)?  Device-resident 2^18 points over the
# 2^20 plan's buckets (c = 16, GLV), K = 32 (the piece K) and 16, plus the new decider Gt test.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_decider.py -x -q --timeout 120 --timeout-method thread -k "h2c or halo2curves" > gpurun_out/r04_q_test.log 2>&1; rc=$?; tail -2 gpurun_out/r04_q_test.log; [ $rc -ne 0 ] && exit $rc
for K in 32 16 64; do
  SVGPU_WINDOW_BITS=16 SVGPU_ACC_K=$K timeout -k 10 200 python bench.py --log-n 18 --no-extras --no-cpu-baseline --config4-log-n 0 --steps 40 > gpurun_out/r04_q_$K.json 2>gpurun_out/r04_q_$K.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r04_q_$K.json'));print('2^18 c=16 K=$K', round(d['ms_per_step'],4), d['breakdown_ms'])"
done
