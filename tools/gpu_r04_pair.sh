#!/bin/bash
# round 4: two Miller steps per Fq12 product in k_decide_wg -- parity, then A/B of SVGPU_DECIDER_PAIR
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_decider.py tests/test_gpu_codec.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_pair_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04_pair_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for pr in 0 1; do
    SVGPU_DECIDER_PAIR=$pr timeout -k 10 120 python3 tools/decider_bench.py 256 2>&1 | tail -1 | sed "s/^/pair=$pr /" || exit 1
  done
done
