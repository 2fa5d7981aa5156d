#!/bin/bash
# round 4: VALU rate microbenchmark + the decider / create_proof GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench_f64 > gpurun_out/ubench_f64.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_decider.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04_decider.log 2>&1
rc=$?
tail -5 gpurun_out/r04_decider.log
cat gpurun_out/ubench_f64.log
exit $rc
