#!/bin/bash
# round 4: VALU rate microbenchmark + the decider / create_proof / batch / thread GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench_f64 > gpurun_out/ubench_f64.log 2>&1 || exit $?
cat gpurun_out/ubench_f64.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_decider.py tests/test_gpu_msm_batch.py tests/test_gpu_threads.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04_a.log 2>&1
rc=$?
tail -15 gpurun_out/r04_a.log
exit $rc
