set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batch.py tests/test_gpu_decider.py -x -q > gpurun_out/msm_pytest.log 2>&1 || { tail -30 gpurun_out/msm_pytest.log; exit 1; }
tail -2 gpurun_out/msm_pytest.log
SWEEP_C=16 SWEEP_K=0 timeout -k 10 300 python tools/msm_sweep.py 20,22,24 > gpurun_out/big_sweep.log 2>&1; rc=$?
cat gpurun_out/big_sweep.log; exit $rc
