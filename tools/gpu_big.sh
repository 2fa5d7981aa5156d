set -o pipefail
mkdir -p gpurun_out
SWEEP_C=16 SWEEP_K=0 timeout -k 10 300 python tools/msm_sweep.py 22,24 > gpurun_out/big_sweep.log 2>&1; rc=$?
cat gpurun_out/big_sweep.log; exit $rc
