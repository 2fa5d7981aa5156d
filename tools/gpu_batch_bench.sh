set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/batch_bench.py > gpurun_out/batch_bench.log 2>&1
rc=$?; cat gpurun_out/batch_bench.log; exit $rc
