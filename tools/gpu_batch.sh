set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python tools/batch_bench.py > gpurun_out/batch_bench.log 2>&1 && \
timeout -k 10 300 python tools/decider_bench.py > gpurun_out/decider_bench.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; cat gpurun_out/batch_bench.log; tail -8 gpurun_out/decider_bench.log; exit $rc
