set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_poseidon.py -x -q > gpurun_out/poseidon_pytest.log 2>&1 && \
timeout -k 10 200 python tools/poseidon_bench.py > gpurun_out/poseidon_bench.log 2>&1
rc=$?; tail -20 gpurun_out/poseidon_pytest.log; cat gpurun_out/poseidon_bench.log; exit $rc
