set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_decider.py tests/test_gpu_codec.py -x -q > gpurun_out/dec_pytest.log 2>&1 || { tail -30 gpurun_out/dec_pytest.log; exit 1; }
tail -1 gpurun_out/dec_pytest.log
timeout -k 10 300 python tools/decider_bench.py > gpurun_out/dec_bench.log 2>&1; rc=$?; cat gpurun_out/dec_bench.log | grep -v amdgpu.ids; exit $rc
