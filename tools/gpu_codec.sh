set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_codec.py -x -q > gpurun_out/codec_pytest.log 2>&1
rc=$?; tail -30 gpurun_out/codec_pytest.log; exit $rc
