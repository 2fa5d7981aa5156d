cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 -u tools/decider_bench.py 256 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 python3 -u tools/decider_bench.py 1 2>&1 | grep -v amdgpu.ids | tail -2
SVGPU_DECIDER_LANES=48 timeout -k 10 120 python3 -u tools/decider_bench.py 256 2>&1 | grep -v amdgpu.ids | tail -2
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_decider.py tests/test_gpu_threads.py tests/test_gpu_codec.py > gpurun_out/pytest_dec.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_dec.log; exit $rc
