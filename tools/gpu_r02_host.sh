cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_host_path.py tests/test_gpu_decider.py tests/test_gpu_codec.py tests/test_gpu_poseidon.py tests/test_gpu_msm_batch.py > gpurun_out/pytest_host.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_host.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u tools/host_api_bench.py 20 2>&1 | grep -v amdgpu.ids
