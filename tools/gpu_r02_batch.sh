cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_msm_batch.py > gpurun_out/pytest_batch.log 2>&1
rc=$?; tail -8 gpurun_out/pytest_batch.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/table_bench.py 2>&1 | grep -v amdgpu.ids | tail -20
