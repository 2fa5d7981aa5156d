# Round-2: new GPU tests (threads, field edges, config 4, batch) then the whole gpu suite.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_field_edges.py tests/test_gpu_threads.py tests/test_gpu_msm_batch.py tests/test_gpu_msm_config4.py \
  > gpurun_out/pytest_new.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; exit $rc
