# round 6: decider without copy/conjugation ops -- decider GPU tests, kernel timing
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06e
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_decider.py tests/test_gpu_threads.py > gpurun_out/r06e/pytest.log 2>&1 || { tail -30 gpurun_out/r06e/pytest.log; exit 1; }
tail -2 gpurun_out/r06e/pytest.log
timeout -k 10 300 python3 tools/decider_bench.py 256 > gpurun_out/r06e/dec.log 2>&1 || { tail -5 gpurun_out/r06e/dec.log; exit 1; }
timeout -k 10 300 python3 tools/decider_bench.py 256 >> gpurun_out/r06e/dec.log 2>&1 || { tail -5 gpurun_out/r06e/dec.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06e/dec.log
