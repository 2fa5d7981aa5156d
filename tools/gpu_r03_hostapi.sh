# Round-3: host-path gpu tests, then tools/host_api_bench.py over the given piece specs.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "host_path or config4" > gpurun_out/ha_pytest.log 2>&1
rc=$?; echo "[pytest] rc=$rc"; tail -2 gpurun_out/ha_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python3 tools/host_api_bench.py 20 "$@" > gpurun_out/ha_bench.log 2>&1
rc=$?; echo "[host_api_bench] rc=$rc"; cat gpurun_out/ha_bench.log | grep -v amdgpu.ids; exit $rc
