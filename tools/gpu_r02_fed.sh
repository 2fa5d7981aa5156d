# Host-fed path with GLV pieces: parity tests, then the host-API timing against the device path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_host_path.py tests/test_gpu_threads.py tests/test_gpu_dist.py > gpurun_out/pytest_fed.log 2>&1 || { tail -30 gpurun_out/pytest_fed.log; exit 1; }
tail -1 gpurun_out/pytest_fed.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --config4-log-n 0 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms_per_step', round(d['ms_per_step'],4), d['breakdown_ms']); print(json.dumps(d['host_api'])[:400])"
