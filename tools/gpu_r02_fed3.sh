# Host-fed path with the automatic piece count: parity tests, host-API timings, bench host_api row.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_host_path.py tests/test_gpu_threads.py > gpurun_out/pytest_fed3.log 2>&1 || { tail -30 gpurun_out/pytest_fed3.log; exit 1; }
tail -1 gpurun_out/pytest_fed3.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --config4-log-n 0 2>/dev/null > gpurun_out/bench_fed3.log
python3 -c "import json; d=json.loads(open('gpurun_out/bench_fed3.log').read().strip().splitlines()[-1]); print('ms_per_step', round(d['ms_per_step'],4)); print(json.dumps(d['host_api'])[:300]); print('cfg5', d['config5_aggregation']['latency_ms'], 'pos', d['poseidon']['ms'])"
