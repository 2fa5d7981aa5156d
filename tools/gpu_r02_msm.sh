# MSM parity (all MSM test files) + headline bench line (no extras) + kernel timeline.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_host_path.py tests/test_gpu_msm_config4.py tests/test_gpu_threads.py > gpurun_out/pytest_msm.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_msm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras --config4-log-n 0 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms_per_step', round(d['ms_per_step'],4), d['breakdown_ms'])"
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof/msmtrace -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-extras --config4-log-n 0 > gpurun_out/prof/msmtrace.log 2>&1 || { tail -5 gpurun_out/prof/msmtrace.log; exit 1; }
python3 tools/trace_gaps.py gpurun_out/prof/msmtrace | tail -16
