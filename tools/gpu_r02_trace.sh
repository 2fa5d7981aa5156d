# Kernel timeline of the 2^20 bench step (per-kernel durations and idle gaps).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras --config4-log-n 0 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms_per_step', round(d['ms_per_step'],4), d['breakdown_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof/msmtrace -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-extras --config4-log-n 0 > gpurun_out/prof/msmtrace.log 2>&1 || { tail -5 gpurun_out/prof/msmtrace.log; exit 1; }
python3 tools/trace_gaps.py gpurun_out/prof/msmtrace | tail -22
