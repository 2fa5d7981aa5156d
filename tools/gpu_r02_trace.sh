# Kernel trace (timestamps) of the headline MSM steps: per-kernel durations and inter-kernel gaps.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/r02trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --config4-log-n 0 > gpurun_out/prof/r02trace.log 2>&1 || { tail -20 gpurun_out/prof/r02trace.log; exit 1; }
python3 tools/trace_gaps.py gpurun_out/prof/r02trace
