# Kernel + memory-copy timeline of the host-buffer MSM's piece pipeline (no counters).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof/hosttrace -o run -- python3 tools/host_path_trace.py > gpurun_out/prof/hosttrace.log 2>&1 || { tail -5 gpurun_out/prof/hosttrace.log; exit 1; }
ls gpurun_out/prof/hosttrace
