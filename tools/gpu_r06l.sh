# Round 6: kernel + copy timeline of the host-fed 2^20 MSM (the tail after the last byte)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06l
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r06l/tr -o run -- python3 tools/host_path_trace.py > gpurun_out/r06l/run.log 2>&1 || exit 1
d=$(dirname $(find gpurun_out/r06l/tr -name 'run_kernel_trace.csv' | head -1))
python3 tools/trace_timeline.py $d -5 > gpurun_out/r06l/timeline.txt
cat gpurun_out/r06l/timeline.txt
