# Round-3 probe: gpu tests, host-buffer MSM timings per piece count, and the kernel + memory-copy
# timeline of one host-fed MSM.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "[$name] failed: stopping"; exit $rc; fi
}
run pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run host_api 300 python3 tools/host_api_bench.py
run prof/hosttrace 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof/hosttrace -o run -- python3 tools/host_path_trace.py
