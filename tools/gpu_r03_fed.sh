# Host-fed MSM pipeline: parity tests, schedule timings, kernel + copy timeline of one call.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "[$name] failed: stopping"; exit $rc; fi
}
run pytest_fed 400 python3 -u -m pytest tests/test_gpu_host_path.py tests/test_gpu_msm.py -x -q --timeout 120 --timeout-method thread
run host_api 300 python3 tools/host_api_bench.py 20 ${FED_SPECS}
run prof/hosttrace 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof/hosttrace -o run -- python3 tools/host_path_trace.py
python3 tools/trace_timeline.py gpurun_out/prof/hosttrace -5 > gpurun_out/tl_arrays.txt; python3 tools/trace_timeline.py gpurun_out/prof/hosttrace -1 > gpurun_out/tl_refs.txt
cat gpurun_out/host_api.log
