# Round evidence in one GPU session: gpu tests, smoke, full bench (with CPU baseline), rocprof
# kernel-trace stats + separate FETCH_SIZE / WRITE_SIZE passes.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -2 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "[$name] failed: stopping"; exit $rc; fi
}
run pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python3 bench.py
run prof/trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --config4-log-n 0
run prof/trace_extras 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace_extras -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
run prof/pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --config4-log-n 0
run prof/pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --config4-log-n 0
