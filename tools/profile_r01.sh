# rocprofv3 kernel-trace stats + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of bench.py.
# trace = the headline command without the next-row extras (its k_accumulate average is the one
# bench.py's roofline uses); trace_extras = bench.py with the batch-MSM / config-5 / Poseidon lines.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/prof/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -3 "gpurun_out/prof/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
step trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --config4-log-n 0
step trace_extras 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace_extras -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --config4-log-n 0
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --config4-log-n 0
find gpurun_out/prof -name "*.csv" | head -20
