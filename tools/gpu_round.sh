# Round evidence in one GPU session (TAG=rNN_final bash tools/gpu_round.sh): gpu tests, smoke, the
# full bench (CPU baseline + config-4 parity), rocprof kernel-trace stats (headline + extras),
# FETCH_SIZE / WRITE_SIZE passes, the FETCH calibration, and two SQ passes (VALU mix, wait cycles),
# each counter group in a run of its own.  Stops at the first failure.  Summary: gpurun_out/prof.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "[$name] failed: stopping"; exit $rc; fi
}
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --config4-log-n 0"
[ -n "$SKIP_TESTS" ] || run pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
[ -n "$SKIP_TESTS" ] || run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
[ -n "$SKIP_BENCH" ] || run bench 600 python3 bench.py
run prof/trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --config4-log-n 0
run prof/trace_extras 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace_extras -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
run prof/pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/pmc_fetch -o run -- python3 $B
run prof/pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/pmc_write -o run -- python3 $B
# the calibration binary is not uploaded (.gpurunignore): build it on the box
[ -x tools/calib_fetch ] || run build_calib 300 /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/calib_fetch.hip -o tools/calib_fetch
run prof/pmc_calib 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/pmc_calib -o run -- ./tools/calib_fetch
run prof/sq_valu 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/prof/sq_valu -o run -- python3 $B
run prof/sq_wait 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM --output-format csv -d gpurun_out/prof/sq_wait -o run -- python3 $B
python3 tools/summarize_profile.py gpurun_out/prof gpurun_out/prof ${TAG:-round} > gpurun_out/prof/summary.log 2>&1 || { tail -5 gpurun_out/prof/summary.log; exit 1; }
tail -3 gpurun_out/prof/summary.log
