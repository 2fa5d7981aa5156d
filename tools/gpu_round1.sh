# One GPU session: gpu tests, smoke, bench.  Stops at the first crash/timeout (rc >= 124).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -4 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "[$name] crashed/timed out: stopping"; exit $rc; fi
  return 0
}
run pytest_gpu 900 python3 -m pytest tests -q -m gpu
run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python3 bench.py
