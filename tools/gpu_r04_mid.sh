# Round-4 mid-round check in one GPU session: every gpu test, smoke, the full bench line.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "[$name] failed: stopping"; exit $rc; fi
}
run r04_pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run r04_smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
run r04_bench 600 python3 bench.py
