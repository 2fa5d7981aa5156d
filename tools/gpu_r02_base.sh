# Round-2 baseline: gpu tests, bench (N=1), and an N=2 gloo rehearsal on one card.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "[$name] failed: stopping"; exit $rc; fi
}
run pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run bench 600 python3 bench.py
SVGPU_DIST_BACKEND=gloo run bench_n2 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2
