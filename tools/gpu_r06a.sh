cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06a
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_decider.py tests/test_gpu_msm_batch.py > gpurun_out/r06a/pytest.log 2>&1 || { tail -30 gpurun_out/r06a/pytest.log; exit 1; }
tail -3 gpurun_out/r06a/pytest.log
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --config4-log-n 0 > gpurun_out/r06a/bench.json 2> gpurun_out/r06a/bench.err || { tail -20 gpurun_out/r06a/bench.err; exit 1; }
echo bench ok
SVGPU_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/r06a/bench_n2.json 2> gpurun_out/r06a/bench_n2.err || { tail -20 gpurun_out/r06a/bench_n2.err; exit 1; }
echo n2 ok
