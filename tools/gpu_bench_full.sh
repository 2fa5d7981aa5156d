set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log
SVGPU_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/bench_n2.log 2>&1 || { tail -20 gpurun_out/bench_n2.log; exit 1; }
tail -1 gpurun_out/bench_n2.log
