set -o pipefail
mkdir -p gpurun_out
for c in 14 15 16; do for k in 16 32 64; do
  SVGPU_WINDOW_BITS=$c SVGPU_ACC_K=$k timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --steps 20 > gpurun_out/bench_c${c}_k$k.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_c${c}_k$k.log').read().strip().splitlines()[-1]); print('c=$c K=$k', round(d['ms_per_step'],4), d['breakdown_ms'])"
done; done
