set -o pipefail
mkdir -p gpurun_out
for ph in 1 2 3; do
  SVGPU_DECIDER_PHASES=$ph timeout -k 10 300 python tools/decider_bench.py > gpurun_out/dec_ph$ph.log 2>&1 || { tail -5 gpurun_out/dec_ph$ph.log; exit 1; }
  echo "phases=$ph $(tail -1 gpurun_out/dec_ph$ph.log)"
done
