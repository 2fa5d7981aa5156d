set -o pipefail
mkdir -p gpurun_out
for lib in libsvgpu_old.so libsvgpu.so libsvgpu_old.so libsvgpu.so; do
  SVGPU_LIB=snark-verifier-axiom_amd/build/$lib SWEEP_C=16 SWEEP_K=0 timeout -k 10 300 python tools/msm_sweep.py 20 > gpurun_out/ab.log 2>&1 || { cat gpurun_out/ab.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/ab.log)"
done
