# A/B of the baseline library (build/libsvgpu_old.so) vs the current build on the 2^20 MSM, after
# the MSM parity tests on the current build.  Usage: bash tools/gpu_ab.sh [log_n]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
LOGN=${1:-20}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batch.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || { tail -30 gpurun_out/pytest_ab.log; exit 1; }
tail -1 gpurun_out/pytest_ab.log
for lib in libsvgpu_old.so libsvgpu.so libsvgpu_old.so libsvgpu.so; do
  SVGPU_LIB=snark-verifier-axiom_amd/build/$lib SWEEP_C=16 SWEEP_K=0 timeout -k 10 300 python3 tools/msm_sweep.py $LOGN > gpurun_out/ab.log 2>&1 || { cat gpurun_out/ab.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/ab.log)"
done
