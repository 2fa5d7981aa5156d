# Time the 2^LOG_N MSM with each library given (alternating, two rounds); every result checked equal.
# Usage: bash tools/gpu_abn.sh LOG_N lib1.so lib2.so ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
LOGN=$1; shift
for r in 1 2; do
  for lib in "$@"; do
    SVGPU_LIB=$lib timeout -k 10 300 python3 tools/msm_sweep_env.py $LOGN SVGPU_GLV=0 > gpurun_out/abn.log 2>&1 || { cat gpurun_out/abn.log; exit 1; }
    echo "$(basename $lib) $(grep '2^' gpurun_out/abn.log | tail -1)"
  done
done
