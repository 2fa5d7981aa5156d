# Interleaved A/B of two builds of libsvgpu.so on the 2^20 MSM: A = build/, B = build_ab/ (same
# sources, different compile flags).  Usage: bash tools/gpu_ab_lib.sh ROUNDS [extra sweep specs]
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=${1:-3}
for r in $(seq 1 $R); do
  echo "== round $r A (build/)"
  SWEEP_ROUNDS=1 SWEEP_REPS=21 timeout -k 10 120 python3 -u tools/msm_sweep_env.py 20 '' || exit 1
  echo "== round $r B (build_ab/)"
  SVGPU_LIB=snark-verifier-axiom_amd/build_ab/libsvgpu.so SWEEP_ROUNDS=1 SWEEP_REPS=21 timeout -k 10 120 python3 -u tools/msm_sweep_env.py 20 '' || exit 1
done
