# round 6: decider A/B on one box -- previous build (copy/conj ops) vs current, interleaved
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06f
for i in 1 2 3; do
  SVGPU_LIB=snark-verifier-axiom_amd/build_ab/libsvgpu_oldec.so timeout -k 10 300 python3 tools/decider_bench.py 256 2>&1 | grep decide
  timeout -k 10 300 python3 tools/decider_bench.py 256 2>&1 | grep decide
done > gpurun_out/r06f/dec_ab.log 2>&1
cat gpurun_out/r06f/dec_ab.log
