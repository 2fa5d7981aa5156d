# round 6: decider A/B on one box, interleaved: pre-round-6 ops / conj folded / + a^2, a^3 reuse
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06f
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_decider.py > gpurun_out/r06f/pytest.log 2>&1 || { tail -30 gpurun_out/r06f/pytest.log; exit 1; }
tail -1 gpurun_out/r06f/pytest.log
for i in 1 2 3; do
  SVGPU_LIB=snark-verifier-axiom_amd/build_ab/libsvgpu_oldec.so timeout -k 10 300 python3 tools/decider_bench.py 256 2>&1 | grep decide
  SVGPU_LIB=snark-verifier-axiom_amd/build_ab/libsvgpu_dec1.so timeout -k 10 300 python3 tools/decider_bench.py 256 2>&1 | grep decide
  timeout -k 10 300 python3 tools/decider_bench.py 256 2>&1 | grep decide
done > gpurun_out/r06f/dec_ab2.log 2>&1
cat gpurun_out/r06f/dec_ab2.log
