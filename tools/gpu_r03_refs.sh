# Round-3: sv_bn254_g1_msm_refs staging / gather variants, one process per env (the knobs are read once).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "host_path" > gpurun_out/rf_pytest.log 2>&1
rc=$?; echo "[pytest] rc=$rc"; tail -2 gpurun_out/rf_pytest.log; [ $rc -ne 0 ] && exit $rc
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 200 python3 tools/host_api_bench.py 20 "" > gpurun_out/rf_bench_$i.log 2>&1
  rc=$?; echo "[$envs] rc=$rc"; grep -E "host|refs" gpurun_out/rf_bench_$i.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
