# Round-3 iteration: MSM gpu tests, then A/B bench lines (SVGPU_* env per line) on the headline.
# Usage: bash tools/gpu_r03_iter.sh "<pytest -k expr or empty>" "ENV=.. ENV=.." "ENV=.." ...
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
sel=$1; shift
if [ -n "$sel" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$sel" > gpurun_out/iter_pytest.log 2>&1
  rc=$?; echo "[pytest] rc=$rc"; tail -3 gpurun_out/iter_pytest.log
  [ $rc -ne 0 ] && exit $rc
fi
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras --config4-log-n 0 > gpurun_out/iter_bench_$i.log 2>&1
  rc=$?
  echo "[bench $i: $envs] rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/iter_bench_$i.log; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/iter_bench_$i.log').read().strip().splitlines()[-1]); print(' ms/step %.4f' % d['ms_per_step'], d.get('breakdown_ms'), 'dec %.4f' % d['kzg']['kernel_ms'])"
done
