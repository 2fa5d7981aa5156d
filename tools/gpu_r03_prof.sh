# Round-3: MSM gpu tests, rocprof kernel stats of the headline bench, then A/B bench lines.
# Usage: bash tools/gpu_r03_prof.sh "<pytest -k expr or empty>" "ENV=.." ...
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
sel=$1; shift
if [ -n "$sel" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$sel" > gpurun_out/iter_pytest.log 2>&1
  rc=$?; echo "[pytest] rc=$rc"; tail -3 gpurun_out/iter_pytest.log
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/iter -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --config4-log-n 0 > gpurun_out/iter_prof.log 2>&1
rc=$?; echo "[rocprof] rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/iter_prof.log; exit $rc; }
f=$(ls gpurun_out/prof/iter/*kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:16]: print('%-40s %6s %10.1f us' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3))"
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras --config4-log-n 0 > gpurun_out/iter_bench_$i.log 2>&1
  rc=$?
  echo "[bench $i: $envs] rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/iter_bench_$i.log; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/iter_bench_$i.log').read().strip().splitlines()[-1]); print(' ms/step %.4f' % d['ms_per_step'], d.get('breakdown_ms'), 'dec %.4f' % d['kzg']['kernel_ms'])"
done
