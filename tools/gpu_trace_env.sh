# rocprofv3 kernel-trace stats of the headline bench (no extras) under each env spec given
# (e.g. SVGPU_RED_LOG=2); prints the MSM kernels' average durations per spec.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_env
i=0
for spec in "$@"; do
  i=$((i+1))
  env $(echo "$spec" | tr ',' ' ') timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_env/t$i -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --config4-log-n 0 > gpurun_out/prof_env/t$i.log 2>&1 || { tail -5 gpurun_out/prof_env/t$i.log; exit 1; }
  f=$(find gpurun_out/prof_env/t$i -name "*kernel_stats.csv" | head -1)
  echo "== $spec"
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    n=r['Name']
    if any(k in n for k in ('k_wsum','k_group_sum','k_fixup','k_accumulate','k_fine','k_bin')): print('  %-40s %8.1f us' % (n.split('(')[0][:40], float(r['AverageNs'])/1e3))
"
done
