# Round 6: per-kernel times of the reduction at L = 4 (default) and L = 2 (SVGPU_RED_LOG=1)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06j
for rl in 2 1; do
  SVGPU_RED_LOG=$rl SWEEP_ROUNDS=1 SWEEP_REPS=20 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/r06j/rl$rl -o run -- python3 tools/msm_sweep_env.py 20 '' > gpurun_out/r06j/rl$rl.log 2>&1 || exit 1
  f=$(find gpurun_out/r06j/rl$rl -name '*kernel_stats.csv' | head -1)
  echo "== RED_LOG=$rl"; grep -v amdgpu gpurun_out/r06j/rl$rl.log | tail -1
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:12]:
    print('%-40s %6s %10.1f us' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3))
"
done
