# rocprofv3 kernel-trace stats of the headline bench command (no extras); prints the top kernels.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --config4-log-n 0 > gpurun_out/prof/trace.log 2>&1 || { tail -20 gpurun_out/prof/trace.log; exit 1; }
tail -1 gpurun_out/prof/trace.log | cut -c1-300
f=$(find gpurun_out/prof/trace -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv,sys
for r in list(csv.DictReader(open('$f')))[:20]: print('%-60s %5s %10.1f' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
"
