# Round 6: where the decider's LDS bank conflicts are: the wide prologue (LDS scratch) vs the old one
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06k
for w in 1 0; do
  SVGPU_DECIDER_WIDE=$w timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU --output-format csv \
    -d gpurun_out/r06k/w$w -o run -- python3 tools/decider_bench.py > gpurun_out/r06k/w$w.log 2>&1 || exit 1
  f=$(find gpurun_out/r06k/w$w -name '*counter_collection.csv' | head -1)
  echo "== WIDE=$w"; grep decide gpurun_out/r06k/w$w.log | tail -1
  python3 -c "
import csv,collections
s=collections.defaultdict(float); n=collections.Counter()
for r in csv.DictReader(open('$f')):
    if 'k_decide_wg' in r['Kernel_Name']:
        s[r['Counter_Name']]+=float(r['Counter_Value']); n[r['Counter_Name']]+=1
for k in s: print(k, s[k]/max(1,n[k]/1), n[k])
"
done
