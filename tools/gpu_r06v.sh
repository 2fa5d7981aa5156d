# Round 6: VALU instructions of k_accumulate in two builds (A = build/, B = build_ab/), one SQ pass each
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06v
for v in A B; do
  if [ $v = B ]; then export SVGPU_LIB=snark-verifier-axiom_amd/build_ab/libsvgpu.so; fi
  SWEEP_ROUNDS=1 SWEEP_REPS=3 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv \
    -d gpurun_out/r06v/$v -o run -- python3 tools/msm_sweep_env.py 20 '' > gpurun_out/r06v/$v.log 2>&1 || exit 1
  f=$(find gpurun_out/r06v/$v -name '*counter_collection.csv' | head -1)
  python3 -c "
import csv,collections
s=collections.defaultdict(list)
for r in csv.DictReader(open('$f')):
    if 'k_accumulate<false, true' in r['Kernel_Name']: s[r['Counter_Name']].append(float(r['Counter_Value']))
v=s['SQ_INSTS_VALU']; sa=s['SQ_INSTS_SALU']
print('$v', 'VALU per launch %.4g per entry-wave %.1f SALU per entry-wave %.1f' % (v[-1], v[-1]/(2**24/64), sa[-1]/(2**24/64)))
"
done
