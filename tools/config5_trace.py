"""Timeline of one config-5 iteration (create_proof + decide) from a rocprofv3 --kernel-trace
--memory-copy-trace CSV directory: python tools/config5_trace.py DIR [ITER] (ITER = -2: the
second-to-last decide delimits the iteration)."""
import csv
import glob
import sys

d = sys.argv[1]
it = int(sys.argv[2]) if len(sys.argv) > 2 else -2
kf = glob.glob(d + '/**/*kernel_trace.csv', recursive=True)
mf = glob.glob(d + '/**/*memory_copy_trace.csv', recursive=True)
ev = []
for k in csv.DictReader(open(kf[0])):
    ev.append((int(k['Start_Timestamp']), int(k['End_Timestamp']), 'K', k['Kernel_Name'].split('(')[0][:48]))
if mf:
    for m in csv.DictReader(open(mf[0])):
        ev.append((int(m['Start_Timestamp']), int(m['End_Timestamp']), 'C', m['Direction']))
ev.sort()
dec = [i for i, e in enumerate(ev) if 'k_decide' in e[3]]
a, b = dec[it - 1], dec[it]
seg = ev[a + 1:b + 1]
t0 = seg[0][0]
busy = 0
for s, e, kind, name in seg:
    busy += e - s
    print('%8.1f %8.1f %7.1f  %s %s' % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, kind, name))
print('span %.1f us, summed durations %.1f us' % ((seg[-1][1] - t0) / 1e3, busy / 1e3))
