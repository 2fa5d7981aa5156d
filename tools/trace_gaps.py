"""Per-kernel duration and the idle gap before each kernel, from a rocprofv3 --kernel-trace CSV:
the last MSM step of a bench run (k_to_mont / k_bin_hist ... k_group_sum)."""
import csv
import glob
import sys

d = sys.argv[1]
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
# last occurrence of the MSM's first kernel
starts = [i for i, n in enumerate(names) if n.startswith("void sv::k_bin_hist")]
steps = []
for s in starts[-4:]:
    e = s
    while e < len(rows) and not names[e].startswith("sv::k_group_sum"):
        e += 1
    steps.append((s, e))
for s, e in steps[-2:]:
    t0 = int(rows[s]["Start_Timestamp"])
    prev_end = t0
    print("---- step (%d kernels)" % (e - s + 1))
    for r in rows[s:e + 1]:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print("%-40s start %8.1f us  dur %8.1f us  gap %6.1f us" % (r["Kernel_Name"][:40], (st - t0) / 1e3, (en - st) / 1e3, (st - prev_end) / 1e3))
        prev_end = en
    print("span %.1f us" % ((int(rows[e]["End_Timestamp"]) - t0) / 1e3))
# call-to-call gap between steps
for (s1, e1), (s2, e2) in zip(steps, steps[1:]):
    print("between steps: %.1f us" % ((int(rows[s2]["Start_Timestamp"]) - int(rows[e1]["End_Timestamp"])) / 1e3))
