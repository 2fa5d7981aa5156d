"""Timeline (kernels + memory copies, us from the segment start) of one MSM call in a rocprofv3
--kernel-trace --memory-copy-trace CSV directory: python tools/trace_timeline.py DIR [CALL]
(CALL = -1: the last call, -5: four calls before it; calls are delimited by k_group_sum / k_group_fin)."""
import csv, sys
d = sys.argv[1]
call = int(sys.argv[2]) if len(sys.argv) > 2 else -1
K=list(csv.DictReader(open(d+'/run_kernel_trace.csv')))
M=list(csv.DictReader(open(d+'/run_memory_copy_trace.csv')))
ev=[]
for k in K: ev.append((int(k['Start_Timestamp']),int(k['End_Timestamp']),'K q%s'%k['Queue_Id'],k['Kernel_Name'].split('(')[0][:40]))
for m in M: ev.append((int(m['Start_Timestamp']),int(m['End_Timestamp']),'C s%s'%m['Stream_Id'],m['Direction'][12:]+' %.1fMB'%0))
ev.sort()
gs=[i for i,e in enumerate(ev) if 'group_sum' in e[3] or 'group_fin' in e[3]]
last_gs=gs[call]
prev_gs=gs[call-1]
seg=ev[prev_gs+1:last_gs+1]
t0=seg[0][0]
for s,e,kind,name in seg:
    print('%8.1f %8.1f %7.1f  %-6s %s'%((s-t0)/1e3,(e-t0)/1e3,(e-s)/1e3,kind,name))
