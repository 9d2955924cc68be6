"""Where a chained owgs_process_batch call spends its GPU time: from a rocprofv3 --kernel-trace --memory-copy-trace
directory of tools/shim_leg.py, the engine launch durations and the kernels and copies around one of them.
  python tools/analysis/chain_timeline.py gpurun_out/.../shimtrace"""
import csv, sys, statistics as S
d = sys.argv[1]
ev = []
for r in csv.DictReader(open(d + '/run_kernel_trace.csv')):
    ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'][:34]))
for r in csv.DictReader(open(d + '/run_memory_copy_trace.csv')):
    ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Direction'][12:]))
ev.sort()
eng = [i for i, e in enumerate(ev) if e[2].startswith('void owgs_engine_kernel')]
print('engine launches', len(eng))
durs = [(ev[i][1]-ev[i][0])/1e3 for i in eng]
print('engine dur: first 250 median %.1f p10 %.1f p90 %.1f' % (S.median(durs[:250]), sorted(durs[:250])[25], sorted(durs[:250])[225]))
# per engine launch: span from the first event within 80us before it (same call) to the D2H after it
spans, pre, post = [], [], []
for i in eng[5:250]:
    t_e0, t_e1 = ev[i][0], ev[i][1]
    j = i
    while j > 0 and t_e0 - ev[j-1][1] < 40_000 and ev[j-1][2] != 'DEVICE_TO_HOST': j -= 1
    k = i
    while k < len(ev)-1 and ev[k+1][0] - t_e1 < 40_000 and ev[k][2] != 'DEVICE_TO_HOST': k += 1
    spans.append((ev[k][1]-ev[j][0])/1e3); pre.append((t_e0-ev[j][0])/1e3); post.append((ev[k][1]-t_e1)/1e3)
print('call span median %.1f us: before engine %.1f, engine %.1f, after %.1f' % (S.median(spans), S.median(pre), S.median(durs[5:250]), S.median(post)))
i = eng[100]
for e in ev:
    if ev[i][0] - 80_000 < e[0] < ev[i][1] + 60_000:
        print('%10.1f %8.1f  %s' % ((e[0]-ev[i][0])/1e3, (e[1]-e[0])/1e3, e[2]))
