"""Do the health exchange's copies run while an engine launch does?  From a rocprofv3 --kernel-trace run_kernel_trace.csv
of bench.py --health-churn [--rccl]: hardware queue and stream of the engine launches and of the copy kernels, and which
copies ran entirely inside an engine launch.
  python tools/analysis/queue_overlap.py gpurun_out/.../run_kernel_trace.csv"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
eng = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Queue_Id'], r['Stream_Id']) for r in rows if 'owgs_engine_kernel' in r['Kernel_Name']]
cp = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Queue_Id'], r['Stream_Id'], r['Kernel_Name'][:30]) for r in rows if 'copyBuffer' in r['Kernel_Name'] or 'nccl' in r['Kernel_Name'].lower()]
print('engine launches', len(eng), 'queues', sorted(set(e[2] for e in eng)), 'streams', sorted(set(e[3] for e in eng)))
inside = [c for c in cp if any(e[0] < c[0] and c[1] < e[1] for e in eng)]
print('copy kernels', len(cp), 'entirely inside an engine launch:', len(inside))
from collections import Counter
print('queues/streams of the overlapping copies:', Counter((c[2], c[3]) for c in inside).most_common(5))
print('queues/streams of all copies:', Counter((c[2], c[3]) for c in cp).most_common(8))
# per engine launch: copies that ran during it
for e in eng[3:9]:
    n = sum(1 for c in cp if e[0] < c[0] < e[1])
    print('engine %.2f ms: %d copies started during it' % ((e[1]-e[0])/1e6, n))
