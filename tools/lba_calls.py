"""Per-call LBA kernel breakdown from a rocprofv3 kernel trace: per solve (k_init_state ..), the
number of LM steps and each kernel's total / per-step microseconds.  Usage: lba_calls.py TRACE.csv"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
short = lambda r: r['Kernel_Name'].split('(')[0].split('::')[-1]
idx = [i for i, r in enumerate(rows) if short(r) == 'k_init_state']
for a, b in zip(idx, idx[1:] + [len(rows)]):
    seg = rows[a:b]
    d = collections.OrderedDict()
    for r in seg:
        d.setdefault(short(r), []).append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
    steps = len(d.get('k_trial_control', [])) or 1
    t0, t1 = int(seg[0]['Start_Timestamp']), max(int(r['End_Timestamp']) for r in seg)
    busy = sum(sum(v) for v in d.values())
    print(f"call: wall {(t1 - t0) / 1e3:.0f} us, kernels {busy:.0f} us, steps {steps}; per step: " +
          ", ".join(f"{k} {sum(v) / steps:.0f}" for k, v in d.items() if len(v) >= steps))
