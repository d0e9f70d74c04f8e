"""Per-scan timeline analysis of a rocprofv3 kernel trace: busy union, idle gaps, per-kernel critical time."""
import csv, sys, collections, re
path = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/trace_cur/run_kernel_trace.csv'
nlast = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = []
for r in csv.DictReader(open(path)):
    n = r['Kernel_Name']
    m = re.match(r'(?:void )?(?:vg::)?([\w:]+)', n)
    short = m.group(1) if m else n
    if 'rocprim' in n:
        k = re.findall(r'detail::(\w+)', n)
        short = 'rocprim.' + (k[1] if len(k) > 1 else k[0])
        if 'unsigned long' in n: short += '.u64'
    rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), short, int(r['Queue_Id']), int(r['Grid_Size_X']) // max(1, int(r['Workgroup_Size_X']))))
rows.sort()
starts = [i for i, r in enumerate(rows) if r[2].endswith('k_scan_begin')]
print('scans', len(starts))
sel = starts[-nlast - 1:]
tot_busy = tot_span = 0
gapk = collections.Counter(); crit = collections.Counter(); cnt = collections.Counter()
for a, b in zip(sel[:-1], sel[1:]):
    seg = rows[a:b]
    t0, t1 = seg[0][0], rows[b][0]
    busy = 0; cur_e = t0; last = None
    for s, e, n, q, g in seg:
        cnt[n] += 1
        if s > cur_e:
            gapk[(last, n)] += s - cur_e
        if e > cur_e:
            crit[n] += e - max(s, cur_e); busy += e - max(s, cur_e); cur_e = e; last = n
    tot_busy += busy; tot_span += t1 - t0
ns = len(sel) - 1
print(f'per scan: span {tot_span/ns/1e3:.1f} us, busy {tot_busy/ns/1e3:.1f} us, idle {(tot_span-tot_busy)/ns/1e3:.1f} us, kernels {sum(cnt.values())/ns:.0f}')
print('--- exclusive (critical) time per kernel, us/scan')
for n, v in crit.most_common(40): print(f'{v/ns/1e3:8.2f}  {cnt[n]/ns:5.1f}  {n}')
print('--- idle gaps (prev -> next), us/scan')
for (p, n), v in gapk.most_common(25): print(f'{v/ns/1e3:8.2f}  {p} -> {n}')
