"""Print the dispatch sequence of one scan from a rocprofv3 kernel trace (start offset, duration, queue, grid)."""
import csv, sys, re
path = sys.argv[1]; which = int(sys.argv[2]) if len(sys.argv) > 2 else -3
rows = []
for r in csv.DictReader(open(path)):
    n = r['Kernel_Name']
    m = re.match(r'(?:void )?(?:vg::)?([\w:]+)', n)
    short = m.group(1) if m else n
    if 'rocprim' in n:
        k = re.findall(r'detail::(\w+)', n)
        short = 'rocprim.' + (k[1] if len(k) > 1 else k[0]) + ('.u64' if 'unsigned long' in n else '') + ('.pairs' if 'unsigned int*, unsigned int*>' in n else '')
    rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), short, r['Queue_Id'], int(r['Grid_Size_X']) // max(1, int(r['Workgroup_Size_X']))))
rows.sort()
st = [i for i, r in enumerate(rows) if r[2].endswith('k_scan_begin')]
a, b = st[which], st[which + 1]
t0 = rows[a][0]
for s, e, n, q, g in rows[a:b]:
    print(f'{(s-t0)/1e3:8.1f} {(e-s)/1e3:7.2f} q{q} g{g:<6} {n}')
