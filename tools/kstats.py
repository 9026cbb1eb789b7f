#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 results database (``rocprofv3 --kernel-trace -d DIR -o run``
writes DIR/run_results.db): calls, average and total microseconds, sorted by total.

    python tools/kstats.py gpurun_out/X/prof/run_results.db [name-filter] [--csv out.csv]
"""
import csv
import sqlite3
import sys

db = sys.argv[1]
args = sys.argv[2:]
out = None
if '--csv' in args:
    i = args.index('--csv')
    out = args[i + 1]
    del args[i:i + 2]
filt = args[0] if args else ''
c = sqlite3.connect(db)
rows = c.execute('select name, count(*), avg("end" - start) / 1000.0, sum("end" - start) / 1000.0, '
                 'min("end" - start) / 1000.0, max("end" - start) / 1000.0 from kernels '
                 'group by name order by sum("end" - start) desc').fetchall()
rows = [r for r in rows if filt in r[0]]
for name, n, avg, tot, lo, hi in rows:
    print(f'{n:6d} {avg:10.2f} {tot:11.1f} {lo:9.2f} {hi:9.2f}  {name[:140]}')
if out:
    with open(out, 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['Name', 'Calls', 'AverageUs', 'TotalUs', 'MinUs', 'MaxUs'])
        w.writerows(rows)
