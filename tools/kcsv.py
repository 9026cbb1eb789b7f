#!/usr/bin/env python3
"""Kernel averages from a rocprofv3 --stats CSV:  python tools/kcsv.py run_kernel_stats.csv [filter]"""
import csv
import sys

filt = sys.argv[2] if len(sys.argv) > 2 else ''
for r in csv.DictReader(open(sys.argv[1])):
    if filt in r['Name']:
        print(f"{float(r['AverageNs']) / 1e3:9.1f} us  x{r['Calls']:>4}  {r['Name'][:100]}")
