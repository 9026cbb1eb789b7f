#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc SQ counter CSVs per kernel: per-dispatch averages, per-wave
instruction counts, and the busy / wait fractions of the wave cycles.
    python3 tools/sq_summary.py DIR [DIR ...]"""
import collections
import csv
import glob
import sys

vals = collections.defaultdict(list)
for d in sys.argv[1:]:
    for f in glob.glob(d + '/**/run_counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'kmp' not in r['Kernel_Name']:
                continue
            vals[(r['Kernel_Name'][:96], r['Counter_Name'])].append(float(r['Counter_Value']))
kernels = sorted({k for k, _ in vals})
for k in kernels:
    avg = {c: sum(v) / len(v) for (kk, c), v in vals.items() if kk == k}
    waves = max(avg.get('SQ_WAVES', 1.0), 1.0)
    cyc = max(avg.get('SQ_WAVE_CYCLES', 1.0), 1.0)
    print(k)
    print('  per dispatch: ' + ', '.join(f'{c}={v:.4g}' for c, v in sorted(avg.items())))
    per_wave = {c[len('SQ_INSTS_'):]: avg[c] / waves for c in avg if c.startswith('SQ_INSTS_')}
    print('  instructions per wave: ' + ', '.join(f'{c}={v:.1f}' for c, v in sorted(per_wave.items())))
    frac = {c: avg[c] / cyc for c in ('SQ_ACTIVE_INST_VALU', 'SQ_ACTIVE_INST_ANY', 'SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY',
                                       'SQ_ACTIVE_INST_LDS', 'SQ_WAIT_INST_LDS') if c in avg}
    print('  fraction of wave cycles: ' + ', '.join(f'{c[3:]}={v:.3f}' for c, v in frac.items()))
    if 'SQ_VALU_MFMA_BUSY_CYCLES' in avg and 'SQ_BUSY_CYCLES' in avg:
        print(f"  MFMA busy cycles / busy cycles = {avg['SQ_VALU_MFMA_BUSY_CYCLES'] / max(avg['SQ_BUSY_CYCLES'], 1):.3f}")
