#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per libfsagg kernel.

usage: pmc_summary.py OUT_JSON DIR [DIR ...]

Each DIR is one rocprofv3 -d output of a single --pmc pass (one counter
group, see tools/pmc.sh).  For every kernel whose name contains 'fsagg' the
mean of each counter over its dispatches is recorded, plus derived figures
when the counters are present: VALU instructions per wave, LDS instructions
per wave, and the HBM bytes per launch (FETCH_SIZE and WRITE_SIZE in KiB;
FETCH_SIZE is reported raw — its gfx950 half-count applies to 16-B-per-lane
reads only, MI355X_MICROARCH.md §HBM, so the caller states the correction).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    for pre in ('(anonymous namespace)::', 'void ', 'fsagg::', 'os::'):
        name = name.replace(pre, '')
    return name.split('(')[0]


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for path in glob.glob(os.path.join(d, '**', '*counter_collection.csv'),
                              recursive=True):
            with open(path) as f:
                for r in csv.DictReader(f):
                    k = r.get('Kernel_Name', '')
                    if 'fsagg' not in k:
                        continue
                    acc[short(k)][r['Counter_Name']].append(
                        float(r['Counter_Value']))
    res = {}
    for k, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        m['dispatches'] = max(len(v) for v in cs.values())
        if m.get('SQ_WAVES'):
            for c in ('SQ_INSTS_VALU', 'SQ_INSTS_LDS', 'SQ_INSTS_SALU',
                      'SQ_INSTS_VMEM'):
                if c in m:
                    m[c + '_per_wave'] = m[c] / m['SQ_WAVES']
        if 'FETCH_SIZE' in m:
            m['fetch_bytes_raw'] = m['FETCH_SIZE'] * 1024
        if 'WRITE_SIZE' in m:
            m['write_bytes'] = m['WRITE_SIZE'] * 1024
        res[k] = m
    with open(out, 'w') as f:
        json.dump(res, f, indent=1, sort_keys=True)
    for k, m in sorted(res.items()):
        print(k, {c: round(v, 1) for c, v in m.items()
                  if c.endswith('per_wave') or c in ('fetch_bytes_raw',
                                                     'write_bytes')})


if __name__ == '__main__':
    main()
