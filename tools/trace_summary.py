#!/usr/bin/env python3
"""Per-kernel duration summary of a rocprofv3 --kernel-trace CSV, split by
a duration threshold so that one kernel template launched at two problem
sizes in the same run (e.g. bench.py's C3 reduction and its 20-client CPU
baseline check) is reported per size.

  trace_summary.py run_kernel_trace.csv SUBSTRING [--min-ms X] [--max-ms Y]
"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
    ap.add_argument('kernel')
    ap.add_argument('--min-ms', type=float, default=0.0)
    ap.add_argument('--max-ms', type=float, default=float('inf'))
    a = ap.parse_args()
    v = []
    names = set()
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            if a.kernel not in r['Kernel_Name']:
                continue
            ms = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
            if a.min_ms <= ms <= a.max_ms:
                v.append(ms)
                names.add(r['Kernel_Name'])
    v.sort()
    print(json.dumps({
        'kernel': sorted(names), 'launches': len(v),
        'avg_ms': round(sum(v) / len(v), 6) if v else None,
        'median_ms': round(v[len(v) // 2], 6) if v else None,
        'min_ms': round(v[0], 6) if v else None,
        'max_ms': round(v[-1], 6) if v else None,
        'filter_ms': [a.min_ms, a.max_ms]}))


if __name__ == '__main__':
    main()
