#!/usr/bin/env python3
"""Dump the per-kernel summary of a rocprofv3 database (the default output
format of rocprofv3 --kernel-trace --stats in ROCm 7: <dir>/<name>_results.db)
as CSV: Name, Calls, TotalDurationNs, AverageNs, Percentage.

    python3 tools/rocpd_stats.py gpurun_out/prof/run_results.db out.csv
"""
import csv
import sqlite3
import sys


def main():
    db, out = sys.argv[1], sys.argv[2]
    con = sqlite3.connect(db)
    rows = con.execute('select name, total_calls, total_duration, average, '
                       'percentage from top_kernels').fetchall()
    with open(out, 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['Name', 'Calls', 'TotalDurationNs', 'AverageNs',
                    'Percentage'])
        for r in rows:
            w.writerow(r)
    for r in rows[:6]:
        print('%-90.90s %6d %12.1f' % (r[0], r[1], r[3]))


if __name__ == '__main__':
    main()
