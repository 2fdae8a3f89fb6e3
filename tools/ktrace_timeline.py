#!/usr/bin/env python3
"""Print the kernel timeline of a rocprofv3 --kernel-trace database
(start offset, duration, gap to the previous kernel, name), the last
``count`` dispatches.  tools only."""
import glob
import sqlite3
import sys


def main():
    db = glob.glob(sys.argv[1] + '/*.db')[0]
    count = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    c = sqlite3.connect(db)
    rows = list(c.execute(
        'select start, end, name from kernels order by start'))[-count:]
    t0 = rows[0][0]
    prev = None
    for s, e, name in rows:
        gap = (s - prev) / 1000.0 if prev is not None else 0.0
        print('%9.1f us  dur %7.1f  gap %6.1f  %s' % (
            (s - t0) / 1000.0, (e - s) / 1000.0, gap, name[:70]))
        prev = e


if __name__ == '__main__':
    main()
