#!/usr/bin/env python3
"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs)
into HBM bytes per launch of one kernel, with the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE reports exactly half
the bytes of a wide coalesced (16 B/lane) streaming read → ×2; WRITE_SIZE is
exact for 16-B streaming stores.  Counters are in KiB.

usage: pmc_traffic.py FETCH_CSV WRITE_CSV KERNEL_SUBSTR CLIENTS PARAMS OUT_JSON
"""
import csv
import json
import sys


def mean_counter(path, kernel, counter):
    vals = [float(r['Counter_Value']) for r in csv.DictReader(open(path))
            if kernel in r['Kernel_Name'] and r['Counter_Name'] == counter]
    if not vals:
        raise SystemExit('no %s rows for %s in %s' % (counter, kernel, path))
    return sum(vals) / len(vals), len(vals)


def main():
    fetch_csv, write_csv, kernel, n, P, out = sys.argv[1:7]
    n, P = int(n), int(P)
    f_kb, nf = mean_counter(fetch_csv, kernel, 'FETCH_SIZE')
    w_kb, nw = mean_counter(write_csv, kernel, 'WRITE_SIZE')
    read_b = f_kb * 1024 * 2   # gfx950: FETCH_SIZE = half of a wide stream
    write_b = w_kb * 1024
    algo = 4.0 * n * P + 4.0 * P + 4.0 * n
    rec = {
        'kernel': kernel, 'clients': n, 'params': P,
        'fetch_size_kib': f_kb, 'write_size_kib': w_kb,
        'dispatches': [nf, nw],
        'hbm_read_bytes_per_launch': read_b,
        'hbm_write_bytes_per_launch': write_b,
        'hbm_bytes_per_launch': read_b + write_b,
        'algorithmic_bytes_per_launch': algo,
        'traffic_over_algorithmic': (read_b + write_b) / algo,
        'correction': 'FETCH_SIZE x2 (gfx950 wide coalesced reads), '
                      'WRITE_SIZE as is; KiB -> bytes',
    }
    with open(out, 'w') as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == '__main__':
    main()
