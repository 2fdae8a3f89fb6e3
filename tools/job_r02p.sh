# row-set weighted sum: the flat kernel's tile for dense chunks (A/B,
# FSAGG_WSUM_ROWS_TILE=1): tests under it, then kernel-only probe times
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
FSAGG_WSUM_ROWS_TILE=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "rows or golden or server or dropin or fullsize" > gpurun_out/t_tile.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_tile.log
[ $rc -eq 0 ] || exit $rc
for T in 0 1 0 1; do
  FSAGG_WSUM_ROWS_TILE=$T timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_tile_$T -o run -- python3 tools/probe_rows_alloc.py > /dev/null 2>&1 || exit 1
  python3 - $T <<'PY'
import csv, glob, statistics, sys
f = glob.glob('gpurun_out/prof_tile_%s/**/*kernel_trace.csv' % sys.argv[1], recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if 'wsum' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
for name in ('wsum_f32_vec_kernel', 'wsum_rows_kernel'):
    d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 for r in rows if name in r['Kernel_Name']]
    half = len(d) // 2
    print('TILE=%s' % sys.argv[1], name, 'slab', round(statistics.median(d[1:half]), 4), 'separate', round(statistics.median(d[half + 1:]), 4))
PY
  rm -rf gpurun_out/prof_tile_$T
done
FSAGG_WSUM_ROWS_TILE=1 timeout -k 10 300 python3 tools/bench_robust.py dropin 2>/dev/null | cut -c1-90
