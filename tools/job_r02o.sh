# kernel-trace of the allocation probe: per-dispatch durations of the flat and
# row-set weighted sums, slab then separate rows
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_probe -o run -- python3 tools/probe_rows_alloc.py > gpurun_out/prof_probe.log 2>&1; echo rc=$? order=${FSAGG_PROBE_ORDER:-forward}
python3 - <<'PY'
import csv, glob, statistics
f = glob.glob('gpurun_out/prof_probe/**/*kernel_trace.csv', recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if 'wsum' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
for name in ('wsum_f32_vec_kernel', 'wsum_rows_kernel'):
    d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 for r in rows if name in r['Kernel_Name']]
    half = len(d) // 2
    first, second = statistics.median(d[1:half]), statistics.median(d[half + 1:])
    print(name, 'first run', round(first, 4), 'second run', round(second, 4), len(d))
PY
