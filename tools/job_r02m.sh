# drop-in aggregate() timings and the kernels under them (same box)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/bench_robust.py dropin > gpurun_out/dropin.jsonl 2> gpurun_out/dropin.err; echo "dropin rc=$?"; cut -c1-110 gpurun_out/dropin.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dropin -o run -- python3 tools/bench_robust.py dropin > gpurun_out/prof_dropin.log 2>&1; echo "prof rc=$?"
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/prof_dropin/run_kernel_stats.csv')):
    if 'fsagg' in r['Name']:
        print('  %-70s calls=%5s avg_ms=%.4f' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e6))
PY
