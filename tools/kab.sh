# A/B of device kernels under env variants: the end-to-end line(s) of
# tools/bench_robust.py <what> and each fsagg kernel's average duration from
# a kernel trace.  Usage: KAB_VARIANTS='A=1|A=2 B=3' bash tools/kab.sh <what>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
what=${1:-krum}
i=0
IFS='|' read -ra VARIANTS <<< "${KAB_VARIANTS:-FSAGG_NONE=0}"
for v in "${VARIANTS[@]}"; do
  i=$((i+1))
  echo "== $what: $v"
  for kv in $v; do export $kv; done
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/kab_${what}_$i -o run -- python3 tools/bench_robust.py $what \
    > gpurun_out/kab_${what}_$i.log 2>&1 || { echo "run failed"; exit 1; }
  grep '^{' gpurun_out/kab_${what}_$i.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print('  ', d.get('config', d.get('rule')), 'ms_median', d.get('ms_median', d.get('ms_aggregate')), 'ok', d.get('parity_sampled_4096_cols', d.get('selection_exact')))"
  python3 - gpurun_out/kab_${what}_$i/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'fsagg' in r['Name']:
        print('   %-70s calls=%s avg_ms=%.4f' % (r['Name'][:70], r['Calls'], float(r['AverageNs']) / 1e6))
PY
  for kv in $v; do unset ${kv%%=*}; done
done
