# A/B of the Krum distance kernels: end-to-end ops.pairdist time (bench_robust
# krum) and the per-kernel average from a kernel trace, per variant.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
# KAB_VARIANTS: '|'-separated, each a space-separated list of VAR=value
i=0
IFS='|' read -ra VARIANTS <<< "${KAB_VARIANTS:-FSAGG_PAIRDIST=flat|FSAGG_PAIRDIST=ring|FSAGG_PAIRDIST=ring FSAGG_RING_MODE=2}"
for v in "${VARIANTS[@]}"; do
  i=$((i+1))
  echo "== $v"
  for kv in $v; do export $kv; done
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/krum_ab_$i -o run -- python3 tools/bench_robust.py krum \
    > gpurun_out/krum_ab_$i.log 2>&1
  grep '^{' gpurun_out/krum_ab_$i.log | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print('e2e', d['ms_median'], d['ms_min'], d['selection_exact'])"
  python3 - gpurun_out/krum_ab_$i/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'pairdist' in r['Name'] or 'chunk_prefix' in r['Name']:
        print('   %-60s calls=%s avg_ms=%.4f' % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e6))
PY
  for kv in $v; do unset ${kv%%=*}; done
done
