#!/bin/bash
# A/B of kernel variants in the probe build (tools/probe, -DFSAGG_PROBE):
# runs CMD once per variant under a kernel trace and prints the command's
# JSON lines plus the average duration of every kernel matching PATTERN.
#   AB_VARIANTS='FSAGG_PROBE_RING=0|FSAGG_PROBE_RING=1 FSAGG_PROBE_RING_SLOTS=4' \
#   AB_PATTERN=pairdist bash tools/ab.sh python3 tools/bench_robust.py krum
# Variants are '|'-separated lists of VAR=value; run from the repo root.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
set -e
export FSAGG_LIB=$PWD/tools/probe/lib/libfsagg.so
IFS='|' read -ra VARIANTS <<< "${AB_VARIANTS:-}"
PATTERN=${AB_PATTERN:-.}
REPS=${AB_REPS:-1}
i=0
for rep in $(seq 1 "$REPS"); do
for v in "${VARIANTS[@]}"; do
  i=$((i+1))
  echo "== [$rep] $v"
  for kv in $v; do export "$kv"; done
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/ab_$i -o run -- "$@" > gpurun_out/ab_$i.log 2>&1
  grep '^{' gpurun_out/ab_$i.log | cut -c1-400 || true
  python3 - gpurun_out/ab_$i/run_kernel_stats.csv "$PATTERN" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[2], r['Name']):
        print('   %-70s calls=%s avg_ms=%.4f' % (r['Name'][:70], r['Calls'],
                                               float(r['AverageNs']) / 1e6))
PY
  for kv in $v; do unset "${kv%%=*}"; done
done
done
