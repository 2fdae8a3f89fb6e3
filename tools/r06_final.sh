#!/bin/bash
# Round 6 final-tree records: the bench line and its kernel trace; the
# robust rules (Krum C4, C5 order statistics, the drop-ins warm and with
# fresh uploads) under a kernel trace; Krum n = 100 / 200 / 256 under a
# kernel trace; the Krum host timeline; the 8-rank share of aggregate().
# Traces go to /tmp; only their kernel summaries come back.
set -u
cd "$(dirname "$0")/.."
F=gpurun_out/r06/final
mkdir -p $F
export TMPDIR=/tmp
P=/tmp/r06prof
stats() {  # stats <trace dir> <name>
  find "$1" -name '*kernel_stats.csv' -exec cp {} "$F/$2_kernel_stats.csv" \;
}
bash tools/gpu_job.sh \
  "timeout -k 10 400 python bench.py > $F/bench.json" \
  "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/bench -o run --output-format csv -- python bench.py --no-pmc > $F/bench_traced.json" \
  "timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $P/robust -o run --output-format csv -- python tools/bench_robust.py krum orderstat dropin dropin_fresh > $F/robust.jsonl" \
  "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/krum_large -o run --output-format csv -- python tools/bench_robust.py krum_large > $F/krum_large.jsonl" \
  "timeout -k 10 300 python tools/time_krum_devsel.py > $F/krum_devsel_warm.txt 2>&1" \
  "FRESH=1 timeout -k 10 300 python tools/time_krum_devsel.py > $F/krum_devsel_fresh.txt 2>&1" \
  "timeout -k 10 300 python tools/bench_share.py --aggregate --world 8 > $F/share_aggregate_n8.jsonl"
rc=$?
stats $P/bench bench; stats $P/robust robust; stats $P/krum_large krum_large
exit $rc
