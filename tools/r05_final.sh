#!/bin/bash
# Round-5 evidence on one fresh box (profiles/r05/): smoke; the bench line
# (with its PMC traffic pass); the E2E line; the bench under a kernel trace
# (roofline.frac reproducible from this round's profiles); the robust
# rules, order statistics and Krum at n = 50 / 100 / 200; the C5 order
# statistics under a kernel trace; the 8-rank share of the plug-in path.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
bash tools/gpu_job.sh pytestall smoke \
  "timeout -k 10 400 python bench.py > gpurun_out/r05/bench.json" \
  "timeout -k 10 500 python bench.py --e2e --no-pmc --no-cpu-baseline > gpurun_out/r05/bench_e2e.json" \
  "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/prof_bench -o run --output-format csv -- python bench.py --no-pmc --no-cpu-baseline > gpurun_out/r05/bench_traced.json" \
  "timeout -k 10 500 python -u tools/bench_robust.py krum orderstat orderstat_large dropin krum_large > gpurun_out/r05/robust.jsonl" \
  "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/prof_os -o run --output-format csv -- python tools/bench_robust.py orderstat > gpurun_out/r05/robust_os_traced.jsonl" \
  "timeout -k 10 300 python tools/bench_share.py --aggregate --world 8 > gpurun_out/r05/share_aggregate_n8.jsonl"
