#!/bin/bash
# Round-5 baseline on a fresh box: the bench line under a kernel trace
# (roofline evidence for this round), then the robust benches.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python bench.py --no-pmc > gpurun_out/bench_traced.json" \
  "timeout -k 10 400 python -u tools/bench_robust.py orderstat dropin > gpurun_out/robust.jsonl"
