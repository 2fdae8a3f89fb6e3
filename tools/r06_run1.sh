#!/bin/bash
# Round 6, first box: the GPU suite as a measurement pass of the trimmed-mean
# error (every check logs its max error in units of ε·Σ|x|/(n−2k), none
# fails on it); the bench line with the new C2 and fresh-upload legs; Krum
# C4 and the drop-in rules (warm and fresh uploads) under a kernel trace;
# the 8-rank share of aggregate().
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
export FSAGG_TRIM_MEASURE=1 FSAGG_ERR_LOG=$PWD/gpurun_out/r06/trimmed_err.jsonl
bash tools/gpu_job.sh pytestall smoke \
  "timeout -k 10 400 python bench.py > gpurun_out/r06/bench.json" \
  "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/prof_krum -o run --output-format csv -- python tools/bench_robust.py krum dropin dropin_fresh > gpurun_out/r06/robust_traced.jsonl" \
  "timeout -k 10 300 python tools/bench_share.py --aggregate --world 8 > gpurun_out/r06/share_aggregate_n8.jsonl"
