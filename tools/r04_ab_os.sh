#!/bin/bash
# Streaming order statistics (n > 255): compaction pass from the last row
# down (product) against the forward pass (tools/probe/osold), interleaved;
# the order-statistic parity tests.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
P="timeout -k 10 300 python -u tools/bench_robust.py orderstat_large"
Q="FSAGG_LIB=tools/probe/osold/libfsagg.so $P"
bash tools/gpu_job.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_golden.py -q -k 'median or trimmed or orderstat or bulyan' --timeout 200 --timeout-method thread > gpurun_out/os.log 2>&1" \
  "$P > gpurun_out/os_ab.jsonl" "$Q >> gpurun_out/os_ab.jsonl" \
  "$P >> gpurun_out/os_ab.jsonl" "$Q >> gpurun_out/os_ab.jsonl"
