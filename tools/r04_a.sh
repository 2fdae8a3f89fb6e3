#!/bin/bash
# Round-4 validation pass: MFMA numerics probe, the changed GPU tests, the
# full-size tests, the robust-rule bench, the plug-in share at N = 8.
set -u
cd "$(dirname "$0")/.."
export FSAGG_TEST_LOG=gpurun_out/stress.jsonl
bash tools/gpu_job.sh \
  "timeout -k 10 300 python -u tools/probe/mfma_numerics.py > gpurun_out/mfma_numerics.jsonl" \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_pairgram.py tests/test_gpu_world2.py tests/test_gpu_wire.py tests/test_gpu_golden.py -v --timeout 200 --timeout-method thread" \
  "timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -v --timeout 200 --timeout-method thread" \
  "timeout -k 10 300 python -u tools/bench_robust.py krum orderstat > gpurun_out/bench_robust.jsonl" \
  "timeout -k 10 300 python -u tools/bench_share.py --aggregate --world 8 > gpurun_out/share_aggregate.jsonl"
