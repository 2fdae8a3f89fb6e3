#!/bin/bash
# Gram staging A/B (product = LDS-staged rows, tools/probe/regs = register
# loads) on the C4 shape in four row placements; the MFMA alignment-window
# probe.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash tools/gpu_job.sh \
  "timeout -k 10 120 python -u tools/probe/mfma_numerics.py window > gpurun_out/mfma_window.jsonl" \
  "timeout -k 10 200 python -u tools/probe_gram_data.py > gpurun_out/gram_ab_staged.jsonl" \
  "FSAGG_LIB=tools/probe/regs/libfsagg.so timeout -k 10 200 python -u tools/probe_gram_data.py > gpurun_out/gram_ab_regs.jsonl" \
  "timeout -k 10 200 python -u tools/probe_gram_data.py > gpurun_out/gram_ab_staged2.jsonl" \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_world2.py -x -q --timeout 200 --timeout-method thread -k 'median or trimmed or sharded or peer or bulyan'"
