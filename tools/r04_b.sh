#!/bin/bash
# Gram staging A/B: the product library (LDS-staged rows) against the
# register-load build, on the C4 shape in four row placements; then a
# kernel trace of the product path.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash tools/gpu_job.sh \
  "timeout -k 10 200 python -u tools/probe_gram_data.py > gpurun_out/gram_ab_staged.jsonl" \
  "FSAGG_LIB=tools/probe/regs/libfsagg.so timeout -k 10 200 python -u tools/probe_gram_data.py > gpurun_out/gram_ab_regs.jsonl" \
  "timeout -k 10 200 python -u tools/probe_gram_data.py > gpurun_out/gram_ab_staged2.jsonl"
