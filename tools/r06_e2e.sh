#!/bin/bash
# E2E host dicts in/out: the native non-temporal pack against torch copies
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
bash tools/gpu_job.sh \
  "timeout -k 10 600 python bench.py --e2e --no-pmc --steps 5 --warmup 2 > gpurun_out/r06/bench_e2e_native.json 2> gpurun_out/r06/bench_e2e_native.log" \
  "FSAGG_NATIVE_PACK=0 timeout -k 10 600 python bench.py --e2e --no-pmc --steps 5 --warmup 2 > gpurun_out/r06/bench_e2e_torch.json 2> gpurun_out/r06/bench_e2e_torch.log"
