#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
bash tools/gpu_job.sh \
  "timeout -k 10 600 python bench.py --e2e --no-pmc --steps 3 --warmup 1 > gpurun_out/r06/e2e_nbuf2.json 2> gpurun_out/r06/e2e_nbuf2.log" \
  "FSAGG_STAGE_BUFFERS=3 timeout -k 10 600 python bench.py --e2e --no-pmc --steps 3 --warmup 1 > gpurun_out/r06/e2e_nbuf3.json 2> gpurun_out/r06/e2e_nbuf3.log" \
  "FSAGG_STAGE_BUFFERS=4 timeout -k 10 600 python bench.py --e2e --no-pmc --steps 3 --warmup 1 > gpurun_out/r06/e2e_nbuf4.json 2> gpurun_out/r06/e2e_nbuf4.log"
