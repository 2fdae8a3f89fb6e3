#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
bash tools/gpu_job.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_server.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06/wire_tests3.log 2>&1" \
  "timeout -k 10 400 python tools/bench_wire.py quant > gpurun_out/r06/wire_quant_native3.jsonl 2> gpurun_out/r06/wire_quant_native3.log"
