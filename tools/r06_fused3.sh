#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_pairgram.py tests/test_gpu_krumsel.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06/fused_tests3.log 2>&1" \
  "KNOB=fused timeout -k 10 300 python tools/ab_gram_stages.py 50 100 200 > gpurun_out/r06/gram_fused_ab3.jsonl" \
  "timeout -k 10 300 python tools/time_krum_devsel.py > gpurun_out/r06/krum_devsel_warm3.txt 2>&1" \
  "FRESH=1 timeout -k 10 300 python tools/time_krum_devsel.py > gpurun_out/r06/krum_devsel_fresh3.txt 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/prof_fused3 -o run --output-format csv -- python tools/time_krum_devsel.py > gpurun_out/r06/krum_devsel_traced3.txt 2>&1"
