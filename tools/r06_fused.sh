#!/bin/bash
# Fused Gram chain tail: bit-identity tests, interleaved A/B against the
# eight-launch chain, the device-select host timeline, a kernel trace.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_pairgram.py tests/test_gpu_krumsel.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06/fused_tests.log 2>&1" \
  "KNOB=fused timeout -k 10 300 python tools/ab_gram_stages.py 50 100 200 > gpurun_out/r06/gram_fused_ab.jsonl" \
  "timeout -k 10 300 python tools/time_krum_devsel.py > gpurun_out/r06/krum_devsel_warm.txt 2>&1" \
  "FRESH=1 timeout -k 10 300 python tools/time_krum_devsel.py > gpurun_out/r06/krum_devsel_fresh.txt 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/prof_fused -o run --output-format csv -- python tools/time_krum_devsel.py > gpurun_out/r06/krum_devsel_traced.txt 2>&1"
