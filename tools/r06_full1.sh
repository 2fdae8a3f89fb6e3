#!/bin/bash
# full GPU suite + smoke on the fused Gram tail; Krum phases after the
# single knob read
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
bash tools/gpu_job.sh pytestall smoke \
  "timeout -k 10 300 python tools/time_krum_devsel.py > gpurun_out/r06/krum_devsel_warm4.txt 2>&1" \
  "FRESH=1 timeout -k 10 300 python tools/time_krum_devsel.py > gpurun_out/r06/krum_devsel_fresh4.txt 2>&1"
