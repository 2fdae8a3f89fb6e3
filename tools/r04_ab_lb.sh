#!/bin/bash
# Layout B: kernel trace of the probe (gaps between back-to-back
# aggregate() calls) and the host phases of aggregate().
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 200 python -u tools/time_dropin_host.py --layout resnet50 > gpurun_out/host_lb.json" \
  "timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lb -o run --output-format csv -- python tools/probe_layout_b.py --rounds 2"
