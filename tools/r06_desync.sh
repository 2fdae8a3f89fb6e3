#!/bin/bash
# Gram main-pass start-offset A/B, and the channel probe with expandable
# allocator segments.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "KNOB=desync CHUNKS=0,13,14,15,25,26,27 timeout -k 10 300 python tools/ab_gram_chunks.py 50 > gpurun_out/r06/gram_desync_ab.jsonl" \
  "PYTORCH_HIP_ALLOC_CONF=expandable_segments:True timeout -k 10 400 python tools/probe_channels.py > gpurun_out/r06/probe_channels_expandable.jsonl"
