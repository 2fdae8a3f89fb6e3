#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "CHUNKS=1024,1536,2048,3072,4096 timeout -k 10 300 python tools/ab_gram_chunks.py 50 100 > gpurun_out/r06/gram_chunks_ab2.jsonl"
