#!/bin/bash
# Host cost of one pinned-ring upload, statement by statement.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 200 python -u tools/probe_upload.py > gpurun_out/upload.json"
