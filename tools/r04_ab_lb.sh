#!/bin/bash
# Layout B A/B on one box: the row-set kernel with short keys' clients
# loaded eight at a time (product) against the previous form
# (tools/probe/nb), interleaved.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
NB=tools/probe/nb/libfsagg.so
bash tools/gpu_job.sh \
  "timeout -k 10 200 python -u tools/probe_layout_b.py > gpurun_out/lb_ab.jsonl" \
  "FSAGG_LIB=$NB timeout -k 10 200 python -u tools/probe_layout_b.py >> gpurun_out/lb_ab.jsonl" \
  "timeout -k 10 200 python -u tools/probe_layout_b.py >> gpurun_out/lb_ab.jsonl" \
  "FSAGG_LIB=$NB timeout -k 10 200 python -u tools/probe_layout_b.py >> gpurun_out/lb_ab.jsonl" \
  "timeout -k 10 200 python -u tools/probe_layout_b.py >> gpurun_out/lb_ab.jsonl" \
  "FSAGG_LIB=$NB timeout -k 10 200 python -u tools/probe_layout_b.py >> gpurun_out/lb_ab.jsonl" || exit $?
bash tools/r04_final.sh
