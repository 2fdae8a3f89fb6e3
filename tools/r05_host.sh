#!/bin/bash
# Round-5 host-path pass: the whole GPU suite, the integer VALU probe, the
# sharded aggregate() share (copy / views, cache on / off) and its host cost.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh pytestall \
  "timeout -k 10 120 ./tools/probe/bin/valu_probe3 > gpurun_out/valu3.txt" \
  "timeout -k 10 300 python -u tools/bench_share.py --aggregate --world 8 > gpurun_out/share_agg.jsonl" \
  "timeout -k 10 300 python -u tools/bench_share.py --aggregate --world 8 --rank 1 > gpurun_out/share_agg_r1.jsonl" \
  "timeout -k 10 200 python -u tools/time_share_host.py --views 1 > gpurun_out/share_host_views.txt" \
  "timeout -k 10 200 python -u tools/time_share_host.py --views 0 > gpurun_out/share_host_copy.txt"
