#!/bin/bash
# configs[2] layout B (161 keys): chunk-order A/B of the row-set kernel,
# host phases of aggregate(), a kernel trace; pairgram parity.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_pairgram.py -q --timeout 200 --timeout-method thread > gpurun_out/pairgram.log 2>&1" \
  "timeout -k 10 200 python -u tools/probe_layout_b.py --plan short_first > gpurun_out/layout_b.jsonl" \
  "timeout -k 10 200 python -u tools/probe_layout_b.py >> gpurun_out/layout_b.jsonl" \
  "timeout -k 10 200 python -u tools/probe_layout_b.py --plan short_first >> gpurun_out/layout_b.jsonl" \
  "timeout -k 10 200 python -u tools/probe_layout_b.py >> gpurun_out/layout_b.jsonl" \
  "timeout -k 10 200 python -u tools/time_dropin_host.py --layout resnet50 > gpurun_out/host_lb.json" \
  "timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lb -o run --output-format csv -- python tools/probe_layout_b.py --rounds 2" || exit $?
bash tools/pmc.sh krum r04 > gpurun_out/pmc_krum.log 2>&1 || exit 1
bash tools/pmc.sh orderstat r04 > gpurun_out/pmc_os.log 2>&1 || exit 1
bash tools/gpu_job.sh "timeout -k 10 300 python -u tools/bench_robust.py dropin > gpurun_out/dropin.jsonl"
