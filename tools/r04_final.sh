#!/bin/bash
# Round-4 evidence pass on the final tree: pytest -m gpu, smoke, the bench
# line, robust benches (Krum n = 50/100/200, C5 order statistics, drop-ins)
# with a kernel trace, the layout-B probe, gRPC ingest, and rank 0's share of
# the sharded aggregate().  Each GPU step is time-limited; a crash-class
# exit stops the job (tools/gpu_job.sh).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh pytestall smoke bench \
  "timeout -k 10 400 python -u tools/bench_robust.py krum krum_large orderstat orderstat_large dropin > gpurun_out/robust.jsonl" \
  "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_robust -o run --output-format csv -- python tools/bench_robust.py krum orderstat dropin" \
  "timeout -k 10 200 python -u tools/probe_layout_b.py > gpurun_out/layout_b.jsonl" \
  "timeout -k 10 200 python -u tools/bench_b64.py --keys 100 > gpurun_out/b64_k100.jsonl" \
  "timeout -k 10 200 python -u tools/bench_share.py --aggregate --world 8 > gpurun_out/share_agg.jsonl"
