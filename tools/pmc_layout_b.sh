#!/bin/bash
# TLB and memory-side counter passes over tools/probe_layout_b.py, one leg
# per run (the row-set kernel on slab views, then on separately allocated
# key tensors): per-kernel means into gpurun_out/pmc_layout_b_<leg>.json.
# Usage: bash tools/pmc_layout_b.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum"
P2="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"
P3="TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_UTCL1_THRASHING_STALL_sum"
for leg in rows_views rows_sep; do
  dirs=""
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    d=gpurun_out/pmc_lb_${leg}_$i
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $d -o run \
      -- python3 tools/probe_layout_b.py --only $leg --no-fill --rounds 2 --calls 5 \
      > $d.log 2>&1 || { echo "pass $leg $i failed"; tail -5 $d.log; exit 1; }
    dirs="$dirs $d"
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_layout_b_${leg}.json $dirs && rm -rf $dirs
done
