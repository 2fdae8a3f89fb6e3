#!/bin/bash
# SQ / GRBM counter passes (one counter group per run) over a driver
# program; per-kernel means into gpurun_out/pmc_<tag>.json.
# Usage: bash tools/pmc_gram2.sh <tag> <driver.py> [args...]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=$1; shift
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS"
P3="SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
dirs=""
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  d=gpurun_out/pmc_${tag}_$i
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv \
    -d $d -o run -- python3 "$@" > $d.log 2>&1 || { echo "pass $i failed"; tail -5 $d.log; exit 1; }
  dirs="$dirs $d"
done
python3 tools/pmc_summary.py gpurun_out/pmc_${tag}.json $dirs && rm -rf $dirs
