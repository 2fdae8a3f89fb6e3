#!/bin/bash
# SQ counter passes over tools/ab_gram_block8.py <n> (per-kernel means into
# gpurun_out/pmc_gram_<tag>.json).  Usage: bash tools/pmc_gram.sh <tag> <n>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=$1; shift
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS"
P3="SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
i=0
dirs=""
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  d=gpurun_out/pmc_gram_${tag}_$i
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv \
    -d $d -o run -- python3 tools/ab_gram_block8.py "$@" \
    > $d.log 2>&1 || { echo "pass $i failed"; tail -5 $d.log; }
  dirs="$dirs $d"
done
python3 tools/pmc_summary.py gpurun_out/pmc_gram_${tag}.json $dirs && rm -rf $dirs
