# PMC passes over the Krum pairwise kernel (tools/bench_robust.py krum), one
# counter group per rocprofv3 run, for the flat and the ring kernels.
# Output: gpurun_out/pmc_<tag>_<pass>/ (csv) and gpurun_out/counters.txt.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS"
for tag in ${KRUM_TAGS:-flat ring}; do
  if [ $tag = flat ]; then export FSAGG_PAIRDIST=flat; else unset FSAGG_PAIRDIST; fi
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv \
      -d gpurun_out/pmc_${tag}_$i -o run -- python3 tools/bench_robust.py krum \
      > gpurun_out/pmc_${tag}_$i.log 2>&1 || { echo "pass $tag $i failed"; exit 1; }
  done
done
