# PMC passes (one rocprofv3 run per counter group) over tools/bench_robust.py.
# usage: bash tools/pmc_orderstat.sh [krum|orderstat]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
W=${1:-orderstat}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc1_$W -o run -- python3 tools/bench_robust.py $W > gpurun_out/pmc1_$W.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc2_$W -o run -- python3 tools/bench_robust.py $W > gpurun_out/pmc2_$W.log 2>&1 || exit $?
