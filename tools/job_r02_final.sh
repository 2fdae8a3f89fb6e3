# round-2 final profile pass: kernel-trace summaries of the headline bench
# and every robust benchmark (incl. the n > 255 sweep), PMC passes of the
# Krum and streaming order-statistic kernels, the bench line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
prof() {  # prof <name> <cmd...>
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/prof_$name -o run -- "$@" > gpurun_out/prof_$name.log 2>&1
  local rc=$?
  echo "[prof_$name] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
prof bench python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
prof robust python3 tools/bench_robust.py krum orderstat orderstat_large dropin
timeout -k 10 300 bash tools/pmc.sh krum final > gpurun_out/pmc_krum.log 2>&1; echo "pmc krum rc=$?"
timeout -k 10 300 bash tools/pmc.sh orderstat_large final > gpurun_out/pmc_osl.log 2>&1; echo "pmc osl rc=$?"
timeout -k 10 300 python3 bench.py > gpurun_out/bench_line.json 2> gpurun_out/bench_line.err; echo "bench rc=$?"
cat gpurun_out/bench_line.json | cut -c1-200
