# Kernel-trace summaries of every benchmark (rocprofv3 --kernel-trace --stats,
# CSV) into gpurun_out/prof_<name>/; copy the *_kernel_stats.csv files you
# want judged into profiles/.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
prof() {  # prof <name> <cmd...>
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/prof_$name -o run -- "$@" > gpurun_out/prof_$name.log 2>&1
  local rc=$?
  echo "[prof_$name] rc=$rc" >> gpurun_out/steps.log
  [ $rc -eq 0 ] || exit $rc
}
prof bench python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
prof robust python3 tools/bench_robust.py
prof wire python3 tools/bench_wire.py ss dissim
prof smalln python3 tools/bench_smalln.py
