# Kernel-trace summary of the drop-in aggregate() calls (tools/bench_robust.py
# dropin) into gpurun_out/prof_dropin/.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/prof_dropin -o run -- python3 tools/bench_robust.py dropin \
  > gpurun_out/prof_dropin.log 2>&1
