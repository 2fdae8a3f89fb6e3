# host-side drop-in changes (virtual-base key table, as_strided emission):
# full GPU tests, then host phases and the drop-in bench
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/time_dropin_host.py > gpurun_out/dropin_host.txt 2>&1; cat gpurun_out/dropin_host.txt
timeout -k 10 300 python3 tools/bench_robust.py dropin > gpurun_out/dropin.jsonl 2> gpurun_out/dropin.err; echo "dropin rc=$?"; cut -c1-120 gpurun_out/dropin.jsonl
