# row-set weighted sum through raw buffer loads: tests, probe, drop-ins
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "rows or golden or server or dropin or fullsize or sharded or world2" > gpurun_out/t_rows.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_rows.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python3 tools/probe_rows_alloc.py && timeout -k 10 100 python3 tools/probe_rows_alloc.py
timeout -k 10 300 python3 tools/bench_robust.py dropin 2>/dev/null | cut -c1-100
