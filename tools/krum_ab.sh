set -e
for v in "FSAGG_PAIRDIST=flat" "FSAGG_RING_BUFS=3" "FSAGG_RING_BUFS=4" "FSAGG_RING_MODE=1" "FSAGG_RING_MODE=2"; do
  echo "== $v"; env $v timeout -k 10 120 python tools/bench_robust.py krum 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['ms_median'], d['ms_min'], d['selection_exact'])"
done
