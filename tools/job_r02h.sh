# Krum pipelined operand reads (FSAGG_PAIR_LDS=pipe): tests, then A/B
mkdir -p gpurun_out
FSAGG_PAIR_LDS=pipe timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "krum or pairdist or bulyan or Krum or fullsize" > gpurun_out/t_krum.log 2>&1; rc=$?; echo "krum pipe tests rc=$rc"; tail -3 gpurun_out/t_krum.log
[ $rc -eq 0 ] || exit $rc
KAB_VARIANTS='FSAGG_NONE=0|FSAGG_PAIR_LDS=pipe|FSAGG_NONE=0|FSAGG_PAIR_LDS=pipe' timeout -k 10 400 bash tools/kab.sh krum
