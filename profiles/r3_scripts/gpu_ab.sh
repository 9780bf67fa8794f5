#!/bin/bash
# A/B of library builds on one bench line: TESTS (pytest -k expr, optional) on
# the in-tree build first, then for each round, each of LIBS ("new" = in-tree,
# else variants/<name>.so) runs bench.py $BARGS.
set -o pipefail
O=gpurun_out/${TAG:-ab}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest ${TFILES:-tests/test_gpu_tile.py} -x -q --timeout 300 --timeout-method thread -k "$TESTS" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
  tail -1 $O/t.log
fi
BARGS=${BARGS:---frames 16384 --steps 1 --warmup 1 --cpu-seconds 0 --extra-snr= --phys-steps 0}
for r in $(seq ${ROUNDS:-2}); do for v in ${LIBS:-base new}; do
  E=""; [ $v != new ] && E="LDPC_HIP_LIB=variants/$v.so"
  env $E $XENV timeout -k 10 300 python -u bench.py $BARGS > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail $O/${v}_$r.err; exit 1; }
  echo "$v.$r $(python tools/bench_summary.py $O/${v}_$r.json)"
done; done
