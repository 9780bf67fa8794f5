#!/bin/bash
# r3/4: tile8 vs split; r1/2: tile8 vs tile_sub (quick A/B, 16,384 frames at 1 dB)
set -o pipefail
O=gpurun_out/${TAG:-t8e}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tile.py -x -q --timeout 300 --timeout-method thread -k "tile8" > $O/t1.log 2>&1 || { tail -40 $O/t1.log; exit 1; }
tail -1 $O/t1.log
B="--frames 16384 --steps 1 --warmup 1 --cpu-seconds 0 --extra-snr= --phys-steps 0"
for code in wimax_2304_0.75A wimax_2304_0.5; do for v in new old; do
  E="LDPC_TILE8=1"; [ $v = old ] && E="LDPC_TILE8=0"
  env $E timeout -k 10 300 python -u bench.py $B --code $code > $O/${code}_$v.json 2> $O/${code}_$v.err && python tools/bench_summary.py $O/${code}_$v.json || { tail $O/${code}_$v.err; exit 1; }
done; done
