#!/bin/bash
# tile_sub_kernel vs the split CN/VN launches on the WiMAX 2304 codes (GPU box)
mkdir -p gpurun_out/subbench
run() {  # name, bench args...
  name=$1; shift
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 "$@" > gpurun_out/subbench/$name.json 2> gpurun_out/subbench/$name.err || { echo "FAIL $name"; tail -3 gpurun_out/subbench/$name.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/subbench/$name.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$name'.ljust(28), round(d['value']), 'cw/s', r['kernel'], 'frac', round(r['frac'],3), 'iters', round(d['avg_iters'],2), 'fer', round(d['fer'],4))"
}
run r12_1db_sub   --code wimax_2304_0.5 --frames 16384 --snr 1.0 --schedule static
run r12_1db_split --code wimax_2304_0.5 --frames 16384 --snr 1.0 --schedule static --split
run r34A_1db_sub   --code wimax_2304_0.75A --frames 16384 --snr 1.0 --schedule static
run r34A_1db_split --code wimax_2304_0.75A --frames 16384 --snr 1.0 --schedule static --split
run r12_3db_sub    --code wimax_2304_0.5 --frames 65536 --chunk 16384 --snr 3.0 --schedule static
run r12_3db_stream --code wimax_2304_0.5 --frames 65536 --chunk 16384 --snr 3.0 --schedule stream
