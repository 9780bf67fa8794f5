# A/B of the streaming decode (bench's extra SNR points) across library variants.
# usage (GPU box): TAG=x VARIANTS="a b" bash tools/gpu_ab_stream.sh
set -o pipefail
O=gpurun_out/${TAG:-abs}; mkdir -p $O
B="--steps 1 --warmup 1 --frames 16384 --cpu-seconds 0 --extra-snr=2.0,3.0"
for round in 1 2; do
  timeout -k 10 200 python bench.py $B > $O/new_$round.json 2>/dev/null || exit 1
  for v in $VARIANTS; do LDPC_HIP_LIB=variants/$v.so timeout -k 10 200 python bench.py $B > $O/${v}_$round.json 2>/dev/null || exit 1; done
done
for f in $O/*.json; do python -c "import json,sys;d=json.load(open('$f'));r=d['roofline'];print('$f',round(d['value']),round(r['frac'],3),[(p['snr_db'],round(p['value']),p['slots']) for p in d['snr_points']])"; done
