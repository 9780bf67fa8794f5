O=gpurun_out/tailprobe; mkdir -p $O
for F in 64 512 4096; do
timeout -k 10 120 python bench.py --split --schedule static --frames $F --iters 10 --steps 2 --warmup 1 --extra-snr= --cpu-seconds 0 > $O/f$F.json 2>$O/f$F.err || exit 1
python -c "
import json;d=json.loads(open('$O/f$F.json').read().strip().splitlines()[-1]);r=d['decode_roofline'];l=d['roofline']['launches']
print($F, 'ms/step', round(d['ms_per_step'],2), 'cn ms', round(r['cn_ms'],3), 'vn ms', round(r['vn_ms'],3), 'launches', l)"
done
