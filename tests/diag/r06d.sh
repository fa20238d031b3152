# Round 6: tile-size threshold A/B on the batch (128 x 1080p) and C4 (16 x 4096^2, 6 octaves):
# levels of at most SGPU_GAUSS_TILE_MB MB take the tile kernels (0: none).   (GPU box)
set -o pipefail
OUT=gpurun_out/r06d
mkdir -p $OUT
for i in 1 2; do
  for mb in 0 16 32 64; do
    SGPU_GAUSS_TILE_MB=$mb timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-e2e --no-c2 --no-match --no-cpu-baseline > $OUT/b$mb-$i.json 2> $OUT/b$mb-$i.err || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/b$mb-$i.json').read().strip().splitlines()[-1]); c=d['c4']; print('mb=$mb', round(d['value']), round(d['ms_per_step'],3), round(d['roofline']['frac'],4), 'c4', round(c['value']), round(c.get('roofline',{}).get('frac',0),4), {k: round(v,3) for k,v in c.get('stage_ms_per_step',{}).items() if v})"
  done
done
# two ranks sharing the GPU over gloo, self-verifying (bench.py --verify)
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --batch 32 --dist-backend gloo --verify --no-match > $OUT/rehearse2.json 2> $OUT/rehearse2.err || exit 1
python3 -c "import json; d=json.loads(open('$OUT/rehearse2.json').read().strip().splitlines()[-1]); print('rehearse2', round(d['value']), d['verify'])"
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --verify --no-c4 --no-e2e --no-c2 --no-match --no-cpu-baseline > $OUT/verify1.json 2> $OUT/verify1.err || exit 1
python3 -c "import json; d=json.loads(open('$OUT/verify1.json').read().strip().splitlines()[-1]); print('verify1', round(d['value']), d['verify'])"
exit 0
