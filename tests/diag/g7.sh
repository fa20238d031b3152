# Two-rank gloo rehearsal of the multi-GPU bench on the one-GPU box, self-verifying (--verify:
# per-image digests all-gathered, a sample recomputed on rank 0), then the N = 1 verify line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --batch 32 --dist-backend gloo --verify > gpurun_out/rehearse2v.json 2> gpurun_out/rehearse2v.err && echo rehearse ok && \
timeout -k 10 300 python bench.py --verify --no-c4 --no-e2e --no-match --no-cpu-baseline --no-c2 > gpurun_out/verify1.json 2> gpurun_out/verify1.err && echo verify1 ok
