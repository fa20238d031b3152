# Multi-rank rehearsal on a one-GPU box: two ranks share the GPU, the exchanges go over gloo
# (bench.py --dist-backend gloo), then the N=1 bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --batch 32 --dist-backend gloo > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err && echo rehearse ok && \
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && echo bench ok
