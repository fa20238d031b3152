# Final round-3 evidence on the GPU box: tests/gpu_round.sh, then the gloo two-rank rehearsal of
# the multi-rank bench and the fail-fast check of --gpus 2 with RCCL on one GPU.
set -o pipefail
bash tests/gpu_round.sh r03i || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --batch 32 --dist-backend gloo --no-c4 --no-e2e --no-c2 > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err && echo rehearse ok || exit 1
tail -c 600 gpurun_out/rehearse2.json
timeout -k 10 120 python bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/failfast.json 2> gpurun_out/failfast.err; echo "gpus 2 on one GPU: rc=$?"; tail -2 gpurun_out/failfast.err
