#!/bin/bash
# 8-rank rehearsal of the multi-GPU bench path on one GPU (gloo; ranks share the card).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
FITOCT_BENCH_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 8 --steps 1 --warmup 0 --iters 50,50 > gpurun_out/reh8.json 2> gpurun_out/reh8.err || { tail -30 gpurun_out/reh8.err; exit 1; }
grep metric gpurun_out/reh8.json
FITOCT_BENCH_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29542 bench.py --config 5 --gpus 8 --steps 1 --warmup 0 > gpurun_out/reh8c5.json 2> gpurun_out/reh8c5.err || { tail -30 gpurun_out/reh8c5.err; exit 1; }
grep metric gpurun_out/reh8c5.json
