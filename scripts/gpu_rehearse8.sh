#!/bin/bash
# 8-rank rehearsal of the multi-GPU bench path on one GPU (gloo; ranks share the card):
# config 3 and config 4 (8 x 1024 = 8192 global chains, R-hat over every rank's gathered
# chains, device_list sub-object) with short W/S, and config 5 (256 files over 8 ranks).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() {   # tag port args...
  local tag=$1 port=$2; shift 2
  FITOCT_BENCH_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 8 --steps 1 --warmup 0 "$@" > gpurun_out/reh8$tag.json 2> gpurun_out/reh8$tag.err || { tail -30 gpurun_out/reh8$tag.err; return 1; }
  grep metric gpurun_out/reh8$tag.json
}
run c3 29541 --config 3 --iters 50,50 && run c4 29543 --config 4 --iters 50,50 && run c5 29542 --config 5
