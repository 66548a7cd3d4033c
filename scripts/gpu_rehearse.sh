#!/bin/bash
# smoke() and a 2-rank rehearsal of the multi-GPU bench path on one GPU (gloo).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
FITOCT_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 0 --iters 150,150 > gpurun_out/reh2.json 2> gpurun_out/reh2.err || { tail -30 gpurun_out/reh2.err; exit 1; }
cat gpurun_out/reh2.json
FITOCT_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --config 5 --gpus 2 --steps 1 --warmup 0 > gpurun_out/reh5.json 2> gpurun_out/reh5.err || { tail -30 gpurun_out/reh5.err; exit 1; }
cat gpurun_out/reh5.json
