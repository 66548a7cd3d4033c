#!/bin/bash
# Round 4: device-list route checks on one GPU -- the multi-device GPU tests (ordering fence,
# batch cancellation, set_init atomicity), bench.py --devices / --device-ids rehearsals
# (entries 0,0 on one card), config 5's strong-scaling estimate, and the torchrun path's
# device-list sub-line rehearsed with gloo ranks sharing GPU 0.  Outputs gpurun_out/r4dl/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4dl
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_multidevice.py -x -v --timeout 200 --timeout-method thread -m gpu > $OUT/pytest_md.log 2>&1 || { tail -30 $OUT/pytest_md.log; exit 1; }
timeout -k 10 300 python3 bench.py --device-ids 0,0 --iters 100,100 --steps 1 --warmup 0 --no-cpu > $OUT/dl_c3.json 2> $OUT/dl_c3.err || { tail -20 $OUT/dl_c3.err; exit 1; }
timeout -k 10 300 python3 bench.py --config 5 --device-ids 0,0 --steps 1 --warmup 0 > $OUT/dl_c5.json 2> $OUT/dl_c5.err || { tail -20 $OUT/dl_c5.err; exit 1; }
timeout -k 10 300 python3 bench.py --config 5 --steps 2 --warmup 1 > $OUT/c5.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
FITOCT_BENCH_BACKEND=gloo FITOCT_BENCH_DEVICE_LIST=0,0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --iters 100,100 --steps 1 --warmup 0 > $OUT/tr2_c3.json 2> $OUT/tr2_c3.err || { tail -20 $OUT/tr2_c3.err; exit 1; }
FITOCT_BENCH_BACKEND=gloo FITOCT_BENCH_DEVICE_LIST=0,0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --config 5 --steps 1 --warmup 0 > $OUT/tr2_c5.json 2> $OUT/tr2_c5.err || { tail -20 $OUT/tr2_c5.err; exit 1; }
echo ALL_OK
