#!/bin/bash
# Round-4 final checks: the whole GPU suite, smoke(), and the 8-rank torchrun path rehearsed on
# one GPU (gloo ranks sharing it) -- with the device-list sub-line over eight entries of GPU 0,
# and without (devices 1..7 do not exist: the sub-line must record its error, not crash the
# line).  Outputs gpurun_out/r4fc/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4fc
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
FITOCT_BENCH_BACKEND=gloo FITOCT_BENCH_DEVICE_LIST=0,0,0,0,0,0,0,0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29551 bench.py --gpus 8 --steps 1 --warmup 0 --iters 50,50 > $OUT/reh8.json 2> $OUT/reh8.err || { tail -30 $OUT/reh8.err; exit 1; }
FITOCT_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29552 bench.py --config 5 --gpus 8 --steps 1 --warmup 0 > $OUT/reh8c5.json 2> $OUT/reh8c5.err || { tail -30 $OUT/reh8c5.err; exit 1; }
python3 -c "
import json
for f in ('reh8', 'reh8c5'):
    d = json.loads(open('$OUT/' + f + '.json').read().strip().splitlines()[-1])
    print(f, d['value'], d['n_gpus'], d['config']['route'], json.dumps(d.get('device_list'))[:300])
"
