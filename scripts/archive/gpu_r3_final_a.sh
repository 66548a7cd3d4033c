#!/bin/bash
# Round-3 final measurements, part A: the whole GPU test suite, the default bench line (with
# its hard-geometry sub-line), rocprofv3 kernel stats of the headline workload.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r3f
mkdir -p $OUT
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-hard > $OUT/trace.out 2>&1 || { tail -5 $OUT/trace.out; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" | head -1 | xargs cat
