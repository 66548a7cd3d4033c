#!/bin/bash
# Round 6 measurement bundle, part A: the whole GPU suite, smoke, the default bench line
# (config 3 + hard-geometry sub-line + CPU baseline), rocprofv3 kernel stats of one config-3
# step, PMC HBM traffic of config 3.  gpurun_out/r6bundle/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6bundle
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 500 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
head -c 400 $OUT/bench.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-hard > $OUT/trace.out 2>&1 || { tail -5 $OUT/trace.out; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" -exec cat {} \; | head -4
bash scripts/pmc_traffic.sh 3 > $OUT/pmc3.out 2>&1 || { tail -5 $OUT/pmc3.out; exit 1; }
tail -2 $OUT/pmc3.out
