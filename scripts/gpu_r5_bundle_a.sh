#!/bin/bash
# Round 5 measurement bundle, part A: the default bench line (config 3 + hard-geometry
# sub-line + CPU baseline), rocprofv3 kernel stats of one config-3 step, PMC HBM traffic of
# config 3.  gpurun_out/r5bundle/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5bundle
mkdir -p $OUT
timeout -k 10 500 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-hard > $OUT/trace.out 2>&1 || { tail -5 $OUT/trace.out; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" -exec cat {} \; | head -5
bash scripts/pmc_traffic.sh 3 > $OUT/pmc3.out 2>&1 || { tail -5 $OUT/pmc3.out; exit 1; }
tail -3 $OUT/pmc3.out
