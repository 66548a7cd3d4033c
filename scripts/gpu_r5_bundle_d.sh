#!/bin/bash
# Round 5 measurement bundle, part D (final tree, after the LDS-ordering commits): the default
# bench line (config 3 + hard geometry + CPU baseline), rocprofv3 kernel stats of one config-3
# step, and the config 2 / 4 / 5 lines with their CPU baselines.  gpurun_out/r5bundle_d/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5bundle_d
mkdir -p $OUT
timeout -k 10 500 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
head -c 300 $OUT/bench.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-hard > $OUT/trace.out 2>&1 || { tail -5 $OUT/trace.out; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" -exec head -2 {} \;
for c in 2 4 5; do
  timeout -k 10 400 python3 bench.py --config $c --steps 2 --warmup 1 > $OUT/config$c.json 2> $OUT/config$c.err || { tail -5 $OUT/config$c.err; exit 1; }
  head -c 250 $OUT/config$c.json; echo
done
