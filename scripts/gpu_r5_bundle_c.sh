#!/bin/bash
# Round 5 measurement bundle, part C (after the tail-threshold change): the default bench line
# (config 3 + hard geometry + CPU baseline), rocprofv3 kernel stats of one config-3 step,
# config 4's line, PMC HBM traffic of configs 3 and 4, and the SQ stall counters of the
# headline's short PMC run.  gpurun_out/r5bundle_c/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5bundle_c
mkdir -p $OUT
timeout -k 10 500 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
head -c 400 $OUT/bench.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-hard > $OUT/trace.out 2>&1 || { tail -5 $OUT/trace.out; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" -exec cat {} \; | head -3
timeout -k 10 400 python3 bench.py --config 4 --steps 2 --warmup 1 > $OUT/config4.json 2> $OUT/config4.err || { tail -5 $OUT/config4.err; exit 1; }
head -c 300 $OUT/config4.json; echo
for c in 3 4; do
  bash scripts/pmc_traffic.sh $c > $OUT/pmc$c.out 2>&1 || { tail -5 $OUT/pmc$c.out; exit 1; }
  tail -2 $OUT/pmc$c.out
done
bash scripts/pmc_stall.sh 0 > $OUT/stall.out 2>&1 || { tail -5 $OUT/stall.out; exit 1; }
tail -3 $OUT/stall.out
