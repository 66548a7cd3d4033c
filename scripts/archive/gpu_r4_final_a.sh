#!/bin/bash
# Round-4 final measurements, part A: the default bench line (hard-geometry sub-line at the
# last step's seed), rocprofv3 kernel stats of the headline workload, PMC HBM traffic of
# config 3.  Outputs gpurun_out/r4f/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4f
mkdir -p $OUT
timeout -k 10 500 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-hard > $OUT/trace.out 2>&1 || { tail -5 $OUT/trace.out; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" | head -1 | xargs cat
timeout -k 10 400 bash scripts/pmc_traffic.sh 3 > $OUT/pmc_c3.out 2>&1 || { tail -5 $OUT/pmc_c3.out; exit 1; }
cat $OUT/pmc_c3.out | tail -3
