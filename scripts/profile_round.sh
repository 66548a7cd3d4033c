#!/bin/bash
# Round profile bundle: default bench line, rocprofv3 kernel-trace stats of the
# same workload, PMC HBM traffic.  Outputs under gpurun_out/round/.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/round
mkdir -p $OUT
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $OUT/trace.out 2>&1
find $OUT/trace -name "*kernel_stats.csv" -exec cat {} \;
bash scripts/pmc_traffic.sh > $OUT/pmc.out 2>&1
cat gpurun_out/pmc_traffic/summary.json
