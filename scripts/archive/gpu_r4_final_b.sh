#!/bin/bash
# Round-4 final measurements, part B: secondary bench lines (configs 2, 4, 5), PMC traffic of
# configs 2, 4, 5 and the SQ stall counters of the config-3 shape.  Outputs gpurun_out/r4f/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4f
mkdir -p $OUT
for c in 2 4 5; do
  timeout -k 10 300 python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu > $OUT/config$c.json 2> $OUT/config$c.err || { tail -5 $OUT/config$c.err; exit 1; }
  cat $OUT/config$c.json
done
for c in 2 4 5; do timeout -k 10 400 bash scripts/pmc_traffic.sh $c > $OUT/pmc_c$c.out 2>&1 || { tail -5 $OUT/pmc_c$c.out; exit 1; }; done
timeout -k 10 200 bash scripts/pmc_stall.sh 0 > $OUT/pmc_stall.out 2>&1 || { tail -5 $OUT/pmc_stall.out; exit 1; }
tail -2 $OUT/pmc_stall.out
