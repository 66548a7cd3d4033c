#!/bin/bash
# Round-3 final measurements, part B: PMC HBM traffic of configs 3, 2, 4, 5 and the
# secondary bench lines (configs 2, 4, 5).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r3f
mkdir -p $OUT
for c in 3 2 4 5; do timeout -k 10 400 bash scripts/pmc_traffic.sh $c > $OUT/pmc_c$c.out 2>&1 || { tail -5 $OUT/pmc_c$c.out; exit 1; }; done
for c in 2 4 5; do
  timeout -k 10 300 python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu > $OUT/config$c.json 2> $OUT/config$c.err || { tail -5 $OUT/config$c.err; exit 1; }
  cat $OUT/config$c.json
done
