#!/bin/bash
# Round 5 measurement bundle, part B: the secondary lines (configs 2, 4, 5, each with its CPU
# baseline) and the PMC HBM traffic of configs 2, 4, 5.  gpurun_out/r5bundle/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5bundle
mkdir -p $OUT
for c in 2 4 5; do
  timeout -k 10 400 python3 bench.py --config $c --steps 2 --warmup 1 > $OUT/config$c.json 2> $OUT/config$c.err || { tail -5 $OUT/config$c.err; exit 1; }
  head -c 600 $OUT/config$c.json; echo
done
for c in 2 4 5; do
  bash scripts/pmc_traffic.sh $c > $OUT/pmc$c.out 2>&1 || { tail -5 $OUT/pmc$c.out; exit 1; }
  tail -2 $OUT/pmc$c.out
done
