#!/bin/bash
# Round 6 measurement bundle, part B: the secondary lines (configs 2, 4, 5 with CPU
# baselines), rocprofv3 kernel stats of one config-2 step, PMC HBM traffic of config 2.
# gpurun_out/r6bundle/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r6bundle
mkdir -p $OUT
for c in ${CONFIGS:-2 4 5}; do
  timeout -k 10 400 python3 bench.py --config $c --steps 2 --warmup 1 > $OUT/config$c.json 2> $OUT/config$c.err || { tail -5 $OUT/config$c.err; exit 1; }
  head -c 300 $OUT/config$c.json; echo
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace2 -o bench -- python3 bench.py --config 2 --steps 1 --warmup 0 --no-cpu > $OUT/trace2.out 2>&1 || { tail -5 $OUT/trace2.out; exit 1; }
for c in ${PMC:-2}; do
  bash scripts/pmc_traffic.sh $c > $OUT/pmc$c.out 2>&1 || { tail -5 $OUT/pmc$c.out; exit 1; }
  tail -2 $OUT/pmc$c.out
done
