#!/bin/bash
# Round-4 final measurements after two-ended trajectories: bench lines of configs 2 and 5
# (config 5 carries its strong-scaling estimate, whose per-GPU shares run one chain per tile)
# and config 5's PMC traffic.  Outputs gpurun_out/r4fd/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4fd
mkdir -p $OUT
for c in 2 5; do
  timeout -k 10 300 python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu > $OUT/config$c.json 2> $OUT/config$c.err || { tail -5 $OUT/config$c.err; exit 1; }
  cat $OUT/config$c.json
done
timeout -k 10 400 bash scripts/pmc_traffic.sh 5 > $OUT/pmc_c5.out 2>&1 || { tail -5 $OUT/pmc_c5.out; exit 1; }
tail -3 $OUT/pmc_c5.out
