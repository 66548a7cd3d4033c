#!/bin/bash
# Secondary bench lines, one launch each after one untimed launch: BASELINE configs 2, 4
# and 5, and config 3 under the reference's hard-geometry profile (Tests/testGamma.R:45,
# with its CPU baseline).  Outputs gpurun_out/secondary/*.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/secondary
mkdir -p $OUT
for c in 2 4 5; do
  timeout -k 10 300 python3 bench.py --config $c --steps 1 --warmup 1 > $OUT/config$c.json 2> $OUT/config$c.err || exit 1
  cat $OUT/config$c.json
done
timeout -k 10 600 python3 bench.py --steps 1 --warmup 0 --adapt-delta 0.99 --max-treedepth 12 > $OUT/hard.json 2> $OUT/hard.err || exit 1
cat $OUT/hard.json
