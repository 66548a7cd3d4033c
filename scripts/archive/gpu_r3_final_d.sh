#!/bin/bash
# Secondary lines (configs 2 and 5) on the final tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r3f
mkdir -p $OUT
for c in 2 5; do
  timeout -k 10 300 python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu > $OUT/final_config$c.json 2> $OUT/final_config$c.err || { tail -5 $OUT/final_config$c.err; exit 1; }
  cut -c1-300 $OUT/final_config$c.json
done
