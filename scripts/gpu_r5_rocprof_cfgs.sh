#!/bin/bash
# Round 5: rocprofv3 kernel stats of one step of configs 2, 4 and 5 (final tree), beside the
# headline's (scripts/gpu_r5_bundle_c.sh).  gpurun_out/r5rocprof/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5rocprof
mkdir -p $OUT
for c in 2 4 5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c$c -o run -- \
    python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu --no-hard > $OUT/c$c.json 2> $OUT/c$c.err || { tail -5 $OUT/c$c.err; exit 1; }
  head -c 200 $OUT/c$c.json; echo
  find $OUT/c$c -name "*kernel_stats.csv" -exec head -3 {} \;
done
