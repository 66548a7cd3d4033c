#!/bin/bash
# Round 4: rocprofv3 kernel stats of config 2 (two-ended trajectories), one step, to back the
# bench line's kernel_ms.  Outputs gpurun_out/r4pc2/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4pc2
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o c2 -- python3 bench.py --config 2 --steps 1 --warmup 0 --no-cpu > $OUT/trace.out 2>&1 || { tail -5 $OUT/trace.out; exit 1; }
grep -h '"value"' $OUT/trace.out | head -1 | cut -c1-300
find $OUT/trace -name "*kernel_stats.csv" | head -1 | xargs head -3
