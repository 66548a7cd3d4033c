#!/bin/bash
# Round-3 measurement bundle: bitwise speculation / migration tests, the default bench line
# (with its hard-geometry sub-line), rocprofv3 kernel stats of the headline workload, PMC
# traffic of configs 3, 2, 4, 5, and the secondary bench lines.  Outputs gpurun_out/r3/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r3
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_migration.py -x -v --timeout 200 --timeout-method thread -m gpu > $OUT/pytest_spec.log 2>&1 || { tail -20 $OUT/pytest_spec.log; exit 1; }
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-hard > $OUT/trace.out 2>&1 || exit 1
for c in 3 2 4 5; do timeout -k 10 400 bash scripts/pmc_traffic.sh $c > $OUT/pmc_c$c.out 2>&1 || exit 1; done
for c in 2 4 5; do
  timeout -k 10 300 python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu > $OUT/config$c.json 2> $OUT/config$c.err || exit 1
done
