#!/bin/bash
# Round 6: the whole GPU suite, then the secondary bench lines (configs 2, 4, 5) without CPU legs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r6suite}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
for c in ${CONFIGS:-2 4 5}; do
  timeout -k 10 300 python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu > $OUT/config$c.json 2> $OUT/config$c.err || { tail -5 $OUT/config$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/config$c.json'));print('config $c', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d.get('strong_scaling_est'))"
done
