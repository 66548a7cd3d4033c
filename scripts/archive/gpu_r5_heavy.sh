#!/bin/bash
# Round 5: heaviest-first migration (try_donate, P.mig_heavy) -- the migration GPU tests
# (draws bitwise against non-migrating launches), then config 3 at full length with and
# without it (FITOCT_MIG_HEAVY=0), same library, interleaved.  Outputs gpurun_out/r5heavy/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5heavy
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_migration.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for r in 1 2 3; do
  for h in 1 0; do
    FITOCT_MIG_HEAVY=$h timeout -k 10 200 python3 bench.py --config 3 --steps 1 --warmup 0 --no-cpu --no-hard \
       2>>$OUT/stderr.log > $OUT/b.json || exit 1
    python3 -c "import json;d=json.load(open('$OUT/b.json'));print('heavy=$h', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d.get('migrations'))" | tee -a $OUT/ab.txt
  done
done
