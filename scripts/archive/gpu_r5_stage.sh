#!/bin/bash
# Round 5: two-ended producers stage the next leaf before writing the last one's record
# (nuts_device.hip produce) -- the two-ended GPU tests on the new library, then configs 2 and
# 3 at full length against gpulib/lib_base.so (the previous tree), interleaved.
# Outputs gpurun_out/r5stage/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5stage
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_spec.py tests/test_gpu_migration.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for r in ${REPS:-1 2}; do
  for c in ${CONFIGS:-2 3}; do
    for l in new base; do
      lp=""; [ $l = base ] && lp=$PWD/gpulib/lib_base.so
      st=1; [ $c = 2 ] && st=3
      FITOCT_LIB_PATH=$lp timeout -k 10 200 python3 bench.py --config $c --steps $st --warmup 1 --no-cpu --no-hard \
         2>>$OUT/stderr.log > $OUT/b.json || exit 1
      python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$l config $c', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" | tee -a $OUT/ab.txt
    done
  done
done
