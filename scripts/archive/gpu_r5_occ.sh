#!/bin/bash
# Round 5: the compressed-bundle library loads and runs (smoke + the ABI/migration GPU tests),
# then the profiling build (gpulib/lib_prof.so) measures config 3's tile occupancy at full
# length with the end-of-launch idle time attributed to k = 0.  Outputs gpurun_out/r5occ/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5occ
mkdir -p $OUT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_migration.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
FITOCT_LIB_PATH=$PWD/gpulib/lib_prof.so timeout -k 10 300 python3 scripts/stamps_occupancy.py > $OUT/occupancy.txt 2>&1 || { tail -20 $OUT/occupancy.txt; exit 1; }
grep -h "occupancy\|kernel\|tile ends" $OUT/occupancy.txt
