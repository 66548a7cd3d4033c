#!/bin/bash
# Round 6: doorbell / poll variants of the gradient waves' wait -- bitwise suites on the
# doorbell variant, then the A/B (LIBS overridable).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/ab_db}
mkdir -p $OUT
if [ -n "$TESTLIB" ]; then
FITOCT_LIB_PATH=$PWD/$TESTLIB timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_pair.py tests/test_gpu_migration.py tests/test_gpu_spec.py tests/test_gpu_batch.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
fi
OUT=$OUT LIBS="${LIBS:-base db2:prof6/lib_db2.so pf2:prof6/lib_pf2.so}" CONFIGS="${CONFIGS:-2 3 5}" REPS="1 2" bash scripts/gpu_ab.sh
