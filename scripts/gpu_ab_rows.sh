#!/bin/bash
# Round 6: basis rows resident in the gradient waves for N <= 512 (FITOCT_ROWS_RES=1 while
# under test) -- parity and bitwise suites with it on, then the same-box A/B on configs 2, 5.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/ab_rows}
mkdir -p $OUT
FITOCT_ROWS_RES=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  ${TESTS:-tests/test_gpu_logp.py tests/test_gpu_pair.py tests/test_gpu_batch.py tests/test_gpu_spec.py tests/test_gpu_sampler.py} > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
OUT=$OUT LIBS="base rows::FITOCT_ROWS_RES=1" CONFIGS="${CONFIGS:-2 5}" REPS="1 2" bash scripts/gpu_ab.sh
