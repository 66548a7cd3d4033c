#!/bin/bash
# Round 4: new GPU tests (testGamma known answer, R bulk route at 8192 chains) and the
# hard-geometry R-hat over step seeds.  Outputs gpurun_out/r4s/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4s
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_sampler.py::test_testgamma_known_answer_on_gpu tests/test_rshim_driver.py::test_bulk_driver_at_config4_chain_count tests/test_gpu_funnel.py::test_headline_funnel_trapping_matches_oracle -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_new.log 2>&1 || { tail -30 $OUT/pytest_new.log; exit 1; }
timeout -k 10 600 python3 -u scripts/hard_seeds.py 1019 1001 1002 1003 1004 1005 > $OUT/hard_seeds.jsonl 2> $OUT/hard_seeds.err || { tail -20 $OUT/hard_seeds.err; exit 1; }
echo ALL_OK
