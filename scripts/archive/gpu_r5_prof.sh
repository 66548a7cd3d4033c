#!/bin/bash
# Round 5: profiling build (ablib/lib_prof.so, FITOCT_PROFILE=1): tile occupancy of config 3
# at full length with and without two-ended tails, the config-2 shape's sweep / leaf costs;
# then (production library) the SQ cycle counters of the headline's short PMC run
# (scripts/pmc_stall.sh).  Outputs gpurun_out/r5prof/ and gpurun_out/pmc_stall0/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5prof
mkdir -p $OUT
(export FITOCT_LIB_PATH=$PWD/ablib/lib_prof.so
 timeout -k 10 300 python3 scripts/stamps_occupancy.py > $OUT/occupancy.txt 2>&1 &&
 FITOCT_NO_TAIL_BIDI=1 timeout -k 10 300 python3 scripts/stamps_occupancy.py > $OUT/occupancy_notail.txt 2>&1 &&
 timeout -k 10 300 python3 scripts/stamps_config2.py > $OUT/config2.txt 2>&1) || exit 1
grep -h "occupancy\|kernel" $OUT/occupancy.txt $OUT/occupancy_notail.txt
bash scripts/pmc_stall.sh 0 || exit 1
