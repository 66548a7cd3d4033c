#!/bin/bash
# Round 5: profiling build (ablib/lib_prof.so, FITOCT_PROFILE=1): tile occupancy of config 3
# at full length (how much of the machine-time the launch's thinned-out tail takes), and the
# config-2 shape's sweep / leaf costs two-ended vs one-ended.  Outputs gpurun_out/r5prof/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5prof
mkdir -p $OUT
export FITOCT_LIB_PATH=$PWD/ablib/lib_prof.so
timeout -k 10 300 python3 scripts/stamps_occupancy.py > $OUT/occupancy.txt 2>&1 || { tail -5 $OUT/occupancy.txt; exit 1; }
cat $OUT/occupancy.txt
timeout -k 10 300 python3 scripts/stamps_config2.py > $OUT/config2.txt 2>&1 || { tail -5 $OUT/config2.txt; exit 1; }
cat $OUT/config2.txt
