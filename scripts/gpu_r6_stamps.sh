#!/bin/bash
# Round 6: profiling-build stamps of one config-2 step, paired tiles on and off
# (prof6/lib_prof.so: FITOCT_VARIANT=prof FITOCT_PROFILE=1 python -m fitoct_amd.build --force,
# copied to prof6/).  gpurun_out/r6stamps/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r6stamps}
mkdir -p $OUT
for v in ${VARIANTS:-pair nopair}; do
  ev=""; [ $v = nopair ] && ev="FITOCT_NO_PAIR=1"
  env $ev FITOCT_LIB_PATH=$PWD/prof6/lib_prof.so FITOCT_STAMPS=1 timeout -k 10 200 python3 bench.py \
     --config ${CONFIG:-2} --steps 1 --warmup 0 --no-cpu --no-hard > $OUT/$v.json 2> $OUT/$v.err || { tail -5 $OUT/$v.err; exit 1; }
  echo "=== $v"; grep 'fitoct stamps' $OUT/$v.err
done
