#!/bin/bash
# WRITE_SIZE (L2 -> memory bytes) of the config-3 launch per A/B library in $AB_DIR
# (one PMC pass each, kernel trace only).  Output: lines "<lib> write_bytes <B>".
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
for l in ${AB_DIR:-ablib}/lib_*.so; do
  n=$(basename $l .so)
  d=gpurun_out/pmcw_$n
  FITOCT_LIB_PATH=$PWD/$l timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d -o run -- python3 bench.py --config ${CFG:-3} --steps 1 --warmup 0 --no-cpu --no-hard > $d.log 2>&1 || { echo "$l failed"; tail -5 $d.log; exit 1; }
  python3 - "$d" "$l" <<'PY'
import csv, glob, sys
tot = 0.0
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "nuts_kernel" in r["Kernel_Name"]:
            tot += float(r["Counter_Value"])
print(sys.argv[2], "write_bytes", tot * 1024)
PY
done
