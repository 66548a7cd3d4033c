#!/bin/bash
# VALU instruction counts with and without the likelihood sweep (prior_PD=1).
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_split
mkdir -p $OUT
for pd in 0 1; do
  timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM --output-format csv -d $OUT/pd$pd -o run -- python3 scripts/prof_small_pd.py $pd > $OUT/pd$pd.log 2>&1
  timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d $OUT/f$pd -o run -- python3 scripts/prof_small_pd.py $pd > $OUT/f$pd.log 2>&1
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, re
for pd in (0, 1):
    agg = collections.defaultdict(float)
    for d in (f"{sys.argv[1]}/pd{pd}", f"{sys.argv[1]}/f{pd}"):
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "nuts_kernel" in r.get("Kernel_Name", ""):
                    agg[r["Counter_Name"]] += float(r["Counter_Value"])
    lf = int(re.search(r"leapfrogs (\d+)", open(f"{sys.argv[1]}/pd{pd}.log").read()).group(1))
    print(f"prior_PD={pd} gradients={lf}: " + ", ".join(f"{k}={v/lf:.1f}" for k, v in sorted(agg.items())) + " (per gradient)")
PY
