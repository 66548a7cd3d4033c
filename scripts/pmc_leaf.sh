#!/bin/bash
# Instruction mix per chain-gradient of the config-2 shape (one chain per tile, N = 512: the
# latency-bound leaf path), with the sweep (prior_PD 0) and without it (1: NUTS work only).
# One counter pass each, kernel-trace only.  Output gpurun_out/pmc_leaf<PD>/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
PD=${1:-0}
OUT=gpurun_out/pmc_leaf$PD
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
want=""
n=0
for c in SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES; do
  if grep -qw "$c" $OUT/avail.txt && [ $n -lt 8 ]; then want="$want $c"; n=$((n+1)); fi
done
echo "counters:$want" | tee $OUT/counters.txt
[ -n "$want" ] || exit 0
timeout -s KILL 120 rocprofv3 --pmc $want --output-format csv -d $OUT/p -o run -- python3 scripts/prof_config2.py $PD > $OUT/run.log 2>&1 || { tail -5 $OUT/run.log; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, re
agg = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/p/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "nuts_kernel" in r.get("Kernel_Name", ""):
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
lf = int(re.search(r"leapfrogs (\d+)", open(sys.argv[1] + "/run.log").read()).group(1))
print(f"gradients={lf}: " + ", ".join(f"{k}={v/lf:.1f}" for k, v in sorted(agg.items())) + " (per gradient, summed over the tile's waves)")
PY
