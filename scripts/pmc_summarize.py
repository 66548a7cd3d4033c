"""Summarise the PMC passes of scripts/pmc_traffic.sh for nuts_kernel.

FETCH_SIZE / WRITE_SIZE are in KiB (rocprofv3 derived counters).  Per
/opt/skills/guides/MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE
reports 1/2 of the bytes of wide coalesced streaming reads -> doubled here;
WRITE_SIZE is exact for 16-B/lane stores.  Both come from the L2 memory-side
request counters (Infinity-Cache hits included), so they bound HBM traffic from
above."""
import csv, glob, json, os, sys, collections
sys.path.insert(0, os.getcwd())
import bench
out = sys.argv[1]
agg = collections.defaultdict(float)
n_disp = collections.Counter()
for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "nuts_kernel" in r.get("Kernel_Name", ""):
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            n_disp[(r["Counter_Name"], r.get("Dispatch_Id", ""))] += 1
fetch_b = agg.get("FETCH_SIZE", 0.0) * 1024
write_b = agg.get("WRITE_SIZE", 0.0) * 1024
workload = (f"fitExpGP+horseshoe N={bench.N_BINS} Nn={bench.NN} {bench.CHAINS} chains/GPU "
            f"W={bench.WARMUP_IT} S={bench.SAMPLES} treedepth<=10")
res = {"workload": workload, "kernel": "nuts_kernel", "launches": 1,
       "fetch_size_bytes_raw": fetch_b, "fetch_bytes_corrected": 2 * fetch_b,
       "write_bytes": write_b, "bytes_per_launch": 2 * fetch_b + write_b,
       "counters": dict(agg),
       "note": "FETCH_SIZE doubled per the gfx950 correction; FETCH/WRITE count L2 memory-side "
               "requests (MALL hits included) -> an upper bound on HBM bytes"}
print(json.dumps(res, indent=1))
