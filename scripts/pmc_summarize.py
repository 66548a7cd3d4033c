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
# the workload as the bench line of the profiled run names it (first pass's JSON line)
line = None
for ln in open(os.path.join(out, "p1.log")):
    ln = ln.strip()
    if ln.startswith("{") and '"metric"' in ln:
        line = json.loads(ln)
workload = line["config"]["workload"] if line else (
    f"fitExpGP+horseshoe N={bench.N_BINS} Nn={bench.NN} {bench.CHAINS} chains/GPU "
    f"W={bench.WARMUP_IT} S={bench.SAMPLES} treedepth<=10")
res = {"workload": workload, "kernel": "nuts_kernel", "launches": 1,
       "fetch_size_bytes_raw": fetch_b, "fetch_bytes_corrected": 2 * fetch_b,
       "write_bytes": write_b, "bytes_per_launch": 2 * fetch_b + write_b,
       "draws_bytes": None, "counters": dict(agg),
       "note": "FETCH_SIZE doubled per the gfx950 correction; FETCH/WRITE count L2 memory-side "
               "requests (MALL hits included) -> an upper bound on HBM bytes"}
if line:
    c = line["config"]
    cols = {"horseshoe": 3 * 15 + 6, "lasso": 15 + 4, "normal": 15 + 5}
    prior = c.get("prior", "normal")
    chains = c.get("chains_per_gpu") or c.get("files_this_rank", 0) * c.get("chains_per_file", 0)
    iters = c.get("warmup_iters", 0) + c.get("samples", 0)
    if not iters:   # batch line: W / S in the workload text
        import re
        m = re.search(r"W=(\d+) S=(\d+)", workload)
        iters = int(m.group(1)) + int(m.group(2)) if m else 0
    res["draws_bytes"] = 8 * chains * iters * (cols.get(prior, 20) + 8)
    res["write_over_draws"] = round(write_b / res["draws_bytes"], 2) if res["draws_bytes"] else None
print(json.dumps(res, indent=1))
