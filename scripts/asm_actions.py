"""Per-action instruction counts of the sampler kernel from a -S listing compiled
with -DFITOCT_ASM_MARKS (the marks are asm comments at action entries; code is
attributed to the most recent mark in text order, so the counts are approximate
where the compiler interleaves actions)."""
import collections
import subprocess
import sys

fam = sys.argv[1] if len(sys.argv) > 1 else "2"
kern = sys.argv[2] if len(sys.argv) > 2 else "nuts_kernelIdLi8ELi15ELi1ELi0ELi2E"
out = "/tmp/marks.s"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-DFITOCT_FAMILY={fam}",
                "-DFITOCT_ASM_MARKS", "-Iinclude", "-Ifitoct_amd/csrc", "-S", "--cuda-device-only",
                "fitoct_amd/csrc/nuts_device.hip", "-o", out], check=True)
L = open(out).read().split("\n")
st = [i for i, l in enumerate(L) if l.startswith("_ZN6fitoct11" + kern)][0]
en = [i for i in range(st, len(L)) if "s_endpgm" in L[i]][-1] if False else \
    next(i for i in range(st, len(L)) if L[i].startswith(".Lfunc_end"))
cur = "entry"
cnt = collections.defaultdict(collections.Counter)
for l in L[st:en]:
    s = l.strip()
    if ";MARK" in s:
        cur = s.split("MARK")[1].strip()
        continue
    if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
        continue
    op = s.split()[0]
    cls = "valu" if op.startswith("v_") else "salu" if op.startswith("s_") else \
        "lds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "buffer_", "flat_", "scratch_")) else "other"
    cnt[cur][cls] += 1
    if op.startswith("v_"):
        cnt[cur]["f64"] += op.endswith("_f64") or "_f64_" in op
for k, c in sorted(cnt.items(), key=lambda kv: -kv[1]["valu"]):
    print(f"{k:24s} valu {c['valu']:5d} (f64 {c['f64']:4d})  salu {c['salu']:5d}  lds {c['lds']:4d}  vmem {c['vmem']:4d}")
