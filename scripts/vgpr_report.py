"""VGPR / spill / scratch per kernel instantiation of one family (hipcc remarks).

    python scripts/vgpr_report.py [family] [filter]
"""
import os
import re
import subprocess
import sys

fam = sys.argv[1] if len(sys.argv) > 1 else "2"
flt = sys.argv[2] if len(sys.argv) > 2 else "nuts_kernel"
r = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-DFITOCT_FAMILY={fam}",
                    "-Iinclude", "-Ifitoct_amd/csrc", "--cuda-device-only", "-c",
                    os.environ.get("SRC", "fitoct_amd/csrc/nuts_device.hip"), "-o", "/tmp/vgpr_report.o",
                    "-Rpass-analysis=kernel-resource-usage"] + os.environ.get("FITOCT_HIPFLAGS", "").split(),
                   capture_output=True, text=True)
cur, rows = None, {}
for line in r.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark: +(VGPRs|VGPRs Spill|ScratchSize \[bytes/lane\]|SGPRs Spill): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1)] = int(m.group(2))
for k, v in rows.items():
    if flt in k:
        print(f"{k:60s} vgpr {v.get('VGPRs')} vspill {v.get('VGPRs Spill')} "
              f"sspill {v.get('SGPRs Spill')} scratch {v.get('ScratchSize [bytes/lane]')}")
