"""Build rshim/libfitoct_drive.so: the R-free half of the R shim (src/fitoct_drive.c)
linked against the in-tree libfitoct.so, so tests/test_rshim_driver.py can call it
through ctypes.  (The .Call half, src/fitoct_R.c, needs R's headers: R CMD INSTALL.)
"""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "src", "fitoct_drive.c")
# FITOCT_SANITIZE=1 (scripts/cpu_sanitized_suite.sh): an ASan/UBSan driver linked to the
# sanitized libfitoct (fitoct_amd/build_san/), so both share one library instance
SANITIZE = os.environ.get("FITOCT_SANITIZE", "0") not in ("", "0")
OUT = os.path.join(HERE, "build_san", "libfitoct_drive.so") if SANITIZE else \
    os.path.join(HERE, "libfitoct_drive.so")
LIBDIR = os.path.join(ROOT, "fitoct_amd", "build_san") if SANITIZE else \
    os.path.join(ROOT, "fitoct_amd")


def build(force: bool = False) -> str:
    lib = os.path.join(LIBDIR, "libfitoct.so")
    if not os.path.exists(lib):
        raise RuntimeError(f"{lib} not built: run `python -m fitoct_amd.build` first")
    newest = max(os.path.getmtime(p) for p in (SRC, SRC[:-1] + "h", lib))
    if not force and os.path.exists(OUT) and os.path.getmtime(OUT) >= newest:
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cc = ["/opt/rocm/lib/llvm/bin/clang", "-fsanitize=address,undefined", "-shared-libsan",
          "-g"] if SANITIZE else ["gcc"]
    rpath = "$ORIGIN/../../fitoct_amd/build_san" if SANITIZE else "$ORIGIN/../fitoct_amd"
    cmd = cc + ["-std=c99", "-O2", "-Wall", "-Wextra", "-Werror", "-fPIC", "-shared",
                "-I", os.path.join(ROOT, "include"), SRC, "-o", OUT,
                "-L", LIBDIR, "-lfitoct", f"-Wl,-rpath,{rpath}"]
    subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    print(build(force=True))
