"""Build libfitoct.so in-tree (hipcc, gfx950).  No torch, no JIT cache: the
shared object sits next to this file so it travels with the repository
snapshot to the GPU box.

    python -m fitoct_amd.build [--force] [--verbose]
    FITOCT_PROFILE=1 python -m fitoct_amd.build --force   # diagnostic cycle-stamp build
    python -m fitoct_amd.build --sanitize   # host code under ASan + UBSan -> build_san/ (CPU suite)
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(ROOT, "include")
LIB = os.path.join(HERE, "libfitoct.so")
OBJDIR = os.path.join(HERE, "build")
# --sanitize: every host translation unit under AddressSanitizer + UBSan (clang's runtime,
# the one hipcc links), device code unchanged; for the CPU suite only
# (scripts/cpu_sanitized_suite.sh), never shipped
SAN_DIR = os.path.join(HERE, "build_san")
SAN_LIB = os.path.join(SAN_DIR, "libfitoct.so")
SAN_FLAGS = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"]
CLANGXX = "/opt/rocm/lib/llvm/bin/clang++"
# FITOCT_VARIANT=name: an A/B variant library (FITOCT_HIPFLAGS / FITOCT_PROFILE) built to
# ablib/lib_<name>.so with its own objects, leaving fitoct_amd/libfitoct.so alone; load it
# with FITOCT_LIB_PATH (scripts/ab_libs.sh)
VARIANT = os.environ.get("FITOCT_VARIANT", "")
ARCH = os.environ.get("FITOCT_ARCH", "gfx950")

# --offload-compress: the gfx950 code objects of the ~100 sampler instantiations per family
# are stored compressed in the fat binary (24 MiB -> ~3 MiB library; the HIP runtime
# decompresses at module load), which keeps the tree pushed to a GPU box small
_KERNEL = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "--offload-compress"]
SOURCES = [
    # (object name, source, compiler, flags).  The sampler source is compiled once
    # per prior family (the family is a template parameter of the kernels).
    ("nuts_normal", "nuts_device.hip", "hipcc", _KERNEL + ["-DFITOCT_FAMILY=0"]),
    ("nuts_lasso", "nuts_device.hip", "hipcc", _KERNEL + ["-DFITOCT_FAMILY=1"]),
    ("nuts_horseshoe", "nuts_device.hip", "hipcc", _KERNEL + ["-DFITOCT_FAMILY=2"]),
    ("nuts_monoexp", "nuts_device.hip", "hipcc", _KERNEL + ["-DFITOCT_FAMILY=3"]),
    ("fitoct_api", "fitoct_api.cpp", "hipcc", [f"--offload-arch={ARCH}", "-O2", "-std=c++17"]),
    ("multi_device", "multi_device.cpp", "hipcc", [f"--offload-arch={ARCH}", "-O2", "-std=c++17"]),
    ("host_model", "host_model.cpp", "g++", ["-O2", "-std=c++17"]),
    ("optimize", "optimize.cpp", "g++", ["-O2", "-std=c++17"]),
    ("stan_output", "stan_output.cpp", "g++", ["-O2", "-std=c++17"]),
]
# FITOCT_PROFILE=1: a diagnostic build whose kernels record cycle stamps
# (read with FITOCT_STAMPS=1); production builds carry no timing code.
PROFILE = os.environ.get("FITOCT_PROFILE", "0") not in ("", "0")
HEADERS = ["kernel_params.h", "philox.h", "host_internal.h", "plan_internal.h"]
# FITOCT_HIPFLAGS="-DX=1 ...": extra device-compile flags for A/B variant libraries
# (built with --force, copied aside, loaded through FITOCT_LIB_PATH)
EXTRA = os.environ.get("FITOCT_HIPFLAGS", "").split()


def _hipcc() -> str:
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build libfitoct)")


def _flags_file() -> str:
    return os.path.join(OBJDIR, "flags.txt")


def _flags() -> str:
    return f"arch={ARCH} profile={int(PROFILE)} extra={' '.join(EXTRA)}"


def _newest_input() -> float:
    paths = [os.path.join(CSRC, s) for _, s, _, _ in SOURCES]
    paths += [os.path.join(CSRC, h) for h in HEADERS]
    paths += [os.path.join(INCLUDE, "fitoct.h"), os.path.abspath(__file__)]
    return max(os.path.getmtime(p) for p in paths)


def _newest_dep(src: str) -> float:
    """Newest mtime of ``src``, the headers it includes (transitively, quoted includes
    resolved in csrc/ and include/) and this build script."""
    import re
    seen, todo, newest = set(), [src], os.path.getmtime(os.path.abspath(__file__))
    while todo:
        p = todo.pop()
        if p in seen or not os.path.exists(p):
            continue
        seen.add(p)
        newest = max(newest, os.path.getmtime(p))
        with open(p, errors="replace") as f:
            for inc in re.findall(r'^\s*#\s*include\s+"([^"]+)"', f.read(), flags=re.M):
                todo += [os.path.join(CSRC, inc), os.path.join(INCLUDE, inc)]
    return newest


def build(force: bool = False, verbose: bool = False, sanitize: bool = False) -> str:
    """Compile every translation unit and link ``fitoct_amd/libfitoct.so`` (or, with
    ``sanitize``, the ASan/UBSan host build ``fitoct_amd/build_san/libfitoct.so``)."""
    objdir, lib = (SAN_DIR, SAN_LIB) if sanitize else (OBJDIR, LIB)
    if VARIANT and not sanitize:
        objdir = os.path.join(ROOT, "ablib", "obj_" + VARIANT)
        lib = os.path.join(ROOT, "ablib", f"lib_{VARIANT}.so")
    flags_file = os.path.join(objdir, "flags.txt")
    same_flags = os.path.exists(flags_file) and open(flags_file).read() == _flags()
    if (not force and same_flags and os.path.exists(lib)
            and os.path.getmtime(lib) >= _newest_input()):
        return lib
    os.makedirs(objdir, exist_ok=True)
    hipcc = _hipcc()

    def compile_one(item):
        name, src, cc, flags = item
        obj = os.path.join(objdir, name + ".o")
        # incremental: an object is rebuilt only if its source or a header it includes
        # changed, or the build flags did (the sampler kernels take minutes to compile)
        if (not force and same_flags and os.path.exists(obj)
                and os.path.getmtime(obj) >= _newest_dep(os.path.join(CSRC, src))):
            return obj
        if PROFILE and cc == "hipcc":
            flags = flags + ["-DFITOCT_PROFILE=1"]
        if cc == "hipcc" and EXTRA:
            flags = flags + EXTRA
        if sanitize:   # host side only: each -fsanitize right after -Xarch_host for hipcc
            flags = flags + ([a for f in SAN_FLAGS for a in ("-Xarch_host", f)]
                             if cc == "hipcc" else SAN_FLAGS + ["-g"])
        exe = hipcc if cc == "hipcc" else (CLANGXX if sanitize else (shutil.which("g++") or "g++"))
        cmd = [exe, *flags, "-fPIC", "-Wall", f"-I{INCLUDE}", f"-I{CSRC}",
               "-I/opt/rocm/include", "-c", os.path.join(CSRC, src), "-o", obj]
        if cc != "hipcc":
            cmd.insert(1, "-D__HIP_PLATFORM_AMD__")
        record = name.startswith("nuts_") and not sanitize
        if record:   # per-kernel VGPR / spill / scratch remarks, kept beside the object
            cmd.append("-Rpass-analysis=kernel-resource-usage")
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if record:
            with open(os.path.join(objdir, name + ".resources.txt"), "w") as f:
                f.write(r.stderr)
        elif verbose and r.stderr.strip():
            print(r.stderr, file=sys.stderr)
        return obj

    with ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = lib + ".tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
    if sanitize:
        cmd += ["-fsanitize=address,undefined", "-shared-libsan"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, lib)
    with open(flags_file, "w") as f:
        f.write(_flags())
    return lib


def kernel_resources(text: str) -> dict:
    """Parse hipcc's ``-Rpass-analysis=kernel-resource-usage`` remarks into
    {mangled kernel name: {"VGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize", ...}}."""
    import re
    cur, rows = None, {}
    for line in text.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            rows[cur] = {}
            continue
        m = re.search(r"remark: +(VGPRs|AGPRs|VGPRs Spill|SGPRs|SGPRs Spill|"
                      r"ScratchSize \[bytes/lane\]|LDS Size \[bytes/block\]): (\d+)", line)
        if m and cur:
            rows[cur][m.group(1).split(" [")[0]] = int(m.group(2))
    return rows


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose="--verbose" in sys.argv,
                sanitize="--sanitize" in sys.argv))
