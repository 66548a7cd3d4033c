"""Which HIP runtime does libfitoct bind to, and does torch interop work?"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fitoct_amd import _lib
L = _lib.lib()
maps = open("/proc/self/maps").read()
print("hip runtimes mapped:", sorted({l.split()[-1] for l in maps.splitlines() if "libamdhip64" in l}))
print("hsa runtimes mapped:", sorted({l.split()[-1] for l in maps.splitlines() if "libhsa-runtime64" in l}))
import torch
print("torch sees", torch.cuda.device_count(), "devices; lib sees", L.fitoct_device_count())
x = torch.ones(4, device="cuda"); print("torch alloc ok", float(x.sum()))
