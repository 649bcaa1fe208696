"""Which HIP runtime does a process get when torch and libmml_hip.so share it? (diagnostic)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
order = sys.argv[1]


def maps():
    return sorted({l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l or "hsa-runtime" in l})


if order == "torch_first":
    import torch
    print("torch avail", torch.cuda.is_available(), torch.cuda.device_count())
    from mymedialite_amd import _native as N
    N.lib()
else:
    from mymedialite_amd import _native as N
    N.lib()
    print("mml devices", N.device_count())
    import torch
    print("torch avail", torch.cuda.is_available(), torch.cuda.device_count())
print(maps())
ctx = N.Context(0)
print("ctx ok")
x = torch.arange(10, device="cuda:0", dtype=torch.int32)
torch.cuda.synchronize()
print("torch ok", x.sum().item())
