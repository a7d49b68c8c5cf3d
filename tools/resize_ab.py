#!/usr/bin/env python3
"""Dev A/B for the resize kernel alone: B x 4096^2 C-channel frames -> 512^2 (Triangle
and Lanczos3) through ik_resize_batch_device of the library at argv[1] (plain ctypes:
works with older builds), HIP events on a stream of our own; prints one JSON line.
argv[2] = C (default 4), argv[3] = B (default 64)."""
import ctypes
import json
import sys

import numpy as np
import torch

S, O = 4096, 512
C = int(sys.argv[2]) if len(sys.argv) > 2 else 4
B = int(sys.argv[3]) if len(sys.argv) > 3 else 64
lib = ctypes.CDLL(sys.argv[1])
lib.ik_init.argtypes = [ctypes.c_int]
f = lib.ik_resize_batch_device
f.restype = ctypes.c_int
f.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_size_t, ctypes.c_size_t,
              ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
              ctypes.c_size_t, ctypes.c_void_p]
assert lib.ik_init(0) == 0
src = torch.empty((B, S, S * C), dtype=torch.uint8, device="cuda")
for i in range(B):
    src[i] = torch.randint(0, 256, (S, S * C), dtype=torch.uint8, device="cuda")
dst = torch.empty((B, O, O * C), dtype=torch.uint8, device="cuda")
st = torch.cuda.Stream()
torch.cuda.synchronize()
res = {}
for filt, name in ((1, "triangle"), (4, "lanczos3")):
    ms = []
    for r in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        assert f(src.data_ptr(), S, S, C, S * C, S * S * C, B, O, O, filt, dst.data_ptr(), O * C, O * O * C,
                 st.cuda_stream) == 0
        e1.record(st)
        e1.synchronize()
        if r:
            ms.append(e0.elapsed_time(e1))
    res[name] = round(float(np.median(ms)), 4)
    flat = dst.view(-1).to(torch.int64)
    res[name + "_sum"] = int((flat * (torch.arange(flat.numel(), device="cuda") % 251 + 1)).sum().item())
print(json.dumps({"lib": sys.argv[1], "C": C, "B": B, **res}))
