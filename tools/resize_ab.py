#!/usr/bin/env python3
"""Dev A/B for the resize kernel alone: 64 x 4096^2 RGBA8 -> 512^2 Triangle through
ik_resize_batch_device of the library at argv[1] (plain ctypes: works with older
builds), HIP events on a stream of our own; prints one JSON line."""
import ctypes
import json
import sys

import numpy as np
import torch

S, O, B = 4096, 512, 64
lib = ctypes.CDLL(sys.argv[1])
lib.ik_init.argtypes = [ctypes.c_int]
f = lib.ik_resize_batch_device
f.restype = ctypes.c_int
f.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_size_t, ctypes.c_size_t,
              ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
              ctypes.c_size_t, ctypes.c_void_p]
assert lib.ik_init(0) == 0
src = torch.randint(0, 256, (B, S, S * 4), dtype=torch.uint8, device="cuda")
dst = torch.empty((B, O, O * 4), dtype=torch.uint8, device="cuda")
st = torch.cuda.Stream()
torch.cuda.synchronize()
res = {}
for filt, name in ((1, "triangle"), (4, "lanczos3")):
    ms = []
    for r in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        assert f(src.data_ptr(), S, S, 4, S * 4, S * S * 4, B, O, O, filt, dst.data_ptr(), O * 4, O * O * 4,
                 st.cuda_stream) == 0
        e1.record(st)
        e1.synchronize()
        if r:
            ms.append(e0.elapsed_time(e1))
    res[name] = round(float(np.median(ms)), 4)
print(json.dumps({"lib": sys.argv[1], **res}))
