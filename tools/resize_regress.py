#!/usr/bin/env python3
"""Dev probe for VERDICT r2 weak-2: is the k_resize_fused slowdown (0.90 -> 1.40 ms
per 64 x 4096^2 -> 512^2 Triangle launch since fbd8c50) in the kernel or in where
its source frames live?  The kernel's code object is unchanged by that commit
(same VGPR/SGPR counts and instruction mix), so this times the same launch
(ik_resize_batch_device, HIP events on torch's stream) on

  A  a fresh 4 GiB torch buffer in a fresh process,
  B  the same buffer after a PNG transform batch has filled the library's
     image pool (the bench's order: headline first, hbm_resident after),
  C  a torch buffer allocated after that batch.

Prints one JSON line."""
import ctypes
import io
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-image-transform_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ikutil  # noqa: E402

ikutil.use_pillow_codecs()
from imagekit import _lib, transform_batch  # noqa: E402

S, O, B = 4096, 512, 64
TRI = 1


STREAM = None


def timed(lib, src, dst, reps=5):
    # a stream of our own: torch's default stream is the null stream (handle 0),
    # which the library would read as "use the thread's stream"
    global STREAM
    if STREAM is None:
        STREAM = torch.cuda.Stream()
    st = STREAM
    ms = []
    for r in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        rc = lib.ik_resize_batch_device(ctypes.c_void_p(src.data_ptr()), S, S, 4, S * 4, S * S * 4, B, O, O, TRI,
                                        ctypes.c_void_p(dst.data_ptr()), O * 4, O * O * 4,
                                        ctypes.c_void_p(st.cuda_stream))
        assert rc == 0, _lib.last_error()
        e1.record(st)
        e1.synchronize()
        if r:
            ms.append(e0.elapsed_time(e1))
    return round(float(np.median(ms)), 4), [round(x, 4) for x in ms]


def main():
    lib = _lib.load()
    assert lib.ik_init(0) == 0
    out = {}
    frames = [ikutil.synth(S, S, 4, seed=s, pattern="S") for s in range(4)]
    torch.cuda.synchronize()
    src = torch.empty((B, S, S * 4), dtype=torch.uint8, device="cuda")
    for i in range(B):
        src[i].copy_(torch.from_numpy(frames[i % 4].reshape(S, S * 4)))
    dst = torch.empty((B, O, O * 4), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    out["A_fresh"] = timed(lib, src, dst)
    from PIL import Image
    pngs = []
    for f in frames:
        b = io.BytesIO()
        Image.fromarray(f, "RGBA").save(b, format="PNG")
        pngs.append(b.getvalue())
    reqs = [pngs[i % 4] for i in range(B)]
    t0 = time.perf_counter()
    for _ in range(2):
        transform_batch(reqs, [(O, O)] * B, [1] * B, [80] * B, filter=TRI, threads=32)
    out["png_batches_s"] = round(time.perf_counter() - t0, 2)
    out["B_same_buffer_after_pool"] = timed(lib, src, dst)
    src2 = torch.empty((B, S, S * 4), dtype=torch.uint8, device="cuda")
    src2.copy_(src)
    torch.cuda.synchronize()
    out["C_new_buffer_after_pool"] = timed(lib, src2, dst)
    out["A2_fresh_again"] = timed(lib, src, dst)
    gb = B * (4 * S * S + 4 * O * O) / 1e9
    for k in list(out):
        if k.startswith(("A", "B", "C")):
            out[k + "_TBps"] = round(gb / out[k][0], 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
