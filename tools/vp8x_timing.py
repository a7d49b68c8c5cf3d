"""Time the exact GPU WebP coder (ik_webp_encode_exact_device) on a batch of 512x512
frames made the bench's way, against libwebp (WebPEncode on the same planes, one thread
per image) -- wall per batch, and the bytes checked equal.  Usage:
python tools/vp8x_timing.py [--n 64] [--iters 3]"""
import argparse
import ctypes
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-image-transform_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

import ikutil  # noqa: E402
from imagekit import DynamicImage, FilterType, _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=64)
ap.add_argument("--iters", type=int, default=3)
ap.add_argument("--threads", type=int, default=16)
ap.add_argument("--no-check", action="store_true", help="dev builds that change the output: skip the byte check")
ap.add_argument("--stamps", action="store_true", help="IK_VP8X_STAMPS builds: per-phase clock sums of image 0's MBs")
args = ap.parse_args()
ik = _lib.load()
assert ik.ik_init(0) == 0
base = [DynamicImage.from_array(ikutil.synth(4096, 4096, 4, seed=s, pattern="S")).resize(512, 512, FilterType.Triangle).to_array()
        for s in range(4)]
imgs = [base[i % 4] for i in range(args.n)]
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_vp8_analysis import _device_yuv_batch  # noqa: E402
dy, stride = _device_yuv_batch(ik, imgs)
outs = (_lib.u8p * args.n)()
lens = (ctypes.c_size_t * args.n)()
times = []
if args.stamps:
    stamps = (ctypes.c_ulonglong * 32)()
    ik.ik_vp8x_stamps(stamps)  # reset
for it in range(args.iters + 1):
    t = time.perf_counter()
    assert ik.ik_webp_encode_exact_device(dy, stride, args.n, 512, 512, 80, ctypes.cast(outs, ctypes.c_void_p),
                                          ctypes.cast(lens, ctypes.c_void_p)) == 0, _lib.last_error()
    times.append((time.perf_counter() - t) * 1e3)
    files = [ctypes.string_at(outs[i], lens[i]) for i in range(args.n)]
    for i in range(args.n):
        ik.ik_buf_free(outs[i])
if args.stamps:
    ik.ik_vp8x_stamps(stamps)
    names = {0: "prologue", 1: "i16", 2: "i16 select", 10: "i4 A: pred+fwd rows",
             13: "i4 B: fwd cols+quant+inv cols", 15: "i4 C: recon+sse+spectral rows",
             16: "i4 D: spectral cols+rate+argmin+copy", 17: "i4 rotate", 3: "i4 tail", 4: "chroma", 5: "outputs"}
    task = {20: "task: ticket+wait+acquire", 21: "task: whole (loop top to loop top)"}
    calls = (args.iters + 1) * 1024  # image 0's MBs per batch (512^2: 32 x 32)
    tot = sum(stamps[i] for i in names)
    for i, nm in names.items():
        print(f"stamp {i:2d} {nm:24s} {stamps[i] / calls:10.0f} cycles/MB  {100.0 * stamps[i] / max(tot, 1):5.1f} %")
    for i, nm in task.items():
        print(f"stamp {i:2d} {nm:36s} {stamps[i] / calls:10.0f} cycles/MB")
orc = ikutil.Oracle()
ref = [orc.webp_encode_rgb(orc.to_rgb8(base[i]), 80.0) for i in range(4)]
assert args.no_check or all(files[i] == ref[i % 4] for i in range(args.n)), "bytes differ from libwebp"
# libwebp on the host, the same frames, args.threads threads
rgb = [np.ascontiguousarray(orc.to_rgb8(base[i % 4])) for i in range(args.n)]
t = time.perf_counter()
with ThreadPoolExecutor(args.threads) as ex:
    list(ex.map(lambda x: orc.webp_encode_rgb(x, 80.0), rgb))
host_ms = (time.perf_counter() - t) * 1e3
print({"n": args.n, "gpu_exact_ms_per_batch": [round(x, 2) for x in times[1:]], "first_call_ms": round(times[0], 2),
       "libwebp_host_ms_per_batch": round(host_ms, 2), "threads": args.threads, "bytes_equal": True})
ik.ik_dev_free(dy)
