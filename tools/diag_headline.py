"""Diagnose headline-batch parity (dev tool): which requests of bench.py's batch
differ from the oracle, under which submission variant, and whether the decoded
pixels (ik_decode_batch) already differ from the source frame."""
import ctypes
import io
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rust-image-transform_amd"), os.path.join(ROOT, "tests")]
import ikutil  # noqa: E402

ikutil.use_pillow_codecs()
import bench  # noqa: E402
from imagekit import DeviceBytes, PinnedBytes, _lib, transform_batch_submit, transform_batch_submit_device  # noqa: E402

lib = _lib.load()
assert lib.ik_init(0) == 0
orc = ikutil.Oracle()
B = int(os.environ.get("B", "64"))
frames = [ikutil.synth(4096, 4096, 4, seed=sd, pattern="S") for sd in bench.shard_seeds(0, 4)]
pngs = bench.make_pngs(frames)
want = [orc.transform(f, 512, 512, ikutil.TRIANGLE, 1, 80)[0] for f in frames]
res = {}


def check(name, outs, src):
    bad = [i for i, o in enumerate(outs) if o != want[src[i]]]
    res[name] = {"bad": bad, "n": len(outs)}
    print(name, "bad", len(bad), bad[:16], flush=True)


def run_dev(name, reqs, depth, threads=32):
    pend = [transform_batch_submit_device(reqs, [(512, 512)] * len(reqs), [1] * len(reqs), [80] * len(reqs),
                                          filter=ikutil.TRIANGLE, threads=threads) for _ in range(depth)]
    for k, p in enumerate(pend):
        check(f"{name}_b{k}", p.wait(), [i % 4 for i in range(len(reqs))])


# the bench's own inputs: one device allocation per request
own = [DeviceBytes(pngs[i % 4]) for i in range(B)]
run_dev("own_depth1", own, 1)
run_dev("own_depth3", own, 3)
alias = [DeviceBytes(p) for p in pngs]
run_dev("alias_depth1", [alias[i % 4] for i in range(B)], 1)
run_dev("own_t1", own, 1, threads=1)
# host inputs
pin = [PinnedBytes(p) for p in pngs]
p = transform_batch_submit([pin[i % 4] for i in range(B)], [(512, 512)] * B, [1] * B, [80] * B,
                           filter=ikutil.TRIANGLE, threads=32)
check("host_pinned", p.wait(), [i % 4 for i in range(B)])
for n in (8, 16, 32):
    run_dev(f"own_n{n}", own[:n], 1)
# decoded pixels of the batch decode path vs the source frames
n = B
bufs = [pngs[i % 4] for i in range(n)]
keep = [ctypes.create_string_buffer(b, len(b)) for b in bufs]
arr = (ctypes.c_void_p * n)(*[ctypes.addressof(k) for k in keep])
lens = (ctypes.c_size_t * n)(*[len(b) for b in bufs])
outs = (ctypes.c_void_p * n)()
st = (ctypes.c_int * n)()
rc = lib.ik_decode_batch(arr, lens, n, outs, None, st)
badpx = []
for i in range(n):
    img = outs[i]
    buf = np.empty((4096, 4096, 4), np.uint8)
    lib.ik_image_to_host(img, buf.ctypes.data, buf.nbytes)
    if not np.array_equal(buf, frames[i % 4]):
        d = np.argwhere(np.any(buf != frames[i % 4], axis=2))
        badpx.append([i, int(len(d)), d[:3].tolist()])
    lib.ik_image_free(img)
res["decode_batch"] = {"rc": rc, "bad": badpx}
print("decode_batch bad", len(badpx), badpx[:8], flush=True)
print(json.dumps(res))
