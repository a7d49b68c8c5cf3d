"""Diagnose the GPU PNG batch decode (dev tool; needs a dev library built with
-DIK_PNG_DUMP, IK_LIB_PATH pointing at it): decode bench.py's 64-frame batch with
ik_decode_batch, then per frame compare (a) the filtered rows + filter types
before the unfilter pass with zlib's inflate of the same stream and (b) the
decoded pixels with the source frame."""
import ctypes
import json
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rust-image-transform_amd"), os.path.join(ROOT, "tests")]
import ikutil  # noqa: E402
import bench  # noqa: E402
from imagekit import _lib  # noqa: E402

lib = _lib.load()
lib.ik_dev_png_dump.restype = ctypes.c_longlong
lib.ik_dev_png_dump.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
assert lib.ik_init(0) == 0
S = 4096
B = int(os.environ.get("B", "64"))
frames = [ikutil.synth(S, S, 4, seed=sd, pattern="S") for sd in bench.shard_seeds(0, 4)]
pngs = bench.make_pngs(frames)


def idat(p):
    out, pos = b"", 8
    while pos < len(p):
        n = int.from_bytes(p[pos:pos + 4], "big")
        if p[pos + 4:pos + 8] == b"IDAT":
            out += p[pos + 8:pos + 8 + n]
        pos += 12 + n
    return zlib.decompress(out)


raw = [np.frombuffer(idat(p), np.uint8).reshape(S, 4 * S + 1) for p in pngs]
report = []
for rep in range(int(os.environ.get("REPS", "2"))):
    keep = [ctypes.create_string_buffer(pngs[i % 4], len(pngs[i % 4])) for i in range(B)]
    arr = (ctypes.c_void_p * B)(*[ctypes.addressof(k) for k in keep])
    lens = (ctypes.c_size_t * B)(*[len(pngs[i % 4]) for i in range(B)])
    outs = (ctypes.c_void_p * B)()
    st = (ctypes.c_int * B)()
    assert lib.ik_decode_batch(arr, lens, B, outs, None, st) == 0
    dump = np.empty(S * 4 * S + S, np.uint8)
    for i in range(B):
        n = lib.ik_dev_png_dump(i, dump.ctypes.data, dump.nbytes)
        r = raw[i % 4]
        rows = dump[:S * 4 * S].reshape(S, 4 * S)
        ft = dump[S * 4 * S:]
        badf = np.nonzero(np.any(rows != r[:, 1:], axis=1))[0]
        badt = np.nonzero(ft != r[:, 0])[0]
        px = np.empty((S, S, 4), np.uint8)
        lib.ik_image_to_host(outs[i], px.ctypes.data, px.nbytes)
        lib.ik_image_free(outs[i])
        badp = np.nonzero(np.any(px.reshape(S, -1) != frames[i % 4].reshape(S, -1), axis=1))[0]
        if len(badf) or len(badt) or len(badp):
            e = {"rep": rep, "img": i, "dump_bytes": int(n), "bad_filtered_rows": badf[:8].tolist(),
                 "n_bad_filtered_rows": int(len(badf)), "bad_ft": badt[:8].tolist(),
                 "bad_pixel_rows": badp[:8].tolist(), "n_bad_pixel_rows": int(len(badp))}
            if len(badf):
                y = int(badf[0])
                cols = np.nonzero(rows[y] != r[y, 1:])[0]
                e["first_bad_filtered"] = [y, cols[:8].tolist(), int(len(cols))]
            print(json.dumps(e), flush=True)
            report.append(e)
print("summary", json.dumps({"bad_images": len(report)}), flush=True)
