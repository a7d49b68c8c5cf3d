"""Diagnose the self-synchronising GPU JPEG decoder (dev tool; needs a dev library
built with -DIK_JPEG_DUMP, IK_LIB_PATH pointing at it, and lib/libik_jpegmodel.so):
decode JPEGs through ik_decode_batch, then compare the GPU's unstuffed bytes,
interval table, lane records and coefficients with the CPU model's and a Python
restatement, and print the lanes around the first wrong block."""
import ctypes
import io
import json
import os
import sys

import numpy as np
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rust-image-transform_amd"), os.path.join(ROOT, "tests")]
import ikutil  # noqa: E402
from imagekit import _lib  # noqa: E402

lib = _lib.load()
lib.ik_dev_jpeg_dump.restype = ctypes.c_longlong
lib.ik_dev_jpeg_dump.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
assert lib.ik_init(0) == 0
assert lib.ik_set_jpeg_reconstruction(0) == 0  # libjpeg-turbo's, as Pillow
M = ctypes.CDLL(os.path.join(ROOT, "rust-image-transform_amd", "lib", "libik_jpegmodel.so"))
M.ikm_jsync_decode.restype = ctypes.c_int
M.ikm_jsync_decode.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                               ctypes.c_size_t, ctypes.POINTER(ctypes.c_longlong)]

REC = np.dtype([("start", "<u8"), ("exit", "<u8"), ("nblk", "<i4"), ("err", "<i4"), ("dc", "<i4", 4),
                ("work", "<i4"), ("pad", "<i4")])
BASE = np.dtype([("block", "<i8"), ("count", "<i4"), ("dc", "<i4", 4), ("head", "<i4")])


def dump(i, what):
    n = lib.ik_dev_jpeg_dump(i, what, None, 0)
    if n < 0:
        return None
    b = np.empty(n, np.uint8)
    lib.ik_dev_jpeg_dump(i, what, b.ctypes.data, n)
    return b


def frame(data):
    p = 2
    while p < len(data):
        m = data[p + 1]
        ln = data[p + 2] << 8 | data[p + 3]
        if m in (0xC0, 0xC1):
            s = data[p + 4:]
            H, W, nc = s[1] << 8 | s[2], s[3] << 8 | s[4], s[5]
            hv = [(s[7 + 3 * i] >> 4, s[7 + 3 * i] & 15) for i in range(nc)]
            return W, H, hv
        p += 2 + ln


def unstuff(data):
    p = 2
    while True:
        m = data[p + 1]
        ln = data[p + 2] << 8 | data[p + 3]
        if m == 0xDA:
            s = p + 2 + ln
            break
        p += 2 + ln
    e = data.rfind(b"\xff\xd9")
    b = data[s:e]
    out, ivl = bytearray(), [0]
    n = len(b)
    for i in range(n):
        prev = b[i - 1] if i else -1
        cur = b[i]
        nxt = b[i + 1] if i + 1 < n else -1
        last = i + 1 == n
        if cur == 0xFF and 0xD0 <= nxt <= 0xD7:
            ivl.append(8 * len(out))
        keep = (last or nxt == 0) if cur == 0xFF else not (prev == 0xFF and (cur == 0 or 0xD0 <= cur <= 0xD7))
        if keep:
            out.append(cur)
    ivl.append(8 * len(out))
    return bytes(out), ivl


def scan_block_map(W, H, hv):
    hmax, vmax = max(h for h, _ in hv), max(v for _, v in hv)
    mcux, mcuy = -(-W // (8 * hmax)), -(-H // (8 * vmax))
    blk0, bws, nb = [], [], 0
    for h, v in hv:
        blk0.append(nb)
        bws.append(mcux * h)
        nb += mcux * h * mcuy * v
    order = []
    for my in range(mcuy):
        for mx in range(mcux):
            for c, (h, v) in enumerate(hv):
                for by in range(v):
                    for bx in range(h):
                        order.append(blk0[c] + (my * v + by) * bws[c] + mx * h + bx)
    return np.array(order), nb


def run(name, data):
    keep = ctypes.create_string_buffer(data, len(data))
    arr = (ctypes.c_void_p * 1)(ctypes.addressof(keep))
    lens = (ctypes.c_size_t * 1)(len(data))
    outs = (ctypes.c_void_p * 1)()
    st = (ctypes.c_int * 1)()
    assert lib.ik_decode_batch(arr, lens, 1, outs, None, st) == 0 and st[0] == 0
    W, H, hv = frame(data)
    px = np.empty((H, W, 3 if len(hv) == 3 else 1), np.uint8)
    lib.ik_image_to_host(outs[0], px.ctypes.data, px.nbytes)
    lib.ik_image_free(outs[0])
    r = {"case": name}
    ref = np.asarray(Image.open(io.BytesIO(data)))
    r["pixel_mismatch"] = int(np.count_nonzero(px.reshape(ref.shape) != ref))
    raw = dump(0, 0)
    if raw is None or len(raw) == 0:
        r["dump"] = "none (host path?)"
        print(json.dumps(r), flush=True)
        return
    ub, ivl = unstuff(data)
    n4 = len(raw) // 4 * 4
    gb = raw[:n4].reshape(-1, 4)[:, ::-1].reshape(-1)
    ka = len(ub)
    r["unstuffed_bytes"] = ka
    r["unstuff_mismatch"] = int(np.count_nonzero(gb[:min(ka, n4)] != np.frombuffer(ub, np.uint8)[:min(ka, n4)]))
    givl = dump(0, 1).view("<i8")
    r["ivl_ok"] = givl.tolist() == ivl
    stat = dump(0, 6).view("<i4")
    r["status"], r["rounds"] = int(stat[0]), int(stat[1])
    recs = dump(0, 2).view(REC)
    bases = dump(0, 3).view(BASE)
    il = dump(0, 5).view("<i4")
    coef = dump(0, 4).view("<i2").reshape(-1, 64)
    mc = np.zeros_like(coef)
    sts = (ctypes.c_longlong * 9)()
    rc = M.ikm_jsync_decode(data, len(data), 1024, 1024, mc.ctypes.data, mc.size, sts)
    r["model_rc"], r["model_stats"] = rc, list(sts)
    order, nb = scan_block_map(W, H, hv)
    badblk = np.nonzero(np.any(coef != mc, axis=1))[0]
    r["lanes"] = int(len(recs))
    r["bad_blocks"] = int(len(badblk))
    r["sum_counts"] = int(bases["count"].sum())
    r["total_blocks"] = int(len(order))
    incons = [l for l in range(1, len(recs)) if l not in set(il.tolist()) and recs[l]["start"] != recs[l - 1]["exit"]]
    r["inconsistent_lanes"] = incons[:10]
    if len(badblk):
        inv = np.empty(nb, np.int64)
        inv[order] = np.arange(len(order))
        sb = inv[badblk]  # scan order of the bad blocks
        r["bad_scan_blocks"] = sorted(sb.tolist())[:20]
        first = int(sb.min())
        lane = int(np.nonzero((bases["block"] <= first) & (first < bases["block"] + bases["count"]))[0][0])
        r["lane_of_first"] = lane
        rows = []
        for l in range(max(0, lane - 2), min(len(recs), lane + 3)):
            rows.append({"lane": l, "start": [int(recs[l]["start"]) & ((1 << 48) - 1), int(recs[l]["start"]) >> 48 & 15],
                         "exit": [int(recs[l]["exit"]) & ((1 << 48) - 1), int(recs[l]["exit"]) >> 48 & 15],
                         "nblk": int(recs[l]["nblk"]), "err": int(recs[l]["err"]), "dc": recs[l]["dc"].tolist(),
                         "base": int(bases[l]["block"]), "count": int(bases[l]["count"]),
                         "bdc": bases[l]["dc"].tolist()})
        r["lanes_near"] = rows
        b0 = int(badblk[0])
        d = np.nonzero(coef[b0] != mc[b0])[0]
        r["first_bad_block"] = {"block": b0, "scan": int(inv[b0]), "pos": d.tolist()[:16],
                                "gpu": coef[b0][d].tolist()[:16], "model": mc[b0][d].tolist()[:16]}
    print(json.dumps(r), flush=True)


def jpeg(px, **kw):
    b = io.BytesIO()
    Image.fromarray(px).save(b, format="JPEG", **kw)
    return b.getvalue()


for (w, h), sub, q in [((640, 480), 0, 50), ((640, 480), 2, 90), ((2000, 1000), 2, 50), ((2000, 1000), 1, 90)]:
    run(f"{w}x{h}_s{sub}_q{q}", jpeg(ikutil.synth(w, h, 3, seed=w + q), quality=q, subsampling=sub))
run("640x480_rst", jpeg(ikutil.synth(640, 480, 3, seed=3), quality=85, restart_marker_rows=1))
