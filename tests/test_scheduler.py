"""CPU: the multi-device work queue's placement policy and cost model (ik_pool.cpp),
through the C ABI with fake devices -- no GPU work.

The reference serves every request from one tokio process (src/main.rs:20; the
handlers call the transform at src/lib.rs:175-191).  SURVEY 8(e) E-2: one process
drives the node's GPUs through a host work queue, least outstanding cost first.
The loadtest's /sign mix (loadtest/src/main.rs:59-60, 84-85) draws w, h in
[200, 800) and f in {webp, jpeg, avif}; AVIF's host AV1 coding costs ~100x a
WebP request, which is what static round-robin balances badly."""
import ctypes
import io
import random

import numpy as np
import pytest

from imagekit import _lib

JPEG, WEBP, AVIF = 0, 1, 2


def plan(costs, ndev, outstanding=None):
    lib = _lib.load()
    n = len(costs)
    c = (ctypes.c_uint64 * n)(*costs)
    a = (ctypes.c_uint32 * n)()
    o = (ctypes.c_uint64 * ndev)(*outstanding) if outstanding else None
    lib.ik_schedule_plan(c, n, ndev, o, a)
    return list(a)


def loads(costs, assign, ndev, outstanding=None):
    ld = list(outstanding) if outstanding else [0] * ndev
    for c, d in zip(costs, assign):
        ld[d] += c
    return ld


def png_bytes(w, h):
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(np.zeros((h, w, 4), np.uint8), "RGBA").save(b, format="PNG")
    return b.getvalue()


def test_request_cost_follows_header_and_encoder():
    lib = _lib.load()
    small, big = png_bytes(64, 48), png_bytes(640, 480)
    cs = lib.ik_request_cost(small, len(small), 32, -1, WEBP)
    cb = lib.ik_request_cost(big, len(big), 32, -1, WEBP)
    assert cb > cs  # decoded bytes come from IHDR, not the (tiny) file size
    assert cb - lib.ik_request_cost(big, len(big), 32, -1, JPEG) > 0
    assert lib.ik_request_cost(big, len(big), 320, 240, AVIF) > 20 * lib.ik_request_cost(big, len(big), 320, 240, JPEG)


def test_least_outstanding_balances_the_sign_mix():
    rnd = random.Random(7)
    lib = _lib.load()
    src = png_bytes(2000, 2000)
    costs = []
    for _ in range(10_000):  # the loadtest's /img request mix
        w, h, f = rnd.randrange(200, 800), rnd.randrange(200, 800), rnd.choice([WEBP, JPEG, AVIF])
        costs.append(int(lib.ik_request_cost(src, len(src), w, h, f)))
    ndev = 8
    lq = loads(costs, plan(costs, ndev), ndev)
    rr = loads(costs, [i % ndev for i in range(len(costs))], ndev)
    mean = sum(costs) / ndev
    assert max(lq) / mean < 1.01          # least-outstanding (LPT): within 1 % of perfect
    assert max(lq) <= max(rr)
    # one 10x request per 8: round-robin piles them all on device 0
    skew = [10_000 if i % 8 == 0 else 1_000 for i in range(800)]
    rr_skew = loads(skew, [i % ndev for i in range(len(skew))], ndev)
    lq_skew = loads(skew, plan(skew, ndev), ndev)
    assert max(rr_skew) / (sum(skew) / ndev) > 4
    assert max(lq_skew) / (sum(skew) / ndev) < 1.01


def test_outstanding_work_is_respected():
    # device 1 already carries a big backlog: new work goes to the others first
    a = plan([100] * 6, 3, outstanding=[0, 10_000, 0])
    assert 1 not in a and a.count(0) == 3 and a.count(2) == 3


@pytest.mark.parametrize("ndev", [1, 2, 3, 8])
def test_every_request_is_placed_once(ndev):
    rnd = random.Random(ndev)
    costs = [rnd.randrange(1, 1 << 30) for _ in range(257)]
    a = plan(costs, ndev)
    assert len(a) == len(costs) and all(0 <= d < ndev for d in a)


def test_multi_device_off_by_default():
    assert _lib.load().ik_logical_device_count() == 0


def split(costs, ndev, min_batch=64, outstanding=None):
    lib = _lib.load()
    n = len(costs)
    c = (ctypes.c_uint64 * n)(*costs)
    o = (ctypes.c_uint64 * ndev)(*outstanding) if outstanding else None
    lo = (ctypes.c_uint32 * (ndev + 1))()
    dev = (ctypes.c_uint32 * ndev)()
    P = lib.ik_schedule_split(c, n, ndev, o, min_batch, lo, dev)
    return [(lo[q], lo[q + 1], dev[q]) for q in range(P)]


def test_512_request_submit_spreads_over_8_devices():
    """A 512-request submit (the driver's 8-GPU bench batch) goes to 8 logical
    devices in parts of 64, one part each (ik_transform_batch_submit's split)."""
    parts = split([1000] * 512, 8)
    assert len(parts) == 8
    assert [hi - lo for lo, hi, _ in parts] == [64] * 8
    assert sorted(d for _, _, d in parts) == list(range(8))
    assert parts[0][0] == 0 and parts[-1][1] == 512
    assert all(parts[q][1] == parts[q + 1][0] for q in range(7))


@pytest.mark.parametrize("n,ndev,want", [(100, 8, [100]), (130, 8, [65, 65]), (64, 8, [64]), (1000, 8, [125] * 8),
                                         (63, 4, [63]), (512, 3, [170, 171, 171])])
def test_parts_are_at_least_the_minimum(n, ndev, want):
    parts = split([1] * n, ndev)
    assert [hi - lo for lo, hi, _ in parts] == want
    assert all(hi - lo >= min(64, n) for lo, hi, _ in parts)
    assert len(set(d for _, _, d in parts)) == len(parts)  # idle devices first


def test_split_respects_outstanding_work():
    # devices 0..3 busy: the 4 parts of a 256-request submit go to devices 4..7
    parts = split([10] * 256, 8, outstanding=[10**6] * 4 + [0] * 4)
    assert sorted(d for _, _, d in parts) == [4, 5, 6, 7]
