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
