"""GPU: the streaming pipeline (ik_pipeline_submit / ik_pipeline_collect), the
batched form of the /img handler's decode -> resize_image -> encode_image chain
(reference src/lib.rs:175-191, src/transform.rs:62-150) with two batches in
flight.  Bar: every batch's bytes identical to ik_pipeline_run on the same
frames (itself pinned against the oracle in test_gpu_pipeline; the exact WebP coder in test_gpu_vp8x),
for every encoder, with batches of different sizes and sources interleaved."""
import ctypes

import numpy as np
import pytest

import ikutil
from imagekit import _lib

pytestmark = pytest.mark.gpu

W, H, C, NW, NH = 320, 240, 4, 96, 72
IK_JPEG, IK_WEBP = 0, 1


def _frames(seed, n):
    return np.stack([ikutil.synth(W, H, C, seed=seed + i, pattern="S" if i % 2 == 0 else "N").reshape(H, W * C)
                     for i in range(n)])


class _Dev:
    def __init__(self, ik, arr):
        self.ik, self.p = ik, ctypes.c_void_p()
        assert ik.ik_dev_alloc(arr.nbytes, ctypes.byref(self.p)) == 0
        assert ik.ik_memcpy_h2d(self.p, arr.ctypes.data, arr.nbytes) == 0

    def free(self):
        self.ik.ik_dev_free(self.p)


def _unpack(out, sizes, n):
    res, off = [], 0
    for i in range(n):
        res.append(bytes(out[off:off + sizes[i]]))
        off += sizes[i]
    return res


@pytest.mark.parametrize("fmt,enc", [(IK_WEBP, 0), (IK_WEBP, 2), (IK_JPEG, 0)])
def test_submit_collect_equals_run(ik, fmt, enc):
    max_b = 4
    batches = [(_frames(100, 4), 4), (_frames(200, 3), 3), (_frames(300, 4), 1), (_frames(400, 2), 2)]
    devs = [_Dev(ik, a) for a, _ in batches]
    p = ctypes.c_void_p()
    cap = max_b * NW * NH * 4 + 65536
    pitch = W * C
    try:
        assert ik.ik_pipeline_create(W, H, C, NW, NH, 4, fmt, 80, max_b, 3, ctypes.byref(p)) == 0, _lib.last_error()
        if fmt == IK_WEBP:
            assert ik.ik_pipeline_set_webp_encoder(p, enc) == 0, _lib.last_error()
        want = []
        for d, (_, n) in zip(devs, batches):
            out = np.zeros(cap, np.uint8)
            sizes = (ctypes.c_size_t * max_b)()
            assert ik.ik_pipeline_run(p, d.p, pitch, H * pitch, n, out.ctypes.data, cap, sizes) == 0, _lib.last_error()
            want.append(_unpack(out, sizes, n))
        # two in flight: submit 0, 1; collect 0; submit 2; collect 1; submit 3; collect 2, 3
        got = []
        n_out = ctypes.c_uint32()

        def collect():
            out = np.zeros(cap, np.uint8)
            sizes = (ctypes.c_size_t * max_b)()
            assert ik.ik_pipeline_collect(p, out.ctypes.data, cap, sizes, ctypes.byref(n_out)) == 0, _lib.last_error()
            got.append(_unpack(out, sizes, n_out.value))

        def submit(i):
            d, (_, n) = devs[i], batches[i]
            assert ik.ik_pipeline_submit(p, d.p, pitch, H * pitch, n) == 0, _lib.last_error()

        submit(0)
        submit(1)
        assert ik.ik_pipeline_submit(p, devs[2].p, pitch, H * pitch, 4) != 0  # a third is refused
        assert ik.ik_pipeline_run(p, devs[2].p, pitch, H * pitch, 4, None, 0, None) != 0
        if fmt == IK_WEBP:
            assert ik.ik_pipeline_set_webp_encoder(p, 2 - enc) != 0
        collect()
        submit(2)
        collect()
        submit(3)
        collect()
        collect()
        assert ik.ik_pipeline_collect(p, None, 0, None, None) != 0  # nothing in flight
        assert [len(g) for g in got] == [n for _, n in batches]
        assert got == want
    finally:
        if p:
            ik.ik_pipeline_destroy(p)
        for d in devs:
            d.free()


def test_destroy_with_batches_in_flight(ik):
    """Destroy drains the stream first: no use-after-free of the pinned slots."""
    d = _Dev(ik, _frames(7, 2))
    p = ctypes.c_void_p()
    try:
        assert ik.ik_pipeline_create(W, H, C, NW, NH, 1, IK_WEBP, 80, 2, 2, ctypes.byref(p)) == 0
        assert ik.ik_pipeline_submit(p, d.p, W * C, H * W * C, 2) == 0
        assert ik.ik_pipeline_submit(p, d.p, W * C, H * W * C, 2) == 0
        ik.ik_pipeline_destroy(p)
        p = None
    finally:
        if p:
            ik.ik_pipeline_destroy(p)
        d.free()
