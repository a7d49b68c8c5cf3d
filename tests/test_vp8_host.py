"""CPU: the host half of the GPU WebP encoder (ik_vp8_enc.cpp: probability
adaptation, boolean coder, header, tokens, RIFF) with the scalar macroblock
reference (tools/vp8_cpu_check.cpp, the same ik_vp8.h code the GPU kernel runs).

The bitstream must decode in libwebp, and with the loop filter off libwebp's
decoded Y/U/V must equal the encoder's own reconstruction bit for bit -- every
predictor, transform, dequantisation and token rule agrees with the decoder.
Rate/quality against libwebp's own encoder (the reference's WebPEncodeRGB) is
checked as a size/PSNR bound (not byte parity: a different, GPU-shaped encoder)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
vp8 = pytest.importorskip("vp8_cpu_check")
import ikutil


def _planes(rec, w, h):
    uw, uh = (w + 1) // 2, (h + 1) // 2
    return (rec[:w * h].reshape(h, w), rec[w * h:w * h + uw * uh].reshape(uh, uw),
            rec[w * h + uw * uh:].reshape(uh, uw))


@pytest.mark.parametrize("wh", [(1, 1), (16, 16), (17, 31), (33, 17), (64, 48), (200, 120)])
@pytest.mark.parametrize("pat", ["S", "N"])
@pytest.mark.parametrize("q", [5.0, 80.0, 100.0])
def test_reconstruction_equals_libwebp_decode(wh, pat, q):
    w, h = wh
    Y, U, V = vp8.yuv_of(ikutil.synth(w, h, 3, seed=w * 7 + h, pattern=pat))
    b, rec = vp8.encode(Y, U, V, q, 0)  # loop filter off
    assert b[:4] == b"RIFF" and b[8:16] == b"WEBPVP8 "
    d = vp8.decode_yuv(b)
    assert d is not None
    for got, want in zip(d, _planes(rec, w, h)):
        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("q", [10.0, 50.0, 80.0, 95.0])
def test_filtered_stream_decodes_and_tracks_quality(q):
    Y, U, V = vp8.yuv_of(ikutil.synth(96, 80, 3, seed=3, pattern="S"))
    b, _ = vp8.encode(Y, U, V, q, -1)
    d = vp8.decode_yuv(b)
    assert d is not None and d[0].shape == (80, 96)
    assert vp8.psnr(d[0], Y) > {10.0: 25, 50.0: 30, 80.0: 33, 95.0: 38}[q]


def test_size_and_psnr_against_libwebp():
    # the reference path (WebPEncodeRGB q80) vs this encoder, both decoded by libwebp
    img = ikutil.synth(256, 256, 3, seed=11, pattern="S")
    ref_n, ref_p, our_n, our_p = vp8.compare_libwebp(img, 80.0)
    assert our_n <= 1.15 * ref_n and our_p >= ref_p - 0.3, (ref_n, ref_p, our_n, our_p)


def test_quality_orders_size():
    Y, U, V = vp8.yuv_of(ikutil.synth(128, 96, 3, seed=5, pattern="S"))
    sizes = [len(vp8.encode(Y, U, V, q, -1)[0]) for q in (10.0, 50.0, 80.0, 100.0)]
    assert sizes == sorted(sizes) and sizes[0] < sizes[-1]


@pytest.mark.parametrize("typ,first", [(0, 1), (0, 0), (1, 0), (2, 0), (3, 0)])
def test_register_token_cost_equals_scan(typ, first):
    """block_cost_fixed (the GPU kernel's unrolled, compile-time-probability form)
    == block_cost's scan, over sparse/dense/large levels and all three contexts."""
    rng = np.random.default_rng(typ * 2 + first)
    for trial in range(1500):
        lv = np.zeros(16, np.int16)
        k = rng.integers(0, 17)
        pos = rng.choice(16, size=k, replace=False)
        mag = rng.choice([1, 1, 1, 2, 3, 4, 5, 6, 7, 9, 10, 11, 18, 19, 34, 35, 66, 67, 200, 2047], size=k)
        lv[pos] = mag * rng.choice([-1, 1], size=k)
        if first:
            lv[0] = 0
        for ctx in range(3):
            g, f = vp8.cost_pair(lv, typ, first, ctx)
            assert g == f, (lv.tolist(), typ, first, ctx, g, f)


def test_pred4_tap_table_equals_pred4():
    """kPred4Tab / pred4_px (the GPU's lane-per-(mode,row) predictor) == pred4 for all
    10 modes and 16 pixels on random contexts."""
    assert vp8.lib.vp8_dev_pred4_mismatches(7, 20000) == 0
