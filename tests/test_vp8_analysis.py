"""CPU: libwebp's method-4 segment analysis, restated (tests/oracle_vp8.py), against
the bytes libwebp itself writes -- the first stage of the reference's WebP coder
(reference src/transform.rs:129-137 -> webp 0.3.1 -> libwebp WebPEncodeRGB).

tests/vp8_parse.py reads each frame's segment map, segment quantisers, base
quantiser, chroma quantiser deltas and segment-tree probabilities back out of the
first partition; the restatement must produce all of them exactly from libwebp's
own YUV420 planes (WebPPictureImportRGB), for every size, pattern and quality here
and for the committed golden WebP bytes (tests/golden/codec_golden.npz).  The GPU
kernel (ik_vp8_analysis.hip) is held to the same bytes by
tests/test_gpu_vp8_analysis.py."""
import os

import numpy as np
import pytest

import ikutil
import oracle_vp8
import vp8_parse

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "codec_golden.npz")


def check_against_bitstream(got, r, where=""):
    """got: {segments (mb_h, mb_w), num_segments, update_map, quant, base_quant, uv_dc,
    uv_ac, probs}; r: vp8_parse.parse(libwebp bytes)."""
    seg = r["segment"]
    assert bool(seg["enabled"]) == (got["num_segments"] > 1), where
    assert bool(seg["update_map"]) == bool(got["update_map"]), where
    if seg["update_map"]:
        np.testing.assert_array_equal(np.asarray(got["segments"]).reshape(r["mb_h"], r["mb_w"]), r["segments"],
                                      err_msg=where)
        assert list(got["probs"]) == list(seg["probs"]), where
    if seg["enabled"]:
        assert list(got["quant"]) == list(seg["quant"]), where
    assert got["base_quant"] == r["quant"]["y_ac_qi"], where
    assert (got["uv_dc"], got["uv_ac"]) == (r["quant"]["uv_dc"], r["quant"]["uv_ac"]), where


@pytest.fixture(scope="module")
def orc():
    return ikutil.Oracle()


@pytest.mark.parametrize("wh", [(1, 1), (16, 16), (17, 31), (32, 16), (64, 48), (100, 70), (333, 222), (512, 512)])
@pytest.mark.parametrize("pat", ["S", "N"])
@pytest.mark.parametrize("q", [10.0, 80.0, 95.0])
def test_restatement_equals_libwebp(orc, wh, pat, q):
    w, h = wh
    rgb = ikutil.synth(w, h, 3, seed=w * 3 + h, pattern=pat)
    r = vp8_parse.parse(orc.webp_encode_rgb(rgb, q))
    assert (r["width"], r["height"]) == (w, h) and not r["overrun"]
    got = oracle_vp8.analyze(*orc.libwebp_import_yuv(rgb), quality=q)
    check_against_bitstream(got, r, f"{w}x{h} {pat} q{q}")


def test_restatement_equals_golden_webp_bytes(orc):
    g = np.load(GOLD)
    for name in ("a", "b", "c", "d"):
        W, H, pat, seed, q = (int(v) for v in g[f"{name}_meta"])
        rgb = ikutil.synth(W, H, 3, seed=seed, pattern="SN"[pat])
        r = vp8_parse.parse(bytes(g[f"{name}_webp"]))
        got = oracle_vp8.analyze(*orc.libwebp_import_yuv(rgb), quality=float(q))
        check_against_bitstream(got, r, name)


def test_parser_reads_libwebp_mode_syntax(orc):
    # the first partition must be consumed exactly: every macroblock's modes decoded
    # with the bytes it has (a mis-read tree would run past the partition)
    for pat in "SN":
        rgb = ikutil.synth(96, 80, 3, seed=7, pattern=pat)
        r = vp8_parse.parse(orc.webp_encode_rgb(rgb, 80.0))
        assert not r["overrun"] and r["mb_w"] == 6 and r["mb_h"] == 5
        assert r["skip_prob"] is None  # method 4 codes with the token buffer: no skip flags
        assert set(np.unique(r["uvmode"])) <= {0, 1, 2, 3}
        assert r["bmodes"].max() <= 9


def test_kmeans_properties():
    # a constant alpha field: one cluster, one segment after SimplifySegments
    p = oracle_vp8.segment_params(np.full(64, 100), np.full(64, 30))
    assert p["num_segments"] == 1 and not p["update_map"]
    # two separated populations: two segments, each MB in its own population's
    a = np.array([10] * 40 + [200] * 24)
    p = oracle_vp8.segment_params(a, np.zeros(64, np.int64))
    seg = p["segments"]
    assert len(set(seg[:40])) == 1 and len(set(seg[40:])) == 1 and seg[0] != seg[-1]
