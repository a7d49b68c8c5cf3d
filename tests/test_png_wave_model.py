"""CPU: the GPU PNG decoder's wave decode pass (ik_png_wave.h: one wave per
decoder lane, 64 self-synchronising sub-lanes over shared Huffman lookup tables,
fix rounds, tokens in pieces), run by its CPU model
(libik_pngmodel.so ikm_inflate_wave: the same sub_decode, code and table
builders and lane algorithm the GPU kernel k_png_wave runs; the unchanged chain
check, expand and marker resolution after it), against zlib.

decode_image on a PNG (reference src/transform.rs:31 -> png 0.18) inflates the
IDAT zlib stream.  Bar: bytes identical to zlib.decompress for every stream
shape zlib produces (dynamic, fixed and stored blocks, every level and
strategy, tiny blocks), planted false candidates and corrupt streams."""
import ctypes
import io
import os
import zlib

import numpy as np
import pytest

import ikutil
from test_png_model import CASES, _idat, filtered

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODEL = os.path.join(ROOT, "rust-image-transform_amd", "lib", "libik_pngmodel.so")
NAMES = ("chunks cand lanes rounds overflows windows sub_passes redo_passes fix_rounds max_rounds blocks "
         "symbol_bits status tokens markers steps wave_steps units").split()


@pytest.fixture(scope="module")
def model():
    if not os.path.exists(MODEL):
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "rust-image-transform_amd"), "lib/libik_pngmodel.so"],
                       check=True, stdout=subprocess.DEVNULL)
    L = ctypes.CDLL(MODEL)
    L.ikm_inflate_wave.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p,
                                   ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    return L


def inflate(model, z, raw_len, chunk):
    out = np.zeros(raw_len + 16, np.uint8)
    n = ctypes.c_uint64()
    st = (ctypes.c_uint64 * 20)()
    rc = model.ikm_inflate_wave(z, len(z), chunk, out.ctypes.data, raw_len, ctypes.byref(n), st)
    return rc, bytes(out[:n.value]), dict(zip(NAMES, list(st)))


@pytest.mark.parametrize("w,h,c,pat,level,strategy", CASES)
@pytest.mark.parametrize("chunk", [4096, 16384, 65536])
def test_wave_inflate_equals_zlib(model, w, h, c, pat, level, strategy, chunk):
    raw = filtered(ikutil.synth(w, h, c, seed=w + h, pattern=pat))
    co = zlib.compressobj(level, zlib.DEFLATED, 15, 8, strategy)
    z = co.compress(raw) + co.flush()
    rc, out, st = inflate(model, z, len(raw), chunk)
    assert rc == 0, st
    assert out == raw


@pytest.mark.parametrize("mem_level", [1, 2, 9])
def test_block_sizes(model, mem_level):
    """zlib's memLevel sets the symbols per block (128 at 1, 32K at 9): from many
    tiny blocks per lane (pieces of several blocks, splits at block boundaries)
    to blocks longer than one staged window (a block's body over windows)."""
    raw = filtered(ikutil.synth(700, 500, 4, seed=11, pattern="S"))
    co = zlib.compressobj(9, zlib.DEFLATED, 15, mem_level)
    z = co.compress(raw) + co.flush()
    rc, out, st = inflate(model, z, len(raw), 16384)
    assert rc == 0 and out == raw, st
    if mem_level == 9:
        assert st["windows"] > st["blocks"]


def test_fixed_code_stream_one_lane(model):
    """Fixed-code blocks give the search no candidates: one lane holds the whole
    stream, and its 64 sub-lanes still decode every block in parallel."""
    raw = filtered(ikutil.synth(1200, 900, 4, seed=12, pattern="S"))
    co = zlib.compressobj(6, zlib.DEFLATED, 15, 8, zlib.Z_FIXED)
    z = co.compress(raw) + co.flush()
    rc, out, st = inflate(model, z, len(raw), 16384)
    assert rc == 0 and out == raw, st
    assert st["lanes"] == 1 and st["rounds"] == 1 and st["sub_passes"] > 60 * st["blocks"]


def test_tiny_flushed_blocks_split(model):
    """A stream flushed every few bytes (Z_SYNC_FLUSH: a short block and an empty
    stored block each time) holds more blocks than a lane's piece table: the lane
    ends early at a block boundary (kLaneSplit) and the chain check starts a new
    lane there, over as many rounds as it takes."""
    raw = filtered(ikutil.synth(64, 48, 4, seed=13, pattern="S"))
    co = zlib.compressobj(6, zlib.DEFLATED, 15)
    z = b"".join(co.compress(raw[i:i + 24]) + co.flush(zlib.Z_SYNC_FLUSH) for i in range(0, len(raw), 24)) + co.flush()
    rc, out, st = inflate(model, z, len(raw), 16384)
    assert rc == 0 and out == raw, st
    assert st["lanes"] > 1 and st["rounds"] > 1, st


@pytest.mark.parametrize("mode,c", [("RGBA", 4), ("RGB", 3), ("L", 1), ("LA", 2)])
def test_pillow_png_streams(model, mode, c):
    from PIL import Image
    img = ikutil.synth(1024, 512, c, seed=5)
    b = io.BytesIO()
    Image.fromarray(img if c > 1 else img[..., 0], mode).save(b, format="PNG")
    z = _idat(b.getvalue())
    raw = zlib.decompress(z)
    rc, out, st = inflate(model, z, len(raw), 16384)
    assert rc == 0 and out == raw, st
    assert st["lanes"] >= 8 and st["rounds"] == 1


@pytest.mark.parametrize("size,seed", [(1024, 8), (640, 480), (1500, 3)])
@pytest.mark.parametrize("chunk", [16384, 65536])
def test_pillow_rgba_frames(model, size, seed, chunk):
    """Pillow's own encoder on bench-pattern RGBA frames: sub-lane pieces that fill
    their token capacity exactly (the padded last group must fit too -- a GPU
    test caught a piece whose last group was not stored)."""
    from PIL import Image
    img = ikutil.synth(size, size, 4, seed=seed, pattern="S")
    b = io.BytesIO()
    Image.fromarray(img, "RGBA").save(b, format="PNG")
    z = _idat(b.getvalue())
    raw = zlib.decompress(z)
    rc, out, st = inflate(model, z, len(raw), chunk)
    assert rc == 0 and out == raw, st


def test_bench_frame_synchronises(model):
    """A bench-pattern 2048^2 RGBA8 frame as Pillow writes it: every lane's
    sub-lanes synchronise within the warm-up (no fix round), and the sub-lanes
    decode each bit once (symbol bits == the streams' body bits)."""
    from PIL import Image
    img = ikutil.synth(2048, 2048, 4, seed=1000, pattern="S")
    b = io.BytesIO()
    Image.fromarray(img, "RGBA").save(b, format="PNG")
    z = _idat(b.getvalue())
    raw = zlib.decompress(z)
    rc, out, st = inflate(model, z, len(raw), 16384)
    assert rc == 0 and out == raw, st
    assert st["redo_passes"] <= st["sub_passes"] // 100, st
    assert abs(st["symbol_bits"] - 8 * len(z)) < 0.01 * 8 * len(z), st


def test_false_candidate_is_dropped(model):
    """A stored block whose payload is a valid-looking dynamic block header: the
    finder takes it as a block start, the chain check must discard it and the
    predecessor must decode through it (test_png_model's stream)."""
    base = zlib.compressobj(6, zlib.DEFLATED, -15)
    bait = (base.compress(ikutil.synth(64, 64, 4, seed=1).tobytes()) + base.flush())[:200]
    payload = bait * 40 + bytes(range(256)) * 64
    co2 = zlib.compressobj(6, zlib.DEFLATED, 15)
    mixed_raw = ikutil.synth(200, 200, 4, seed=2).tobytes() + payload
    z2 = co2.compress(ikutil.synth(200, 200, 4, seed=2).tobytes()) + co2.flush(zlib.Z_FULL_FLUSH)
    co3 = zlib.compressobj(0, zlib.DEFLATED, -15)
    z2 = z2 + co3.compress(payload) + co3.flush()
    co = zlib.compressobj(0, zlib.DEFLATED, 15)
    z = co.compress(payload) + co.flush()
    for stream, raw in ((z, payload), (z2, mixed_raw)):
        rc, out, st = inflate(model, stream, len(raw), 4096)
        assert rc == 0 and out == raw, st


def test_corrupt_stream_is_rejected(model):
    raw = filtered(ikutil.synth(256, 256, 4, seed=3))
    for k in range(8):
        z = bytearray(zlib.compress(raw, 6))
        z[len(z) * (k + 1) // 10] ^= 0x5A
        rc, out, st = inflate(model, bytes(z), len(raw), 4096)
        assert rc != 0 or out != raw  # never a silent "success" with the original bytes
        if rc == 0:
            with pytest.raises(zlib.error):
                zlib.decompress(bytes(z))


def test_deep_marker_chain(model):
    from test_gpu_png import own_png
    img = ikutil.synth(300, 2500, 4, seed=50, pattern="S")
    z = _idat(own_png(img, idat_size=65536))
    raw = zlib.decompress(z)
    rc, out, st = inflate(model, z, len(raw), 16384)
    assert rc == 0 and out == raw, st
