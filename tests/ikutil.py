"""Test helpers: the CPU oracle (oracle/lib/libik_oracle.so) and synthetic images.

TEST INFRASTRUCTURE ONLY -- the oracle is the checker, never the product.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "lib", "libik_oracle.so")

u8p = ctypes.POINTER(ctypes.c_uint8)
NEAREST, TRIANGLE, CATMULLROM, GAUSSIAN, LANCZOS3 = range(5)


def pillow_codec_libs() -> dict:
    """Paths of the libwebp / libavif copies bundled with Pillow in this image.

    The product library loads its codecs only from IK_LIBWEBP / IK_LIBAVIF or the
    system sonames (the image has libwebp.so.7 1.2.2 and no system libavif); the
    harness (tests, bench, tools) names Pillow's copies explicitly, so AVIF can be
    coded here and the WebP byte tests compare libwebp 1.6.0 with the oracle's
    system 1.2.2."""
    import glob
    import PIL
    d = os.path.join(os.path.dirname(os.path.dirname(PIL.__file__)), "pillow.libs")
    out = {}
    for key, pat in (("IK_LIBWEBP", "libwebp-*.so*"), ("IK_LIBAVIF", "libavif-*.so*")):
        hits = sorted(glob.glob(os.path.join(d, pat)))
        if hits:
            out[key] = hits[0]
    return out


def use_pillow_codecs() -> dict:
    """Point IK_LIBWEBP / IK_LIBAVIF at Pillow's copies unless already set (call
    before the first encode: the library reads them once)."""
    libs = pillow_codec_libs()
    for k, v in libs.items():
        os.environ.setdefault(k, v)
    return {k: os.environ.get(k) for k in ("IK_LIBWEBP", "IK_LIBAVIF")}


def build_oracle() -> str:
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                       stdout=subprocess.DEVNULL)
    return ORACLE_SO


def _p(a: np.ndarray):
    return a.ctypes.data_as(u8p)


class Oracle:
    def __init__(self):
        self.lib = ctypes.CDLL(build_oracle())
        L = self.lib
        L.iko_resize_image_dims.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int64,
                                            ctypes.c_int64, ctypes.POINTER(ctypes.c_uint32),
                                            ctypes.POINTER(ctypes.c_uint32)]
        L.iko_jpeg_encode_rgb.restype = ctypes.c_long
        L.iko_webp_encode_rgb.restype = ctypes.c_long
        L.iko_webp_encode_rgb.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_float, ctypes.POINTER(u8p)]
        L.iko_transform_u8.restype = ctypes.c_long
        L.iko_transform_u8.argtypes = [u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, ctypes.POINTER(u8p),
                                       ctypes.POINTER(ctypes.c_uint32),
                                       ctypes.POINTER(ctypes.c_uint32)]

    def resize(self, src: np.ndarray, nw: int, nh: int, f: int) -> np.ndarray:
        src = np.ascontiguousarray(src)
        if src.ndim == 2:
            src = src[:, :, None]
        H, W, C = src.shape
        out = np.zeros((nh, nw, C), np.uint8)
        assert self.lib.iko_resize_u8(_p(src), W, H, C, nw, nh, f, _p(out)) == 0
        return out

    def resize_image_dims(self, W, H, w, h):
        ow, oh = ctypes.c_uint32(), ctypes.c_uint32()
        self.lib.iko_resize_image_dims(W, H, -1 if w is None else w, -1 if h is None else h,
                                       ctypes.byref(ow), ctypes.byref(oh))
        return ow.value, oh.value

    def to_rgb8(self, img: np.ndarray) -> np.ndarray:
        img = np.ascontiguousarray(img)
        h, w, c = img.shape
        out = np.zeros((h, w, 3), np.uint8)
        self.lib.iko_to_rgb8(_p(img), w * h, c, _p(out))
        return out

    def webp_yuv420(self, rgb: np.ndarray):
        rgb = np.ascontiguousarray(rgb)
        h, w, _ = rgb.shape
        uw, uh = (w + 1) // 2, (h + 1) // 2
        y = np.zeros((h, w), np.uint8)
        u = np.zeros((uh, uw), np.uint8)
        v = np.zeros((uh, uw), np.uint8)
        self.lib.iko_webp_rgb_to_yuv420(_p(rgb), w, h, 3 * w, _p(y), w, _p(u), _p(v), uw)
        return y, u, v

    def libwebp_import_yuv(self, rgb: np.ndarray):
        """libwebp 1.2.2's own WebPPictureImportRGB planes (pins webp_yuv420)."""
        rgb = np.ascontiguousarray(rgb)
        h, w, _ = rgb.shape
        uw, uh = (w + 1) // 2, (h + 1) // 2
        y = np.zeros((h, w), np.uint8)
        u = np.zeros((uh, uw), np.uint8)
        v = np.zeros((uh, uw), np.uint8)
        assert self.lib.iko_libwebp_import_yuv(_p(rgb), w, h, 3 * w, _p(y), _p(u), _p(v)) == 0
        return y, u, v

    def webp_encode_rgb(self, rgb: np.ndarray, q: float) -> bytes:
        rgb = np.ascontiguousarray(rgb)
        h, w, _ = rgb.shape
        out = u8p()
        n = self.lib.iko_webp_encode_rgb(_p(rgb), w, h, 3 * w, q, ctypes.byref(out))
        assert n > 0
        b = ctypes.string_at(out, n)
        self.lib.iko_free(out)
        return b

    def jpeg_encode_rgb(self, rgb: np.ndarray, q: int) -> bytes:
        rgb = np.ascontiguousarray(rgb)
        h, w, _ = rgb.shape
        out = u8p()
        n = self.lib.iko_jpeg_encode_rgb(_p(rgb), w, h, q, ctypes.byref(out))
        assert n > 0
        b = ctypes.string_at(out, n)
        self.lib.iko_free(out)
        return b

    def jpeg_coeffs(self, rgb: np.ndarray, q: int) -> np.ndarray:
        rgb = np.ascontiguousarray(rgb)
        h, w, _ = rgb.shape
        nm = ((w + 7) // 8) * ((h + 7) // 8)
        out = np.zeros((nm, 3, 64), np.int16)
        self.lib.iko_jpeg_coeffs_rgb(_p(rgb), w, h, q, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)))
        return out

    JPEG_LIBJPEG, JPEG_ZUNE = 0, 1

    def jpeg_decode(self, data: bytes, mode: int = 1) -> np.ndarray:
        """decode_image on a JPEG (oracle/jpeg_dec.c): mode 1 = zune-jpeg 0.4.21
        restatement (the reference's decoder), 0 = libjpeg-turbo restatement.
        Returns (h, w, 3) RGB8 or (h, w, 1) L8."""
        out = u8p()
        w, h, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self.lib.iko_jpeg_decode.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(u8p),
                                             ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                             ctypes.POINTER(ctypes.c_int)]
        rc = self.lib.iko_jpeg_decode(data, len(data), mode, ctypes.byref(out), ctypes.byref(w), ctypes.byref(h),
                                      ctypes.byref(c))
        if rc != 0:
            raise ValueError("oracle: cannot decode this JPEG")
        a = np.frombuffer(ctypes.string_at(out, w.value * h.value * c.value), np.uint8).reshape(h.value, w.value,
                                                                                                   c.value).copy()
        self.lib.iko_free(out)
        return a

    def transform(self, img: np.ndarray, w, h, f: int, fmt: int, q: int):
        img = np.ascontiguousarray(img)
        H, W, C = img.shape
        out = u8p()
        ow, oh = ctypes.c_uint32(), ctypes.c_uint32()
        n = self.lib.iko_transform_u8(_p(img), W, H, C, -1 if w is None else w,
                                      -1 if h is None else h, f, fmt, q, ctypes.byref(out),
                                      ctypes.byref(ow), ctypes.byref(oh))
        assert n > 0
        b = ctypes.string_at(out, n)
        self.lib.iko_free(out)
        return b, (ow.value, oh.value)


def splitmix64(seed: int, n: int) -> np.ndarray:
    """SplitMix64 stream (uint64) -- the deterministic source of synthetic pixels."""
    x = (np.uint64(seed) + np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15))
    z = x
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def synth(w: int, h: int, c: int = 4, seed: int = 0, pattern: str = "S", alpha: str = "opaque") -> np.ndarray:
    """Pattern S: gradients + 16px checker + +-8 noise; pattern N: uniform noise.
    alpha (C = 2, 4): "opaque" = 255; "random" = uniform noise (independent of the
    colour channels); "edge" = 0 on the left half (colour still set), 255 right."""
    with np.errstate(over="ignore"):
        r = splitmix64(0x1A6E0000 + seed, w * h).reshape(h, w)
    if pattern == "N":
        px = np.stack([(r >> np.uint64(8 * k)) & np.uint64(255) for k in range(c)], -1).astype(np.uint8)
    else:
        yy, xx = np.mgrid[0:h, 0:w]
        base = [xx * 255 // max(w - 1, 1), yy * 255 // max(h - 1, 1), ((xx >> 4) ^ (yy >> 4)) & 255]
        noise = [((r >> np.uint64(8 * k)) & np.uint64(15)).astype(np.int64) - 8 for k in range(3)]
        chans = [np.clip(base[k] + noise[k], 0, 255) for k in range(3)]
        if c == 1:
            px = chans[0][..., None]
        elif c == 2:
            px = np.stack([chans[0], np.full_like(chans[0], 255)], -1)
        else:
            px = np.stack(chans + ([np.full_like(chans[0], 255)] if c == 4 else []), -1)
        px = px.astype(np.uint8)
    if c in (2, 4):
        if alpha == "random":
            px[..., -1] = ((r >> np.uint64(40)) & np.uint64(255)).astype(np.uint8)
        elif alpha == "edge":
            px[..., -1] = 255
            px[:, : w // 2, -1] = 0
        else:
            px[..., -1] = 255
    return np.ascontiguousarray(px)


# The sources of the GPU PNG decode path: PMC traffic files (profiles/pmc_png.json,
# tools/pmc_png_traffic.py) record their hash, and bench.py quotes a traffic figure
# only when it was collected on the code it is measuring.
PNG_PATH_SOURCES = ["ik_png.hip", "ik_inflate.h", "ik_png_decode.cpp", "ik_png_plan.h", "ik_png.h", "ik_unfilter.h",
                    "ik_png_wave.h"]


def png_code_sha16() -> str:
    import hashlib
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rust-image-transform_amd", "csrc")
    h = hashlib.sha256()
    for n in PNG_PATH_SOURCES:
        p = os.path.join(csrc, n)
        if os.path.exists(p):
            h.update(n.encode())
            h.update(open(p, "rb").read())
    return h.hexdigest()[:16]
