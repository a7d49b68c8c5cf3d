"""Independent numpy restatement of the reference resize path (TEST INFRASTRUCTURE).

Second, independently written restatement of image 0.25.8 `imageops::resize`
(src/imageops/sample.rs: vertical_sample then horizontal_sample) as called by
reference src/transform.rs:85-89, and of the transform.rs:74-82 +
DynamicImage::resize dimension policy.  It exists only to cross-check the C
oracle (oracle/resize.c) bit for bit, catching op-order slips in either.

f32 discipline: every product and sum is a separate numpy float32 operation
(no fused multiply-add); sinf/expf come from glibc through ctypes, exactly what
rustc's f32::sin/exp lower to on x86_64-linux-gnu; rounding is half away from
zero (Rust f32::round), done in f64 on values that are exact in f32.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np

_libm = ctypes.CDLL("libm.so.6")
_libm.sinf.restype = ctypes.c_float
_libm.sinf.argtypes = [ctypes.c_float]
_libm.expf.restype = ctypes.c_float
_libm.expf.argtypes = [ctypes.c_float]

F = np.float32
PI = F(math.pi)
NEAREST, TRIANGLE, CATMULLROM, GAUSSIAN, LANCZOS3 = range(5)
SUPPORT = {NEAREST: F(0), TRIANGLE: F(1), CATMULLROM: F(2), GAUSSIAN: F(3), LANCZOS3: F(3)}


def _sinc(t: np.float32) -> np.float32:
    a = F(t * PI)
    if t == 0:
        return F(1)
    return F(F(_libm.sinf(float(a))) / a)


def _kernel(f: int, x: np.float32) -> np.float32:
    x = F(x)
    ax = F(abs(x))
    if f == NEAREST:
        return F(1)
    if f == TRIANGLE:
        return F(F(1) - ax) if ax < 1 else F(0)
    if f == LANCZOS3:
        return F(_sinc(x) * _sinc(F(x / F(3)))) if ax < 3 else F(0)
    if f == CATMULLROM:
        b, c = F(0), F(0.5)
        if ax < 1:
            a2 = F(ax * ax)
            a3 = F(a2 * ax)
            k = F(F(F(12) - F(9) * b - F(6) * c) * a3) + F(F(F(-18) + F(12) * b + F(6) * c) * a2)
            k = F(k + F(F(6) - F(2) * b))
        elif ax < 2:
            a2 = F(ax * ax)
            a3 = F(a2 * ax)
            k = F(F(-b - F(6) * c) * a3) + F(F(F(6) * b + F(30) * c) * a2)
            k = F(k + F(F(F(-12) * b - F(48) * c) * ax))
            k = F(k + F(F(8) * b + F(24) * c))
        else:
            k = F(0)
        return F(k / F(6))
    if f == GAUSSIAN:
        r = F(0.5)
        c = F(F(1) / F(F(np.sqrt(F(F(2) * PI))) * r))
        e = F(_libm.expf(float(F(F(-F(x * x)) / F(F(2) * F(r * r))))))
        return F(c * e)
    raise ValueError(f)


def axis_weights(n_in: int, n_out: int, f: int):
    """sample.rs weight computation: returns [(left, np.float32 weights)] per output index."""
    ratio = F(F(n_in) / F(n_out))
    sratio = F(1) if ratio < 1 else ratio
    support = F(SUPPORT[f] * sratio)
    out = []
    for o in range(n_out):
        c = F(F(F(o) + F(0.5)) * ratio)
        left = int(math.floor(F(c - support)))
        left = min(max(left, 0), n_in - 1)
        right = int(math.ceil(F(c + support)))
        right = min(max(right, left + 1), n_in)
        c = F(c - F(0.5))
        ws = [_kernel(f, F(F(F(i) - c) / sratio)) for i in range(left, right)]
        s = F(0)
        for w in ws:
            s = F(s + w)
        out.append((left, np.array([F(w / s) for w in ws], dtype=F)))
    return out


def _round_half_away(t: np.ndarray, maxv: float = 255.0, dtype=np.uint8) -> np.ndarray:
    t = np.clip(t.astype(np.float64), 0.0, maxv)
    return np.floor(t + 0.5).astype(dtype)  # t >= 0; exact in f64


def resize(src: np.ndarray, nw: int, nh: int, f: int) -> np.ndarray:
    """imageops::resize on an (H, W, C) uint8 or uint16 array (16-bit samples: the
    same f32 sequence, clamped to u16::MAX)."""
    H, W, C = src.shape
    wide = src.dtype == np.uint16
    if (nw, nh) == (W, H):
        return src.copy()
    tmp = np.zeros((nh, W, C), dtype=F)
    for oy, (left, ws) in enumerate(axis_weights(H, nh, f)):
        t = np.zeros((W, C), dtype=F)
        for k, w in enumerate(ws):
            t = t + src[left + k].astype(F) * w
        tmp[oy] = t
    out = np.zeros((nh, nw, C), dtype=np.uint16 if wide else np.uint8)
    for ox, (left, ws) in enumerate(axis_weights(W, nw, f)):
        t = np.zeros((nh, C), dtype=F)
        for k, w in enumerate(ws):
            t = t + tmp[:, left + k, :] * w
        out[:, ox, :] = _round_half_away(t, 65535.0, np.uint16) if wide else _round_half_away(t)
    return out


def resize_dimensions(w: int, h: int, nw: int, nh: int, fill: bool = False):
    wr = nw / w
    hr = nh / h
    r = max(wr, hr) if fill else min(wr, hr)
    # Rust f64::round is half away from zero
    rw = max(int(math.floor(w * r + 0.5)), 1)
    rh = max(int(math.floor(h * r + 0.5)), 1)
    return rw, rh


def resize_image_dims(W: int, H: int, w, h):
    """src/transform.rs:62-90 + DynamicImage::resize -> final (w, h)."""
    if w is None and h is None:
        return W, H
    if w is None:
        ratio = F(F(h) / F(H))
        tw = int(np.floor(np.float64(F(F(W) * ratio)) + 0.5))
    else:
        tw = w
    if h is None:
        ratio = F(F(w) / F(W))
        th = int(np.floor(np.float64(F(F(H) * ratio)) + 0.5))
    else:
        th = h
    tw, th = max(tw, 1), max(th, 1)
    if (tw, th) == (W, H):
        return W, H
    return resize_dimensions(W, H, tw, th)
