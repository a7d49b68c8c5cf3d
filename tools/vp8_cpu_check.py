"""Dev tool: check the scalar VP8 encoder's bitstream against libwebp's decoder.
With the loop filter off, libwebp's decoded Y/U/V must equal the encoder's own
reconstruction exactly; with it on, report PSNR and size next to libwebp's own
encoder on the same YUV planes."""
import ctypes, os, subprocess, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ikutil
so = "/tmp/vp8_cpu_check.so"
subprocess.check_call(["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-o", so,
                       os.path.join(ROOT, "tools/vp8_cpu_check.cpp"),
                       os.path.join(ROOT, "rust-image-transform_amd/csrc/ik_vp8_enc.cpp")])
lib = ctypes.CDLL(so)
lib.vp8_dev_encode.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p]
lib.vp8_dev_cost_pair.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
lib.vp8_dev_pred4_mismatches.argtypes = [ctypes.c_uint, ctypes.c_int]
webp = ctypes.CDLL("libwebp.so.7")
webp.WebPDecodeYUV.restype = ctypes.POINTER(ctypes.c_uint8)
webp.WebPDecodeYUV.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                               ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)), ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)),
                               ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
webp.WebPFree.argtypes = [ctypes.c_void_p]


def yuv_of(img):
    r, g, b = [img[..., k].astype(np.float64) for k in range(3)]
    Y = np.clip(np.round(0.257 * r + 0.504 * g + 0.098 * b + 16), 0, 255).astype(np.uint8)
    h, w = Y.shape
    pad = np.pad(img, ((0, h & 1), (0, w & 1), (0, 0)), mode="edge").astype(np.float64)
    avg = (pad[0::2, 0::2] + pad[1::2, 0::2] + pad[0::2, 1::2] + pad[1::2, 1::2]) / 4
    U = np.clip(np.round(-0.148 * avg[..., 0] - 0.291 * avg[..., 1] + 0.439 * avg[..., 2] + 128), 0, 255).astype(np.uint8)
    V = np.clip(np.round(0.439 * avg[..., 0] - 0.368 * avg[..., 1] - 0.071 * avg[..., 2] + 128), 0, 255).astype(np.uint8)
    return Y, U, V


def decode_yuv(b):
    w, h, ys, uvs = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    u, v = ctypes.POINTER(ctypes.c_uint8)(), ctypes.POINTER(ctypes.c_uint8)()
    buf = ctypes.create_string_buffer(b, len(b))
    y = webp.WebPDecodeYUV(buf, len(b), ctypes.byref(w), ctypes.byref(h), ctypes.byref(u), ctypes.byref(v),
                           ctypes.byref(ys), ctypes.byref(uvs))
    if not y:
        return None
    W, H = w.value, h.value
    uw, uh = (W + 1) // 2, (H + 1) // 2
    Y = np.array([np.ctypeslib.as_array(y, (ys.value * H,))[r * ys.value:r * ys.value + W] for r in range(H)])
    U = np.array([np.ctypeslib.as_array(u, (uvs.value * uh,))[r * uvs.value:r * uvs.value + uw] for r in range(uh)])
    V = np.array([np.ctypeslib.as_array(v, (uvs.value * uh,))[r * uvs.value:r * uvs.value + uw] for r in range(uh)])
    webp.WebPFree(y)
    return Y, U, V


def encode(Y, U, V, q, filt):
    h, w = Y.shape
    out = np.zeros(w * h * 4 + 4096, np.uint8)
    n = ctypes.c_size_t()
    rec = np.zeros(w * h + 2 * U.size, np.uint8)
    assert lib.vp8_dev_encode(np.ascontiguousarray(Y).ctypes.data, np.ascontiguousarray(U).ctypes.data,
                              np.ascontiguousarray(V).ctypes.data, w, h, q, filt, out.ctypes.data, out.size,
                              ctypes.byref(n), rec.ctypes.data) == 0
    return bytes(out[:n.value]), rec


def cost_pair(lv, typ, first, ctx):
    lv = np.ascontiguousarray(lv, dtype=np.int16)
    g, f = ctypes.c_int(), ctypes.c_int()
    assert lib.vp8_dev_cost_pair(lv.ctypes.data, typ, first, ctx, ctypes.byref(g), ctypes.byref(f)) == 0
    return g.value, f.value


def psnr(a, b):
    m = np.mean((a.astype(float) - b.astype(float)) ** 2)
    return 99 if m == 0 else 10 * np.log10(255 ** 2 / m)


if __name__ == "__main__":
    for (w, h, pat) in [(16, 16, "S"), (33, 17, "S"), (64, 48, "N"), (200, 120, "S"), (512, 512, "S")]:
        img = ikutil.synth(w, h, 3, seed=w + h, pattern=pat)
        Y, U, V = yuv_of(img)
        b, rec = encode(Y, U, V, 80.0, 0)
        d = decode_yuv(b)
        assert d is not None, f"libwebp cannot decode {w}x{h}"
        Yd, Ud, Vd = d
        ry = rec[:w * h].reshape(h, w)
        uw, uh = (w + 1) // 2, (h + 1) // 2
        ru = rec[w * h:w * h + uw * uh].reshape(uh, uw)
        rv = rec[w * h + uw * uh:].reshape(uh, uw)
        exact = np.array_equal(Yd, ry) and np.array_equal(Ud, ru) and np.array_equal(Vd, rv)
        b2, _ = encode(Y, U, V, 80.0, -1)
        Yf, _, _ = decode_yuv(b2)
        print(f"{w}x{h} {pat}: bytes={len(b2)} recon==libwebp-decode(no filter): {exact}  "
              f"PSNR-Y={psnr(Yf, Y):.2f}")


def compare_libwebp(img, q=80.0):
    import io
    from PIL import Image
    h, w, _ = img.shape
    webp.WebPEncodeRGB.restype = ctypes.c_size_t
    webp.WebPEncodeRGB.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                   ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8))]
    o = ctypes.POINTER(ctypes.c_uint8)()
    a = np.ascontiguousarray(img)
    n = webp.WebPEncodeRGB(a.ctypes.data, w, h, w * 3, q, ctypes.byref(o))
    ref = ctypes.string_at(o, n)
    webp.WebPFree(o)
    Y, U, V = yuv_of(img)
    ours, _ = encode(Y, U, V, q, -1)
    dr = np.asarray(Image.open(io.BytesIO(ref)).convert("RGB"))
    do = np.asarray(Image.open(io.BytesIO(ours)).convert("RGB"))
    return len(ref), psnr(dr, img), len(ours), psnr(do, img)


if __name__ == "__main__":
    for pat, w, h in [("S", 512, 512), ("N", 128, 128)]:
        img = ikutil.synth(w, h, 3, seed=7, pattern=pat)
        print(pat, w, h, "libwebp bytes/psnr=%d/%.2f  ours=%d/%.2f" % compare_libwebp(img))
    # a natural-ish image: smooth gradients + shapes
    yy, xx = np.mgrid[0:512, 0:512]
    nat = np.stack([(128 + 100 * np.sin(xx / 37.0) * np.cos(yy / 23.0)), (xx * 0.4 + yy * 0.1) % 256,
                    255 * ((xx - 256) ** 2 + (yy - 256) ** 2 < 150 ** 2)], -1).clip(0, 255).astype(np.uint8)
    print("natural", "libwebp bytes/psnr=%d/%.2f  ours=%d/%.2f" % compare_libwebp(nat))
