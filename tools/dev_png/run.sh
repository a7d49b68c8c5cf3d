# Dev: host PNG decode timing on this machine (libdeflate vs zlib inflate, whole decode).
set -e
cd "$(dirname "$0")"
python - <<'PY'
import sys, io, time, ctypes, struct, zlib
sys.path.insert(0, "../../tests")
import ikutil
from PIL import Image
im = ikutil.synth(4096, 4096, 4, seed=0)
b = io.BytesIO(); Image.fromarray(im, "RGBA").save(b, format="PNG"); d = b.getvalue()
open("s.png", "wb").write(d); im.tofile("s.raw")
i = 8; idat = b""
while i < len(d):
    n = struct.unpack(">I", d[i:i+4])[0]
    if d[i+4:i+8] == b"IDAT": idat += d[i+8:i+8+n]
    i += 12 + n
t = time.time(); r = zlib.decompress(idat); print("zlib inflate ms", round((time.time()-t)*1e3, 1))
L = ctypes.CDLL("libdeflate.so.0"); L.libdeflate_alloc_decompressor.restype = ctypes.c_void_p
dec = L.libdeflate_alloc_decompressor(); out = ctypes.create_string_buffer(len(r)); got = ctypes.c_size_t()
for _ in range(3):
    t = time.time(); L.libdeflate_zlib_decompress(ctypes.c_void_p(dec), idat, len(idat), out, len(r), ctypes.byref(got))
    print("libdeflate inflate ms", round((time.time()-t)*1e3, 1))
PY
g++ -O2 png_decode_timing.cpp -o /tmp/png_t -L../../rust-image-transform_amd/lib -limagekit_hip -Wl,-rpath,$(pwd)/../../rust-image-transform_amd/lib
/tmp/png_t
IK_PNG_ZLIB=1 /tmp/png_t
