"""Dev tool: phase clocks of the GPU VP8 kernel (IK_VP8_STAMPS) on a 32-image 512^2 batch."""
import ctypes, os, sys
if os.environ.get("STAMPS", "1") == "1":
    os.environ["IK_VP8_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-image-transform_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import ikutil
from imagekit import _lib
lib = _lib.load(); assert lib.ik_init(0) == 0
W = H = 2048; O = 512
img = ikutil.synth(W, H, 4, seed=1, pattern="S")
for B in [int(b) for b in os.environ.get("B", "32").split(",")]:
    src = np.stack([img.reshape(H, W * 4)] * B)
    d = ctypes.c_void_p(); assert lib.ik_dev_alloc(src.nbytes, ctypes.byref(d)) == 0
    assert lib.ik_memcpy_h2d(d, src.ctypes.data, src.nbytes) == 0
    p = ctypes.c_void_p()
    assert lib.ik_pipeline_create(W, H, 4, O, O, 1, 1, 80, B, 16, ctypes.byref(p)) == 0
    assert lib.ik_pipeline_set_webp_encoder(p, 1) == 0
    for i in range(3):
        assert lib.ik_pipeline_run_device(p, d, W * 4, H * W * 4, B) == 0
        print("batch", B, "vp8 ms", round(lib.ik_pipeline_kernel_ms(p, 2), 3), flush=True)
    lib.ik_pipeline_destroy(p)
    lib.ik_dev_free(d)
