"""Dev tool: time the fused resize kernel (HIP events) over a batch of 4096^2 RGBA8
frames for several filters / workgroup targets.  Usage: python tools/sweep_resize.py"""
import ctypes, os, sys, time, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-image-transform_amd"), os.path.join(ROOT, "tests")]
import torch
from imagekit import _lib
import ikutil
lib = _lib.load(); assert lib.ik_init(0) == 0
S, O = int(os.environ.get("S", 4096)), int(os.environ.get("O", 512))
B = int(os.environ.get("B", 32))
pitch = S * 4
img = ikutil.synth(S, S, 4, seed=1, pattern="S")
src = torch.empty((B, S, pitch), dtype=torch.uint8, device="cuda")
for i in range(B):
    src[i].copy_(torch.from_numpy(img.reshape(S, pitch)))
torch.cuda.synchronize()
res = {}
for f in [int(x) for x in os.environ.get("FILTERS", "1,4").split(",")]:
    for tgt, fl, br in [(t, fl, br) for t in os.environ.get("TARGETS", "8192").split(",")
                        for fl in os.environ.get("FLUSH", "").split(",")
                        for br in os.environ.get("BANDS", "").split(",")]:
        os.environ["IK_TARGET_WG"] = tgt
        for k, v in (("IK_FLUSH_ROWS", fl), ("IK_BAND_ROWS", br)):
            if v: os.environ[k] = v
            else: os.environ.pop(k, None)
        p = ctypes.c_void_p()
        assert lib.ik_pipeline_create(S, S, 4, O, O, f, 1, 80, B, 1, ctypes.byref(p)) == 0, _lib.last_error()
        ms = []
        for i in range(8):
            assert lib.ik_pipeline_run_device(p, ctypes.c_void_p(src.data_ptr()), pitch, S * pitch, B) == 0
            if i >= 2:
                ms.append(lib.ik_pipeline_kernel_ms(p, 0))
        lib.ik_pipeline_destroy(p)
        m = float(np.median(ms))
        gbs = B * (4 * S * S + 4 * O * O) / (m * 1e-3) / 1e9
        print(f"filter={f} target_wg={tgt} flush={fl or 'auto'} band={br or 'auto'} resize_ms={m:.4f} ({m/B*1e3:.1f} us/img) GB/s={gbs:.0f} frac={gbs/8000:.3f}", flush=True)
