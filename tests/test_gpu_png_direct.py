"""GPU: the direct-rows expand (IK_PNG_DIRECT=1, not the default: ik_png_decode.cpp
png_direct_rows).  Expand writes the image rows and filter types itself and lists the
window markers; k_png_marks resolves them and k_png_ftflags checks the filter types --
no resolve pass over the u16 symbols.  A flat image (markers through every unit)
overflows the marker list, and the batch takes the resolve pass after all.

The switch is read once per process, so a child process decodes the batch; its
pixels must equal the sources, all through the GPU path.  (decode_image, reference
src/transform.rs:31 -> png 0.18.)"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
sys.path[:0] = [{pkg!r}, {tests!r}]
import numpy as np
import ikutil
from imagekit import _lib, decode_image_batch
from test_gpu_png import own_png, pil_png
lib = _lib.load()
assert lib.ik_init(0) == 0, _lib.last_error()
assert lib.ik_set_png_gpu_min(0) == 0
flat = np.zeros((2048, 2048, 4), np.uint8); flat[..., 0] = 200; flat[..., 3] = 255
imgs = [ikutil.synth(1024, 768, 4, seed=91, pattern="S"), ikutil.synth(700, 1300, 4, seed=92, pattern="N"),
        ikutil.synth(333, 222, 3, seed=93, pattern="S"), ikutil.synth(1500, 900, 4, seed=94, pattern="S")]
datas = [pil_png(imgs[0]), own_png(imgs[1], idat_size=65536), pil_png(imgs[2]), own_png(imgs[3])]
def run(ds, ims):
    out = decode_image_batch(ds)
    for (d, fmt), im in zip(out, ims):
        np.testing.assert_array_equal(d.to_array().reshape(im.shape), im)
run(datas, imgs)                                   # markers within the list
run(datas + [own_png(flat, filters=0, idat_size=65536)], imgs + [flat])  # the list overflows
import ctypes
c = (ctypes.c_ulonglong * 2)()
assert lib.ik_png_counters(c) == 0
assert c[1] == 0, f"{{c[1]}} stream(s) took the host decoder"
print("direct rows ok", c[0])
"""


def test_direct_rows_expand_equals_sources():
    code = CHILD.format(pkg=os.path.join(ROOT, "rust-image-transform_amd"), tests=os.path.join(ROOT, "tests"))
    env = dict(os.environ, IK_PNG_DIRECT="1", IK_TIMING="1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "direct rows ok" in r.stdout
    assert "resolve pass" in r.stderr  # the flat image's batch overflowed the marker list
