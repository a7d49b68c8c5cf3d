"""GPU: orderly teardown (ik_shutdown; VERDICT r3 "Next" 6).

A child process runs batches through the stage threads and worker pools and then
simply exits: the package's atexit hook calls ik_shutdown, which ends the
library's threads and frees its streams, arenas and pools while the HIP runtime
is alive.  The process must exit with rc 0 and no fault (round 3 recorded a
SIGSEGV in __cxa_finalize at process exit).  A second child shuts down
explicitly, then runs another batch (the library comes back up) and exits."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import io, sys
sys.path[:0] = [{pkg!r}, {tests!r}]
import numpy as np
from PIL import Image
import ikutil
ikutil.use_pillow_codecs()
from imagekit import DeviceBytes, _lib, transform_batch, transform_batch_submit, transform_batch_submit_device
lib = _lib.load()
assert lib.ik_init(0) == 0, _lib.last_error()
px = ikutil.synth(1200, 900, 4, seed=3, pattern="S")
b = io.BytesIO(); Image.fromarray(px, "RGBA").save(b, format="PNG"); png = b.getvalue()
b = io.BytesIO(); Image.fromarray(np.ascontiguousarray(px[..., :3]), "RGB").save(b, format="JPEG", quality=90,
                                                                                restart_marker_rows=1)
jpg = b.getvalue()
reqs = [png, jpg] * 4
p = transform_batch_submit(reqs, [(300, 300)] * 8, [1, 0] * 4, [80] * 8, filter=4, threads=4)
q = transform_batch_submit_device([DeviceBytes(png)] * 4, [(256, 256)] * 4, [1] * 4, [80] * 4, filter=1)
assert all(p.wait()) and all(q.wait())
if {explicit}:
    assert lib.ik_shutdown() == 0
    out = transform_batch(reqs[:2], [(128, 128)] * 2, [1, 0], [80, 80], filter=4)
    assert all(out)
print("CHILD_OK", flush=True)
"""


@pytest.mark.parametrize("explicit", [False, True])
def test_process_exits_cleanly_after_batches(explicit):
    code = CHILD.format(pkg=os.path.join(ROOT, "rust-image-transform_amd"), tests=os.path.join(ROOT, "tests"),
                        explicit=explicit)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180, cwd=ROOT)
    assert "CHILD_OK" in r.stdout, r.stdout + r.stderr
    assert r.returncode == 0, f"exit status {r.returncode}\n{r.stderr[-3000:]}"
    assert "SIGSEGV" not in r.stderr and "Segmentation" not in r.stderr, r.stderr[-3000:]


DAEMON_CHILD = r"""
import io, sys, threading, time
sys.path[:0] = [{pkg!r}, {tests!r}]
import numpy as np
from PIL import Image
import ikutil
ikutil.use_pillow_codecs()
from imagekit import ImageKitError, _lib, transform_batch
lib = _lib.load()
assert lib.ik_init(0) == 0, _lib.last_error()
px = ikutil.synth(800, 600, 4, seed=5, pattern="S")
b = io.BytesIO(); Image.fromarray(px, "RGBA").save(b, format="PNG"); png = b.getvalue()
b = io.BytesIO(); Image.fromarray(np.ascontiguousarray(px[..., :3]), "RGB").save(b, format="JPEG", quality=90)
jpg = b.getvalue()
started = threading.Event()
def serve():  # a server's daemon request thread: submits until the process ends
    while True:
        try:
            transform_batch([png, jpg] * 3, [(200, 200)] * 6, [1, 0] * 3, [80] * 6, filter=4, threads=4)
        except ImageKitError:
            return  # the library was closed under it (ik_close): calls fail, they do not crash
        started.set()
for _ in range(2):
    threading.Thread(target=serve, daemon=True).start()
assert started.wait(120)
time.sleep(0.5)
print("CHILD_OK", flush=True)
"""


def test_exit_with_daemon_threads_inside_the_library():
    """the atexit teardown (ik_close) runs while daemon threads
    are still inside ik_transform_batch; it waits for their calls to return, later
    calls fail with an error, and the process exits with rc 0."""
    code = DAEMON_CHILD.format(pkg=os.path.join(ROOT, "rust-image-transform_amd"), tests=os.path.join(ROOT, "tests"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180, cwd=ROOT)
    assert "CHILD_OK" in r.stdout, r.stdout + r.stderr
    assert r.returncode == 0, f"exit status {r.returncode}\n{r.stderr[-3000:]}"
    assert "SIGSEGV" not in r.stderr and "Segmentation" not in r.stderr, r.stderr[-3000:]


def test_device_inputs_run_on_their_device(ik):
    """a batch of device-resident inputs runs on the device that holds
    them, whatever the calling thread's current device is (two GPUs needed)."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("one GPU on this box: the inputs' device is the caller's")
    import io
    from PIL import Image
    import ikutil
    from imagekit import DeviceBytes, _lib, transform_batch_submit_device
    px = ikutil.synth(640, 480, 4, seed=9, pattern="S")
    b = io.BytesIO()
    Image.fromarray(px, "RGBA").save(b, format="PNG")
    assert ik.ik_init(1) == 0, _lib.last_error()
    d = DeviceBytes(b.getvalue())  # allocated on device 1
    assert ik.ik_init(0) == 0, _lib.last_error()  # the caller now on device 0
    got = transform_batch_submit_device([d] * 2, [(320, 320)] * 2, [1] * 2, [80] * 2, filter=4).wait()
    want = transform_batch_submit_device([d], [(320, 320)], [1], [80], filter=4).wait()
    assert got[0] == got[1] == want[0]
