"""Wall time of decode_image on lossy WebP: the GPU decoder (ik_vp8d*) against libwebp on
the host (IK_WEBP_DECODE=host), one request at a time and as a batch
(decode_image_batch, which decodes its WebP items on parallel host threads, each
driving the GPU path or libwebp).  Prints one JSON line per case."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rust-image-transform_amd"))

import ikutil  # noqa: E402
import webp_tool as wt  # noqa: E402
from imagekit import decode_image, decode_image_batch  # noqa: E402


def timed(fn, reps):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    cases = [(512, 512, 80), (1920, 1080, 80), (2560, 1440, 80), (3000, 2000, 80), (4096, 4096, 80)]
    for w, h, q in cases:
        data = wt.encode(ikutil.synth(w, h, 3, seed=1, pattern="S"), q)
        reps = 20 if w * h <= 1 << 21 else 5
        res = {"case": f"{w}x{h} q{q}", "bytes": len(data)}
        for mode in ("gpu", "host", "auto"):
            os.environ["IK_WEBP_DECODE"] = mode
            res[f"{mode}_ms"] = round(timed(lambda: decode_image(data), reps), 3)
        batch = [wt.encode(ikutil.synth(w, h, 3, seed=s, pattern="S"), q) for s in range(16)] if w * h <= 1 << 21 else None
        if batch:
            for mode in ("gpu", "host"):
                os.environ["IK_WEBP_DECODE"] = mode
                res[f"{mode}_batch16_ms"] = round(timed(lambda: decode_image_batch(batch), 3), 3)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
