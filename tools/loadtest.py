"""Load driver for BASELINE configs[3] (the reference's loadtest, loadtest/src/main.rs:80-100):
/img requests for 2000x2000 JPEG sources ("picsum.photos/2000/2000") with w, h drawn
from [200, 800) and f = webp, q = 80, run through ik_transform_batch (batched device
decode, per-request resize_image + encode_image on host threads with their own HIP
streams).  No HTTP, signatures or caches: only the transform path.

Sharding: one process per GPU under torch.distributed.run; rank r serves requests
i = r (mod world) -- independent requests, no data-path collective (RCCL only for
the start/stop barrier and the max-over-ranks wall time).

Prints one JSON line: requests/s over all ranks, per-batch latency percentiles,
decoded MPix/s.  --formats webp,jpeg,avif mixes output formats (the /sign mix,
loadtest/src/main.rs:59-60); --restart adds RSTn markers per MCU row to the sources
(GPU entropy decoding); without it the sources decode on the host entropy path.

Usage: python tools/loadtest.py [--requests 1024 --batch 64 --sources 8 --threads 16]
"""
import argparse
import io
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-image-transform_amd"), os.path.join(ROOT, "tests")]


def make_requests(n, sources, fmts, seed):
    """The /img mix of loadtest/src/main.rs:80-100: (source, w, h, format) with w, h
    drawn from [200, 800) (:84-85) and the format from the allowed list (:59-60)."""
    rng = np.random.default_rng(seed)
    return [(int(rng.integers(0, sources)), int(rng.integers(200, 800)), int(rng.integers(200, 800)),
             fmts[int(rng.integers(0, len(fmts)))]) for _ in range(n)]


def shard(reqs, rank, world):
    """Round-robin: rank r serves requests r, r + world, ... (independent requests)."""
    return reqs[rank::world]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=64, help="requests per ik_transform_batch call")
    ap.add_argument("--sources", type=int, default=8, help="distinct 2000x2000 JPEG sources")
    ap.add_argument("--size", type=int, default=2000)
    ap.add_argument("--formats", default="webp")
    ap.add_argument("--quality", type=int, default=80)
    ap.add_argument("--restart", action="store_true")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend="nccl" if torch.cuda.is_available() else "gloo")
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    from PIL import Image
    import ikutil
    from imagekit import ImageFormat, _lib, transform_batch
    lib = _lib.load()
    assert lib.ik_init(local) == 0, _lib.last_error()

    S = args.size
    srcs = []
    for k in range(args.sources):
        buf = io.BytesIO()
        kw = {"restart_marker_rows": 1} if args.restart else {}
        Image.fromarray(ikutil.synth(S, S, 3, seed=100 + k, pattern="S")).save(buf, format="JPEG", quality=85, **kw)
        srcs.append(buf.getvalue())
    fmts = [ImageFormat[f] for f in args.formats.split(",")]
    mine = shard(make_requests(args.requests, args.sources, fmts, args.seed), rank, world)

    def run_batch(chunk):
        return transform_batch([srcs[s] for s, _, _, _ in chunk], [(w, h) for _, w, h, _ in chunk],
                               [f for _, _, _, f in chunk], [args.quality] * len(chunk), threads=args.threads)

    run_batch(mine[:min(len(mine), 8)])  # warm-up: plans, streams, pinned staging

    def barrier():
        if dist is not None:
            dist.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    lat, out_bytes = [], 0
    for i in range(0, len(mine), args.batch):
        chunk = mine[i:i + args.batch]
        tb = time.perf_counter()
        res = run_batch(chunk)
        lat.append((time.perf_counter() - tb) * 1e3)
        out_bytes += sum(len(r) for r in res)
    elapsed = time.perf_counter() - t0
    barrier()
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}" if torch.cuda.is_available() else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        print(json.dumps({
            "metric": "loadtest /img requests/s (2000^2 JPEG sources, w,h in [200,800), q80)",
            "value": round(args.requests / elapsed, 1), "unit": "requests/s", "n_gpus": world,
            "requests": args.requests, "batch": args.batch, "formats": args.formats,
            "sources_restart_markers": bool(args.restart),
            "batch_latency_ms": {"p50": round(float(np.percentile(lat, 50)), 2),
                                 "p95": round(float(np.percentile(lat, 95)), 2)},
            "decoded_mpix_per_s": round(args.requests * S * S / elapsed / 1e6, 1),
            "output_bytes_per_request": out_bytes // max(1, len(mine)),
            "host_threads_per_gpu": args.threads,
        }))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
