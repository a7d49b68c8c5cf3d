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

Dynamic queue (default when run as one process): the library serves every visible
GPU itself (ik_init(-1); IK_DEVICES picks them), and --clients threads call
ik_transform_batch concurrently, as request handlers would; each call's requests go
to the devices with the least outstanding work.

CPU leg (--cpu-seconds S): the same request mix through the reference CPU path
restated -- Pillow's libjpeg-turbo decode (zune-jpeg is absent), the oracle's
image 0.25.8 Lanczos3 resize and libwebp -- on nproc forked worker processes for
about S seconds, before anything touches the GPU.

Usage: python tools/loadtest.py [--requests 10000 --batch 64 --sources 8 --threads 16 --clients 4]
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
import ikutil  # noqa: E402

ikutil.use_pillow_codecs()  # codec libraries named explicitly (IK_LIBWEBP / IK_LIBAVIF)


def make_requests(n, sources, fmts, seed):
    """The /img mix of loadtest/src/main.rs:80-100: (source, w, h, format) with w, h
    drawn from [200, 800) (:84-85) and the format from the allowed list (:59-60)."""
    rng = np.random.default_rng(seed)
    return [(int(rng.integers(0, sources)), int(rng.integers(200, 800)), int(rng.integers(200, 800)),
             fmts[int(rng.integers(0, len(fmts)))]) for _ in range(n)]


def shard(reqs, rank, world):
    """Round-robin: rank r serves requests r, r + world, ... (independent requests)."""
    return reqs[rank::world]


_CPU = {}


def _cpu_one(k):
    orc, srcs, reqs, q = _CPU["orc"], _CPU["srcs"], _CPU["reqs"], _CPU["q"]
    s, w, h, f = reqs[k % len(reqs)]
    img = orc.jpeg_decode(srcs[s], mode=1)  # the zune-jpeg 0.4.21 restatement (the reference's decoder)
    fmt = {"jpeg": 0, "webp": 1, "avif": 2}[f]
    if fmt == 2:
        return 0  # the oracle has no AVIF encoder: the leg covers the webp/jpeg requests
    orc.transform(img, w, h, 4, fmt, q)
    return 1


def cpu_leg(args, srcs, reqs):
    """Reference CPU path restated on the same requests: nproc forked processes, one
    request each at a time, for about args.cpu_seconds (started before GPU use)."""
    import multiprocessing as mp

    import ikutil
    _CPU.update(orc=ikutil.Oracle(), srcs=srcs, reqs=reqs, q=args.quality)
    _cpu_one(0)
    t0 = time.perf_counter()
    for k in range(4):
        _cpu_one(k)
    t1 = (time.perf_counter() - t0) / 4
    sys.path.insert(0, ROOT)
    from bench import effective_cores, host_info  # host facts as bench.py records them
    host = host_info()
    nproc = effective_cores(host)  # one process per core the job may use (min of nproc, cgroup quota, affinity)
    per = max(2, min(16, int(args.cpu_seconds / max(t1, 1e-3))))
    print(f"[loadtest] cpu leg: {nproc} processes x {per} requests ({t1 * 1e3:.0f} ms each on one core)",
          file=sys.stderr, flush=True)
    with mp.get_context("fork").Pool(nproc) as pool:
        pool.map(_cpu_one, range(nproc), chunksize=1)
        t0 = time.perf_counter()
        done = sum(pool.map(_cpu_one, range(nproc * per), chunksize=per))
        wall = time.perf_counter() - t0
    return {"value": round(done / wall, 1), "unit": "requests/s", "processes": nproc, "cores": nproc,
            "requests": done, "wall_s": round(wall, 2),
            "kind": "port (oracle zune-jpeg restatement decode + image 0.25.8 Lanczos3 resize + libwebp)",
            "single_thread_requests_per_s": round(1 / t1, 2), "host": host}


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
    ap.add_argument("--clients", type=int, default=0,
                    help="client threads calling ik_transform_batch at once (0 = one per logical device)")
    ap.add_argument("--cpu-seconds", type=float, default=0.0, help="CPU leg of about this long (0 = none)")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="1: each client submits its next batch (ik_transform_batch_submit) before waiting for "
                         "the previous one's bytes, so one batch's libwebp coding runs beside the next one's GPU work")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    from PIL import Image
    import ikutil
    S = args.size
    srcs = []
    for k in range(args.sources):
        buf = io.BytesIO()
        kw = {"restart_marker_rows": 1} if args.restart else {}
        Image.fromarray(ikutil.synth(S, S, 3, seed=100 + k, pattern="S")).save(buf, format="JPEG", quality=85, **kw)
        srcs.append(buf.getvalue())
    fmt_names = args.formats.split(",")
    reqs = make_requests(args.requests, args.sources, fmt_names, args.seed)
    cpu = cpu_leg(args, srcs, reqs) if args.cpu_seconds > 0 and rank == 0 and world == 1 else None

    import threading

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend="nccl" if torch.cuda.is_available() else "gloo")
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    from imagekit import ImageFormat, _lib, transform_batch, transform_batch_submit
    lib = _lib.load()
    queue = world == 1
    assert lib.ik_init(-1 if queue else local) == 0, _lib.last_error()
    ndev = lib.ik_logical_device_count() if queue else 1
    if args.clients <= 0:
        args.clients = max(1, ndev)
    mine = [(s, w, h, ImageFormat[f]) for s, w, h, f in shard(reqs, rank, world)]

    def run_batch(chunk):
        return transform_batch([srcs[s] for s, _, _, _ in chunk], [(w, h) for _, w, h, _ in chunk],
                               [f for _, _, _, f in chunk], [args.quality] * len(chunk), threads=args.threads)

    run_batch(mine[:min(len(mine), 8)])  # warm-up: plans, streams, pinned staging

    def barrier():
        if dist is not None:
            dist.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    chunks = [mine[i:i + args.batch] for i in range(0, len(mine), args.batch)]
    lat, out_bytes = [], [0]
    lock = threading.Lock()
    nxt = [0]

    def done(tb, res):
        dt = (time.perf_counter() - tb) * 1e3
        with lock:
            lat.append(dt)
            out_bytes[0] += sum(len(r) for r in res)
            if len(lat) % 20 == 0:
                print(f"[loadtest] {len(lat) * args.batch} requests", file=sys.stderr, flush=True)

    def client():  # a request handler: takes the next batch, waits for its bytes
        pend = None  # (start time, PendingBatch) of the batch submitted last (--pipeline)
        while True:
            with lock:
                chunk = chunks[nxt[0]] if nxt[0] < len(chunks) else None
                nxt[0] += 1
            if chunk is None:
                if pend is not None:
                    done(pend[0], pend[1].wait())
                return
            tb = time.perf_counter()
            if not args.pipeline:
                done(tb, run_batch(chunk))
                continue
            p = transform_batch_submit([srcs[s] for s, _, _, _ in chunk], [(w, h) for _, w, h, _ in chunk],
                                       [f for _, _, _, f in chunk], [args.quality] * len(chunk), threads=args.threads)
            if pend is not None:
                done(pend[0], pend[1].wait())
            pend = (tb, p)

    barrier()
    t0 = time.perf_counter()
    ts = [threading.Thread(target=client) for _ in range(max(1, args.clients))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    elapsed = time.perf_counter() - t0
    barrier()
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}" if torch.cuda.is_available() else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    out_bytes = out_bytes[0]
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
            "filter": "lanczos3 (the reference's)",
            "pipelined": bool(args.pipeline),
            "dispatch": (f"in-library dynamic queue over {ndev} logical device(s), {args.clients} client threads"
                         if queue else f"{world} processes, round-robin shards"),
            "cpu_leg": cpu,
        }))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
