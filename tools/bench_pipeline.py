#!/usr/bin/env python3
"""tools/bench_pipeline.py -- the device-resident pipeline bench (round 1's bench.py):
frames already decoded in HBM -> resize -> encode, for the configs[2] (JPEG q85,
Lanczos3, 256-image batches) and configs[4] (8192^2 -> 1024^2 AVIF q60) shapes and
for kernel / roofline work on the resize.  The headline metric (PNG bytes in host
memory -> WebP bytes in host memory) is bench.py at the repo root.

Workload (BASELINE.json configs[1]): synthetic 4096x4096 RGBA8 images already
resident in HBM ("RGBA8 synthetic": the decoded DynamicImage the reference's
resize_image receives; raw frames need no entropy decode) -> resize_image to
512x512 (Triangle = "bilinear" per configs[1]; --filter lanczos3 for the
reference's own filter) -> encode_image WebP q80.  One step = one batch through
libimagekit_hip.so's pipeline: ONE resize launch over the batch, ONE WebP
colour-convert launch, D2H of the YUV planes, libwebp VP8 coding of every image
on the host thread pool.  Encoded bytes end in host memory.  Batches go through
ik_pipeline_submit / ik_pipeline_collect with two in flight, so the host coding
of batch i overlaps the device stage of batch i+1 (--sync: one at a time).

value = input pixels of all images of all ranks / max-over-ranks wall time of
the K timed steps.  roofline = the resize kernel (the dominant device kernel):
algorithmic bytes per launch (4*W*H + 4*w*h per image) /
its average duration from HIP events on the pipeline's stream.  cpu_baseline =
the oracle restatement of the reference CPU path (image 0.25.8 resize + libwebp
WebPEncodeRGB) timed on this host's cores on a bounded sample.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N>1 under
torch.distributed.run (one rank per GPU, RCCL only for barrier/max).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-image-transform_amd"), os.path.join(ROOT, "tests")]
import ikutil  # noqa: E402

ikutil.use_pillow_codecs()  # codec libraries named explicitly (IK_LIBWEBP / IK_LIBAVIF)

METRIC = "transform MPix/s (decode+resize+encode) 4096²→512² WebP q80; 1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
FILTERS = {"nearest": 0, "triangle": 1, "catmullrom": 2, "gaussian": 3, "lanczos3": 4}
ENCODERS = {"libwebp": 0, "exact": 2}
CPU_CODER = {"webp": "libwebp", "jpeg": "image-crate JPEG", "avif": "libavif/aom speed 4 (Pillow, rav1e absent)"}
FORMATS = {"jpeg": 0, "webp": 1, "avif": 2}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=64, help="images per GPU per step")
    ap.add_argument("--alt-batch", type=int, default=256, help="images per GPU per step for the other WebP encoder")
    ap.add_argument("--alt-steps", type=int, default=4)
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--out", type=int, default=512)
    ap.add_argument("--filter", default="triangle", choices=sorted(FILTERS))
    ap.add_argument("--quality", type=int, default=80)
    ap.add_argument("--format", default="webp", choices=["webp", "jpeg", "avif"],
                    help="webp: the headline (configs[1]); jpeg: configs[2]-style runs (GPU Huffman coding); "
                         "avif: configs[4]-style runs (--size 8192 --out 1024 --filter lanczos3 --quality 60)")
    ap.add_argument("--threads", type=int, default=16, help="host entropy-coder threads per rank")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="cpu_baseline sample wall-time budget (s)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--device-only", action="store_true", help="time resize+colour kernels only")
    ap.add_argument("--webp-encoder", default="libwebp", choices=["libwebp", "exact"],
                    help="libwebp: host VP8 coder, bytes identical to the reference; gpu: gfx950 VP8 encoder")
    ap.add_argument("--sync", action="store_true", help="one batch in flight (ik_pipeline_run per step)")
    ap.add_argument("--no-alt-encoder", action="store_true", help="skip timing the other WebP encoder")
    ap.add_argument("--png-images", type=int, default=64,
                    help="images per rank for each decode-inclusive leg (PNG and JPEG sources through ik_transform_batch; 0 = skip)")
    return ap.parse_args()


def shard_seeds(rank: int, batch: int, distinct: int = 4):
    """Synthetic frames of rank `rank`: disjoint seed ranges, so ranks never share work."""
    return [1000 * rank + i for i in range(min(batch, distinct))]


def reduce_max(value: float, dist, device) -> float:
    """Max over ranks (the slowest rank defines the job's wall time)."""
    if dist is None:
        return value
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def aggregate_mpix(world: int, batch: int, steps: int, size: int, elapsed: float) -> float:
    """Whole-job throughput: input pixels of all ranks / max-over-ranks wall time."""
    return world * batch * steps * size * size / elapsed / 1e6


def synth_rgba(w, h, seed):
    import ikutil
    return ikutil.synth(w, h, 4, seed=seed, pattern="S")


def png_leg(args, frames, world, dist, device, barrier, kind="png"):
    """Decode-inclusive figure beside `value`: the same frames as encoded files through
    ik_transform_batch, with encoded input and output bytes in host memory.
    kind "png": PNG RGBA8 (Pillow's zlib level 6; SURVEY 8(d) D-2's container for
    configs[1]) -- host inflate + unfilter (png 0.18 via image), device resize, encode.
    kind "jpeg": baseline JPEG q90 4:2:0 with a restart marker per MCU row (D-2's
    container for configs[2]) -- GPU entropy decoding, IDCT, upsampling and colour."""
    import io

    from PIL import Image

    from imagekit import transform_batch
    pngs = []
    for im in frames[:2]:
        b = io.BytesIO()
        if kind == "png":
            Image.fromarray(im, "RGBA").save(b, format="PNG")
        else:
            Image.fromarray(np.ascontiguousarray(im[..., :3]), "RGB").save(b, format="JPEG", quality=90,
                                                                         restart_marker_rows=1)
        pngs.append(b.getvalue())
    n, O, fmt, f = args.png_images, args.out, FORMATS[args.format], FILTERS[args.filter]

    def run(k):
        res = transform_batch([pngs[i % len(pngs)] for i in range(k)], [(O, O)] * k, [fmt] * k,
                              [args.quality] * k, filter=f, threads=args.threads)
        assert all(r for r in res)

    run(2)
    barrier()
    t0 = time.perf_counter()
    run(n)
    el = time.perf_counter() - t0
    barrier()
    el = reduce_max(el, dist, device)
    res = {"source": "PNG RGBA8 (zlib level 6), host inflate + unfilter" if kind == "png" else
                     "JPEG q90 4:2:0, RSTn per MCU row, GPU entropy decoding", "images_per_gpu": n,
           "bytes_per_source_image": sum(len(p) for p in pngs) // len(pngs),
           "value": round(aggregate_mpix(world, n, 1, args.size, el), 2), "unit": "MPix/s",
           "ms_per_image_per_gpu": round(el / n * 1e3, 3)}
    if world == 1 and not args.no_cpu_baseline and args.format != "avif":
        # CPU proxy of the same decode-inclusive transform: Pillow's PNG decoder (zlib +
        # libpng-style unfilter, standing in for png 0.18) + the oracle resize + encode,
        # one image per thread, two rounds of args.threads images
        import ikutil
        orc = ikutil.Oracle()
        threads = max(1, min(args.threads, os.cpu_count() or 1))

        def one(k):
            px = np.asarray(Image.open(io.BytesIO(pngs[k % len(pngs)])).convert("RGBA" if kind == "png" else "RGB"))
            b, _ = orc.transform(px, O, O, f, fmt, args.quality)
            assert b

        t0 = time.perf_counter()
        for r in range(2):
            ts = [threading.Thread(target=one, args=(r * threads + i,)) for i in range(threads)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
        cw = time.perf_counter() - t0
        res["cpu_proxy"] = {"value": round(2 * threads * args.size * args.size / cw / 1e6, 2), "unit": "MPix/s",
                            "cores": threads, "sample": f"{2 * threads} {kind.upper()} images, Pillow decode + oracle "
                                                        f"resize + {CPU_CODER[args.format]}, {cw:.1f}s wall"}
    return res


def cpu_baseline(args, img: np.ndarray):
    """Reference CPU transform restated (oracle/, test infrastructure) on a bounded sample."""
    import ikutil
    orc = ikutil.Oracle()
    threads = max(1, min(args.threads, os.cpu_count() or 1))
    H, W, C = img.shape
    f = FILTERS[args.filter]
    done = [0]
    lock = threading.Lock()

    def one():
        if args.format == "avif":  # oracle resize + libavif/aom (Pillow's, one thread), speed 4 as ravif's
            import io

            from PIL import Image
            px = orc.resize(img, args.out, args.out, f)
            bio = io.BytesIO()
            Image.fromarray(px[..., :3]).save(bio, format="AVIF", quality=args.quality, speed=4, max_threads=1)
            assert bio.getvalue()[4:8] == b"ftyp"
        else:
            b, dims = orc.transform(img, args.out, args.out, f, FORMATS[args.format], args.quality)
            assert dims == (args.out, args.out) and b[:2] in (b"RI", b"\xff\xd8")
        with lock:
            done[0] += 1

    # single-thread time of one warm image sizes the sample: `rounds` rounds of one
    # image per thread ~ args.cpu_seconds of wall time (10-30 s of CPU work in all)
    one()
    t0 = time.perf_counter()
    one()
    t1 = time.perf_counter() - t0
    rounds = max(1, int(args.cpu_seconds / max(t1, 1e-3)))
    rounds = min(rounds, 400)
    done[0] = 0
    t0 = time.perf_counter()
    for _ in range(rounds):
        ts = [threading.Thread(target=one) for _ in range(threads)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    wall = time.perf_counter() - t0
    n = done[0]
    return {
        "value": round(n * W * H / wall / 1e6, 3),
        "unit": "MPix/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{n} x {W}x{H} RGBA8 -> {args.out}x{args.out} {args.filter} + "
                  f"{CPU_CODER[args.format]} q{args.quality}, "
                  f"one image per thread, {threads} threads, {wall:.1f}s wall",
        "value_1core": round(W * H / t1 / 1e6, 3),
        "host": host_info(),
    }


def host_info():
    """the GPU box host's CPU model and core count beside the CPU number."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(),
            "affinity": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # run directly with --gpus N: start the one-rank-per-GPU job as a child
        # (nothing has touched the GPU yet) and pass its exit status on
        import socket
        import subprocess
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
        raise SystemExit(subprocess.run(cmd).returncode)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    import torch
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend="nccl" if torch.cuda.is_available() else "gloo")
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    from imagekit import _lib
    lib = _lib.load()
    if lib.ik_init(local) != 0:
        raise SystemExit(f"ik_init({local}) failed: {_lib.last_error()}")

    S, O, B = args.size, args.out, args.batch
    f = FILTERS[args.filter]
    pitch = S * 4
    # inputs resident in HBM before the timed region: 4 distinct synthetic frames tiled over the batch
    NB = max(B, 0 if (args.device_only or args.no_alt_encoder or args.format != "webp") else args.alt_batch)
    distinct = [synth_rgba(S, S, seed=sd) for sd in shard_seeds(rank, NB)]
    src = torch.empty((NB, S, pitch), dtype=torch.uint8, device=f"cuda:{local}")
    for i in range(NB):  # distinct frames over PCIe once, the rest device to device
        if i < len(distinct):
            src[i].copy_(torch.from_numpy(distinct[i].reshape(S, pitch)))
        else:
            src[i].copy_(src[i % len(distinct)])
    torch.cuda.synchronize()

    pipe = ctypes.c_void_p()
    fmt = FORMATS[args.format]
    if lib.ik_pipeline_create(S, S, 4, O, O, f, fmt, args.quality, B, args.threads, ctypes.byref(pipe)):
        raise SystemExit(f"pipeline: {_lib.last_error()}")
    if fmt == 1 and lib.ik_pipeline_set_webp_encoder(pipe, ENCODERS[args.webp_encoder]):
        raise SystemExit(f"webp encoder: {_lib.last_error()}")
    out_cap = B * O * O * 4 + (1 << 20)
    out = np.empty(out_cap, np.uint8)
    sizes = (ctypes.c_size_t * B)()

    src_ptr = ctypes.c_void_p(src.data_ptr())
    n_done = ctypes.c_uint32()

    def kernel_ms():
        return tuple(lib.ik_pipeline_kernel_ms(pipe, k) for k in range(4))

    def submit():
        if lib.ik_pipeline_submit(pipe, src_ptr, pitch, S * pitch, B):
            raise SystemExit(f"pipeline submit: {_lib.last_error()}")

    def collect():
        if lib.ik_pipeline_collect(pipe, out.ctypes.data, out_cap, sizes, ctypes.byref(n_done)):
            raise SystemExit(f"pipeline collect: {_lib.last_error()}")
        assert n_done.value == B
        return kernel_ms()

    def run_steps(k):
        """k batches; with --sync one run per batch, else two in flight (the host
        stage of batch i overlaps the device stage of batch i+1)"""
        if args.device_only:
            res = []
            for _ in range(k):
                if lib.ik_pipeline_run_device(pipe, src_ptr, pitch, S * pitch, B):
                    raise SystemExit(f"pipeline run: {_lib.last_error()}")
                res.append(kernel_ms())
            return res
        if args.sync:
            res = []
            for _ in range(k):
                submit()
                res.append(collect())
            return res
        res = []
        submit()
        for _ in range(k - 1):
            submit()
            res.append(collect())
        res.append(collect())
        return res

    if args.warmup:
        run_steps(args.warmup)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    kms = run_steps(args.steps)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    barrier()
    elapsed = reduce_max(elapsed, dist, f"cuda:{local}")

    if not args.device_only:
        assert (bytes(out[:2]) in (b"RI", b"\xff\xd8") or bytes(out[4:8]) == b"ftyp") and all(s > 0 for s in sizes)
    resize_ms = float(np.mean([k[0] for k in kms]))
    colour_ms = float(np.mean([k[1] for k in kms]))
    vp8_ms = float(np.mean([k[2] for k in kms]))
    host_ms = float(np.mean([k[3] for k in kms]))
    out_bytes = int(sum(sizes))

    # the other WebP encoder end to end on frames of the same batch (a few steps,
    # its own batch size: the GPU VP8 wavefront is latency-bound, so it wants more
    # images per launch)
    alt_enc = {}
    if not args.device_only and not args.no_alt_encoder and fmt == 1:
        other = "exact" if args.webp_encoder == "libwebp" else "libwebp"
        AB = args.alt_batch
        p3 = ctypes.c_void_p()
        if lib.ik_pipeline_create(S, S, 4, O, O, f, 1, args.quality, AB, args.threads, ctypes.byref(p3)) == 0:
            if lib.ik_pipeline_set_webp_encoder(p3, ENCODERS[other]) == 0:
                acap = AB * O * O * 4 + (1 << 20)
                aout = np.empty(acap, np.uint8)
                asz = (ctypes.c_size_t * AB)()
                nd = ctypes.c_uint32()

                def asub():
                    assert lib.ik_pipeline_submit(p3, src_ptr, pitch, S * pitch, AB) == 0, _lib.last_error()

                def acol():
                    assert lib.ik_pipeline_collect(p3, aout.ctypes.data, acap, asz, ctypes.byref(nd)) == 0, \
                        _lib.last_error()
                    return lib.ik_pipeline_kernel_ms(p3, 2), lib.ik_pipeline_kernel_ms(p3, 3)

                asub()
                acol()
                barrier()
                t1 = time.perf_counter()
                asub()
                ak = []
                for _ in range(args.alt_steps - 1):
                    asub()
                    ak.append(acol())
                ak.append(acol())
                barrier()
                te = reduce_max(time.perf_counter() - t1, dist, f"cuda:{local}")
                alt_enc = {"encoder": other, "batch_per_gpu": AB, "steps": args.alt_steps,
                           "value": round(aggregate_mpix(world, AB, args.alt_steps, S, te), 2),
                           "ms_per_step": round(te / args.alt_steps * 1e3, 3),
                           "vp8_kernel_ms": round(float(np.mean([k[0] for k in ak])), 4),
                           "host_stage_ms": round(float(np.mean([k[1] for k in ak])), 3),
                           "output_bytes_per_image": int(sum(asz)) // AB}
            lib.ik_pipeline_destroy(p3)
    bytes_per_img = 4 * S * S + 4 * O * O
    achieved = B * bytes_per_img / (resize_ms * 1e-3) / 1e9
    value = aggregate_mpix(world, B, args.steps, S, elapsed)

    # the other filter's kernel on the same batch (device-only), for DESIGN.md
    alt = {}
    alt_name = "lanczos3" if args.filter != "lanczos3" else "triangle"
    p2 = ctypes.c_void_p()
    if lib.ik_pipeline_create(S, S, 4, O, O, FILTERS[alt_name], 1, args.quality, B, 1, ctypes.byref(p2)) == 0:
        ms = []
        for i in range(6):
            lib.ik_pipeline_run_device(p2, ctypes.c_void_p(src.data_ptr()), pitch, S * pitch, B)
            if i >= 2:
                ms.append(lib.ik_pipeline_kernel_ms(p2, 0))
        m = float(np.mean(ms))
        alt = {"filter": alt_name, "resize_ms": round(m, 4),
               "achieved_GBps": round(B * bytes_per_img / (m * 1e-3) / 1e9, 1)}
        lib.ik_pipeline_destroy(p2)
    # the FMA resize mode (within 1 LSB; the default stays bit-exact) on both filters, device-only
    fma = {}
    if lib.ik_set_resize_mode(1) == 0:
        for name in (args.filter, alt_name):
            p4 = ctypes.c_void_p()
            if lib.ik_pipeline_create(S, S, 4, O, O, FILTERS[name], 1, args.quality, B, 1, ctypes.byref(p4)) == 0:
                ms = []
                for i in range(6):
                    lib.ik_pipeline_run_device(p4, ctypes.c_void_p(src.data_ptr()), pitch, S * pitch, B)
                    if i >= 2:
                        ms.append(lib.ik_pipeline_kernel_ms(p4, 0))
                m = float(np.mean(ms))
                fma[name] = {"resize_ms": round(m, 4), "achieved_GBps": round(B * bytes_per_img / (m * 1e-3) / 1e9, 1)}
                lib.ik_pipeline_destroy(p4)
        lib.ik_set_resize_mode(0)
    lib.ik_pipeline_destroy(pipe)

    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_resize.json")
    if os.path.exists(pmc):
        try:
            d = json.load(open(pmc))
            key = f"{args.filter}_{S}_{O}_b{B}"
            if key in d:
                traffic = d[key]["hbm_bytes_per_launch"]
        except Exception:
            traffic = None

    png = jpg = {}
    if args.png_images > 0 and not args.device_only and args.format != "avif":
        png = png_leg(args, distinct, world, dist, f"cuda:{local}", barrier)
        jpg = png_leg(args, distinct, world, dist, f"cuda:{local}", barrier, kind="jpeg")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, distinct[0])

    if rank == 0:
        line = {
            "metric": METRIC if args.format == "webp" else
                      f"transform MPix/s (resize+encode) {S}²→{O}² {args.filter} {args.format.upper()} q{args.quality} "
                      f"(configs[{2 if args.format == 'jpeg' else 4}] shape)",
            "value": round(value, 2),
            "unit": "MPix/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {
                "workload": f"{S}x{S} RGBA8 frames resident in HBM -> resize_image {O}x{O} "
                            f"({args.filter}) -> encode_image {args.format} q{args.quality}; bytes to host",
                "batch_per_gpu": B, "filter": args.filter, "format": args.format,
                "quality": args.quality, "host_threads_per_gpu": args.threads,
                "webp_encoder": args.webp_encoder,
                "libwebp": "%d.%d.%d" % (lib.ik_libwebp_version() >> 16, (lib.ik_libwebp_version() >> 8) & 255,
                                         lib.ik_libwebp_version() & 255),
                "device_only": bool(args.device_only), "batches_in_flight": 1 if args.sync else 2, "parallelism": f"images sharded, {world} rank(s)",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic,
                "kernel": "k_resize_fused",
                "kernel_ms": round(resize_ms, 4),
                "bytes_per_launch": B * bytes_per_img,
            },
            "colour_kernel_ms": round(colour_ms, 4),
            "vp8_kernel_ms": round(vp8_ms, 4),
            "host_stage_ms": round(host_ms, 3),
            "output_bytes_per_image": out_bytes // B,
            "alt_webp_encoder": alt_enc,
            "alt_filter_kernel": alt,
            "resize_fma_mode": fma,
            "decode_inclusive_png": png,
            "decode_inclusive_jpeg": jpg,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
