#!/usr/bin/env python3
"""bench.py -- transform MPix/s (decode+resize+encode) 4096^2 -> 512^2 WebP q80.

Headline `value` (BASELINE.json metric): synthetic 4096x4096
RGBA8 frames as PNG files (Pillow, zlib level 6, adaptive filters; the configs[1]
frame in the container SURVEY D-2 names), one device allocation per request,
already resident in HBM when the timed region starts (the measurement contract);
one step is one batch through ik_transform_batch_submit_device / _wait --
decode_image (GPU chunk walk, gather + IDAT CRCs, inflate + unfilter, ik_png.hip),
resize_image to 512x512 (Triangle = configs[1]'s "bilinear"), encode_image WebP
q80 (libwebp, byte-identical to the reference's webp 0.3.1 path) -- ending with
the WebP bytes in host memory; --inflight batches are outstanding.  value = input
pixels of all ranks / max-over-ranks wall time of the K timed steps (every timed
batch waited for).  The host threads the GPU path may use are stated (--threads,
default 32 = an 8-GPU node's 256 cores / 8).

pcie_inclusive: the same steps with the PNG files in HOST memory (page-locked, as a
server reads request bodies with ik_host_alloc) through ik_transform_batch_submit,
so the compressed bytes cross PCIe inside the timed region (upload of one batch
under another's kernels).

Beside it, in the same JSON line:
  cpu_baseline   the same PNG bytes through the reference CPU path restated
                 (oracle/: png decode + image 0.25.8 resize + libwebp), one image
                 per worker at a time, on 1 core and on every core the job can
                 use (min of nproc, the cgroup CPU quota and the affinity mask;
                 SURVEY D-6: the reference runs one synchronous transform per
                 tokio worker), plus the linear physical-core bound (a bound).
  roofline       the dominant device kernel of the step by HIP-event time, its
                 algorithmic bytes per launch / its duration vs 8 TB/s; the
                 resize kernel's own roofline in roofline_resize.
  pageable_input the same steps with the PNG files in ordinary host memory.
  hbm_resident   the old headline: the same frames already decoded in HBM ->
                 ik_pipeline (one resize launch per batch, WebP colour kernel,
                 libwebp on the host threads), two batches in flight.
  decode_inclusive_jpeg   the same frames as JPEG q90 4:2:0 with restart markers
                 (configs[2]'s container) through ik_transform_batch.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N>1 under
torch.distributed.run (one rank per GPU; RCCL only for barrier / max).
"""
from __future__ import annotations

import argparse
import ctypes
import io
import json
import os
import resource
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "rust-image-transform_amd"), os.path.join(ROOT, "tests")]

METRIC = "transform MPix/s (decode+resize+encode) 4096²→512² WebP q80; 1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
FILTERS = {"nearest": 0, "triangle": 1, "catmullrom": 2, "gaussian": 3, "lanczos3": 4}
FORMATS = {"jpeg": 0, "webp": 1, "avif": 2}
# ik_png_last_timing fields reported (index -> name; include/imagekit_hip.h)
PNG_STAGES = {0: "upload_host", 1: "upload_device", 14: "gather_crc", 15: "kernel_stage_wait_find", 13: "find",
              2: "decode", 3: "expand", 4: "resolve", 5: "unfilter", 6: "kernel_stage_wall",
              16: "find_beside_previous_batch"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=64, help="PNG requests per GPU per step")
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--out", type=int, default=512)
    ap.add_argument("--filter", default="triangle", choices=sorted(FILTERS))
    ap.add_argument("--quality", type=int, default=80)
    ap.add_argument("--format", default="webp", choices=sorted(FORMATS), help="output format (encode_image)")
    ap.add_argument("--source", default="png", choices=["png", "jpeg-rst", "jpeg"],
                    help="input container: PNG (configs[1]), or JPEG q90 4:2:0 with a restart marker per MCU "
                         "row / without (configs[2]'s sources)")
    ap.add_argument("--distinct", type=int, default=4, help="distinct PNG frames per rank (tiled over the batch)")
    ap.add_argument("--threads", type=int, default=32, help="host threads per GPU (stated budget)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target wall time of each cpu_baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--webp-encoder", default="auto", choices=["auto", "libwebp", "exact"],
                    help="auto (the library default, IK_WEBP_AUTO): a batch's same-geometry groups on the exact GPU "
                         "coder (libwebp's method-4 decisions on the GPU, byte-identical files); exact: every image "
                         "on it; libwebp: libwebp on host threads")
    ap.add_argument("--alt-steps", type=int, default=6,
                    help="steps of the extra leg with the other WebP coder (0 = skip)")
    ap.add_argument("--no-extras", action="store_true", help="skip the hbm_resident / JPEG legs")
    ap.add_argument("--hbm-batch", type=int, default=64)
    ap.add_argument("--hbm-steps", type=int, default=6)
    ap.add_argument("--jpeg-images", type=int, default=64)
    ap.add_argument("--pipeline", type=int, default=1,
                    help="1: steps are ik_transform_batch_submit calls with --inflight batches outstanding, so "
                         "one batch's upload, another's kernels and a third's libwebp coding overlap; 0: one "
                         "blocking ik_transform_batch per step")
    ap.add_argument("--inflight", type=int, default=3,
                    help="batches submitted before the oldest is waited for (upload / kernels / host coders "
                         "of three batches overlap)")
    ap.add_argument("--no-pcie-leg", action="store_true", help="skip the pcie_inclusive leg (host-memory inputs)")
    ap.add_argument("--pageable", action="store_true",
                    help="inputs in ordinary host memory (default: page-locked, ik_host_alloc)")
    ap.add_argument("--pageable-steps", type=int, default=4,
                    help="steps of the extra leg with pageable inputs (0 = skip)")
    ap.add_argument("--inproc-devices", type=int, default=0,
                    help="drive N logical devices from this one process (ik_init(-1), IK_DEVICES)")
    ap.add_argument("--inproc-map", default="",
                    help="physical device of each logical device, e.g. 0,0 (default 0..N-1)")
    return ap.parse_args()


def shard_seeds(rank: int, n: int):
    """Synthetic frames of rank `rank`: disjoint seed ranges, so ranks never share work."""
    return [1000 * rank + i for i in range(n)]


def reduce_max(value: float, dist, device) -> float:
    """Max over ranks (the slowest rank defines the job's wall time)."""
    if dist is None:
        return value
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_floats(vals, dist, device, world):
    """[rank][k] = vals[k] of every rank (rank 0's own list without a process group)"""
    if dist is None:
        return [list(vals)]
    import torch
    t = torch.tensor(vals, dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [[float(x) for x in o.tolist()] for o in out]


def aggregate_mpix(world: int, per_rank_images: int, size: int, elapsed: float) -> float:
    """Whole-job throughput: input pixels of all ranks / max-over-ranks wall time."""
    return world * per_rank_images * size * size / elapsed / 1e6


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
    quota = None  # the cgroup's CPU quota in cores (a GPU box shares its host: nproc shows the whole machine)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            quota = None if q <= 0 else round(q / per, 2)
        except (OSError, ValueError):
            pass
    return {"cpu_model": model, "nproc": os.cpu_count(), "cgroup_cpu_quota_cores": quota,
            "affinity": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
            "physical_cores": physical_cores()}


def codec_path(lib, fmt) -> str:
    buf = ctypes.create_string_buffer(4096)
    lib.ik_codec_library(fmt, buf, len(buf))
    return buf.value.decode("utf-8", "replace")


def make_pngs(frames):
    from PIL import Image
    out = []
    for im in frames:
        b = io.BytesIO()
        Image.fromarray(im, "RGBA").save(b, format="PNG")  # zlib level 6, adaptive filters
        out.append(b.getvalue())
    return out


def make_jpegs(frames, rst):
    from PIL import Image
    out = []
    for im in frames:
        b = io.BytesIO()
        kw = {"restart_marker_rows": 1} if rst else {}
        Image.fromarray(np.ascontiguousarray(im[..., :3]), "RGB").save(b, format="JPEG", quality=90, subsampling=2,
                                                                     **kw)
        out.append(b.getvalue())
    return out


_CPU = {}  # the oracle and the inputs, inherited by the forked cpu_baseline workers


def _cpu_one(k):
    """One reference-path transform on the CPU (oracle/): PNG bytes -> WebP bytes."""
    import ikutil
    L, pngs, O, f, fmt, q = (_CPU[x] for x in ("L", "pngs", "O", "f", "fmt", "q"))
    data = pngs[k % len(pngs)]
    px = ikutil.u8p()
    if data[:4] == b"\x89PNG":
        w, h, c = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        n = L.iko_png_decode(data, len(data), ctypes.byref(px), ctypes.byref(w), ctypes.byref(h), ctypes.byref(c))
    else:  # JPEG: the zune-jpeg 0.4.21 restatement (the reference's decoder)
        w, h, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        n = L.iko_jpeg_decode(data, len(data), 1, ctypes.byref(px), ctypes.byref(w), ctypes.byref(h), ctypes.byref(c))
        n = 1 if n == 0 else -abs(n) - 1
    assert n > 0, n
    out = ikutil.u8p()
    ow, oh = ctypes.c_uint32(), ctypes.c_uint32()
    m = L.iko_transform_u8(px, w.value, h.value, c.value, O, O, f, fmt, q, ctypes.byref(out),
                           ctypes.byref(ow), ctypes.byref(oh))
    L.iko_free(px)
    assert m > 0 and (ow.value, oh.value) == (O, O)
    L.iko_free(out)
    return 1


def cpu_baseline(args, pngs):
    """The reference CPU path restated (oracle/: PNG decode + image 0.25.8 resize +
    libwebp WebPEncodeRGB) on the same PNG bytes, one image per worker at a time:
    on 1 core and on one worker process per effective core.  Workers are forked processes, as
    independent requests are: threads of one process serialise on the allocator
    and on first-touch page faults of the ~100 MB per image (measured: 256 threads
    reached only 9x one thread).  Runs before anything initialises the GPU (the
    pools fork).  Each sample is sized to about args.cpu_seconds of wall."""
    import multiprocessing as mp

    import ikutil
    orc = ikutil.Oracle()
    L = orc.lib
    L.iko_png_decode.restype = ctypes.c_long
    L.iko_png_decode.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ikutil.u8p),
                                 ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                 ctypes.POINTER(ctypes.c_uint32)]
    L.iko_jpeg_decode.restype = ctypes.c_int
    L.iko_jpeg_decode.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ikutil.u8p),
                                  ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                  ctypes.POINTER(ctypes.c_int)]
    _CPU.update(L=L, pngs=pngs, O=args.out, f=FILTERS[args.filter], fmt=FORMATS[args.format], q=args.quality)
    _cpu_one(0)
    t0 = time.perf_counter()
    _cpu_one(1)
    t1 = time.perf_counter() - t0
    n1 = max(2, int(args.cpu_seconds / max(t1, 1e-3)))
    t0 = time.perf_counter()
    for k in range(n1):
        _cpu_one(k)
    w1 = time.perf_counter() - t0

    def pool_rate(nw):
        per = max(2, min(8, int(args.cpu_seconds / 2 / max(t1, 1e-3))))
        with mp.get_context("fork").Pool(nw) as pool:
            pool.map(_cpu_one, range(nw), chunksize=1)  # every worker warm (library state, page tables)
            t0 = time.perf_counter()
            done = sum(pool.map(_cpu_one, range(nw * per), chunksize=per))
            return done, time.perf_counter() - t0

    host = host_info()
    nproc = os.cpu_count() or 1
    eff = effective_cores(host)
    done, wn = pool_rate(eff)
    S, O = args.size, args.out
    v1 = round(n1 * S * S / w1 / 1e6, 2)
    phys = host.get("physical_cores") or nproc
    return {
        "value": round(done * S * S / wn / 1e6, 2),
        "unit": "MPix/s",
        "cores": eff,
        "cores_basis": "effective cores = min(nproc, cgroup CPU quota, affinity); the job cannot use more",
        "nproc": nproc,
        "kind": "port",
        "sample": (f"{done} x {S}x{S} RGBA8 PNG (host memory) -> oracle PNG decode (CRC, libdeflate inflate, "
                   f"unfilter)" if args.source == "png" else
                   f"{done} x {S}x{S} JPEG q90 4:2:0 ({args.source}, host memory) -> oracle zune-jpeg restatement "
                   f"decode") + f" -> image 0.25.8 resize {O}x{O} {args.filter} -> {args.format} q{args.quality} "
                  f"({'libwebp' if args.format == 'webp' else 'restated image JpegEncoder' if args.format == 'jpeg' else 'libavif/aom'}); "
                  f"one image per worker process at a time, {eff} processes on {eff} effective cores, {wn:.1f}s wall",
        "value_1core": v1,
        "sample_1core": f"{n1} images on 1 thread, {w1:.1f}s wall",
        # not a measurement: the 1-core rate times the host's physical cores, what
        # an uncapped host could at best reach with one transform per core
        "cpu_linear_bound_physical": round(v1 * phys, 1),
        "physical_cores": phys,
        "host": host,
    }


def effective_cores(host) -> int:
    """Cores this job can actually use: min(nproc, cgroup quota, affinity)."""
    c = host.get("nproc") or 1
    if host.get("cgroup_cpu_quota_cores"):
        c = min(c, max(1, int(host["cgroup_cpu_quota_cores"])))
    if host.get("affinity"):
        c = min(c, host["affinity"])
    return max(1, c)


def physical_cores():
    """Distinct (package, core) pairs in sysfs: hardware threads folded."""
    import glob
    seen = set()
    for d in glob.glob("/sys/devices/system/cpu/cpu[0-9]*/topology"):
        try:
            seen.add((open(d + "/physical_package_id").read().strip(), open(d + "/core_id").read().strip()))
        except OSError:
            pass
    return len(seen) or None


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
    S, O, B = args.size, args.out, args.batch
    if args.inproc_devices > 0:
        # one process driving several logical devices through the library's own
        # dispatch (ik_init(-1)); --inproc-map names their physical devices
        devs = [int(x) for x in args.inproc_map.split(",")] if args.inproc_map else list(range(args.inproc_devices))
        os.environ["IK_DEVICES"] = ",".join(str(d) for d in devs[:args.inproc_devices])
    import ikutil
    # the codec libraries are explicit dependencies of libimagekit_hip.so
    # (IK_LIBWEBP / IK_LIBAVIF, else the system sonames): name the copies used here
    ikutil.use_pillow_codecs()
    frames = [ikutil.synth(S, S, 4, seed=sd, pattern="S") for sd in shard_seeds(rank, args.distinct)]
    pngs = make_pngs(frames) if args.source == "png" else make_jpegs(frames, args.source == "jpeg-rst")
    # the CPU leg first: its worker pools fork, and nothing may have touched the GPU yet
    cpu = cpu_baseline(args, pngs) if rank == 0 and world == 1 and not args.no_cpu_baseline else None
    dist = None
    import torch
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend="nccl" if torch.cuda.is_available() else "gloo")
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    from imagekit import (DeviceBytes, PinnedBytes, _lib, transform_batch, transform_batch_submit,
                          transform_batch_submit_device)
    lib = _lib.load()
    if lib.ik_init(-1 if args.inproc_devices > 0 else local) != 0:
        raise SystemExit(f"ik_init failed: {_lib.last_error()}")
    WEBP_ENC = {"libwebp": 0, "exact": 2, "auto": 3}
    if lib.ik_set_webp_encoder(WEBP_ENC[args.webp_encoder]) != 0:
        raise SystemExit(f"ik_set_webp_encoder failed: {_lib.last_error()}")
    dev = f"cuda:{local}"
    # request bodies in page-locked host memory (ik_host_alloc), as a server reads
    # them: the upload DMAs them in place (--pageable: ordinary Python bytes)
    inputs = pngs if args.pageable else [PinnedBytes(p) for p in pngs]
    reqs = [inputs[i % len(inputs)] for i in range(B)]
    # the headline's inputs: every request its own device allocation in HBM (PNG:
    # the GPU walks and gathers them in place).  JPEG sources are parsed on the host
    # (markers, restart scan), so they stay in page-locked host memory.
    dreqs = [DeviceBytes(pngs[i % len(pngs)]) for i in range(B)] if args.source == "png" else reqs
    magic = {"webp": lambda r: r[:4] == b"RIFF", "jpeg": lambda r: r[:2] == b"\xff\xd8",
             "avif": lambda r: r[4:8] == b"ftyp"}[args.format]

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    f = FILTERS[args.filter]

    def resize_kernel(C: int) -> str:  # the resampler this geometry takes (k_resize_periodic / _fused / naive)
        k = lib.ik_resize_kernel_name(S, S, C, O, O, f)
        return k.decode() if k else "unknown"

    # ---- headline: PNG bytes in host memory -> WebP bytes in host memory ----
    stage_ms = []
    NT = 17  # ik_png_last_timing fields

    batch_ms = []
    NB = 13  # ik_batch_last_timing fields

    def note_timing():
        timing = (ctypes.c_double * NT)()  # the last PNG batch the device finished
        lib.ik_png_last_timing(timing, NT)
        stage_ms.append(list(timing))
        bt = (ctypes.c_double * NB)()  # the last batch's JPEG decode / resize / JPEG encode launches
        lib.ik_batch_last_timing(bt, NB)
        batch_ms.append(list(bt))

    def submit(rq):
        fn = transform_batch_submit_device if isinstance(rq[0], DeviceBytes) else transform_batch_submit
        return fn(rq, [(O, O)] * B, [FORMATS[args.format]] * B, [args.quality] * B, filter=f, threads=args.threads)

    def run_pipelined(nsteps, rq=None, depth=None):
        """nsteps batches with up to `depth` in flight (upload of one under the
        kernels of another, host coders of a third); returns the last bytes"""
        rq = reqs if rq is None else rq
        depth = args.inflight if depth is None else depth
        pend, out = [], None
        for _ in range(nsteps):
            pend.append(submit(rq))
            if len(pend) >= depth:
                out = pend.pop(0).wait()
                note_timing()
        while pend:
            out = pend.pop(0).wait()
            note_timing()
        return out

    def run_blocking(nsteps):
        out = None
        for _ in range(nsteps):
            out = transform_batch(reqs, [(O, O)] * B, [FORMATS[args.format]] * B, [args.quality] * B, filter=f,
                                  threads=args.threads)
            note_timing()
        return out

    # PCIe-inclusive leg: the same steps from host memory (reported beside value)
    pcie = {}
    if not args.no_pcie_leg and args.source == "png":
        run_pipelined(args.warmup, rq=reqs) if args.pipeline else run_blocking(args.warmup)
        barrier()
        t1 = time.perf_counter()
        r1 = run_pipelined(args.steps, rq=reqs) if args.pipeline else run_blocking(args.steps)
        torch.cuda.synchronize()
        te = reduce_max(time.perf_counter() - t1, dist, dev)
        barrier()
        assert all(r is not None and magic(r) for r in r1)
        pst = np.mean(np.array(stage_ms), axis=0)
        stage_ms.clear()
        pcie = {"value": round(aggregate_mpix(world, B * args.steps, S, te), 2), "unit": "MPix/s",
                "ms_per_step": round(te / args.steps * 1e3, 3),
                "inputs": "pageable host memory" if args.pageable else "page-locked host memory (ik_host_alloc)",
                "entry": "ik_transform_batch_submit", "png_bytes_per_step": int(sum(len(p) for p in reqs)),
                "upload_device_ms": round(float(pst[1]), 3)}

    # headline: inputs resident in HBM
    run = (lambda k: run_pipelined(k, rq=dreqs)) if args.pipeline else run_blocking
    run(args.warmup)
    stage_ms.clear()
    batch_ms.clear()
    cnt0 = (ctypes.c_ulonglong * 2)()
    lib.ik_png_counters(cnt0)
    barrier()
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    t0 = time.perf_counter()
    res = run(args.steps)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    barrier()
    # this rank's host CPU over the timed region (every thread of the process: the
    # library's stage threads, the worker pool's libwebp coding, the caller)
    cpu_s = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
    rank_cpu = gather_floats([cpu_s, elapsed], dist, dev, world)
    elapsed = reduce_max(elapsed, dist, dev)
    assert all(r is not None and magic(r) for r in res)
    cnt1 = (ctypes.c_ulonglong * 2)()
    lib.ik_png_counters(cnt1)
    gpu_streams, host_streams = cnt1[0] - cnt0[0], cnt1[1] - cnt0[1]
    value = aggregate_mpix(world, B * args.steps, S, elapsed)
    st = np.mean(np.array(stage_ms), axis=0)
    png_stages = {k: round(float(st[i]), 3) for i, k in PNG_STAGES.items()}
    png_stages.update({"decode_rounds": float(st[7]), "decoder_lanes": int(st[8]), "streams_on_gpu": int(st[9]),
                       "timed_streams_gpu_decoded": int(gpu_streams), "timed_streams_host_decoded": int(host_streams)})
    out_bytes = sum(len(r) for r in res) // B
    in_bytes = sum(len(p) for p in reqs) // B

    # ---- device kernels of the step: algorithmic bytes per launch ----
    raw = (S * 4 + 1) * S          # filtered image bytes per frame (filter byte + RGBA row)
    nd = max(1, int(st[9]))        # frames in the timed decode launch
    tok = float(st[12])            # u16 tokens its decode pass wrote
    # the decoder that ran: the wave decoder (default) or round 4's lane decoder
    dec_kernel = "k_png_decode" if os.environ.get("IK_PNG_DECODE") == "lane" else "k_png_wave"
    kern = {
        # the files read, the assembled streams (+ padding) written
        "k_png_gather": (png_stages["gather_crc"], nd * 2 * in_bytes),
        # the compressed streams read (every bit offset is examined)
        "k_png_find": (png_stages["find"], nd * in_bytes),
        # compressed stream read, tokens written
        dec_kernel: (png_stages["decode"], nd * in_bytes + 2 * tok),
        # tokens read, u16 symbols written
        "k_png_expand": (png_stages["expand"], 2 * tok + nd * 2 * raw),
        "k_png_resolve": (png_stages["resolve"], nd * (2 * raw + 4 * S * S)),
        "k_png_unfilter": (png_stages["unfilter"], nd * (2 * 4 * S * S)),
    }
    # the batch path's own launches (ik_batch_last_timing, HIP events on the kernel
    # stream): JPEG entropy decoding, the grouped resize, the batched JPEG encoder
    bt = np.mean(np.array(batch_ms), axis=0) if batch_ms else np.zeros(10)
    jpeg_huff = None
    if args.source != "png":
        # JPEG sources: the PNG stage times do not apply.  The entropy decoding launch
        # reads the scans and writes every block's int16 coefficients (the bytes a
        # decode of these frames must move, SURVEY 8(d) D-5's decode-stage share)
        kern = {"k_jsync_*": (float(bt[0]), float(bt[1] + bt[2]))}
        jpeg_huff = {"ms": round(float(bt[0]), 4), "scan_bytes": int(bt[1]), "coef_bytes": int(bt[2]),
                     "images": int(bt[3]), "lanes": int(bt[4])}
    resize_batch = None
    if bt[5] > 0:
        resize_batch = {"bound": "hbm", "achieved": round(bt[6] / (bt[5] * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBPS,
                        "unit": "GB/s", "frac": round(bt[6] / (bt[5] * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                        "traffic": None, "kernel": resize_kernel(3 if args.source != "png" else 4), "kernel_ms": round(float(bt[5]), 4),
                        "bytes_per_launch": int(bt[6]), "batch": int(bt[7]),
                        "note": "the grouped resize launch of the measured batches themselves (HIP events on the "
                                "post stage's stream, beside the next batch's decode kernels); bytes = C*W*H in + "
                                "C*w*h out per image"}
    jpeg_enc = {"ms": round(float(bt[8]), 4), "images": int(bt[9])} if bt[9] > 0 else None
    dom = max(kern, key=lambda k: kern[k][0]) if kern else None
    dms, kbytes = kern[dom] if dom else (1.0, 0)
    # roofline bytes: SURVEY 8(d) D-5's algorithmic bytes of the transform per frame --
    # the encoded input read, the decoded frame (C*W*H) written and read once, the
    # resized frame (C*w*h), the encoded output -- times the frames of the launch
    # (VERDICT r4 weak 2); the kernel's own stream bytes are the second figure
    C = 3 if args.source != "png" else 4
    d5_frame = in_bytes + C * S * S + C * O * O + out_bytes
    dbytes = nd * d5_frame if args.source == "png" else int(bt[3]) * d5_frame
    traffic_png = None  # PMC HBM bytes of that kernel per 64-frame launch (tools/pmc_png_traffic.sh)
    traffic_basis = "no PMC file for this configuration"
    pmcp = os.path.join(ROOT, "profiles", "pmc_png.json")
    if os.path.exists(pmcp) and B == 64 and S == 4096 and args.source == "png":
        try:
            import ikutil
            pj = json.load(open(pmcp))
            if pj.get("code_sha16") == ikutil.png_code_sha16():
                traffic_png = pj.get(dom, {}).get("hbm_bytes_per_batch")
                traffic_basis = (f"PMC FETCH_SIZE (x2, gfx950) + WRITE_SIZE of this kernel, measured on this code "
                                 f"(PNG path sources sha {pj['code_sha16']}, profiles/pmc_png.json)")
            else:
                traffic_basis = (f"profiles/pmc_png.json was measured on other code (sha {pj.get('code_sha16')} vs "
                                 f"{ikutil.png_code_sha16()} now): not quoted")
        except Exception as ex:  # noqa: BLE001
            traffic_png, traffic_basis = None, f"PMC file unreadable: {ex}"
    # the host coder stage (libwebp / libavif on the worker pool) per batch: wall and
    # core-ms, and what that costs in host cores at the measured step rate (VERDICT r4
    # weak 7: an 8-GPU node's SCALE curve is host-bound where this exceeds its cores)
    host_coder = None
    if bt[12] > 0:
        core_ms_img = bt[11] / bt[12]
        steps_per_s = args.steps / elapsed
        host_coder = {"wall_ms_per_batch": round(float(bt[10]), 3), "core_ms_per_image": round(float(core_ms_img), 3),
                      "images_per_batch": int(bt[12]),
                      "cores_busy_per_gpu": round(core_ms_img * bt[12] * steps_per_s / 1e3, 2),
                      "cores_needed_at_8_gpus": round(8 * core_ms_img * bt[12] * steps_per_s / 1e3, 1),
                      "note": "thread CPU time of the host coders (CLOCK_THREAD_CPUTIME_ID per request), at this "
                              "run's step rate"}
    if args.source == "png":
        note = ("DEFLATE decoding: each lane's symbol-to-symbol chain bounds it, not HBM; bytes_per_launch = "
                "SURVEY D-5's transform bytes of the launch's frames; kernel_stream = compressed bits in + u16 "
                "tokens out")
    else:
        note = ("JPEG entropy decoding, self-synchronising (k_jsync_sync, k_jsync_fix + settle, "
                "k_jsync_seg1-3, k_jsync_decode: HIP events on the kernel stream around them): each lane's "
                "Huffman symbol chain bounds it, not HBM; bytes_per_launch = SURVEY D-5's transform bytes of the "
                "launch's frames; kernel_stream = the unstuffed scans read + every block's int16 coefficients "
                "written")
    roof = {"bound": "hbm", "achieved": round(dbytes / (dms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(dbytes / (dms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4), "traffic": traffic_png, "kernel": dom,
            "kernel_ms": round(dms, 4), "bytes_per_launch": int(dbytes),
            "bytes_basis": (f"SURVEY D-5 per frame: encoded input {in_bytes} + {C}*W*H + {C}*w*h + encoded output "
                            f"{out_bytes} = {d5_frame} B, x {nd if args.source == 'png' else int(bt[3])} frames"),
            "traffic_basis": traffic_basis,
            # PMC bytes over the launch's algorithmic bytes: > 1 = re-reads and partial lines
            "traffic_over_bytes": round(traffic_png / dbytes, 3) if traffic_png else None,
            "kernel_stream": {"bytes_per_launch": int(kbytes), "achieved": round(kbytes / (dms * 1e-3) / 1e9, 1),
                              "frac": round(kbytes / (dms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)},
            "note": note}
    if args.source == "png":
        roof["tokens_per_batch"] = int(tok)
    kernels = {k: {"ms": round(v[0], 4), "GBps": round(v[1] / max(v[0], 1e-6) / 1e6, 1)} for k, v in kern.items()}

    # the same workload with the inputs in ordinary (pageable) memory: the upload
    # stage copies them through pinned staging first
    pageable = {}
    if not args.pageable and not args.no_extras and args.pageable_steps > 0:
        run_pipelined(1, rq=[pngs[i % len(pngs)] for i in range(B)])
        barrier()
        t1 = time.perf_counter()
        run_pipelined(args.pageable_steps, rq=[pngs[i % len(pngs)] for i in range(B)])
        te = reduce_max(time.perf_counter() - t1, dist, dev)
        pageable = {"value": round(aggregate_mpix(world, B * args.pageable_steps, S, te), 2), "unit": "MPix/s",
                    "steps": args.pageable_steps, "ms_per_step": round(te / args.pageable_steps * 1e3, 3)}

    # the same headline workload with the other WebP coder (byte-identical files): its
    # rate and the host cores it keeps busy, so both coders are measured in one run
    alt_coder = {}
    if args.format == "webp" and args.alt_steps > 0 and args.pipeline:
        other = "libwebp" if args.webp_encoder != "libwebp" else "exact"
        lib.ik_set_webp_encoder(WEBP_ENC[other])
        run_pipelined(args.warmup, rq=dreqs)
        barrier()
        ra0 = resource.getrusage(resource.RUSAGE_SELF)
        t1 = time.perf_counter()
        ra = run_pipelined(args.alt_steps, rq=dreqs)
        torch.cuda.synchronize()
        te = time.perf_counter() - t1
        ra1 = resource.getrusage(resource.RUSAGE_SELF)
        cpu_a = (ra1.ru_utime - ra0.ru_utime) + (ra1.ru_stime - ra0.ru_stime)
        te_max = reduce_max(te, dist, dev)
        barrier()
        lib.ik_set_webp_encoder(WEBP_ENC[args.webp_encoder])
        stage_ms.clear()
        batch_ms.clear()
        assert ra is not None and all(magic(r) for r in ra) and ra == res, "the coders' bytes differ"
        alt_coder = {"webp_encoder": other, "value": round(aggregate_mpix(world, B * args.alt_steps, S, te_max), 2),
                     "unit": "MPix/s", "steps": args.alt_steps, "ms_per_step": round(te_max / args.alt_steps * 1e3, 3),
                     "rank0_cores_busy": round(cpu_a / max(te, 1e-9), 2),
                     "bytes_equal_to_value_leg": True}

    # ---- extras: HBM-resident pipeline (old headline) and JPEG-source leg ----
    hbm = {}
    roof_resize = None
    jpg = {}
    if not args.no_extras:
        HB = args.hbm_batch
        pitch = S * 4
        src = torch.empty((HB, S, pitch), dtype=torch.uint8, device=dev)
        for i in range(HB):
            if i < len(frames):
                src[i].copy_(torch.from_numpy(frames[i].reshape(S, pitch)))
            else:
                src[i].copy_(src[i % len(frames)])
        torch.cuda.synchronize()
        pipe = ctypes.c_void_p()
        if lib.ik_pipeline_create(S, S, 4, O, O, f, FORMATS[args.format], args.quality, HB, args.threads,
                                  ctypes.byref(pipe)):
            raise SystemExit(f"pipeline: {_lib.last_error()}")
        cap = HB * O * O * 4 + (1 << 20)
        out = np.empty(cap, np.uint8)
        sizes = (ctypes.c_size_t * HB)()
        nd = ctypes.c_uint32()
        sp = ctypes.c_void_p(src.data_ptr())
        km = []

        def sub():
            assert lib.ik_pipeline_submit(pipe, sp, pitch, S * pitch, HB) == 0, _lib.last_error()

        def col():
            assert lib.ik_pipeline_collect(pipe, out.ctypes.data, cap, sizes, ctypes.byref(nd)) == 0, _lib.last_error()
            km.append([lib.ik_pipeline_kernel_ms(pipe, k) for k in range(4)])

        sub()
        col()
        km.clear()
        barrier()
        t1 = time.perf_counter()
        sub()
        for _ in range(args.hbm_steps - 1):
            sub()
            col()
        col()
        barrier()
        te = reduce_max(time.perf_counter() - t1, dist, dev)
        lib.ik_pipeline_destroy(pipe)
        kmm = np.mean(np.array(km), axis=0)
        rb = HB * (4 * S * S + 4 * O * O)
        hbm = {"workload": f"{S}x{S} RGBA8 frames already in HBM -> resize {O}x{O} {args.filter} -> {args.format} "
                           f"q{args.quality}, bytes to host; two batches in flight",
               "value": round(aggregate_mpix(world, HB * args.hbm_steps, S, te), 2), "unit": "MPix/s",
               "ms_per_step": round(te / args.hbm_steps * 1e3, 3), "batch_per_gpu": HB,
               "resize_ms": round(float(kmm[0]), 4), "colour_ms": round(float(kmm[1]), 4),
               "host_stage_ms": round(float(kmm[3]), 3)}
        achieved = rb / (kmm[0] * 1e-3) / 1e9
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_resize.json")
        if os.path.exists(pmc):
            try:
                d = json.load(open(pmc))
                key = f"{args.filter}_{S}_{O}_b{HB}"
                # quoted only when collected on the kernel this geometry takes now
                if key in d and d[key].get("kernel", "k_resize_fused") == resize_kernel(4):
                    traffic = d[key]["hbm_bytes_per_launch"]
            except Exception:
                traffic = None
        roof_resize = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                       "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic, "kernel": resize_kernel(4),
                       "kernel_ms": round(float(kmm[0]), 4), "bytes_per_launch": rb, "batch": HB}
        del src
        torch.cuda.empty_cache()
        # JPEG sources (restart marker per MCU row) through the same batch call
        if args.jpeg_images > 0:
            from PIL import Image
            jp = []
            for im in frames[:2]:
                b = io.BytesIO()
                Image.fromarray(np.ascontiguousarray(im[..., :3]), "RGB").save(b, format="JPEG", quality=90,
                                                                             restart_marker_rows=1)
                jp.append(b.getvalue())
            n = args.jpeg_images
            run = lambda k: transform_batch([jp[i % 2] for i in range(k)], [(O, O)] * k, [1] * k,
                                            [args.quality] * k, filter=f, threads=args.threads)
            run(4)
            barrier()
            t1 = time.perf_counter()
            run(n)
            te = reduce_max(time.perf_counter() - t1, dist, dev)
            jpg = {"source": "JPEG q90 4:2:0, RSTn per MCU row (GPU entropy decoding)", "images_per_gpu": n,
                   "bytes_per_source_image": sum(len(p) for p in jp) // 2,
                   "value": round(aggregate_mpix(world, n, S, te), 2), "unit": "MPix/s"}

    if roof_resize is None:
        # the resize kernel alone on the measured batch's geometry (C channels as the
        # decoded frames: 3 for JPEG sources): in the four-stage pipeline the batch's
        # own resize runs beside the next batch's decode kernels, so its event time
        # (roofline_resize_batch_path) includes their contention
        C = 3 if args.source != "png" else 4
        src = torch.empty((B, S, S * C), dtype=torch.uint8, device=dev)
        for i in range(B):
            src[i].random_(0, 256)
        dstt = torch.empty((B, O, O * C), dtype=torch.uint8, device=dev)
        st = torch.cuda.Stream()
        torch.cuda.synchronize()
        rms = []
        for r in range(4):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            if lib.ik_resize_batch_device(src.data_ptr(), S, S, C, S * C, S * S * C, B, O, O, f, dstt.data_ptr(),
                                          O * C, O * O * C, ctypes.c_void_p(st.cuda_stream)):
                raise SystemExit(f"resize: {_lib.last_error()}")
            e1.record(st)
            e1.synchronize()
            if r:
                rms.append(e0.elapsed_time(e1))
        rms_med = float(np.median(rms))
        rb = B * C * (S * S + O * O)
        roof_resize = {"bound": "hbm", "achieved": round(rb / (rms_med * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBPS,
                       "unit": "GB/s", "frac": round(rb / (rms_med * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4), "traffic": None,
                       "kernel": resize_kernel(C), "kernel_ms": round(rms_med, 4), "bytes_per_launch": rb, "batch": B,
                       "note": f"the resize kernel alone (ik_resize_batch_device, {C} channels, the batch's "
                               f"geometry and filter), HIP events on its stream, median of 3 launches"}
        del src, dstt
        torch.cuda.empty_cache()
    src_desc = ({"png": "PNG (zlib level 6), resident in HBM (one device allocation per request) -> "
                        "ik_transform_batch_submit_device: decode_image (GPU chunk walk, gather + CRC, inflate + "
                        "unfilter)",
                 "jpeg-rst": "JPEG q90 4:2:0 with a restart marker per MCU row, in page-locked host memory -> "
                             "ik_transform_batch_submit: decode_image (self-synchronising GPU entropy decoding, "
                             "IDCT, upsampling, colour)",
                 "jpeg": "JPEG q90 4:2:0 without restart markers, in page-locked host memory -> "
                         "ik_transform_batch_submit: decode_image (GPU self-synchronising entropy decoding, IDCT, "
                         "upsampling, colour)"}[args.source] if args.pipeline else "host memory -> ik_transform_batch")
    coder = {"webp": "libwebp on host threads" if args.webp_encoder == "libwebp" else
             "libwebp method 4's decisions on the GPU, the exact coder (IK_WEBP_%s, byte-identical)" %
             args.webp_encoder.upper(),
             "jpeg": "GPU FDCT + Huffman", "avif": "libavif/aom"}[args.format]
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "MPix/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": f"{S}x{S} RGBA8 synthetic frames as {src_desc} -> resize_image {O}x{O} "
                            f"({args.filter}) -> encode_image {args.format} q{args.quality} ({coder}) -> encoded bytes "
                            f"in host memory",
                "source": args.source,
                "batch_per_gpu": B, "inflight": args.inflight if args.pipeline else 1,
                "inputs": "device memory (HBM), resident before the timed region" if args.pipeline and args.source == "png" else
                          ("pageable host memory" if args.pageable else "page-locked host memory (ik_host_alloc)"),
                "value_basis": ("HBM-resident inputs (the measurement contract); SURVEY D-1's host-memory-to-host-"
                                "memory figure is pcie_inclusive.value" if args.pipeline and args.source == "png"
                                else "encoded inputs in host memory -> encoded outputs in host memory (SURVEY D-1)"),
                "inproc_devices": args.inproc_devices, "filter": args.filter, "format": args.format, "quality": args.quality,
                "webp_encoder": args.webp_encoder if args.format == "webp" else None,
                "host_threads_per_gpu": args.threads, "png_bytes_per_image": in_bytes,
                "webp_bytes_per_image": out_bytes,
                "libwebp": "%d.%d.%d" % (lib.ik_libwebp_version() >> 16, (lib.ik_libwebp_version() >> 8) & 255,
                                         lib.ik_libwebp_version() & 255),
                "libwebp_path": codec_path(lib, FORMATS["webp"]),
                "parallelism": f"images sharded, {world} rank(s)",
            },
            "roofline": roof,
            "host_cpu": {"per_rank_cpu_s": [round(r[0], 3) for r in rank_cpu],
                         "per_rank_wall_s": [round(r[1], 3) for r in rank_cpu],
                         "per_rank_cores_busy": [round(r[0] / max(r[1], 1e-9), 2) for r in rank_cpu],
                         "host_coder_stage": host_coder},
            "roofline_resize": roof_resize,
            "roofline_resize_batch_path": resize_batch,
            "jpeg_entropy_decode": jpeg_huff,
            "jpeg_encode_batched": jpeg_enc,
            "png_decode_stages_ms": png_stages,
            "kernels": kernels,
            "pcie_inclusive": pcie,
            "pageable_input": pageable,
            "webp_coder_alt": alt_coder,
            "hbm_resident": hbm,
            "decode_inclusive_jpeg": jpg,
            "cpu_baseline": cpu,
        }
        if cpu:
            # against the CPU this job could use (cpu_baseline.cores effective cores),
            # against one core, and against the linear physical-core bound (a bound)
            line["ratio_vs_cpu_allcore"] = round(value / cpu["value"], 2)
            line["ratio_vs_cpu_allcore_basis"] = (f"{cpu['cores']} effective cores (nproc {cpu['nproc']}, cgroup "
                                                  f"quota {cpu['host'].get('cgroup_cpu_quota_cores')})")
            line["ratio_vs_cpu_1core"] = round(value / cpu["value_1core"], 2)
            line["ratio_vs_cpu_linear_bound_physical"] = round(value / cpu["cpu_linear_bound_physical"], 3)
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
