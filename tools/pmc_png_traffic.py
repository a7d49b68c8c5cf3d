"""Per-launch HBM bytes of the PNG decode kernels from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
runs of bench.py (tools/pmc_png_traffic.sh).  FETCH_SIZE is doubled (MI355X_MICROARCH.md: on
gfx950 it reports half the bytes of a wide streaming read); the factor measured on
tools/bw_probe.hip pattern 0 (known byte count) is recorded beside it.  WRITE_SIZE is taken
as is (exact for 16-B-per-lane streaming stores, the token / symbol / row stores here).

usage: python tools/pmc_png_traffic.py FETCH_DIR WRITE_DIR CALIB_DIR OUT_JSON
"""
import csv, json, os, subprocess, sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import ikutil  # noqa: E402  (png_code_sha16: the code the counters were measured on)

KERNELS = ["k_png_decode", "k_png_expand", "k_png_resolve", "k_png_unfilter", "k_png_find", "k_png_wave"]


def per_kernel(d, counter):
    """kernel -> (sum over its dispatches of the counter (KB), dispatches)"""
    tot, n = {}, {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if r["Counter_Name"] != counter:
            continue
        for k in KERNELS + ["k_strip"]:
            if k in r["Kernel_Name"]:
                tot[k] = tot.get(k, 0.0) + float(r["Counter_Value"])
                n[k] = n.get(k, 0) + 1
    return tot, n


def main():
    fdir, wdir, cdir, out = sys.argv[1:5]
    f, nf = per_kernel(fdir, "FETCH_SIZE")
    w, nw = per_kernel(wdir, "WRITE_SIZE")
    c, nc = per_kernel(cdir, "FETCH_SIZE")
    known = 32 * 4096 * 4096 * 4  # tools/bw_probe.py pattern 0: each byte of 32 x 4096^2 RGBA8 read once
    calib = known / (c["k_strip"] / nc["k_strip"] * 1024.0) if c.get("k_strip") else None
    res = {"note": "per 64-frame batch (bench.py headline; counter sums over the run's dispatches / dispatch "
                   "count); fetch doubled per MI355X_MICROARCH.md (gfx950 FETCH_SIZE = half of a streaming "
                   "read), confirmed by the bw_probe calibration factor (known bytes / FETCH_SIZE bytes)",
           "bw_probe_fetch_factor": calib,
           "code_sha16": ikutil.png_code_sha16()}
    try:
        res["git_head"] = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], capture_output=True,
                                         text=True).stdout.strip() or None
    except OSError:
        res["git_head"] = None
    for k in KERNELS:
        if k not in f or k not in w:
            continue
        # one dispatch per kernel per batch (round 3: k_png_find too); the run may hold
        # more than one batch, so the sums are divided by the dispatch count
        fetch = f[k] * 1024.0 * 2.0 / nf[k]
        write = w[k] * 1024.0 / nw[k]
        res[k] = {"hbm_bytes_per_batch": int(fetch + write), "fetch_bytes_corrected": int(fetch),
                  "write_bytes": int(write), "fetch_size_kb_raw_total": f[k], "write_size_kb_raw_total": w[k],
                  "dispatches": nf[k]}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
