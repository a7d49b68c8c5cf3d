"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs into per-launch HBM bytes of the
fused resize kernel (profiles/pmc_resize.json), with the read counter calibrated
on tools/bw_probe.hip pattern 0 (the same 8-byte-lane strip reads, known byte
count) as MI355X_MICROARCH.md's HBM section prescribes.

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR CALIB_DIR KEY BATCH S O [FIRST COUNT]
(FIRST/COUNT select the dispatches of one configuration, e.g. bench.py's main filter
 = the first warmup+steps launches, its alt filter = the rest).  IK_PMC_KERNEL names the
kernel (default k_resize_fused; k_resize_periodic for integer ratios); it is recorded.
"""
import csv, json, os, sys


def per_dispatch(d, counter, name, first=0, count=None):
    f = os.path.join(d, "run_counter_collection.csv")
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
            if r["Counter_Name"] == counter and name in r["Kernel_Name"]]
    vals = vals[first:first + count] if count else vals[first:]
    return sum(vals) / len(vals), len(vals)


def main():
    fdir, wdir, cdir, key, B, S, O = sys.argv[1:8]
    first, count = (int(sys.argv[8]), int(sys.argv[9])) if len(sys.argv) > 9 else (0, None)
    B, S, O = int(B), int(S), int(O)
    kname = os.environ.get("IK_PMC_KERNEL", "k_resize_fused")
    fetch_kb, nf = per_dispatch(fdir, "FETCH_SIZE", kname, first, count)
    write_kb, nw = per_dispatch(wdir, "WRITE_SIZE", kname, first, count)
    cal_kb, nc = per_dispatch(cdir, "FETCH_SIZE", "k_strip")
    known = 32 * 4096 * 4096 * 4  # tools/bw_probe.py: 32 images of 4096^2 RGBA8 (fixed), each byte read once
    calib = known / (cal_kb * 1024.0)
    fetch = fetch_kb * 1024.0 * calib
    write = write_kb * 1024.0
    algo = B * (4 * S * S + 4 * O * O)
    out_path = os.environ.get("IK_PMC_OUT") or os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_resize.json")
    d = json.load(open(out_path)) if os.path.exists(out_path) else {}
    d[key] = {
        "kernel": kname,
        "hbm_bytes_per_launch": int(fetch + write),
        "fetch_bytes_corrected": int(fetch), "write_bytes": int(write),
        "fetch_size_kb_raw": fetch_kb, "write_size_kb_raw": write_kb,
        "fetch_calibration_factor": calib, "calibration": "tools/bw_probe.hip pattern 0, 8 B/lane strip reads, known bytes",
        "algorithmic_bytes_per_launch": algo, "traffic_over_algorithmic": (fetch + write) / algo,
        "dispatches": {"fetch": nf, "write": nw, "calib": nc},
    }
    json.dump(d, open(out_path, "w"), indent=1)
    print(json.dumps(d[key], indent=1))


if __name__ == "__main__":
    main()
