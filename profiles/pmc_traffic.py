"""Turn rocprofv3 PMC passes into per-kernel HBM bytes per launch.

    python profiles/pmc_traffic.py FETCH_DIR WRITE_DIR [out.json]

FETCH_DIR / WRITE_DIR hold the csv output of
    rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv ...
    rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv ...
(separate passes: FETCH_SIZE and WRITE_SIZE do not fit one TCC pass).
Corrections (MI355X_MICROARCH.md, HBM): FETCH_SIZE is in KiB and on gfx950
reports half the bytes of a 16-B/lane streaming read, so it is doubled;
WRITE_SIZE (KiB) is exact for 16-B/lane streaming stores.  Infinity-Cache hits
are counted by these memory-side counters, not excluded.
"""
import csv
import glob
import hashlib
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL_SOURCES = ["gpu-gmres_amd/csrc/kernels.hip", "gpu-gmres_amd/csrc/solver.hip",
                  "gpu-gmres_amd/csrc/kernels.h", "gpu-gmres_amd/csrc/gg_internal.h"]


def src_sha():
    """sha256 (16 hex digits) over the kernel sources, in a fixed order"""
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        with open(os.path.join(REPO, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def short(name):
    """'void gg::(anonymous namespace)::k_trsv_wave2d<false, 2, false>(gg::Gate, ...)'
    -> 'k_trsv_wave2d<false, 2, false>'"""
    name = re.sub(r"^void ", "", name.strip())
    name = name.split("(gg::")[0] if "(gg::" in name else name
    m = re.search(r"(k_[A-Za-z0-9_]+(<[^()]*>)?)", name)
    return m.group(1) if m else name


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                k = short(row["Kernel_Name"])
                v = float(row["Counter_Value"])
                key = row.get("Dispatch_Id") or row.get("Correlation_Id")
                e = acc.setdefault(k, {})
                e[key] = e.get(key, 0.0) + v          # sum over XCD / shader-engine instances
    # a launch whose gate was closed (the solve converged while later launches
    # of its chunk were already enqueued) reads its control block and returns:
    # its dispatches are dropped from the average (below 1 % of the kernel's
    # largest dispatch), counted in "gated"
    out = {}
    for k, e in acc.items():
        vals = list(e.values())
        hi = max(vals)
        keep = [v for v in vals if v >= 0.01 * hi] if hi > 64.0 else vals
        out[k] = (sum(keep) / len(keep), len(keep), len(vals) - len(keep))
    return out


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), "pmc_traffic.json")
    fetch = per_kernel(fdir, "FETCH_SIZE")
    write = per_kernel(wdir, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        fk, fn, fg = fetch.get(k, (0.0, 0, 0))
        wk, wn, wg = write.get(k, (0.0, 0, 0))
        rd = 2.0 * fk * 1024.0
        wr = wk * 1024.0
        res[k] = {"fetch_kib_raw": round(fk, 3), "write_kib_raw": round(wk, 3),
                  "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                  "hbm_bytes_per_launch": rd + wr, "dispatches": [fn, wn], "gated": [fg, wg]}
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE --kernel-trace (separate passes)",
           "correction": "read = 2 x FETCH_SIZE KiB (gfx950 16-B/lane streaming reads); write = WRITE_SIZE KiB",
           # the kernel sources these counters were taken on: bench.py drops the
           # traffic figure when the sources have changed since (stale counters)
           "src_sha": src_sha(),
           "kernels": res}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    for k, v in res.items():
        print(f"{k:45s} read {v['read_bytes_per_launch']/1e6:9.3f} MB  write {v['write_bytes_per_launch']/1e6:9.3f} MB")


if __name__ == "__main__":
    main()
