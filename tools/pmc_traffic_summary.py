"""HBM bytes per launch of one kernel from separate FETCH_SIZE / WRITE_SIZE passes (tools/gpu_pmc.sh).

    python tools/pmc_traffic_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write --json out.json

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of a
16 B/lane streaming read, so it is doubled; WRITE_SIZE is taken as is; KB = 1024 B.  The figure per
launch is the launch-weighted mean over the kernel's roles (template instances)."""
import argparse
import collections
import csv
import glob
import json
import os


def _sums(d, counter):
    per = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].split("(")[0]
            per[k] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    return per, {k: len(v) for k, v in disp.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--json")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--algorithmic", type=float, default=None, help="algorithmic bytes per launch")
    a = ap.parse_args()
    fs, fn = _sums(a.fetch_dir, "FETCH_SIZE")
    ws, wn = _sums(a.write_dir, "WRITE_SIZE")
    roles, tot, n_all = {}, 0.0, 0
    for k in sorted(fs):
        n = fn[k]
        fkb, wkb = fs[k] / n, ws.get(k, 0.0) / max(wn.get(k, 1), 1)
        b = 2 * fkb * 1024 + wkb * 1024
        roles[k] = {"launches": n, "fetch_size_kb_raw": round(fkb, 1), "write_size_kb": round(wkb, 1),
                    "hbm_bytes_per_launch": int(b)}
        tot += b * n
        n_all += n
        print(f"{k}: x{n} FETCH {fkb:.1f} KB (x2) WRITE {wkb:.1f} KB -> {b / 1e6:.2f} MB/launch")
    out = {"kernel": a.kernel, "units": "bytes per launch",
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), tools/gpu_pmc.sh",
           "correction": "FETCH_SIZE x2 (gfx950 reports half the bytes of 16 B/lane reads, MI355X_MICROARCH.md "
                         "HBM section); KB = 1024 B; Infinity-Cache hits are counted",
           "roles": roles, "hbm_bytes_per_launch": int(tot / max(n_all, 1))}
    if a.algorithmic:
        out["algorithmic_bytes_per_launch"] = a.algorithmic
        out["traffic_over_algorithmic"] = round(out["hbm_bytes_per_launch"] / a.algorithmic, 3)
    print("mean", out["hbm_bytes_per_launch"] / 1e6, "MB/launch")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
