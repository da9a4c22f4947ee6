"""Per-kernel rocprofv3 counter summaries joined with kernel-trace durations (round 5).

    python tools/pmc_r5_summary.py mfma  <pmc_dir> <trace_dir> --json profiles/r05_mfma_busy.json
    python tools/pmc_r5_summary.py hbm   <fetch_dir> <write_dir> <trace_dir> --json profiles/r05_b128_f32_pmc.json
    python tools/pmc_r5_summary.py stall <pass_dir> [<pass_dir> ...] <trace_dir> --json profiles/r05_stalls.json

mfma: SQ_VALU_MFMA_BUSY_CYCLES (cycles an MFMA occupies its SIMD, summed over SIMDs: 32 per
v_mfma_f32_32x32x16_bf16, 16 per 16x16x32, MI355X_MICROARCH.md cycle-constants table) per dispatch
over the SIMD-cycles of the dispatch's duration in the plan-mode kernel trace at the 2.4 GHz peak
clock x 1024 SIMDs: a lower bound of the MFMA-busy fraction (the chip holds a lower clock under
load).  GRBM_GUI_ACTIVE is reported but not used as the denominator: it reads high on dispatches
shorter than ~0.3 ms (MI355X_MICROARCH.md, DVFS item).

hbm: FETCH_SIZE x 2 (gfx950 reports half the bytes of 16 B/lane reads) + WRITE_SIZE, KB = 1024 B,
per dispatch (separate passes, eager bench steps), over the kernel's mean duration in the plan-mode
trace of the same workload: achieved GB/s and the fraction of 8 TB/s.  Infinity-Cache hits are
counted in FETCH_SIZE (MI355X_MICROARCH.md HBM section), so this is traffic leaving L2, an upper
bound of HBM bytes.
"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics

CLOCK_HZ = 2.4e9
SIMDS = 256 * 4
HBM_PEAK_GBS = 8000.0


def short(name):
    n = name.split("(")[0]
    return n[5:] if n.startswith("void ") else n


def counters(d):
    per = collections.defaultdict(lambda: collections.defaultdict(list))  # (kernel, grid) -> counter -> values
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            per[(short(r["Kernel_Name"]), int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


def durations(d):
    per = collections.defaultdict(list)  # (kernel, grid) -> us
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            per[(short(r["Kernel_Name"]), g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return per


def mfma(a):
    pmc, dur = counters(a.dirs[0]), durations(a.dirs[1])
    out = []
    for key, cs in sorted(pmc.items()):
        busy = statistics.median(cs.get("SQ_VALU_MFMA_BUSY_CYCLES", [0.0]))
        if busy <= 0:
            continue
        n_mfma = statistics.median(cs.get("SQ_INSTS_MFMA", [0.0]))
        us = statistics.mean(dur[key]) if key in dur else None
        rec = {"kernel": key[0], "grid": key[1], "dispatches": len(cs["SQ_VALU_MFMA_BUSY_CYCLES"]),
               "mfma_busy_cycles": busy, "mfma_insts": n_mfma,
               "busy_cycles_per_mfma": round(busy / n_mfma, 2) if n_mfma else None,
               "sq_busy_cycles": statistics.median(cs.get("SQ_BUSY_CYCLES", [0.0])),
               "grbm_gui_active": statistics.median(cs.get("GRBM_GUI_ACTIVE", [0.0])),
               "trace_us": round(us, 2) if us else None,
               "mfma_busy_frac": round(busy / (us * 1e-6 * CLOCK_HZ * SIMDS), 4) if us else None}
        out.append(rec)
    out.sort(key=lambda r: -(r["trace_us"] or 0) * (dur and len(dur.get((r["kernel"], r["grid"]), [])) or 1))
    for r in out:
        print(f"{r['kernel'][:40]:40s} g{r['grid']:8d} {r['trace_us'] or 0:7.2f} us  MFMA busy {r['mfma_busy_frac'] or 0:.3f}"
              f"  ({r['busy_cycles_per_mfma']} cyc/MFMA)")
    return {"source": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE "
                      "GRBM_COUNT over eager bench steps (64^3 B=4 bf16); durations: plan-mode kernel trace of the bench",
            "mfma_busy_frac": "SQ_VALU_MFMA_BUSY_CYCLES / (trace duration x 2.4 GHz x 1024 SIMDs): lower bound",
            "kernels": out}


def hbm(a):
    f, w, dur = counters(a.dirs[0]), counters(a.dirs[1]), durations(a.dirs[2])
    out = []
    for key in sorted(set(f) | set(w)):
        fk = statistics.mean(f[key]["FETCH_SIZE"]) if key in f and "FETCH_SIZE" in f[key] else 0.0
        wk = statistics.mean(w[key]["WRITE_SIZE"]) if key in w and "WRITE_SIZE" in w[key] else 0.0
        b = (2 * fk + wk) * 1024
        us = statistics.mean(dur[key]) if key in dur else None
        launches = len(dur.get(key, []))
        rec = {"kernel": key[0], "grid": key[1], "fetch_kb_raw": round(fk, 1), "write_kb": round(wk, 1),
               "bytes_per_launch": int(b), "trace_us": round(us, 2) if us else None,
               "launches_in_trace": launches,
               "gbs": round(b / (us * 1e-6) / 1e9, 1) if us else None,
               "hbm_frac": round(b / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4) if us else None}
        out.append(rec)
    out.sort(key=lambda r: -(r["trace_us"] or 0) * max(r["launches_in_trace"], 1))
    for r in out[:40]:
        print(f"{r['kernel'][:44]:44s} g{r['grid']:8d} {r['bytes_per_launch'] / 1e6:8.2f} MB {r['trace_us'] or 0:8.2f} us "
              f"{r['gbs'] or 0:8.1f} GB/s ({r['hbm_frac'] or 0:.3f})")
    return {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes, eager bench steps) of bench.py "
                      "--size 128 --batch 1 --precision f32; durations: the plan-mode kernel trace of the same command",
            "correction": "FETCH_SIZE x 2 (gfx950, MI355X_MICROARCH.md HBM section), KB = 1024 B; Infinity-Cache hits "
                          "are counted (bytes leaving L2: an upper bound of HBM bytes)",
            "peak_gbs": HBM_PEAK_GBS, "kernels": out}


def stall(a):
    """Per-kernel instruction mix and wait fractions from several SQ passes: per dispatch medians,
    ratios of counters in the same units (wave-cycles for SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_*)."""
    per = collections.defaultdict(dict)
    for d in a.dirs[:-1]:
        for key, cs in counters(d).items():
            for c, v in cs.items():
                per[key][c] = statistics.median(v)
    dur = durations(a.dirs[-1])
    out = []
    for key, c in per.items():
        g = lambda n: c.get(n, 0.0)
        wc = g("SQ_WAVE_CYCLES")
        mf = g("SQ_INSTS_MFMA")
        us = statistics.mean(dur[key]) if key in dur else None
        rec = {"kernel": key[0], "grid": key[1], "trace_us": round(us, 2) if us else None,
               "launches_in_trace": len(dur.get(key, [])),
               "valu_per_mfma": round(g("SQ_INSTS_VALU") / mf, 2) if mf else None,
               "lds_per_mfma": round(g("SQ_INSTS_LDS") / mf, 2) if mf else None,
               "vmem_rd_per_mfma": round(g("SQ_INSTS_VMEM_RD") / mf, 2) if mf else None,
               "salu_per_mfma": round(g("SQ_INSTS_SALU") / mf, 2) if mf else None,
               "lds_conflict_frac": round(g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE"), 3) if g("SQ_LDS_IDX_ACTIVE") else None}
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                      "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_ANY"):
                if n in c:
                    rec[n[3:].lower() + "_frac"] = round(c[n] / wc, 3)
        rec["raw"] = {k: c[k] for k in sorted(c)}
        out.append(rec)
    out.sort(key=lambda r: -(r["trace_us"] or 0) * max(r["launches_in_trace"], 1))
    for r in out[:45]:
        print(f"{r['kernel'][:38]:38s} g{r['grid']:8d} {r['trace_us'] or 0:6.1f}us valu/mfma {r['valu_per_mfma']} "
              f"lds/mfma {r['lds_per_mfma']} vmem/mfma {r['vmem_rd_per_mfma']} confl {r['lds_conflict_frac']} "
              f"wait {r.get('wait_any_frac')} winst {r.get('wait_inst_any_frac')} wlds {r.get('wait_inst_lds_frac')} "
              f"valu {r.get('active_inst_valu_frac')} lds {r.get('active_inst_lds_frac')} vmem {r.get('active_inst_vmem_frac')}")
    return {"source": "rocprofv3 --pmc passes (8 SQ counters each) over eager bench steps (64^3 B=4 bf16); durations: "
                      "plan-mode kernel trace", "kernels": out}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["mfma", "hbm", "stall"])
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--json")
    a = ap.parse_args()
    res = {"mfma": mfma, "hbm": hbm, "stall": stall}[a.what](a)
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
