"""Per-kernel summary of an SQ-counter pass (tools/gpu_pmc_sq_step.sh): instructions per dispatch
(VALU / MFMA / VMEM / LDS), VALU per MFMA, and the share of wave cycles spent waiting.

    python tools/pmc_sq_summary.py gpurun_out/pmc_sq_step/run_counter_collection.csv [--json out.json]
"""
import argparse
import collections
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--json")
    a = ap.parse_args()
    per = collections.defaultdict(lambda: collections.defaultdict(float))  # (kernel, grid) -> counter sums
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(a.csv)):
        key = (r["Kernel_Name"].split("(")[0], int(r["Grid_Size"]))
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[key].add(r["Dispatch_Id"])
    out = []
    for (k, grid), c in sorted(per.items()):
        n = len(disp[(k, grid)])
        mfma = c["SQ_INSTS_MFMA"] / n
        rec = {"kernel": k, "grid": grid, "dispatches": n,
               "valu_per_dispatch": c["SQ_INSTS_VALU"] / n, "mfma_per_dispatch": mfma,
               "vmem_per_dispatch": c["SQ_INSTS_VMEM"] / n, "lds_per_dispatch": c["SQ_INSTS_LDS"] / n,
               "valu_per_mfma": c["SQ_INSTS_VALU"] / c["SQ_INSTS_MFMA"] if c["SQ_INSTS_MFMA"] else None,
               "wait_frac": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"] if c["SQ_WAVE_CYCLES"] else None,
               "wait_inst_frac": c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"] if c["SQ_WAVE_CYCLES"] else None,
               "active_inst_frac": c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"] if c["SQ_WAVE_CYCLES"] else None}
        out.append(rec)
        vpm = f"{rec['valu_per_mfma']:.1f}" if rec["valu_per_mfma"] else "-"
        print(f"{k[:40]:40s} grid {grid:8d} x{n}: VALU {rec['valu_per_dispatch']:.3g} MFMA {mfma:.3g} "
              f"(VALU/MFMA {vpm}) VMEM {rec['vmem_per_dispatch']:.3g} LDS {rec['lds_per_dispatch']:.3g} "
              f"wait {rec['wait_frac']:.2f} active {rec['active_inst_frac']:.2f}")
    if a.json:
        json.dump({"source": "rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY "
                   "SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_MFMA over 3 eager bench steps "
                   "(tools/gpu_pmc_sq_step.sh); per-dispatch averages per (kernel, grid)",
                   "kernels": out}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
