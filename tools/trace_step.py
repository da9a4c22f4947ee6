"""Per-step view of a rocprofv3 kernel trace (``--kernel-trace``; CSV or the SQLite ``*_results.db``).

    python tools/trace_step.py gpurun_out/prof/run_kernel_trace.csv [--steps 20] [--drop-last 10] [--list]

Splits the trace into steps at the generator's Adam launch (the last launch of a step), then
reports for the last ``--steps`` steps: wall time per step, GPU busy time (union of kernel
intervals over all streams), idle gaps, and the per-kernel totals; ``--list`` prints one step's
launches in order with their stream, start offset and duration.
"""
import argparse
import collections
import csv


def load_rows(path):
    """Kernel-trace rows from a rocprofv3 CSV or its default SQLite output (``*_results.db``)."""
    if not path.endswith(".db"):
        return list(csv.DictReader(open(path)))
    import sqlite3
    c = sqlite3.connect(path)
    q = "select name, start, end, queue_id, grid_x, workgroup_x from kernels"
    return [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e, "Queue_Id": qid, "Grid_Size_X": gx,
             "Workgroup_Size_X": wx} for n, s, e, qid, gx, wx in c.execute(q)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--list", action="store_true")
    ap.add_argument("--drop-last", type=int, default=10, help="trailing steps to skip (bench.py's roofline steps)")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = sorted(load_rows(a.trace), key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("cg::adam_kernel")]
    ends = adam[1::2]  # two Adam launches per step: critic, then generator
    if a.drop_last:
        ends = ends[:-a.drop_last]
    ends = ends[-(a.steps + 1):]
    steps = [rows[ends[i] + 1:ends[i + 1] + 1] for i in range(len(ends) - 1)]
    walls, busys = [], []
    per = collections.defaultdict(float)
    cnt = collections.Counter()
    for st in steps:
        t0 = int(st[0]["Start_Timestamp"])
        t1 = max(int(r["End_Timestamp"]) for r in st)
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in st)
        busy, cs, ce = 0, iv[0][0], iv[0][1]
        for s, e in iv[1:]:
            if s > ce:
                busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        walls.append(t1 - t0)
        busys.append(busy)
        for r in st:
            nm = r["Kernel_Name"].split("(")[0]
            per[nm] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / len(steps)
            cnt[nm] += 1
    n = len(steps)
    print(f"steps {n}: wall {sum(walls) / n / 1e3:.1f} us, busy {sum(busys) / n / 1e3:.1f} us, "
          f"launches/step {len(steps[-1])}")
    tot = sum(per.values())
    print(f"sum of kernel durations {tot / 1e3:.1f} us/step")
    for nm, t in sorted(per.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f"{t / 1e3:9.1f} us {cnt[nm] // n:4d}x  {nm[:110]}")
    if a.list:
        st = steps[-1]
        t0 = int(st[0]["Start_Timestamp"])
        prev_end = t0
        for r in st:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            print(f"{(s - t0) / 1e3:8.1f} +{(e - s) / 1e3:7.1f} gap {(s - prev_end) / 1e3:6.1f} "
                  f"q{r['Queue_Id']} g{r['Grid_Size_X']}/{r['Workgroup_Size_X']} {r['Kernel_Name'].split('(')[0][:90]}")
            prev_end = max(prev_end, e)


if __name__ == "__main__":
    main()
