"""One plan-mode step of a rocprofv3 kernel trace as a timeline: stream, start offset, duration,
gap since the previous launch on the same stream, kernel, grid.

    python tools/step_timeline.py gpurun_out/prof/run_kernel_trace.csv [--anchor k7m_w2n] [--summary]

Steps are cut at a kernel that runs once per full step (``--anchor``); the median-length step
among the steady ones (the timed plan steps) is printed.
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--anchor", default="k7m_w2n")
    ap.add_argument("--summary", action="store_true", help="per-kernel totals of that step only")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.anchor in r["Kernel_Name"]]
    spans = [(idx[k], idx[k + 1]) for k in range(len(idx) - 1)]
    lens = collections.Counter(e - s for s, e in spans)
    n_common = lens.most_common(1)[0][0]
    cands = [(s, e) for s, e in spans if e - s == n_common]
    s, e = cands[len(cands) // 2]
    seg = rows[s:e]
    t0 = int(seg[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in seg)
    qs, last_end = {}, {}
    busy = collections.defaultdict(float)
    for r in seg:
        q = qs.setdefault(r["Queue_Id"], len(qs))
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (st - last_end.get(q, st)) / 1e3
        last_end[q] = max(last_end.get(q, 0), en)
        busy[r["Kernel_Name"].split("(")[0][:60]] += (en - st) / 1e3
        if not a.summary:
            print(f"{q} {(st - t0) / 1e3:8.1f} {(en - st) / 1e3:7.1f} gap {gap:6.1f}  {r['Kernel_Name'][:64]} g{r['Grid_Size_X']}")
    print(f"step: {len(seg)} launches, {(t1 - t0) / 1e3:.1f} us from first start to last end, {len(qs)} queues")
    if a.summary:
        for k, v in sorted(busy.items(), key=lambda kv: -kv[1]):
            print(f"{v:8.1f} us  {k}")


if __name__ == "__main__":
    main()
