#!/usr/bin/env python3
"""Per-step kernel breakdown from a rocprofv3 ``*_kernel_trace.csv``.

Steps are delimited by a marker kernel (default: the embedding kernel, first node of every
DAG step); the last ``--steps`` complete steps are averaged. Prints, per (kernel, grid),
calls/step, mean µs and total µs/step, plus the step wall span.

    python tools/analyze_trace.py gpurun_out/prof/llama3-8b_kernel_trace.csv --steps 5
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"Cfg<([^>]*)>", name)
    base = name.replace("(anonymous namespace)::", "").replace("at::native::", "")
    base = re.sub(r"^void ", "", base)
    base = re.sub(r"[(<].*", "", base)
    if m:
        base += f"<{m.group(1).replace(' ', '')}>"
    return base[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--marker", default="embedding_kernel")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--per-dispatch", action="store_true",
                    help="also list every dispatch of the last step in order (duration, gap to the previous end)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(starts) < a.steps + 1:
        print(f"only {len(starts)} markers found")
        starts = starts + [len(rows)]
    sel_lo, sel_hi = starts[-a.steps - 1], starts[-1]
    sel = rows[sel_lo:sel_hi]
    nst = a.steps
    agg = defaultdict(lambda: [0, 0.0])
    busy = 0.0
    for r in sel:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        key = (short(r["Kernel_Name"]), f'{r["Grid_Size_X"]}x{r["Grid_Size_Y"]}x{r["Grid_Size_Z"]}/{r["Workgroup_Size_X"]}')
        agg[key][0] += 1
        agg[key][1] += d
        busy += d
    span = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e3 / nst
    print(f"steps={nst} kernels/step={len(sel) / nst:.0f} busy/step={busy / nst:.1f}us span/step={span:.1f}us")
    print(f"{'kernel':60s} {'grid/block':>22s} {'calls':>6s} {'mean_us':>9s} {'us/step':>9s} {'%':>5s}")
    for (k, g), (n, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:a.top]:
        print(f"{k:60s} {g:>22s} {n / nst:6.1f} {t / n:9.2f} {t / nst:9.1f} {100 * t / busy:5.1f}")
    if a.per_dispatch:
        last = rows[starts[-2]:starts[-1]] if len(starts) >= 2 else sel
        print(f"\nlast step, {len(last)} dispatches in order:")
        print(f"{'#':>3s} {'kernel':60s} {'grid/block':>22s} {'us':>8s} {'gap_us':>7s}")
        prev = None
        for i, r in enumerate(last):
            s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            gap = (s0 - prev) / 1e3 if prev is not None else 0.0
            prev = e0
            g = f'{r["Grid_Size_X"]}x{r["Grid_Size_Y"]}x{r["Grid_Size_Z"]}/{r["Workgroup_Size_X"]}'
            print(f"{i:3d} {short(r['Kernel_Name']):60s} {g:>22s} {(e0 - s0) / 1e3:8.2f} {gap:7.2f}")


if __name__ == "__main__":
    main()
