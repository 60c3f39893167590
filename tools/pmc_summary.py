#!/usr/bin/env python3
"""Per-kernel hardware-counter table from rocprofv3 ``--pmc`` runs.

Reads one or more ``*_counter_collection.csv`` files (one per counter pass of the same
program), groups the dispatches by kernel (and grid size), averages every counter over the
dispatches, and derives what the raw numbers mean on gfx950:

* ``mfma_util``  = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CU_CYCLES x 4 SIMDs)  (matrix-pipe busy share)
* ``waves``      = SQ_WAVES (per dispatch); ``wait_share`` = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
* ``l2_hit``     = TCC_HIT / (TCC_HIT + TCC_MISS)
* ``hbm_rd_MB``  = TCC_EA0_RDREQ_DRAM x 64 B  (MI355X_MICROARCH.md: EA read requests are
  tallied at 64 B while a wide read moves 128 B — double it against a byte count)
* ``lds_conf``   = SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS
* ``waves_cu``   = 4 x SQ_WAVE_CYCLES / SQ_BUSY_CU_CYCLES: mean waves resident on a busy CU
  (calibrated on the 8-wave, one-workgroup-per-CU expert tiles, which read 8.0; a 4-wave
  workgroup reads ~4 at one workgroup per CU and ~8 at two)

    python tools/pmc_summary.py gpurun_out/pmc_lmhead_* [--match gemm]     (files or directories)
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"Cfg<([^>]*)>", name)
    base = name.replace("(anonymous namespace)::", "")
    base = re.sub(r"^void ", "", base)
    base = re.sub(r"[(<].*", "", base)
    if m:
        base += f"<{m.group(1).replace(' ', '')}>"
    return base[:56]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csvs", nargs="+")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    # (kernel, grid) -> counter -> [values per dispatch]
    vals = defaultdict(lambda: defaultdict(list))
    paths = []
    for p in a.csvs:
        paths += sorted(glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True)) \
            if os.path.isdir(p) else [p]
    for path in paths:
        per = defaultdict(lambda: defaultdict(float))  # (dispatch, kernel, grid) -> counter -> value
        for r in csv.DictReader(open(path)):
            k = (r.get("Dispatch_Id"), short(r["Kernel_Name"]), r.get("Grid_Size", ""))
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        for (_, kern, grid), cs in per.items():
            if a.match and a.match not in kern:
                continue
            for c, v in cs.items():
                vals[(kern, grid)][c].append(v)
    cols = ["n", "waves", "mfma_util", "wait_share", "l2_hit", "hbm_rd_MB", "lds_conf", "waves_cu"]
    print(f"{'kernel':56s} {'grid':>9s} " + " ".join(f"{c:>10s}" for c in cols))
    for (kern, grid), cs in sorted(vals.items(), key=lambda kv: -max((len(v) for v in kv[1].values()), default=0)):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        n = max(len(v) for v in cs.values())

        def ratio(a_, b_, scale=1.0):
            return f"{m[a_] / (m[b_] * scale):.3f}" if a_ in m and b_ in m and m[b_] else "-"
        row = {
            "n": str(n),
            "waves": f"{m['SQ_WAVES']:.0f}" if "SQ_WAVES" in m else "-",
            "mfma_util": ratio("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CU_CYCLES", 4.0),
            "wait_share": ratio("SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES"),
            "l2_hit": (f"{m['TCC_HIT_sum'] / (m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.3f}"
                       if m.get("TCC_HIT_sum", 0) + m.get("TCC_MISS_sum", 0) else "-"),
            "hbm_rd_MB": f"{m['TCC_EA0_RDREQ_DRAM_sum'] * 64 / 1e6:.2f}" if "TCC_EA0_RDREQ_DRAM_sum" in m else "-",
            "lds_conf": ratio("SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS"),
            "waves_cu": ratio("SQ_WAVE_CYCLES", "SQ_BUSY_CU_CYCLES", 0.25),
        }
        print(f"{kern:56s} {grid:>9s} " + " ".join(f"{row[c]:>10s}" for c in cols))
        raw = " ".join(f"{c}={v:.4g}" for c, v in sorted(m.items()))
        print(f"    {raw}")


if __name__ == "__main__":
    main()
