#!/usr/bin/env python3
"""Summarise rocprofv3 PMC runs (tools/profile_counters.sh) into a Markdown table.

    python tools/summarize_counters.py gpurun_out/pmc > profiles/r1/counters.md

Per (workload, kernel) it reports the median per-dispatch value of every counter collected
and a few derived quantities:
  valu_per_sample   SQ_INSTS_VALU * 64 / samples  (wave-level instruction count -> per lane)
  f64_ops_per_clk   (FMA_F64*2 + ADD_F64 + MUL_F64 + TRANS_F64) * 64 / GRBM_GUI_ACTIVE*8 ...
  eff_clock_ghz     GRBM_GUI_ACTIVE / 8 XCDs / kernel time  (MI355X_MICROARCH 'DVFS give-back')
  valu_busy         SQ_ACTIVE_INST_VALU * 4 / (SQ_BUSY_CYCLES * 4 SIMD ...) approximated
"""
from __future__ import annotations

import collections
import csv
import glob
import os
import statistics
import sys


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    n = n.replace("miint::", "").replace("(miint::DivMode)", "div")
    depth, out = 0, []
    for ch in n:  # drop the parameter list, keep template arguments
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out)[:90]


def load(dirpath: str):
    rows = []
    for f in glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows.extend(csv.DictReader(fh))
    return rows


def main(root: str) -> None:
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    durations = collections.defaultdict(list)
    for d in sorted(glob.glob(os.path.join(root, "*_G*"))):
        if not os.path.isdir(d):
            continue
        workload = os.path.basename(d).rsplit("_G", 1)[0]
        for r in load(d):
            k = (workload, short(r.get("Kernel_Name", "?")))
            try:
                v = float(r["Counter_Value"])
            except (KeyError, ValueError):
                continue
            per[k][r["Counter_Name"]].append(v)
            try:
                durations[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            except (KeyError, ValueError):
                pass
    print("| workload | kernel | dispatch us (median) | counter medians | derived |")
    print("|---|---|---|---|---|")
    for (w, kname), ctrs in sorted(per.items()):
        if "rocclr" in kname:
            continue
        med = {c: statistics.median(v) for c, v in ctrs.items()}
        dur = statistics.median(durations[(w, kname)]) / 1e3 if durations[(w, kname)] else 0.0
        derived = []
        if "GRBM_GUI_ACTIVE" in med and dur > 0:
            derived.append(f"eff_clock {med['GRBM_GUI_ACTIVE'] / 8 / (dur * 1e3):.2f} GHz")
        if "SQ_ACTIVE_INST_VALU" in med and "SQ_BUSY_CYCLES" in med and med["SQ_BUSY_CYCLES"]:
            derived.append(f"VALU_active/busy {med['SQ_ACTIVE_INST_VALU'] / med['SQ_BUSY_CYCLES']:.2f}")
        if "SQ_INSTS_LDS" in med and "SQ_INSTS_VALU" in med and med["SQ_INSTS_VALU"]:
            derived.append(f"LDS/VALU {med['SQ_INSTS_LDS'] / med['SQ_INSTS_VALU']:.2e}")
        cs = ", ".join(f"{c}={v:.4g}" for c, v in sorted(med.items()))
        print(f"| {w} | `{kname}` | {dur:.1f} | {cs} | {'; '.join(derived)} |")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
