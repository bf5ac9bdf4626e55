#!/usr/bin/env python3
"""Speed-of-light table of the hot kernels from rocprofv3 PMC runs (tools/profile_counters.sh).

    python tools/roofline.py gpurun_out/pmc > profiles/r2/roofline.md

For every (workload, kernel) whose median dispatch is at least --min-us long:
  valu_bound_us  (4 cycles x non-transcendental VALU + 16 x SQ_INSTS_VALU_TRANS_F64) /
                 (1024 SIMDs x 2.4 GHz): a wave64 fp64 or packed-fp32 VALU instruction occupies
                 its SIMD for 4 cycles, a v_rcp_f64 for 16 (valu_rate_probe: 4.69 vs 16.3
                 nominal cycles, profiles/r2/valu_rate_probe2.jsonl); the issue-limited time of
                 the whole dispatch at the nominal clock. (Plain fp32 VALU issues in ~2.6, so
                 fp32 kernels with many unpacked ops are over-charged here.)
  hbm_bound_us   (FETCH_SIZE + WRITE_SIZE) / 8 TB/s (MI355X spec; ~6.3-6.9 TB/s is what a
                 streaming kernel reaches, profiles/r1 and r2 trainscan rows), when collected
  sol            max(bounds) / measured median dispatch time: the fraction of the tighter
                 roofline the kernel reaches
  valu_per_sample, when the workload's sample count is known (Riemann workloads: 1e9; the
                 2-D multi-step dispatch runs T2D_REPLAY integrations of its field)
  clock_ghz      GRBM_GUI_ACTIVE / 8 XCDs / measured median: the shader clock the dispatch
                 actually ran at (the counter sums the 8 XCDs' busy cycles; its window runs a
                 few us past the dispatch, so only dispatches >= 500 us get a clock)
  valu_at_clock  the VALU bound priced at that clock / measured: issue efficiency with the
                 clock taken out (packed-fp32 kernels run at ~2.1 GHz under the power limit
                 where fp64 runs at ~2.3: at 2.4 GHz pricing they look 10 points worse than
                 their issue rate is)
Counters of one workload come from several runs (one counter group each); per counter the
median over that workload's dispatches of the kernel is used.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import statistics

SIMDS = 256 * 4
CLOCK_HZ = 2.4e9
VALU_CYCLES = 4
TRANS_F64_CYCLES = 16
HBM_BPS = 8.0e12

SAMPLES = {  # samples per dispatch of the Riemann workloads (miint bench default N)
    "pi4_series": 1e9, "pi4_ieee": 1e9, "pi4_fp32": 1e9, "sin": 1e9, "sin_ocml": 1e9,
    "train": 1e9, "poly": 1e9, "table": 1e9, "table2d": 4096 * 4096, "trainscan": 18e6,
    "pi4_fp32acc": 1e9, "pi4_series_exact": 1e9, "sin_fast": 1e9, "train_fast": 1e9, "table2d_slice8": 512 * 4096,
    "pi4_series_exact_share8": 1.25e8, "pi4_series_g": 1e9,
    "share8_20": 1.25e8, "share8_64": 1.25e8,
    "materialize": 18e6,
}

# integrations per 2-D multi-step dispatch (Table2DPlan::graph_steps, auto since round 5: a
# replay holds 2^33 samples; round 4's profiles ran 32)
T2D_REPLAY = {"table2d": 512, "table2d_slice8": 1024}


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    n = n.replace("miint::", "").replace("(miint::DivMode)", "div")
    depth, out = 0, []
    for ch in n:
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out)[:70]


def collect(root: str):
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for d in sorted(glob.glob(os.path.join(root, "*_G*"))):
        if not os.path.isdir(d):
            continue
        workload = os.path.basename(d).rsplit("_G", 1)[0]
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            seen = set()
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    k = (workload, short(r.get("Kernel_Name", "?")))
                    try:
                        ctr[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                    except (KeyError, ValueError):
                        continue
                    did = (r.get("Dispatch_Id"), r.get("Correlation_Id"))
                    if did not in seen:
                        seen.add(did)
                        try:
                            dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                        except (KeyError, ValueError):
                            pass
    return ctr, dur


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("root", nargs="?", default="gpurun_out/pmc")
    ap.add_argument("--min-us", type=float, default=4.0)
    a = ap.parse_args()
    ctr, dur = collect(a.root)
    print("| workload | kernel | median us | VALU insts | VALU/sample | VALU bound us | "
          "HBM bytes | HBM bound us | speed of light | clock GHz | VALU issue at that clock |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for (w, kname), cs in sorted(ctr.items()):
        if "rocclr" in kname or not dur[(w, kname)]:
            continue
        t_us = statistics.median(dur[(w, kname)]) / 1e3
        if t_us < a.min_us:
            continue
        med = {c: statistics.median(v) for c, v in cs.items()}
        valu = med.get("SQ_INSTS_VALU")
        trans = med.get("SQ_INSTS_VALU_TRANS_F64", 0.0)
        vb = ((valu - trans) * VALU_CYCLES + trans * TRANS_F64_CYCLES) / (SIMDS * CLOCK_HZ) * 1e6 \
            if valu else None
        nbytes = None
        if "FETCH_SIZE" in med or "WRITE_SIZE" in med:  # kilobytes
            nbytes = (med.get("FETCH_SIZE", 0.0) + med.get("WRITE_SIZE", 0.0)) * 1024
        hb = nbytes / HBM_BPS * 1e6 if nbytes else None
        bound = max(b for b in (vb, hb, 0.0) if b is not None)
        samples = SAMPLES.get(w, 0) * (T2D_REPLAY.get(w, 32)
                                       if w.startswith("table2d") and "multistep" in kname else 1)
        per = f"{valu * 64 / samples:.2f}" if valu and samples else "—"
        grbm = med.get("GRBM_GUI_ACTIVE")
        # the counter window spans a few us past the dispatch: only long dispatches give a clock
        ghz = grbm / 8 / (t_us * 1e-6) / 1e9 if grbm and t_us >= 500 else None
        at_clock = (f"{vb * CLOCK_HZ / (ghz * 1e9) / t_us:.0%}" if ghz and vb else "—")
        tail = f" {'—' if ghz is None else f'{ghz:.2f}'} | {at_clock} |"
        print(f"| {w} | `{kname}` | {t_us:.1f} | {valu:.3g} | {per} | "
              f"{vb:.1f} | {'—' if nbytes is None else f'{nbytes:.3g}'} | "
              f"{'—' if hb is None else f'{hb:.1f}'} | {bound / t_us:.0%} |" + tail
              if valu else
              f"| {w} | `{kname}` | {t_us:.1f} | — | — | — | "
              f"{'—' if nbytes is None else f'{nbytes:.3g}'} | {'—' if hb is None else f'{hb:.1f}'} | "
              f"{bound / t_us:.0%} |" + tail)


if __name__ == "__main__":
    main()
