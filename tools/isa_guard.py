#!/usr/bin/env python3
"""ISA / resource regression guard for the hot gfx950 kernels (runs on the CPU box).

The Riemann kernels sit at 84-96 % of their VALU issue bound (profiles/r2/roofline.md), and
that rests on exact register allocation and instruction selection: register-pinned constants
(integrands.hpp Pi4::init), 8 resident waves per SIMD (<= 64 VGPRs, <= 96 SGPRs,
riemann.hip occupancy_hint), no scratch. A compiler or source change can lose 10-50 %
without any test failing. This tool compiles the kernel files device-only to gfx950
assembly (hipcc --cuda-device-only -S, no GPU needed), and for every guarded instantiation
reads the compiler's kernel-info block (TotalNumSgprs, NumVgprs, NumAgprs, ScratchSize,
Occupancy) and the VALU count of its hot loop (the loop body with the most VALU
instructions = one tile of the lane loop for the series kernels; for the multi-step kernels
the step loop around it, i.e. a tile plus the per-step overhead).

    python tools/isa_guard.py --write   # refresh tools/isa_baseline.json
    python tools/isa_guard.py           # compare; exit 1 on a regression

Regression = hot-loop VALU more than 3 % above the baseline, scratch where the baseline has
none (or more than it has), a scratch access in a hot loop that had none, or fewer waves per
SIMD than the baseline. (Improvements print a note: refresh the baseline with --write.)
The per-sample loop this replaces is riemann.cpp:34-41.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BASELINE = os.path.join(REPO, "tools", "isa_baseline.json")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# extra -D switches of an A/B variant (e.g. ISA_DEFS="-DMIINT_MS_CHUNK=4"), compared against
# the default build's baseline
DEFS = os.environ.get("ISA_DEFS", "").split()
VALU_SLACK = 1.03

# name -> (kernel file, symbol regex, samples per hot-loop iteration or 0 = not one tile)
CH = r"riemann_chained_kernel(?:_o8)?ILNS_7DivModeE"
MS = r"riemann_multistep_kernel(?:_o8)?ILNS_7DivModeE"
GUARDED = {
    "pi4_series": ("riemann", CH + r"0ENS_3Pi4EE", 384),
    "pi4_ieee": ("riemann", CH + r"1ENS_3Pi4EE", 32),
    "pi4_series_exact": ("riemann", CH + r"3ENS_3Pi4EE", 384),
    "sin_series": ("riemann", CH + r"0ENS_3SinEE", 192),
    "sin_ieee": ("riemann", CH + r"1ENS_3SinEE", 32),
    "train_series": ("riemann", CH + r"0ENS_8TrainVelEE", 128),
    "train_ieee": ("riemann", CH + r"1ENS_8TrainVelEE", 32),
    "table_series": ("riemann", CH + r"0ENS_5TableEE", 0),
    "pi4f32_series": ("riemann", CH + r"0ENS0_6Pi4F32EE", 192),
    "pi4f32_ieee": ("riemann", CH + r"1ENS0_6Pi4F32EE", 32),
    "poly7_series": ("riemann", CH + r"0ENS_4PolyILi7EEE", 64),
    # the multi-step kernels (graph batches by default): the hot loop found is the step loop
    # around a tile, so no per-sample figure; max_block_valu is one tile's straight line
    "ms_pi4_series": ("riemann", MS + r"0ENS_3Pi4ELb0EE", 0),
    "ms_pi4_series_exact": ("riemann", MS + r"3ENS_3Pi4ELb0EE", 0),
    "ms_pi4f32_series": ("riemann", MS + r"0ENS0_6Pi4F32ELb0EE", 0),
    "ms_sin_series": ("riemann", MS + r"0ENS_3SinELb0EE", 0),
    "ms_sin_ieee": ("riemann", MS + r"1ENS_3SinELb0EE", 0),
    "ms_train_series": ("riemann", MS + r"0ENS_8TrainVelELb0EE", 0),
    "ms_poly7_series": ("riemann", MS + r"0ENS_4PolyILi7EEELb0EE", 0),
    "ms_table_series": ("riemann", MS + r"0ENS_5TableELb0EE", 0),
    "ms_table_ieee": ("riemann", MS + r"1ENS_5TableELb0EE", 0),
    # the same step loops with the in-launch close after them (RiemannConfig::close "launch")
    "msc_pi4_series_exact": ("riemann", MS + r"3ENS_3Pi4ELb1EE", 0),
    "msc_pi4_series": ("riemann", MS + r"0ENS_3Pi4ELb1EE", 0),
    "table2d_stream_0_16": ("table", r"table2d_stream_kernelILi0ELi16ELb0EE", 0),
    "table2d_stream_0_30": ("table", r"table2d_stream_kernelILi0ELi30ELb0EE", 0),
    "table2d_stream_1_16": ("table", r"table2d_stream_kernelILi1ELi16ELb0EE", 0),
    "table2d_stream_1_30": ("table", r"table2d_stream_kernelILi1ELi30ELb0EE", 0),
    "table2d_stream_2_16": ("table", r"table2d_stream_kernelILi2ELi16ELb0EE", 0),
    "table2d_stream_2_30": ("table", r"table2d_stream_kernelILi2ELi30ELb0EE", 0),
    # the 2-D multi-step kernels: the 30-row tile must keep 5 waves per SIMD (<= 96 VGPRs at
    # the 5 workgroups per CU its LDS allows; at 3 the 4096^2 grid would no longer be resident
    # and the plan would fall back to chained replays)
    "table2d_ms_16": ("table", r"table2d_multistep_kernelILi16EE", 0),
    "table2d_ms_30": ("table", r"table2d_multistep_kernelILi30EE", 0),
}


def compile_asm(stem: str, outdir: str) -> str:
    out = os.path.join(outdir, stem + ".s")
    subprocess.run([HIPCC, "-std=c++17", "-O3", "-fPIC", "-I" + os.path.join(REPO, "csrc", "include"),
                    "--offload-arch=gfx950", "--cuda-device-only", "-S", *DEFS,
                    os.path.join(REPO, "csrc", "kernels", stem + ".hip"), "-o", out],
                   check=True, capture_output=True, text=True)
    with open(out) as f:
        return f.read()


def functions(text: str):
    """(symbol, body, kernel-info block) of every kernel in a gfx950 .s file."""
    for m in re.finditer(r"^(_Z\S+):[^\n]*\n", text, re.M):
        name = m.group(1)
        end = text.find("\n.Lfunc_end", m.end())
        if end < 0:
            continue
        info_at = text.find("; Kernel info:", end)
        nxt = text.find("\n_Z", end)
        info = text[info_at:nxt if nxt > 0 else len(text)] if info_at > 0 else ""
        yield name, text[m.end():end], info


def cfg(body: str):
    """Basic blocks of a function body: (instructions, successor indices) per block."""
    blocks, labels, cur = [], {}, []

    def close():
        blocks.append(cur)

    for ln in body.splitlines():
        s = ln.split(";")[0].strip()
        if not s:
            continue
        if s.endswith(":"):
            if cur:
                close()
                cur = []
            labels[s[:-1]] = len(blocks)
            continue
        if s.startswith("."):
            continue
        cur.append(s)
        op = s.split()[0]
        if op.startswith("s_cbranch") or op in ("s_branch", "s_endpgm", "s_setpc_b64"):
            close()
            cur = []
    if cur:
        close()
    succ = []
    for i, ins in enumerate(blocks):
        last = ins[-1].split() if ins else [""]
        out = []
        if last[0].startswith("s_cbranch") or last[0] == "s_branch":
            if last[-1] in labels:
                out.append(labels[last[-1]])
        if not (last[0] in ("s_branch", "s_endpgm", "s_setpc_b64")) and i + 1 < len(blocks):
            out.append(i + 1)
        succ.append(out)
    return blocks, succ


def loops(body: str):
    """Instruction lists of every natural loop (a back edge to a block that dominates its
    source, and every block that reaches the source without passing the header). A backward
    jump of the block layout that is not a loop (a block placed after a loop that re-enters
    the code before it) has no dominating target and is not counted."""
    blocks, succ = cfg(body)
    n = len(blocks)
    if n == 0:
        return
    pred = [[] for _ in range(n)]
    for i, ss in enumerate(succ):
        for j in ss:
            pred[j].append(i)
    full = set(range(n))
    dom = [full.copy() for _ in range(n)]
    dom[0] = {0}
    changed = True
    while changed:
        changed = False
        for i in range(1, n):
            new = set.intersection(*(dom[p] for p in pred[i])) if pred[i] else set()
            new = new | {i}
            if new != dom[i]:
                dom[i], changed = new, True
    heads: dict = {}
    for i, ss in enumerate(succ):
        for h in ss:
            if h in dom[i]:  # back edge i -> h
                body_set = heads.setdefault(h, {h})
                stack = [i]
                while stack:
                    b = stack.pop()
                    if b not in body_set:
                        body_set.add(b)
                        stack.extend(pred[b])
    for h, members in heads.items():
        yield [ins for b in sorted(members) for ins in blocks[b]]


def field(info: str, key: str) -> int:
    m = re.search(rf"^; {key}: (\d+)", info, re.M)
    return int(m.group(1)) if m else -1


def blocks(body: str):
    """VALU count of every basic block (label to label)."""
    cur, out = "entry", {}
    for ln in body.splitlines():
        s = ln.split(";")[0].strip()
        if not s:
            continue
        if s.endswith(":"):
            cur = s[:-1]
            continue
        if s.startswith("."):
            continue
        if s.startswith("v_"):
            out[cur] = out.get(cur, 0) + 1
    return out


def stats(body: str, info: str, tile: int) -> dict:
    hot_loop = max(loops(body), key=lambda lp: sum(1 for s in lp if s.startswith("v_")),
                   default=[])
    hot = sum(1 for s in hot_loop if s.startswith("v_"))
    out = {"sgpr": field(info, "TotalNumSgprs"), "vgpr": field(info, "NumVgprs"),
           "agpr": field(info, "NumAgprs"), "scratch": field(info, "ScratchSize"),
           "occupancy": field(info, "Occupancy"), "hot_loop_valu": hot,
           "hot_loop_scratch_ops": sum(1 for s in hot_loop if s.startswith("scratch_")),
           # the longest straight-line block: one tile's samples on one path (a loop with
           # branches, e.g. the kIeee sin / cos kernels, holds several such paths)
           "max_block_valu": max(blocks(body).values(), default=0)}
    if tile:
        out["valu_per_sample"] = round(hot / tile, 4)
        out["block_valu_per_sample"] = round(out["max_block_valu"] / tile, 4)
    return out


def measure(names=None) -> dict:
    want = {k: v for k, v in GUARDED.items() if names is None or k in names}
    res: dict = {}
    with tempfile.TemporaryDirectory() as d:
        for stem in sorted({v[0] for v in want.values()}):
            text = compile_asm(stem, d)
            fns = list(functions(text))
            for key, (st, pat, tile) in want.items():
                if st != stem:
                    continue
                rx = re.compile(pat)
                hit = next(((n, b, i) for n, b, i in fns if rx.search(n)), None)
                if hit is None:
                    res[key] = {"missing": pat}
                    continue
                res[key] = dict(stats(hit[1], hit[2], tile), symbol=hit[0])
    return res


def compare(base: dict, now: dict) -> list[str]:
    bad = []
    for key, b in base.items():
        n = now.get(key)
        if n is None or "missing" in n:
            bad.append(f"{key}: kernel not found")
            continue
        if n["scratch"] > b["scratch"]:  # the baseline's scratch is 0 for all but two
            bad.append(f"{key}: {n['scratch']} bytes of scratch (baseline {b['scratch']})")
        if n["hot_loop_scratch_ops"] > b.get("hot_loop_scratch_ops", 0):
            bad.append(f"{key}: {n['hot_loop_scratch_ops']} scratch accesses in the hot loop")
        if n["occupancy"] < b["occupancy"]:
            bad.append(f"{key}: occupancy {n['occupancy']} < baseline {b['occupancy']} waves/SIMD")
        if n["hot_loop_valu"] > b["hot_loop_valu"] * VALU_SLACK:
            bad.append(f"{key}: hot loop {n['hot_loop_valu']} VALU > baseline "
                       f"{b['hot_loop_valu']} + 3 %")
        if n.get("max_block_valu", 0) > b.get("max_block_valu", 1 << 30) * VALU_SLACK:
            bad.append(f"{key}: longest block {n['max_block_valu']} VALU > baseline "
                       f"{b['max_block_valu']} + 3 %")
    return bad


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--write", action="store_true", help="refresh the baseline JSON")
    ap.add_argument("--baseline", default=BASELINE)
    a = ap.parse_args(argv)
    now = measure()
    if a.write:
        with open(a.baseline, "w") as f:
            json.dump(now, f, indent=1, sort_keys=True)
            f.write("\n")
        print(json.dumps(now, indent=1, sort_keys=True))
        return 0
    with open(a.baseline) as f:
        base = json.load(f)
    for k in sorted(now):
        n, b = now[k], base.get(k, {})
        if "missing" not in n and b and n["hot_loop_valu"] < b.get("hot_loop_valu", 0):
            print(f"note: {k} improved: {b['hot_loop_valu']} -> {n['hot_loop_valu']} VALU "
                  "(refresh with --write)")
    bad = compare(base, now)
    for line in bad:
        print("REGRESSION", line)
    print(json.dumps(now, indent=1, sort_keys=True))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
