#!/usr/bin/env python3
"""Count instructions per loop body in a gfx950 assembly dump (`make asm` -> build/asm/*.s).

    python tools/isa_count.py build/asm/riemann.s 'riemann_fused_kernelILNS_7DivModeE0ENS_3Pi4E'

For every kernel whose symbol matches the regex: the register counts from the metadata and,
for each loop (a basic block range closed by a branch back to an earlier label), the number
of VALU (v_*), fp64 VALU, SALU (s_*), LDS (ds_*) and memory instructions in it. This is how
the per-tile VALU counts quoted in integrands.hpp and docs/ARCHITECTURE.md are obtained.
"""
from __future__ import annotations

import re
import sys


def kernels(text: str):
    for m in re.finditer(r"^(\S+):\s*(?:;.*)?\n", text, re.M):
        name = m.group(1)
        if name.startswith(".") or not name.startswith("_Z"):
            continue
        end = text.find("\n.Lfunc_end", m.end())
        yield name, text[m.end():end if end > 0 else len(text)]


def classify(op: str) -> str:
    if op.startswith(("ds_",)):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "mem"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


def loops(body: str):
    lines = body.splitlines()
    labels = {}
    ins = []  # (label-index position, op)
    for ln in lines:
        s = ln.split(";")[0].strip()
        if not s:
            continue
        if s.endswith(":"):
            labels[s[:-1]] = len(ins)
            continue
        if s.startswith("."):
            continue
        ins.append(s)
    for i, s in enumerate(ins):
        op = s.split()[0]
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = s.split()[-1]
            if tgt in labels and labels[tgt] <= i:
                yield tgt, ins[labels[tgt]:i + 1]


def main() -> int:
    path, pat = sys.argv[1], re.compile(sys.argv[2])
    text = open(path).read()
    for name, body in kernels(text):
        if not pat.search(name):
            continue
        meta = text[text.find(f".name:           {name}"):]
        sg = re.search(r"\.sgpr_count:\s+(\d+)", meta)
        vg = re.search(r"\.vgpr_count:\s+(\d+)", meta)
        print(f"{name}\n  sgpr {sg.group(1) if sg else '?'}  vgpr {vg.group(1) if vg else '?'}")
        for lbl, block in loops(body):
            cnt: dict[str, int] = {}
            f64 = 0
            for s in block:
                op = s.split()[0]
                k = classify(op)
                cnt[k] = cnt.get(k, 0) + 1
                if k == "valu" and re.sub(r"_e(32|64)$", "", op).endswith("_f64"):
                    f64 += 1
            print(f"  loop {lbl}: {len(block)} instr, valu {cnt.get('valu', 0)} (f64 {f64}), "
                  f"salu {cnt.get('salu', 0)}, lds {cnt.get('lds', 0)}, mem {cnt.get('mem', 0)}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
