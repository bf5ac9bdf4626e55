#!/usr/bin/env python3
"""--block sweep (the reference's SP, cintegrate.cu:17-18,124-127: threads per block) with
`miint bench`: every supported workgroup size at the default grid (the same waves per CU)
for a few integrands and two N (the headline 1e9 and a 1/8 share of it).

    python tools/block_sweep.py [--jsonl FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MIINT = os.path.join(REPO, "build", "bin", "miint")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", default="64,128,256,512,1024")
    ap.add_argument("--cases", default="pi4:series:1e9,pi4:series:1.25e8,sin:ieee:1e9,"
                                       "sin:series:1e9,table:series:1e9")
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--jsonl", default="")
    a = ap.parse_args(argv)
    for case in a.cases.split(","):
        integ, div, n = case.split(":")
        for b in a.blocks.split(","):
            p = subprocess.run([MIINT, "bench", "--integrand", integ, "--div", div, "--n", n,
                                "--block", b, "--iters", str(a.iters)],
                               capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(p.stderr, file=sys.stderr)
                return p.returncode
            row = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
            row["div"] = div
            print(json.dumps(row), flush=True)
            if a.jsonl:
                with open(a.jsonl, "a") as f:
                    f.write(json.dumps(row) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
