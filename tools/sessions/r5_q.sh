#!/bin/bash
# r5 session Q: PMC counters of the 2-D field and its 1/8 slice at HEAD (adaptive replays)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc
ONLY="table2d table2d_slice8" bash tools/profile_counters.sh && \
python3 tools/roofline.py gpurun_out/pmc > gpurun_out/r5/q_roofline_t2d.md
echo "exit $?"
