#!/bin/bash
# Round 6: where a wave's cycles go at the 1/8 share vs G = 1 (wait / instruction-fetch
# counters, tools/profile_counters.sh group G5), 20-step multi-step dispatches.
set -o pipefail
ONLY="g1_w share8_w" bash tools/profile_counters.sh > gpurun_out/pmc_wait.log 2>&1 &&
python3 tools/summarize_counters.py gpurun_out/pmc > gpurun_out/pmc_wait.md
rc=$?; echo "rc=$rc"; cat gpurun_out/pmc_wait.md | head -30; exit $rc
