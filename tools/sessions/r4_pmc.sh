# PMC roofline of the hot kernels at HEAD (round 4): counters per workload, then the table
set -uo pipefail
mkdir -p gpurun_out/r4
rm -rf gpurun_out/pmc
ONLY="pi4_series pi4_fp32 pi4_fp32acc pi4_series_exact table2d table2d_slice8 sin train poly table" \
  timeout -k 10 900 bash tools/profile_counters.sh > gpurun_out/r4/pmc.log 2>&1 || { tail -20 gpurun_out/r4/pmc.log; exit 1; }
python3 tools/roofline.py gpurun_out/pmc > gpurun_out/r4/roofline.md
cat gpurun_out/r4/roofline.md
