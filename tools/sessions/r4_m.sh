# round 4 session M: the PMC roofline of every hot kernel at the final HEAD
set -uo pipefail
mkdir -p gpurun_out/r4
bash tools/sessions/r4_pmc.sh > gpurun_out/r4/pmc_session_m.txt 2>&1 || { tail -20 gpurun_out/r4/pmc_session_m.txt; exit 1; }
cat gpurun_out/r4/roofline.md
