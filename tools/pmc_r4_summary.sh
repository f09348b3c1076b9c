#!/bin/bash
# Fold the tools/pmc_r4.sh passes (gpurun_out/pmc_r4/) into profiles/pmc_traffic.json and
# profiles/pmc_valu.json (CPU side; run after the GPU call merged gpurun_out/ back).
R="$(cd "$(dirname "$0")/.." && pwd)"
O="$R/gpurun_out/pmc_r4"
S="python3 $R/tools/pmc_summary.py"
set -e
$S --alg "$R/profiles/pmc_valu.json" race_level3_4_PYB_GND_DRAG_DW_fp32_4096 "$O/r4g_alg_fp32" 16384
for P in fp64 fp32; do
  $S "$R/profiles/pmc_traffic.json" \
    "PYB_${P}_4096" "$O/h_f_$P" "$O/h_w_$P" \
    "race_level0_2_PYB_${P}_2048" "$O/r3_f_$P" "$O/r3_w_$P" \
    "race_level3_4_PYB_DW_${P}_4096" "$O/r4_f_$P" "$O/r4_w_$P" \
    "race_level3_4_PYB_GND_DRAG_DW_${P}_4096" "$O/r4g_f_$P" "$O/r4g_w_$P"
  $S --valu "$R/profiles/pmc_valu.json" \
    "PYB_${P}_4096" "$O/h_fl_$P" "$O/h_bu_$P" \
    "race_level0_2_PYB_${P}_2048" "$O/r3_fl_$P" "$O/r3_bu_$P" \
    "race_level3_4_PYB_DW_${P}_4096" "$O/r4_fl_$P" "$O/r4_bu_$P" \
    "race_level3_4_PYB_GND_DRAG_DW_${P}_4096" "$O/r4g_fl_$P" "$O/r4g_bu_$P"
done
