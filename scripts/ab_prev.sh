#!/bin/bash
# Build the committed K1 (git HEAD, or $1) as library variant "prev" for same-call A/B
# against the working tree's product library: bash scripts/ab_prev.sh [rev]
# (the i4 recipe table it includes is taken from the same revision)
cd "$(dirname "$0")/.."
rev="${1:-HEAD}"
git show "$rev":go-webp_amd/csrc/device/pred4_table.inc > go-webp_amd/csrc/device/_ab_prev_pred4_table.inc
git show "$rev":go-webp_amd/csrc/device/vp8_recon_filter.hip |
  sed 's/#include "pred4_table.inc"/#include "_ab_prev_pred4_table.inc"/' > go-webp_amd/csrc/device/_ab_prev.hip
make -s -j8 -C go-webp_amd/csrc VARIANT=prev K1SRC=device/_ab_prev.hip
