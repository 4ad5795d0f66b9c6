#!/bin/bash
# Build the committed K1 (git HEAD, or $1) as library variant "prev" for same-call A/B
# against the working tree's product library: bash scripts/ab_prev.sh [rev]
cd "$(dirname "$0")/.."
git show "${1:-HEAD}":go-webp_amd/csrc/device/vp8_recon_filter.hip > go-webp_amd/csrc/device/_ab_prev.hip
make -s -j8 -C go-webp_amd/csrc VARIANT=prev K1SRC=device/_ab_prev.hip
