#!/bin/bash
# Build the whole library of a committed revision (default HEAD) as variant "prev"
# (go-webp_amd/webp_amd/libgowebp_amd_prev.so) for same-call A/Bs against the working tree:
#   bash scripts/build_prev_lib.sh [rev]      then   WG_LIB_VARIANT=prev python bench.py ...
cd "$(dirname "$0")/.."
rev="${1:-HEAD}"
tmp=$(mktemp -d)
git archive "$rev" go-webp_amd/csrc include | tar -x -C "$tmp"
make -s -j8 -C "$tmp/go-webp_amd/csrc" OUT="$PWD/go-webp_amd/webp_amd/libgowebp_amd_prev.so" BUILD="$tmp/build" \
  && echo "built libgowebp_amd_prev.so from $rev"
rm -rf "$tmp"
