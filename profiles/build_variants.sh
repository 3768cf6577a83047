#!/bin/bash
# Build kernel variants side by side for A/B timing (SURFCASCADE_LIB selects one).
#   bash profiles/build_variants.sh name1 "-DFOO=1" name2 "-DBAR=2" ...
R=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -ge 2 ]; do
  make -s -C "$R/surfcascade_amd/csrc" OUT="$R/surfcascade_amd/lib/variants/$1" EXTRA="$2" -j8 || exit 1
  shift 2
done
