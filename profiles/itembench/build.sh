#!/bin/bash
# Builds libitembench.so (gfx950) next to this script.
cd "$(dirname "$0")" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared \
  -ffp-contract=off -fno-slp-vectorize -Wno-unused-result -I../../include -I../../surfcascade_amd/csrc \
  $EXTRA -o libitembench.so itembench.hip
