#!/bin/bash
# Builds the FETCH_SIZE calibration binary (gfx950) next to this script.
cd "$(dirname "$0")" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -o fetch_calib fetch_calib.hip
