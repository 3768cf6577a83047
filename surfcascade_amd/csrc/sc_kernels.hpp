// sc_kernels.hpp -- launch interface of the gfx950 kernels (sc_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "surfcascade.h"

namespace sc {

// One scale level of the window pyramid (ObjDetector.cpp:178-182).
struct LevelInfo {
    int l, lh;          // window width / height
    int nx, ny;         // grid windows per row / rows
    long long grid_base;  // first grid index of the level (canonical order)
    float thr;          // (float)(l*lh) * prefilter_k   (ObjDetector.cpp:188)
    int pad;
};

// Projected template patch of one weak classifier at one level
// (ProjectPatches + GetRectsFromPatch, DenseSURFFeatureExtractor.cpp:459-484,
// 360-377): corner offsets relative to the window origin.
struct ProjPatch {
    int16_t dx, dy;  // projected patch origin
    int16_t c;       // cell edge
    int16_t shape;   // 0: 2x2, 1: 1x4 (tall), 2: 4x1 (wide)
};

struct RowScanArgs {
    const uint8_t *frames;
    long long frame_bytes;  // distance between frames
    int stride;             // bytes per image row
    int W, H;
    float *table;
    long long frame_stride;  // floats between frame tables
    int pitch;               // floats per table row (cells*8)
};

struct WindowArgs {
    const float *table;
    long long frame_stride;
    int pitch;
    const int2 *rows;  // (level, y)
    const LevelInfo *levels;
    const ProjPatch *proj;  // [n_levels][K]
    const float4 *w;        // [K][9]: w[0..32] + 3 pad
    const double *bias;     // [K]
    const float *theta;     // [S]
    const int *stage_off;   // [S+1]
    int K, n_stages, step;
    double stride_score;
    sc_det_record *out;
    int capacity;
    int *counters;  // [0] total, [1+f] per frame
    unsigned long long *visited;
    // debug (grid-indexed per frame) -- only written when non-null
    int16_t *dbg_p;
    float *dbg_s;
    uint8_t *dbg_v;
    long long grid_per_frame;
    int lds_nx;  // windows per row the dynamic LDS is sized for
};

void launch_rowscan(const RowScanArgs &a, int n_frames, hipStream_t s);
void launch_colscan(float *table, long long frame_stride, int pitch, int W, int H,
                    int n_frames, hipStream_t s);
void launch_windows(const WindowArgs &a, int n_rows, int n_frames, bool debug, hipStream_t s);
size_t window_lds_bytes(int nx_max);

}  // namespace sc
