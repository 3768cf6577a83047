// sc_kernels.hpp -- launch interface of the gfx950 kernels
// (sc_integral.hip: rowscan, colscan; sc_windows.hip: cascade, walk).
//
// Integral-table layout in HBM ("phase-split"): the reference's table is
// S[y][x][8 channels] (F256Dat, DenseSURFFeatureExtractor.h:21-25).  Windows
// of one row sit at x = step*j, so the corner a weak classifier reads for
// window j is at x = step*j + off: always the same phase off % step.  We store
// each table row as `step` phase planes of Qp cells, so consecutive windows
// read consecutive cells.  Two cell formats (TableGeom::cs/hs):
//   interleaved (cs 2): a cell is 32 B, channels 0-7 together
//       float4 (y, x, half) = y*rowp + 2*((x%step)*Qp + x/step) + half
//   channel-split (cs 1): halves (channels 0-3 | 4-7) in separate planes
//       float4 (y, x, half) = y*rowp + (half*step + x%step)*Qp + x/step
// Values are bit-identical to the reference table; only the addressing
// differs (sc_debug_dump converts back).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "surfcascade.h"

// Timing ablations (segments that start without their hand-off, walks that
// store nothing, extra round trips / exp per item) give wrong results or
// deliberately slow the kernels: a build that sets one must say it is an
// ablation build, and then reports it (sc_build_info "ablation": true).
#if !defined(SC_ABLATION_BUILD) &&                                                   \
    ((defined(SC_ABL_NOWAIT) && SC_ABL_NOWAIT) || (defined(SC_ABL_EXTRA_RT) && SC_ABL_EXTRA_RT) || \
     (defined(SC_ABL_EXTRA_EXP) && SC_ABL_EXTRA_EXP) || defined(SC_NO_WALK) ||                    \
     (defined(SC_WALK_STORE) && SC_WALK_STORE == 0))
#error "timing ablation flag set: build with -DSC_ABLATION_BUILD (never the product library)"
#endif

namespace sc {

constexpr int kXcds = 8;        // MI355X: 8 XCDs, one L2 each
constexpr int kQueueStride = 64;  // ints between per-XCD queue words (own 256-B line each)
constexpr int kMaxSubQ = 8;       // chain kernel: dequeue counters per XCD queue, at most
constexpr int kQueueWords = kXcds * kMaxSubQ * kQueueStride;  // the queue buffer
// chain kernel: segments per row, chosen per launch (WalkArgs::nseg, a power
// of 2 dividing kXcds); XCD x serves segment x / (kXcds / nseg) and, of that
// segment, part x % (kXcds / nseg) of the row list (contiguous parts)

struct TableGeom {
    int W, H, step;
    int ph;    // phase planes per row half: step, or 2*step (windows of one parity adjacent)
    int Qp;    // cells per phase plane (>= ceil((W+1)/ph), multiple of 16)
    int rowp;  // float4 per table row = 2*ph*Qp
    int cs;    // float4 per cell step: 1 (channel-split halves) or 2 (8 channels together)
    int hs;    // float4 from a cell's channels 0-3 to its channels 4-7: ph*Qp or 1
    long long frame4;  // float4 per frame table = (H+1)*rowp
    unsigned phm;      // ceil(2^32 / ph): x / ph = umulhi(x, phm) for the columns of a frame (host check)
    // float4 index of (x, half) within a table row
    __host__ __device__ int at(int x, int h) const {
        return cs * ((x % ph) * Qp + x / ph) + h * hs;
    }
    // at(x, 0) with the division by ph as a multiply-high (kernels)
    __device__ __forceinline__ int at0(unsigned x) const {
        const unsigned q = __umulhi(x, phm);
        return cs * ((int)(x - q * (unsigned)ph) * Qp + (int)q);
    }
    // origin cell of grid window j (x = step*j) within its table row: windows
    // of one parity sit in consecutive cells when ph = 2*step
    __host__ __device__ int win_cell(int j) const {
        return ph == step ? cs * j : cs * ((j & 1) * step * Qp + (j >> 1));
    }
};

// One scale level of the window pyramid (ObjDetector.cpp:178-182).
struct LevelInfo {
    int l, lh;            // window width / height
    int nx, ny;           // grid windows per row / rows
    long long grid_base;  // first grid index of the level (canonical order)
    float thr;            // (float)(l*lh) * prefilter_k   (ObjDetector.cpp:188)
    int pre_col[2];       // cell of column x+l relative to x, by window parity
    int pre_row;          // lh*rowp
    float scale;          // (float)l / tmpl_w   (DenseSURFFeatureExtractor.cpp:463)
    int pad;
};

// A fitted patch projected to one level (ProjectPatches + GetRectsFromPatch,
// DenseSURFFeatureExtractor.cpp:459-484, 360-377), as table offsets relative
// to the window's origin cell.  shape 0: 2x2 cells, 1: 1x4 (tall), 2: 4x1.
struct ProjPatch {
    int shape;
    int row0;     // dy*rowp
    int rowstep;  // c*rowp
    int col[5];   // ((dx+i*c)%step)*Qp + (dx+i*c)/step, i = 0..gw
    __device__ __forceinline__ int colq(int q) const { return col[q]; }
};

// A fitted patch as the template rect it was projected from: the chain
// kernel projects it per item (ProjectPatches :459-484 + GetRectsFromPatch
// :360-377, the same f32 multiplies and truncations as the host table) from
// a 16-B record in LDS instead of fetching a ProjPatch from HBM: one
// dependent global round trip less per item.
//   x = px, y = py, z = the template side ProjectPatches scales (ph for
//   square / wide, pw for tall), w = shape (0 2x2, 1 1x4 tall, 2 4x1 wide)
struct InlinePatch {
    int shape, row0, rowstep;
    int x0;   // window column of the patch's left edge + the parity base column
    int c;    // cell side
    int cb;   // at0(parity base column)
    unsigned phm;
    int ph, Qp, cs;  // TableGeom (wave-uniform)
    __device__ __forceinline__ int colq(int q) const {
        const unsigned x = (unsigned)(x0 + q * c), qq = __umulhi(x, phm);
        return cs * ((int)(x - qq * (unsigned)ph) * Qp + (int)qq) - cb;
    }
};

constexpr int kStrip = 32;  // integral passes: pixels per strip (per 32-lane half wave)

struct RowScanArgs {
    const uint8_t *frames;
    long long frame_bytes;  // distance between frames
    int stride;             // bytes per image row
    float4 *table;
    TableGeom g;
    uint32_t *carry;        // [frame][H][ceil(W/kStrip)][8] exclusive strip prefixes
    // int arrays the step needs zeroed (counters, queues, hand-off words):
    // rowcarry's workgroups clear them on the way instead of one fill
    // dispatch each
    int *zero[4];
    long long zero_n[4];
    int rfull_n;  // rowcarry4: frames [0, rfull_n) also get their exact row prefixes R written
                  // into the table (the two-pass column pass's input; rowfull then skipped)
    uint32_t *colblk;  // one-frame column pass in row segments (colseg): exact 32-row column
                       // sums, [ceil(H/32)][rowp*4] (null: colsum4)
};

// Cascade kernel: persistent workgroups of 4 independent waves; a task is
// one strip (1/(8*n_sub) of a row's windows) of a band of up to band_rows
// consecutive grid rows of one (frame, level).  XCD x serves the strips
// [x*n_sub, (x+1)*n_sub) of every band from its own queue (steals from the
// others when empty), so the rows its L2 sees stay in a narrow column band.
// One strip of one band, precomputed on the host (one load per task).
struct TaskDesc {
    int t_off;    // table offset (float4) of the band's first row: y*rowp
    int g_off;    // grid index (within a frame) of the strip's first window
    int nw;       // windows per row of the strip (0: empty strip)
    int nr;       // grid rows in the band
    int g_row;    // grid index distance between the band's rows (= level nx)
    int level;
    float thr;    // prefilter threshold (float)(l*lh)*k   (ObjDetector.cpp:188)
    int pre_row;  // lh*rowp
    int pre_col[2];  // LevelInfo::pre_col
    int j0;       // the strip's first window in its row
    int pad;
};

struct CascadeArgs {
    const float4 *table;
    TableGeom g;
    const TaskDesc *tasks;  // [n_bands][kXcds*n_sub]
    const ProjPatch *proj;  // [n_levels][2 parities][K]
    const int4 *rects;      // [K]: template rect record of each weak (InlinePatch)
    const float4 *w;        // [K][9]: w[0..32] + 3 pad
    const double *bias;     // [K]
    const float *theta;     // [S]
    const int *stage_off;   // [S+1]
    const int16_t *order;   // [K]: per stage, local weak indices sorted by patch shape
    int K, n_stages;
    int chunk_min;          // survivors from which a stage runs one lane per window
    int n_bands, n_frames, n_sub;
    int strip_max;          // max windows per row of one strip (LDS sizing)
    int band_rows;          // max grid rows per band
    long long grid_per_frame;
    int *queues;            // [kXcds] task counters, zeroed per launch
    int8_t *st_p;           // [frame][grid]: stage reached (-1 prefilter reject)
    float *st_s;            // [frame][grid]: last stage score
};

// Walk kernel: one wave per (frame, row); the adaptive-stride x chain over
// the row's per-window results (ObjDetector.cpp:185-217).
struct WalkArgs {
    const int2 *rows;
    const LevelInfo *levels;
    int n_rows, n_stages, step;
    int n_levels;
    double stride_score;
    long long grid_per_frame;
    const int8_t *st_p;
    const float *st_s;
    sc_det_record *out;
    int capacity;
    int *counters;  // [0] total, [1+f] per frame
    unsigned *row_visited;  // [frame][row] words; their sum = windows the x chain visited (walk kernel: per row)
    uint8_t *dbg_v;  // optional [frame][grid] visited flags
    int row_max;     // chain kernel: most windows in one row segment (LDS sizing)
    int *entry;      // chain kernel: [frame*rows][kXcds] chain entry + 1 per segment (zeroed)
    int *err;        // chain kernel: hand-off timeouts, summed over launches and calls (must stay 0)
    int *err_host;   // chain kernel: 1 once err is raised, in mapped host memory (sc_synchronize reads it
                     // after the stream drains, with no device copy)
    int *fired;      // chain kernel: this launch's watchdog has fired (zeroed per launch)
    int *spec;       // chain kernel: speculative rounds of this launch (zeroed per launch)
    int drop_task1;  // test only: row task + 1 whose segment-0 hand-off is dropped (0: none)
    int drop_walk1;  // test only: fused column walk + 1 whose completion count is dropped (0: none)
    int frame0;      // chain kernel: first frame of this launch (record frame index)
    int nseg;        // chain kernel: segments per row (8; 4 for one-frame launches)
    int seg_shift;   // chain kernel: log2(kXcds / nseg)
    int subq;        // chain kernel: dequeue counters per XCD queue (1..kMaxSubQ; 4 for one-frame launches)
    int n_wide;      // chain kernel, SC_WIDECAP builds: the last n_wide rows of `rows` are the wide levels',
                     // dealt from their own queue (sub-queue word kMaxSubQ - 1); 0: one list
    int wide_cap;    // ... at most wide_cap of a CU's task slots hold a wide row while narrow rows are left
    int spec_max;    // chain kernel, one-frame launches: speculative rounds per waiting task (2*kBatch windows each)
    int slots;       // chain kernel: task slots a wave fills (1 or kSlots = 2)
    unsigned long long *prof;  // chain kernel, SC_PROF_CHAIN builds: phase cycle totals (or null)
    // Fused integral (chain kernel): colstrip's column walks of frames
    // [int_f0, n_frames) of this launch run inside the chain kernel as a
    // second task type; frames below int_f0 have their tables already.
    // The walk = colstrip_kernel's (frame, 64-column strip, half) walk.
    const uint8_t *frames;     // this launch's first frame
    long long frame_bytes;
    int stride;
    const uint32_t *carry;     // rowcarry's carries of this launch's first frame
    int int_f0;                // first frame the launch integrates
    int int_walks;             // walks to run: (n_frames - int_f0) * walks_per_frame (0: none)
    int walks_per_frame;       // 2 * ceil(W / 64)
    int *int_ctl;              // [0] walk dequeue counter, [1 + f] walks finished of frame f (zeroed)
};

// Hard-negative mining (sc_mine.hip, FillNegSamples): candidate selection
// over the cascade kernel's per-window results, then descriptors.
constexpr int kMineBlock = 1024;  // grid windows per selection block

struct MineWindow {
    int frame, level, x, y, l;
    float score;  // last stage score
};

// A batch of n_frames images of one size: per-window results [frame][grid];
// selection blocks of kMineBlock windows never straddle two frames (bpf
// blocks per frame), so block counts also give per-frame counts.
struct MineArgs {
    const int8_t *st_p;
    const float *st_s;
    long long grid;           // windows per frame
    int n_frames, bpf;
    int n_stages, step, n_levels;
    const LevelInfo *levels;
    int *block_count;         // [n_frames * bpf] candidates per block
    int *block_offset;        // [n_frames * bpf] exclusive prefix (device scan), saturated at INT32_MAX
    int *frame_count;         // [1 + n_frames]: [0] all candidates (saturated), [1+f] frame f's
    MineWindow *out;
    int capacity;
};

struct FeatureArgs {
    const float4 *table;  // frame 0's table (frame f's at + f * g.frame4)
    TableGeom g;
    const MineWindow *windows;
    int n_windows, n_patches;
    const int *n_valid;  // when set, *n_valid (saturated total) bounds the windows described
    const ProjPatch *proj_all;  // [n_levels][2 parities][n_patches]: every template patch
    float *out;                 // [n_windows][n_patches][32]
};

void launch_mine_count(const MineArgs &a, hipStream_t s);
void launch_mine_scan(const MineArgs &a, hipStream_t s);
void launch_mine_scatter(const MineArgs &a, hipStream_t s);
void launch_features(const FeatureArgs &a, hipStream_t s);

// integral pass 1 (rowcarry4 / rowcarry), sc_integral.hip; returns whether
// the R rows of frames [0, a.rfull_n) were written (rowcarry4)
// *colblk_done: the one-frame column-block sums (a.colblk) were computed in the same launch
bool launch_rowscan(const RowScanArgs &a, int n_frames, hipStream_t s, bool *colblk_done = nullptr);
// two_pass: rowfull + colsum (small batches; rowfull skipped when have_r), else colstrip
void launch_colscan(const RowScanArgs &a, int n_frames, bool two_pass, hipStream_t s, bool have_r = false,
                    bool colblk_done = false);
int colseg_segments();  // row segments of the one-frame column pass (0: colsum4)
int colblk_rows();      // rows per exact column-block sum of the one-frame column pass
// Per-detector launch configuration: the device's CU count (queried once
// per detector, no process-wide cache) and the SC_OPT_* launch options.
struct LaunchCfg {
    int cus;
    int lds_weights;  // -1 auto, 0 off, 1 on (when the model fits)
    int wgs_per_cu;   // 0: occupancy limit
    int chain_waves;  // chain kernel waves per workgroup: 0 auto (16 when the LDS holds them), 12, 16
};

// returns the number of workgroups launched
int launch_cascade(const CascadeArgs &a, const LaunchCfg &c, hipStream_t s);
void launch_walk(const WalkArgs &a, int n_frames, hipStream_t s);
// Lazy grid: the walk drives the cascade (chain kernel, sc_windows.hip); the
// cascade args' st_p / st_s, when not null, receive the evaluated windows
// (others keep the caller's fill).  Returns the number of workgroups.
int launch_chain(const CascadeArgs &a, const WalkArgs &w, const LaunchCfg &c, hipStream_t s,
                 int *waves_out = nullptr);  // waves_out: the workgroup's waves (12 / 16)
// sc_selftest.hip: exhaustive sqrt_rn / rcp_rn check (sc_selftest_rn).  The
// ranges the shortened sequences are stated for (sc_device.hpp) and checked
// over bit pattern by bit pattern (tests/test_gpu_rn.py); build_geometry
// rejects a frame whose Normalize operands could leave them.
constexpr double kRnSqrtLo = 0x1p-96, kRnSqrtHi = 0x1.fffffep127;  // sqrt_rn: [2^-96, FLT_MAX]
constexpr double kRnRcpLo = 0x1p-20, kRnRcpHi = 0x1p40;            // rcp_rn: [2^-20, 2^40]
void launch_rn_check(int op, uint32_t lo, uint32_t hi, unsigned long long *out, int cus, hipStream_t s);
size_t chain_lds_bytes(int K, int seg_max, int n_levels);
// whether a multi-frame chain launch runs the 16-wave kernel (weights in LDS,
// a table within 128 MiB); otherwise 10 (larger tables) or 12 waves
bool chain_batch_waves16(int K, int row_max, int n_levels, long long frame4);
size_t cascade_lds_bytes(int K, int strip_max, int band_rows);

}  // namespace sc
