// sc_integral.hip -- gfx950 (CDNA4) integral-table kernels of the detect path.
//
// The table S[y][x][c] is OpenCV's integral_ of the 8 T2bFilter gradient
// planes (DenseSURFFeatureExtractor.cpp:73-76, 199-349): the row prefix
// R_y[x] = sum_{x'<x} g_c(y, x') is an exact integer, the column sum is the
// f32 recurrence S[y+1][x] = fl(S[y][x] + R_y[x]) taken sequentially in y
// (SURVEY.md App. A.2).  Two passes, the table written exactly once:
//   rowcarry : one wave per (frame, row): gradients of the row in strips of
//              kStrip pixels; exclusive per-strip prefix ("carry") of the 8
//              channels (u32, exact) -> carry[frame][y][strip][8].  Also
//              zeroes table row 0 and column 0.
//   colstrip : one wave per (frame, 64-px strip, channel half): for y =
//              0..H-1 the strip's gradients again, an exact in-strip prefix
//              (wave scan) plus the carry gives R_y, then S += R_y in f32 --
//              the reference's association order -- and one store per table
//              half-cell.
// rowcarry lanes = half*32 + column, colstrip lanes = column; half 0 owns
// channels 0-3 (dx, dy), half 1 channels 4-7 (du, dv): one table half-cell.
//
// Every f32 operation is the one the reference performs, in its order;
// compiled with -ffp-contract=off, no fast-math.  Table layout: sc_kernels.hpp.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "sc_integral_dev.hpp"
#include "sc_kernels.hpp"

namespace sc {

namespace {

using namespace idev;

#ifndef SC_COL_UNROLL
#define SC_COL_UNROLL 16
#endif
constexpr int kColUnroll = SC_COL_UNROLL;  // rows per colstrip block (two blocks of loads in flight)
#ifndef SC_COL_WAVES  // colstrip: waves per SIMD the register budget must allow
#define SC_COL_WAVES 1
#endif

#ifndef SC_COLBLK  // one-frame column pass: rows per exact column-block sum (colseg's starts)
#define SC_COLBLK 32
#endif
constexpr int kColBlk = SC_COLBLK;

#ifndef SC_RC_ROWS  // rowcarry: rows (waves) per workgroup
#define SC_RC_ROWS 1
#endif
constexpr int kRcRows = SC_RC_ROWS;

__global__ __launch_bounds__(64 * kRcRows) void rowcarry_kernel(RowScanArgs a) {
    const int y = blockIdx.x * kRcRows + (int)(threadIdx.x >> 6), frame = blockIdx.y, lane = threadIdx.x & 63;
    const int h = lane >> 5, c = lane & 31;
    const TableGeom g = a.g;
    const int W = g.W, H = g.H, ns = (W + kStrip - 1) / kStrip;
    {   // the step's zeroed int arrays, grid-strided over the workgroups
        const long long nt = (long long)gridDim.x * gridDim.y * 64 * kRcRows;
        const long long i0 = ((long long)blockIdx.y * gridDim.x + blockIdx.x) * 64 * kRcRows + threadIdx.x;
#pragma unroll
        for (int k = 0; k < 4; k++)
            for (long long i = i0; i < a.zero_n[k]; i += nt) a.zero[k][i] = 0;
    }
    if (y >= H) return;
    const uint8_t *img = a.frames + (long long)frame * a.frame_bytes;
    float4 *tab = a.table + (long long)frame * g.frame4;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (y == 0)  // table row 0 is all zeros
        for (int i = lane; i < g.rowp; i += 64) tab[i] = z4;
    if (lane < 2) tab[(long long)(y + 1) * g.rowp + lane * g.hs] = z4;  // column 0

    uint4 *out = reinterpret_cast<uint4 *>(a.carry) + ((long long)frame * H + y) * ns * 2 + h;
    uint32_t run[4] = {0u, 0u, 0u, 0u};
#ifndef SC_RC_KB
#define SC_RC_KB 4
#endif
    constexpr int kB = SC_RC_KB;  // strips whose pixel loads are in flight together
    for (int s0 = 0; s0 < ns; s0 += kB) {
        Px4 px[kB];
#pragma unroll
        for (int k = 0; k < kB; k++) {
            const int x = min((s0 + k) * kStrip + c, W - 1);
            px[k] = load_px(img, a.stride, W, H, y, x, h);
        }
#pragma unroll
        for (int k = 0; k < kB; k++) {
            const int s = s0 + k;
            if (s >= ns) break;
            uint2 p = (s * kStrip + c < W) ? grad_packed(px[k]) : make_uint2(0u, 0u);
            // strip totals of each 32-lane half: its scan's last lane
            p.x = half_scan(p.x);
            p.y = half_scan(p.y);
            const uint32_t tx = h ? __builtin_amdgcn_readlane(p.x, 63) : __builtin_amdgcn_readlane(p.x, 31);
            const uint32_t ty = h ? __builtin_amdgcn_readlane(p.y, 63) : __builtin_amdgcn_readlane(p.y, 31);
            if (c == 0) out[(long long)s * 2] = make_uint4(run[0], run[1], run[2], run[3]);
            run[0] += tx & 0xffffu;
            run[1] += tx >> 16;
            run[2] += ty & 0xffffu;
            run[3] += ty >> 16;
        }
    }
}

// rowcarry with dword pixel loads (frames whose rows start 4-B aligned):
// one wave per (row, frame), 4 columns per lane, 256 columns per pass.  The
// byte-load form issues 4 loads per lane per 32-column strip and is bound by
// the texture-address unit (TA busy ~80 % of its time: one instruction costs
// the same whatever it moves); here a pass is 3 dword loads per lane (rows
// y-1, y, y+1), the x-1 / x+4 neighbours come from the adjacent lanes by DPP
// wave shifts (the pass's edges from the neighbouring passes), and the 8
// channel sums of a lane's 4 columns go through one wave scan per channel
// pair.  Same gradients, same exact u32 strip carries as rowcarry_kernel.
__device__ __forceinline__ uint32_t byte_of(unsigned long long w, int i) {
    return (uint32_t)(w >> (8 * i)) & 0xffu;
}

// the step's zeroed int arrays, grid-strided over the launch's threads
__device__ __forceinline__ void zero_arrays(const RowScanArgs &a, long long i0, long long nt) {
#pragma unroll
    for (int k = 0; k < 4; k++)
        for (long long i = i0; i < a.zero_n[k]; i += nt) a.zero[k][i] = 0;
}

// a row's dword at x0 (4-B aligned: frame and stride are); the row's last
// partial dword byte by byte, so no load reads past column W - 1 (a device
// caller's buffer may end at the last row's W-th byte).  The bytes past W
// read as 0 and are never used (x = W - 1 clamps x + 1 to itself).
__device__ __forceinline__ uint32_t ld4(const uint8_t *row, int x0, int W) {
    if (x0 + 4 <= W) return *reinterpret_cast<const uint32_t *>(row + x0);
    uint32_t v = 0u;
    for (int k = 0; k < 4 && x0 + k < W; k++) v |= (uint32_t)row[x0 + k] << (8 * k);
    return v;
}

// bytes x0-1 .. x0+4 of a row around this lane's dword v (lanes l-1 / l+1 by
// wave_shr / wave_shl; lane 0's left byte and lane 63's right byte come in)
__device__ __forceinline__ unsigned long long byte_window(uint32_t v, uint32_t left, uint32_t right) {
    const uint32_t l = (uint32_t)__builtin_amdgcn_update_dpp((int)(left << 24), (int)v, 0x138, 0xf, 0xf, false) >> 24;
    const uint32_t r = (uint32_t)__builtin_amdgcn_update_dpp((int)right, (int)v, 0x130, 0xf, 0xf, false) & 0xffu;
    return ((unsigned long long)r << 40) | ((unsigned long long)v << 8) | l;
}

// The 8 T2bFilter gradients of column x0 + j (j = 0..3) from the byte
// windows of rows y-1, y, y+1, accumulated into G (x = W-1: x+1 clamps to x)
__device__ __forceinline__ void grad8(unsigned long long U, unsigned long long C, unsigned long long D, int j,
                                      bool last, uint32_t (&G)[8]) {
    const int il = j, im = j + 1, ir = last ? j + 1 : j + 2;
    // half 0: (C[x-1], C[x+1]), (U[x], D[x]); half 1: (U[x-1], D[x+1]), (D[x-1], U[x+1])
    const uint32_t a0 = byte_of(C, il), b0 = byte_of(C, ir), c0_ = byte_of(U, im), d0_ = byte_of(D, im);
    const uint32_t a1 = byte_of(U, il), b1 = byte_of(D, ir), c1_ = byte_of(D, il), d1_ = byte_of(U, ir);
    G[0] += sat_sub(a0, b0); G[1] += sat_sub(b0, a0); G[2] += sat_sub(c0_, d0_); G[3] += sat_sub(d0_, c0_);
    G[4] += sat_sub(a1, b1); G[5] += sat_sub(b1, a1); G[6] += sat_sub(c1_, d1_); G[7] += sat_sub(d1_, c1_);
}

__device__ __forceinline__ void rowcarry4_row(const RowScanArgs &a, int y, int frame, int lane) {
    const TableGeom g = a.g;
    const int W = g.W, H = g.H, ns = (W + kStrip - 1) / kStrip;
    const uint8_t *img = a.frames + (long long)frame * a.frame_bytes;
    float4 *tab = a.table + (long long)frame * g.frame4;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (y == 0)  // table row 0 is all zeros
        for (int i = lane; i < g.rowp; i += 64) tab[i] = z4;
    if (lane < 2) tab[(long long)(y + 1) * g.rowp + lane * g.hs] = z4;  // column 0

    const uint8_t *ru = img + (long long)(y > 0 ? y - 1 : 0) * a.stride;
    const uint8_t *rc = img + (long long)y * a.stride;
    const uint8_t *rd = img + (long long)(y < H - 1 ? y + 1 : H - 1) * a.stride;
    uint4 *out = reinterpret_cast<uint4 *>(a.carry) + ((long long)frame * H + y) * ns * 2;
    const int np = (W + 255) / 256;
    // a pass's dwords (rows u, c, d), loaded one pass ahead
    auto load = [&](int p, uint32_t &u, uint32_t &c, uint32_t &d) {
        const int x0 = p * 256 + 4 * lane;
        u = c = d = 0u;
        if (p < np && x0 < W) {
            u = ld4(ru, x0, W);
            c = ld4(rc, x0, W);
            d = ld4(rd, x0, W);
        }
    };
    uint32_t u0, c0, d0;
    load(0, u0, c0, d0);
    // the byte left of the pass (x0 - 1 of lane 0): the previous pass's last;
    // x = 0 clamps to itself
    uint32_t lu = u0 & 0xffu, lc = c0 & 0xffu, ld = d0 & 0xffu;
    uint32_t run[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    // frames whose column pass is colsum (two-pass): their R rows are written
    // here, so rowfull_kernel does not run for them
    const bool write_r = frame < a.rfull_n;
    for (int p = 0; p < np; p++) {
        uint32_t u1, c1, d1;
        load(p + 1, u1, c1, d1);
        // the byte right of the pass (x0 + 4 of lane 63): the next pass's first
        const uint32_t nu = (uint32_t)__builtin_amdgcn_readlane((int)u1, 0) & 0xffu;
        const uint32_t nc = (uint32_t)__builtin_amdgcn_readlane((int)c1, 0) & 0xffu;
        const uint32_t nd = (uint32_t)__builtin_amdgcn_readlane((int)d1, 0) & 0xffu;
        const unsigned long long U = byte_window(u0, lu, nu), C = byte_window(c0, lc, nc), D = byte_window(d0, ld, nd);
        const int x0 = p * 256 + 4 * lane;
        uint32_t G[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
        uint32_t Pc[4][8];  // the lane's inclusive prefix through column j (R rows: rowfull's cells)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int x = x0 + j;
            if (x < W) grad8(U, C, D, j, x + 1 >= W, G);
#pragma unroll
            for (int ch = 0; ch < 8; ch++) Pc[j][ch] = G[ch];
        }
        // 16-bit channel pairs: a pass's prefix stays < 64 x 4 x 255 < 2^16
        uint32_t q[4] = {G[0] | (G[1] << 16), G[2] | (G[3] << 16), G[4] | (G[5] << 16), G[6] | (G[7] << 16)};
        uint32_t e[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t incl = wave_scan(q[k]);
            e[k] = incl - q[k];  // exclusive: the columns of the pass left of this lane
            q[k] = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);  // the pass's totals
        }
        if (write_r) {  // R_y[x+1] = the exact row prefix through column x, into table row y+1
            float4 *trow = tab + (long long)(y + 1) * g.rowp;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int x = x0 + j;
                if (x < W) {
                    uint4 r0, r1;
                    r0.x = run[0] + (e[0] & 0xffffu) + Pc[j][0]; r0.y = run[1] + (e[0] >> 16) + Pc[j][1];
                    r0.z = run[2] + (e[1] & 0xffffu) + Pc[j][2]; r0.w = run[3] + (e[1] >> 16) + Pc[j][3];
                    r1.x = run[4] + (e[2] & 0xffffu) + Pc[j][4]; r1.y = run[5] + (e[2] >> 16) + Pc[j][5];
                    r1.z = run[6] + (e[3] & 0xffffu) + Pc[j][6]; r1.w = run[7] + (e[3] >> 16) + Pc[j][7];
                    reinterpret_cast<uint4 *>(trow)[g.at(x + 1, 0)] = r0;
                    reinterpret_cast<uint4 *>(trow)[g.at(x + 1, 1)] = r1;
                }
            }
        }
        const int s = p * 8 + (lane >> 3);  // 32-column strip starting at this lane (lane % 8 == 0)
        if ((lane & 7) == 0 && s < ns) {
            out[(long long)s * 2] = make_uint4(run[0] + (e[0] & 0xffffu), run[1] + (e[0] >> 16),
                                               run[2] + (e[1] & 0xffffu), run[3] + (e[1] >> 16));
            out[(long long)s * 2 + 1] = make_uint4(run[4] + (e[2] & 0xffffu), run[5] + (e[2] >> 16),
                                                   run[6] + (e[3] & 0xffffu), run[7] + (e[3] >> 16));
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            run[2 * k] += q[k] & 0xffffu;
            run[2 * k + 1] += q[k] >> 16;
        }
        lu = (uint32_t)__builtin_amdgcn_readlane((int)u0, 63) >> 24;
        lc = (uint32_t)__builtin_amdgcn_readlane((int)c0, 63) >> 24;
        ld = (uint32_t)__builtin_amdgcn_readlane((int)d0, 63) >> 24;
        u0 = u1; c0 = c1; d0 = d1;
    }
}

__global__ __launch_bounds__(64) void rowcarry4_kernel(RowScanArgs a) {
    zero_arrays(a, ((long long)blockIdx.y * gridDim.x + blockIdx.x) * 64 + threadIdx.x,
                (long long)gridDim.x * gridDim.y * 64);
    rowcarry4_row(a, blockIdx.x, blockIdx.y, threadIdx.x);
}

// One frame: rowcarry4's rows and the exact kColBlk-row column-block sums of
// the R rows (colseg's segment starts) in ONE launch.  A block sum is computed
// from the pixels, not from the R rows rowcarry writes, so the two roles are
// independent: sum_{y in blk} R_y(x+1) = sum_{x' <= x} (sum_{y in blk}
// g_y(x')), i.e. the block's column sums of the 8 gradient planes, prefixed
// along x once per block instead of once per row (exact u32: at most kColBlk
// * 255 * W).  Workgroups [0, n_row_wg) are rowcarry4's (kRcbWaves rows each),
// the others one block each: wave w takes the 256-column passes w, w +
// kRcbWaves, ...; a pass's totals cross the waves through LDS for the
// carry of the passes to its right.  Replaces colblock_kernel's launch and
// its read of the R rows (50 MB at 1080p) by a read of the block's pixels.
#ifndef SC_RCB_WAVES  // merged rowcarry4 + block-sum launch: waves per workgroup
#define SC_RCB_WAVES 8  // (one frame: rowscan + colseg 0.0608 ms; 4: 0.0724, 16: 0.0665; profiles/r5/f)
#endif
constexpr int kRcbWaves = SC_RCB_WAVES;
#ifndef SC_CB_ROWS  // block role: image rows whose loads are in flight together
#define SC_CB_ROWS 8
#endif
constexpr int kCbRows = SC_CB_ROWS;
__device__ __forceinline__ void colblk_pixels(const RowScanArgs &a, int bb, int wv, int lane) {
    const TableGeom g = a.g;
    const int W = g.W, H = g.H, np = (W + 255) / 256;
    const int y0 = bb * kColBlk, y1 = min(H, y0 + kColBlk);
    const long long rs = (long long)g.rowp * 4;  // floats per table row (colblk's row stride)
    __shared__ uint32_t s_tot[kRcbWaves][8];      // this chunk's pass totals
    __shared__ uint32_t s_run[8];                 // the totals of the chunks done
    if (threadIdx.x < 8) s_run[threadIdx.x] = 0u;
    for (int c0 = 0; c0 < np; c0 += kRcbWaves) {
        const int p = c0 + wv, x0 = p * 256 + 4 * lane;
        uint32_t S[4][8];  // the block's column sums of the lane's 4 columns
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int ch = 0; ch < 8; ch++) S[j][ch] = 0u;
        if (p < np) {
            // lane 0's left byte: the previous pass's last (x = 0: itself);
            // lane 63's right byte: the next pass's first
            const int xl = p > 0 ? p * 256 - 1 : 0, xr = (p + 1) * 256;
            for (int yb = y0; yb < y1; yb += kCbRows) {
                // rows yb-1 .. yb+kCbRows (clamped like rowcarry's): loads first,
                // in flight together, then the rows' gradients
                uint32_t dw[kCbRows + 2], lb[kCbRows + 2], rb[kCbRows + 2];
#pragma unroll
                for (int k = 0; k < kCbRows + 2; k++) {
                    const int yy = min(max(yb - 1 + k, 0), H - 1);
                    const uint8_t *row = a.frames + (long long)yy * a.stride;
                    dw[k] = x0 < W ? ld4(row, x0, W) : 0u;
                    lb[k] = row[xl];  // (wave-uniform; as scalar loads: +22 % rowscan, profiles/r5/h)
                    rb[k] = xr < W ? row[xr] : 0u;
                }
#pragma unroll
                for (int k = 0; k < kCbRows; k++) {
                    if (yb + k >= y1) break;
                    const unsigned long long Uw = byte_window(dw[k], lb[k], rb[k]);
                    const unsigned long long Cw = byte_window(dw[k + 1], lb[k + 1], rb[k + 1]);
                    const unsigned long long Dw = byte_window(dw[k + 2], lb[k + 2], rb[k + 2]);
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        if (x0 + j < W) grad8(Uw, Cw, Dw, j, x0 + j + 1 >= W, S[j]);
                }
            }
        }
        // in-pass inclusive prefix along x: the lane's 4 columns, then the wave
        uint32_t E[8], T[8];
#pragma unroll
        for (int ch = 0; ch < 8; ch++) {
            S[1][ch] += S[0][ch];
            S[2][ch] += S[1][ch];
            S[3][ch] += S[2][ch];
            const uint32_t incl = wave_scan(S[3][ch]);
            E[ch] = incl - S[3][ch];  // the pass's columns left of this lane
            T[ch] = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        }
        if (lane == 0)
#pragma unroll
            for (int ch = 0; ch < 8; ch++) s_tot[wv][ch] = p < np ? T[ch] : 0u;
        __syncthreads();
        if (p < np) {
            uint32_t cy[8];  // every column left of this pass, over the block's rows
#pragma unroll
            for (int ch = 0; ch < 8; ch++) {
                cy[ch] = s_run[ch] + E[ch];
                for (int w2 = 0; w2 < wv; w2++) cy[ch] += s_tot[w2][ch];
            }
            uint4 *row = reinterpret_cast<uint4 *>(a.colblk + (long long)bb * rs);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int x = x0 + j;
                if (x < W) {
                    row[g.at(x + 1, 0)] = make_uint4(cy[0] + S[j][0], cy[1] + S[j][1], cy[2] + S[j][2], cy[3] + S[j][3]);
                    row[g.at(x + 1, 1)] = make_uint4(cy[4] + S[j][4], cy[5] + S[j][5], cy[6] + S[j][6], cy[7] + S[j][7]);
                }
            }
        }
        __syncthreads();
        if (threadIdx.x < 8) {
            uint32_t t = 0u;
            for (int w2 = 0; w2 < kRcbWaves; w2++) t += s_tot[w2][threadIdx.x];
            s_run[threadIdx.x] += t;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(64 * kRcbWaves) void rowcarry4_colblk_kernel(RowScanArgs a, int n_row_wg) {
    const int wv = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
    zero_arrays(a, (long long)blockIdx.x * 64 * kRcbWaves + threadIdx.x, (long long)gridDim.x * 64 * kRcbWaves);
    if ((int)blockIdx.x < n_row_wg) {  // (the whole workgroup takes one role: the barriers below are the block role's)
        const int y = (int)blockIdx.x * kRcbWaves + wv;
        if (y < a.g.H) rowcarry4_row(a, y, 0, lane);
        return;
    }
    colblk_pixels(a, (int)blockIdx.x - n_row_wg, wv, lane);
}

#ifndef SC_COL_XCD
#define SC_COL_XCD 1
#endif
// Which (frame, half, strip) a column-walk workgroup takes.  The hardware
// deals workgroup b (linear id) to XCD b % kXcds; with SC_COL_XCD each XCD
// gets a contiguous run of (frame, half, strip) ids instead, strip fastest,
// so the 128-B lines two neighbouring strips share at a phase-plane run's
// ends are written through one L2 (adjacent ids on two XCDs leave two
// partial dirty copies of each such line).
struct ColBlock {
    int s, h, frame;
};
__device__ __forceinline__ ColBlock col_block() {
    const int ns64 = gridDim.x >> 1;
#if SC_COL_XCD
    const int nb = gridDim.x * gridDim.y, b = blockIdx.x + blockIdx.y * gridDim.x;
    const int x = b % kXcds, q = nb / kXcds, r = nb % kXcds;
    const int lb = x * q + min(x, r) + b / kXcds;  // a bijection onto [0, nb)
    const int f = lb / gridDim.x, rem = lb - f * gridDim.x;
    return ColBlock{rem % ns64, rem / ns64, f};
#else
    (void)ns64;
    return ColBlock{(int)blockIdx.x >> 1, (int)blockIdx.x & 1, (int)blockIdx.y};
#endif
}

// One wave per (frame, 64-column strip, channel half): lane = column, so a
// row's stores are long runs within each phase plane of the half.
__global__ __launch_bounds__(64, SC_COL_WAVES) void colstrip_kernel(RowScanArgs a) {
    const ColBlock cb_ = col_block();
    const int s = cb_.s, h = cb_.h, frame = cb_.frame, lane = threadIdx.x;
    const TableGeom g = a.g;
    const int W = g.W, H = g.H, ns = (W + kStrip - 1) / kStrip;  // carries per 32-px strip
    const int x = s * 2 * kStrip + lane;
    const bool live = x < W;
    const int xs = live ? x : W - 1;  // dead lanes still join the scan with zeros
    const uint8_t *img = a.frames + (long long)frame * a.frame_bytes;
    float4 *cellp = a.table + (long long)frame * g.frame4 + g.at(x + 1, h);  // row 0 of the column
    // the exclusive carry at column 64*s is the 32-px strip 2*s's
    const uint4 *cin = reinterpret_cast<const uint4 *>(a.carry) + (long long)frame * H * ns * 2 +
                       (long long)(2 * s) * 2 + h;
    // software pipeline: the loads of block b+1 are in flight while block b
    // is scanned and stored
    Px4 pa[kColUnroll];
    uint4 ca[kColUnroll];
    auto load_block = [&](int y0, Px4 (&px)[kColUnroll], uint4 (&cr)[kColUnroll]) {
#pragma unroll
        for (int k = 0; k < kColUnroll; k++) {
            const int y = min(y0 + k, H - 1);
            px[k] = load_px(img, a.stride, W, H, y, xs, h);
            cr[k] = cin[(long long)y * ns * 2];
        }
    };
    load_block(0, pa, ca);
    float S0 = 0.0f, S1 = 0.0f, S2 = 0.0f, S3 = 0.0f;  // table row 0
    for (int y0 = 0; y0 < H; y0 += kColUnroll) {
        Px4 pb[kColUnroll];
        uint4 cb[kColUnroll];
        load_block(y0 + kColUnroll < H ? y0 + kColUnroll : y0, pb, cb);
#pragma unroll
        for (int k = 0; k < kColUnroll; k++) {
            const int y = y0 + k;  // rows past H: harmless extra steps, not stored
            uint2 p = live ? grad_packed(pa[k]) : make_uint2(0u, 0u);
            p.x = wave_scan(p.x);  // 16-bit channel pairs: 64 px x 255 < 2^16
            p.y = wave_scan(p.y);
            // R_y[x+1] exact (< 2^24), then the f32 column step
            S0 = S0 + (float)(ca[k].x + (p.x & 0xffffu));
            S1 = S1 + (float)(ca[k].y + (p.x >> 16));
            S2 = S2 + (float)(ca[k].z + (p.y & 0xffffu));
            S3 = S3 + (float)(ca[k].w + (p.y >> 16));
            if (live && y < H) cellp[(long long)(y + 1) * g.rowp] = make_float4(S0, S1, S2, S3);
        }
#pragma unroll
        for (int k = 0; k < kColUnroll; k++) {
            pa[k] = pb[k];
            ca[k] = cb[k];
        }
    }
}

// Small batches (a single frame's colstrip is 60 waves walking 1080 rows:
// 0.21 ms of latency) split colstrip in two passes over the table:
//   rowfull : one wave per (frame, row, 64-column strip, half): the same
//             gradients, in-strip scan and carry as colstrip, writing the
//             exact row prefix R_y[x+1] (u32 x 4) into the table cell;
//   colsum  : one wave per (frame, strip, half), lane = column: S += (float)R
//             down the column in place, loads of the next rows in flight.
// The f32 operations and their order are colstrip's (S_{y+1} = S_y + R_y);
// the table is written twice and read once, so large batches keep colstrip.
__global__ __launch_bounds__(64) void rowfull_kernel(RowScanArgs a) {
    const int s = blockIdx.x >> 1, h = blockIdx.x & 1, y = blockIdx.y, frame = blockIdx.z, lane = threadIdx.x;
    const TableGeom g = a.g;
    const int W = g.W, H = g.H, ns = (W + kStrip - 1) / kStrip;
    const int x = s * 2 * kStrip + lane;
    const bool live = x < W;
    const uint8_t *img = a.frames + (long long)frame * a.frame_bytes;
    const Px4 px = load_px(img, a.stride, W, H, y, live ? x : W - 1, h);
    uint2 p = live ? grad_packed(px) : make_uint2(0u, 0u);
    p.x = wave_scan(p.x);
    p.y = wave_scan(p.y);
    const uint4 c = reinterpret_cast<const uint4 *>(a.carry)[(((long long)frame * H + y) * ns + 2 * s) * 2 + h];
    const uint4 R = make_uint4(c.x + (p.x & 0xffffu), c.y + (p.x >> 16), c.z + (p.y & 0xffffu), c.w + (p.y >> 16));
    if (live)
        reinterpret_cast<uint4 *>(a.table)[(long long)frame * g.frame4 + (long long)(y + 1) * g.rowp + g.at(x + 1, h)] = R;
}

constexpr int kSumAhead = 16;  // colsum: rows of loads in flight
__global__ __launch_bounds__(64) void colsum_kernel(RowScanArgs a) {
    const ColBlock cb_ = col_block();
    const int s = cb_.s, h = cb_.h, frame = cb_.frame, lane = threadIdx.x;
    const TableGeom g = a.g;
    const int W = g.W, H = g.H;
    const int x = s * 2 * kStrip + lane;
    if (x >= W) return;  // (no cross-lane work in this pass)
    float4 *cellp = a.table + (long long)frame * g.frame4 + g.at(x + 1, h) + g.rowp;  // table row 1
    const uint4 *rp = reinterpret_cast<const uint4 *>(cellp);
    float S0 = 0.0f, S1 = 0.0f, S2 = 0.0f, S3 = 0.0f;
    uint4 ra[kSumAhead];
#pragma unroll
    for (int k = 0; k < kSumAhead; k++) ra[k] = rp[(long long)min(k, H - 1) * g.rowp];
    for (int y0 = 0; y0 < H; y0 += kSumAhead) {
        uint4 rb[kSumAhead];
#pragma unroll
        for (int k = 0; k < kSumAhead; k++) rb[k] = rp[(long long)min(y0 + kSumAhead + k, H - 1) * g.rowp];
#pragma unroll
        for (int k = 0; k < kSumAhead; k++) {
            const int y = y0 + k;
            S0 = S0 + (float)ra[k].x;  // the f32 column step, colstrip's order
            S1 = S1 + (float)ra[k].y;
            S2 = S2 + (float)ra[k].z;
            S3 = S3 + (float)ra[k].w;
            if (y < H) cellp[(long long)y * g.rowp] = make_float4(S0, S1, S2, S3);
        }
#pragma unroll
        for (int k = 0; k < kSumAhead; k++) ra[k] = rb[k];
    }
}

#ifndef SC_COLSUM4
#define SC_COLSUM4 1
#endif
// colsum with one lane per (column, channel): 4 waves per (strip, half), each
// 16 columns x 4 channels, one dword per row and lane, so a lane keeps 4x
// the rows of loads in flight in the same registers (the walk is bound by
// the load latency: 120 walks for a 1080p frame, one per SIMD at most).
#ifndef SC_SUM_AHEAD4
#define SC_SUM_AHEAD4 48
#endif
constexpr int kSumAhead4 = SC_SUM_AHEAD4;
__global__ __launch_bounds__(64) void colsum4_kernel(RowScanArgs a) {
    const int nb = gridDim.x * gridDim.y, b = blockIdx.x + blockIdx.y * gridDim.x;
    const int xq = b % kXcds, q = nb / kXcds, r = nb % kXcds;
    const int lb = xq * q + min(xq, r) + b / kXcds;  // XCD-aware: neighbours through one L2
    const int frame = lb / gridDim.x, rem = lb - frame * gridDim.x;
    const int s = rem >> 3, h = (rem >> 2) & 1, sub = rem & 3, lane = threadIdx.x;
    const TableGeom g = a.g;
    const int W = g.W, H = g.H;
    const int x = s * 2 * kStrip + sub * 16 + (lane >> 2), ch = lane & 3;
    if (x >= W) return;  // (no cross-lane work in this pass)
    float *cellp = reinterpret_cast<float *>(a.table + (long long)frame * g.frame4 + g.at(x + 1, h) + g.rowp) + ch;
    const uint32_t *rp = reinterpret_cast<const uint32_t *>(cellp);
    const long long rs = (long long)g.rowp * 4;  // floats per table row
    float S = 0.0f;
    uint32_t ra[kSumAhead4];
#pragma unroll
    for (int k = 0; k < kSumAhead4; k++) ra[k] = rp[min(k, H - 1) * rs];
    for (int y0 = 0; y0 < H; y0 += kSumAhead4) {
        uint32_t rb[kSumAhead4];
#pragma unroll
        for (int k = 0; k < kSumAhead4; k++) rb[k] = rp[min(y0 + kSumAhead4 + k, H - 1) * rs];
#pragma unroll
        for (int k = 0; k < kSumAhead4; k++) {
            S = S + (float)ra[k];  // the f32 column step, colstrip's order
            if (y0 + k < H) cellp[(y0 + k) * rs] = S;
        }
#pragma unroll
        for (int k = 0; k < kSumAhead4; k++) ra[k] = rb[k];
    }
}

// colsum in table order: a wave owns 64 consecutive floats of every table row
// (8 cells x 8 channels when the 8 channels sit together, 16 cells x 4
// otherwise), lane = (cell, channel), so each row's load and store is two
// whole 128-B lines instead of colsum4's 16 columns spread over the `ph`
// phase planes.  Cells of the plane padding (and column 0) are skipped; the
// per-element f32 step and its order are colsum4's.
#ifndef SC_COLSUM_PLANE
#define SC_COLSUM_PLANE 1
#endif
__global__ __launch_bounds__(64) void colsum_plane_kernel(RowScanArgs a) {
    const TableGeom g = a.g;
    const int frame = blockIdx.y, lane = threadIdx.x;
    const int fi = blockIdx.x * 64 + lane;  // float within a table row
    const int f4 = fi >> 2, plane_cells = g.ph * g.Qp;
    const int ci = g.cs == 2 ? f4 >> 1 : f4 % plane_cells;  // cell index within its half
    const int col = (ci % g.Qp) * g.ph + ci / g.Qp;         // table column (x + 1)
    if (col < 1 || col > g.W) return;  // (no cross-lane work in this pass)
    float *cellp = reinterpret_cast<float *>(a.table + (long long)frame * g.frame4 + g.rowp) + fi;  // table row 1
    const uint32_t *rp = reinterpret_cast<const uint32_t *>(cellp);
    const long long rs = (long long)g.rowp * 4;  // floats per table row
    const int H = g.H;
    float S = 0.0f;
    uint32_t ra[kSumAhead4];
#pragma unroll
    for (int k = 0; k < kSumAhead4; k++) ra[k] = rp[min(k, H - 1) * rs];
    for (int y0 = 0; y0 < H; y0 += kSumAhead4) {
        uint32_t rb[kSumAhead4];
#pragma unroll
        for (int k = 0; k < kSumAhead4; k++) rb[k] = rp[min(y0 + kSumAhead4 + k, H - 1) * rs];
#pragma unroll
        for (int k = 0; k < kSumAhead4; k++) {
            S = S + (float)ra[k];  // the f32 column step, colstrip's order
            if (y0 + k < H) cellp[(y0 + k) * rs] = S;
        }
#pragma unroll
        for (int k = 0; k < kSumAhead4; k++) ra[k] = rb[k];
    }
}

// One frame's column pass in parallel row segments (colblock + colseg).
// colsum4's step S_{y+1} = S_y + (float)R_y is exact while the column's
// running sum stays <= 2^24: the R_y are non-negative integers below 2^24,
// so every partial sum up to that bound is an integer f32 holds exactly.  So
// the wave of segment k ([ya, yb) of 1/SC_COLSEG of the height) starts a
// column from the exact integer sum of the rows above ya (from exact 32-row
// block sums) whenever that sum is <= 2^24.  A column whose sum passes 2^24
// above yb continues in the same wave, step by step in order, down to row H;
// the later segments leave it alone (each row is read and written by one
// wave only: the pass is in place).  The same bits as the sequential walk for
// every input; the walk is as long as the column's last exact segment start
// allows (a 1080p bench frame passes 2^24 from row 939 on).
// row segments: 5 (column pass 0.0314 ms per 1080p frame with the block sums
// from rowcarry4's launch; 4: 0.0334, 3: 0.0385, profiles/r5/h; colsum4's one
// walk: 0.053).  More segments start later rows, and a column whose sum has
// passed 2^24 above a start is walked on by its last exact segment: at 6 the
// bench frames' last start (row 960) is past their 2^24 crossing (row 939)
#ifndef SC_COLSEG
#define SC_COLSEG 5
#endif
__global__ __launch_bounds__(64) void colblock_kernel(RowScanArgs a) {
    const TableGeom g = a.g;
    const int fi = blockIdx.x * 64 + threadIdx.x, blk = blockIdx.y;  // float within a table row
    const int y0 = blk * kColBlk, y1 = min(g.H, y0 + kColBlk);
    const long long rs = (long long)g.rowp * 4;
    const uint32_t *rp = reinterpret_cast<const uint32_t *>(a.table + g.rowp) + fi;  // R_y at table row y+1
    uint32_t s = 0u;  // (< 32 * 255 * W: exact; padding cells sum garbage nobody reads)
#pragma unroll 8
    for (int y = y0; y < y1; y++) s += rp[y * rs];
    a.colblk[blk * rs + fi] = s;
}

__global__ __launch_bounds__(64) void colseg_kernel(RowScanArgs a, int seg_len) {
    const TableGeom g = a.g;
    const int lane = threadIdx.x, fi = blockIdx.x * 64 + lane;
    const int H = g.H, ya = blockIdx.y * seg_len, yb = min(H, ya + seg_len);
    const int f4 = fi >> 2, plane_cells = g.ph * g.Qp;
    const int ci = g.cs == 2 ? f4 >> 1 : f4 % plane_cells;  // colsum_plane's cell -> column map
    const int col = (ci % g.Qp) * g.ph + ci / g.Qp;
    const bool live = col >= 1 && col <= g.W && ya < H;
    float *cellp = reinterpret_cast<float *>(a.table + g.rowp) + fi;
    const uint32_t *rp = reinterpret_cast<const uint32_t *>(cellp);
    const long long rs = (long long)g.rowp * 4;
    // exact sums above ya and above yb (yb < H: a multiple of kColBlk)
    unsigned long long ea = 0ull, eb = 0ull;
    if (live) {
        for (int i = 0; i < ya / kColBlk; i++) ea += a.colblk[i * rs + fi];
        eb = ea;
        if (yb < H)
            for (int i = ya / kColBlk; i < yb / kColBlk; i++) eb += a.colblk[i * rs + fi];
    }
    const bool act = live && ea <= (1ull << 24);            // this segment starts the column exactly
    const int end = !act ? ya : (yb < H && eb <= (1ull << 24)) ? yb : H;  // else it walks on to H
    int ye = end;  // the wave's last row (all lanes take part: no early exit above)
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) ye = max(ye, __shfl_xor(ye, o));
    ye = __builtin_amdgcn_readfirstlane(ye);
    if (!act) return;  // (no cross-lane work below)
    float S = (float)(uint32_t)ea;  // exact
    uint32_t ra[kSumAhead4];  // colsum4's walk over [ya, end)
#pragma unroll
    for (int k = 0; k < kSumAhead4; k++) ra[k] = rp[min(ya + k, end - 1) * rs];
    for (int y0 = ya; y0 < ye; y0 += kSumAhead4) {
        uint32_t rb[kSumAhead4];
#pragma unroll
        for (int k = 0; k < kSumAhead4; k++) rb[k] = rp[min(y0 + kSumAhead4 + k, end - 1) * rs];
#pragma unroll
        for (int k = 0; k < kSumAhead4; k++) {
            S = S + (float)ra[k];
            if (y0 + k < end) cellp[(y0 + k) * rs] = S;
        }
#pragma unroll
        for (int k = 0; k < kSumAhead4; k++) ra[k] = rb[k];
    }
}

}  // namespace

int colseg_segments() { return SC_COLSEG; }
int colblk_rows() { return kColBlk; }

#ifndef SC_RC_DWORD  // rowcarry4 (dword loads) when the rows start 4-B aligned
#define SC_RC_DWORD 1
#endif
// colseg's row segments for a frame of height H: seg rows each (a multiple of
// kColBlk), nseg of them; block sums are needed above the last one's start
__host__ __device__ inline void colseg_geometry(int H, int &seg, int &nseg) {
    seg = ((H + SC_COLSEG - 1) / SC_COLSEG + kColBlk - 1) / kColBlk * kColBlk;
    nseg = (H + seg - 1) / seg;
}

#ifndef SC_RC_COLBLK  // one frame: the column-block sums inside rowcarry4's launch (from the pixels)
#define SC_RC_COLBLK 1
#endif
bool launch_rowscan(const RowScanArgs &a, int n_frames, hipStream_t s, bool *colblk_done) {
    const bool aligned = ((uintptr_t)a.frames & 3u) == 0 && (a.stride & 3) == 0;
    if (colblk_done) *colblk_done = false;
    if (SC_RC_DWORD && aligned) {
        int seg = 0, nseg = 0;
        colseg_geometry(a.g.H, seg, nseg);
        if (SC_RC_COLBLK && SC_COLSEG > 1 && n_frames == 1 && a.colblk && nseg > 1) {
            const int n_row_wg = (a.g.H + kRcbWaves - 1) / kRcbWaves, nblk = (nseg - 1) * seg / kColBlk;
            hipLaunchKernelGGL(rowcarry4_colblk_kernel, dim3(n_row_wg + nblk), dim3(64 * kRcbWaves), 0, s, a,
                               n_row_wg);
            if (colblk_done) *colblk_done = true;
            return a.rfull_n > 0;
        }
        hipLaunchKernelGGL(rowcarry4_kernel, dim3(a.g.H, n_frames), dim3(64), 0, s, a);
        return a.rfull_n > 0;
    }
    RowScanArgs b = a;
    b.rfull_n = 0;
    hipLaunchKernelGGL(rowcarry_kernel, dim3((a.g.H + kRcRows - 1) / kRcRows, n_frames), dim3(64 * kRcRows), 0, s, b);
    return false;
}

void launch_colscan(const RowScanArgs &a, int n_frames, bool two_pass, hipStream_t s, bool have_r, bool colblk_done) {
    const int ns64 = (a.g.W + 2 * kStrip - 1) / (2 * kStrip);
    if (two_pass) {
        if (!have_r)  // (rowcarry4 wrote the R rows already)
            hipLaunchKernelGGL(rowfull_kernel, dim3(ns64 * 2, a.g.H, n_frames), dim3(64), 0, s, a);
        // table order from 2 frames (C2's two prebuilt frames: 0.087 -> 0.062
        // ms); one frame: colblock + colseg (0.048 ms), colsum4's one walk per
        // column 0.053, colsum_plane 0.059 (profiles/r3/g51, r4/colseg)
        if (SC_COLSUM_PLANE && n_frames >= 2) {
            hipLaunchKernelGGL(colsum_plane_kernel, dim3(a.g.rowp / 16, n_frames), dim3(64), 0, s, a);
        } else if (SC_COLSEG > 1 && n_frames == 1 && a.colblk) {
            int seg = 0, nseg = 0;
            colseg_geometry(a.g.H, seg, nseg);
            // (block sums only above the last segment's start: nothing reads the
            // rest; computed by rowcarry4's launch unless the frame took rowcarry)
            if (nseg > 1 && !colblk_done)
                hipLaunchKernelGGL(colblock_kernel, dim3(a.g.rowp / 16, (nseg - 1) * seg / kColBlk), dim3(64), 0, s, a);
            hipLaunchKernelGGL(colseg_kernel, dim3(a.g.rowp / 16, nseg), dim3(64), 0, s, a, seg);
        } else if (SC_COLSUM4) {
            hipLaunchKernelGGL(colsum4_kernel, dim3(ns64 * 8, n_frames), dim3(64), 0, s, a);
        } else {
            hipLaunchKernelGGL(colsum_kernel, dim3(ns64 * 2, n_frames), dim3(64), 0, s, a);
        }
    } else {
        hipLaunchKernelGGL(colstrip_kernel, dim3(ns64 * 2, n_frames), dim3(64), 0, s, a);
    }
}

}  // namespace sc
