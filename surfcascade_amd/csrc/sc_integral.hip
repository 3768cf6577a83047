// sc_integral.hip -- gfx950 (CDNA4) integral-table kernels of the detect path.
//
//   rowscan  : T2bFilter gradients (DenseSURFFeatureExtractor.cpp:199-349)
//              fused with the exact integer row prefix of cv::integral
//              (:73-76); writes R_y[x] (exact in f32) into table row y+1.
//   colscan  : the f32 column recurrence S[y+1][x] = S[y][x] + R_y[x],
//              sequential in y per (x, channel) -- the association order of
//              OpenCV's scalar integral_.
//
// Every f32/f64 operation is the one the reference performs, in its order;
// the file is compiled with -ffp-contract=off (no FMA contraction), IEEE
// sqrt / division (hipcc default), no fast-math.  Table layout: sc_kernels.hpp.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>

#include "sc_kernels.hpp"

namespace sc {

namespace {

constexpr int kRowThreads = 256;
constexpr int kRowPx = 4;                      // pixels per thread
constexpr int kRowSeg = kRowThreads * kRowPx;  // pixels per segment

__device__ __forceinline__ uint32_t sat_sub(uint32_t a, uint32_t b) { return a > b ? a - b : 0u; }

// ---------------------------------------------------------------------------
// rowscan: gradients + exact integer row prefix -> table row y+1
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kRowThreads) void rowscan_kernel(RowScanArgs a) {
    __shared__ uint8_t s_img[3][kRowSeg + 16];
    __shared__ __attribute__((aligned(16))) float s_out[kRowSeg * 8];
    __shared__ uint32_t s_wsum[kRowThreads / 64][8];

    const int y = blockIdx.x, frame = blockIdx.y, tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    const TableGeom g = a.g;
    const int W = g.W, H = g.H, step = g.step, Qp = g.Qp;
    const uint8_t *img = a.frames + (long long)frame * a.frame_bytes;
    const uint8_t *rows[3] = {img + (long long)(y > 0 ? y - 1 : 0) * a.stride,
                              img + (long long)y * a.stride,
                              img + (long long)(y < H - 1 ? y + 1 : H - 1) * a.stride};
    float4 *tab = a.table + (long long)frame * g.frame4;
    float4 *out = tab + (long long)(y + 1) * g.rowp;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);

    if (y == 0)  // table row 0 is all zeros
        for (int i = tid; i < g.rowp; i += kRowThreads) tab[i] = z4;
    if (tid == 0) {  // column 0 (phase 0, q 0) of this row
        out[0] = z4;
        out[(long long)step * Qp] = z4;
    }

    uint32_t carry[8];
#pragma unroll
    for (int c = 0; c < 8; c++) carry[c] = 0;

    for (int seg = 0; seg < W; seg += kRowSeg) {
        // stage the three source rows of this segment (x = seg-1 .. seg+kRowSeg)
        for (int i = tid; i < kRowSeg + 2; i += kRowThreads) {
            int x = seg - 1 + i;
            x = x < 0 ? 0 : (x > W - 1 ? W - 1 : x);
#pragma unroll
            for (int r = 0; r < 3; r++) s_img[r][i] = rows[r][x];
        }
        __syncthreads();

        const int x0 = seg + tid * kRowPx;
        uint32_t pre[kRowPx][8];  // inclusive in-thread prefix [px][ch]
        uint32_t acc[8];
#pragma unroll
        for (int c = 0; c < 8; c++) acc[c] = 0;
#pragma unroll
        for (int px = 0; px < kRowPx; px++) {
            const int x = x0 + px;
            if (x < W) {
                const int xn = (x < W - 1 ? x + 1 : W - 1) - seg + 1;
                const int xp = (x > 0 ? x - 1 : 0) - seg + 1;
                const int xc = x - seg + 1;
                const uint32_t u_c = s_img[0][xc], d_c = s_img[2][xc];
                const uint32_t c_n = s_img[1][xn], c_p = s_img[1][xp];
                const uint32_t u_n = s_img[0][xn], u_p = s_img[0][xp];
                const uint32_t d_n = s_img[2][xn], d_p = s_img[2][xp];
                acc[0] += sat_sub(c_p, c_n);  // dx: In = I[y][x+1], Ip = I[y][x-1]
                acc[1] += sat_sub(c_n, c_p);
                acc[2] += sat_sub(u_c, d_c);  // dy: In = I[y+1][x], Ip = I[y-1][x]
                acc[3] += sat_sub(d_c, u_c);
                acc[4] += sat_sub(u_p, d_n);  // du: In = I[y+1][x+1], Ip = I[y-1][x-1]
                acc[5] += sat_sub(d_n, u_p);
                acc[6] += sat_sub(d_p, u_n);  // dv: In = I[y-1][x+1], Ip = I[y+1][x-1]
                acc[7] += sat_sub(u_n, d_p);
            }
#pragma unroll
            for (int c = 0; c < 8; c++) pre[px][c] = acc[c];
        }
        // exclusive scan of the per-thread totals across the workgroup (exact ints)
        uint32_t incl[8];
#pragma unroll
        for (int c = 0; c < 8; c++) incl[c] = acc[c];
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
#pragma unroll
            for (int c = 0; c < 8; c++) {
                uint32_t v = __shfl_up(incl[c], off, 64);
                if (lane >= off) incl[c] += v;
            }
        }
        if (lane == 63)
#pragma unroll
            for (int c = 0; c < 8; c++) s_wsum[wv][c] = incl[c];
        __syncthreads();
        uint32_t base[8], seg_total[8];
#pragma unroll
        for (int c = 0; c < 8; c++) {
            uint32_t b = 0, t = 0;
#pragma unroll
            for (int w = 0; w < kRowThreads / 64; w++) {
                if (w < wv) b += s_wsum[w][c];
                t += s_wsum[w][c];
            }
            base[c] = carry[c] + b + incl[c] - acc[c];
            seg_total[c] = t;
        }
        // R values (exact integers < 2^24, exact in f32) staged in LDS
#pragma unroll
        for (int px = 0; px < kRowPx; px++) {
            float4 lo, hi;
            lo.x = (float)(base[0] + pre[px][0]);
            lo.y = (float)(base[1] + pre[px][1]);
            lo.z = (float)(base[2] + pre[px][2]);
            lo.w = (float)(base[3] + pre[px][3]);
            hi.x = (float)(base[4] + pre[px][4]);
            hi.y = (float)(base[5] + pre[px][5]);
            hi.z = (float)(base[6] + pre[px][6]);
            hi.w = (float)(base[7] + pre[px][7]);
            float4 *d = reinterpret_cast<float4 *>(s_out + (tid * kRowPx + px) * 8);
            d[0] = lo;
            d[1] = hi;
        }
        __syncthreads();
        // phase-split stores: cell X = seg+1+i -> (X % step, X / step)
        for (int i = tid; i < kRowSeg; i += kRowThreads) {
            const int X = seg + 1 + i;
            if (X <= W) {
                const int q = X / step, p = X - q * step;
                const float4 *src = reinterpret_cast<const float4 *>(s_out + i * 8);
                out[(long long)p * Qp + q] = src[0];
                out[(long long)(step + p) * Qp + q] = src[1];
            }
        }
#pragma unroll
        for (int c = 0; c < 8; c++) carry[c] += seg_total[c];
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// colscan: S[y+1][x] = fl(S[y][x] + R_y[x]), sequential in y (in place)
// ---------------------------------------------------------------------------
constexpr int kColBlk = 32;

__global__ __launch_bounds__(64) void colscan_kernel(float *table, TableGeom g) {
    const int fi = blockIdx.x * 64 + threadIdx.x;  // float index within a row
    if (fi >= g.rowp * 4) return;
    {   // skip padding cells (x > W) -- never written, never read
        const int f4 = fi >> 2, plane = f4 / g.Qp, q = f4 - plane * g.Qp;
        const int p = plane % g.step;
        if (q * g.step + p > g.W) return;
    }
    const long long pitch = (long long)g.rowp * 4;
    const int H = g.H;
    float *col = table + (long long)blockIdx.y * g.frame4 * 4 + fi;
    float acc = 0.0f;  // row 0
    float cur[kColBlk], nxt[kColBlk];
#pragma unroll
    for (int k = 0; k < kColBlk; k++) cur[k] = (1 + k <= H) ? col[(1 + k) * pitch] : 0.0f;
    for (int y = 1; y <= H; y += kColBlk) {
        const int yn = y + kColBlk;
#pragma unroll
        for (int k = 0; k < kColBlk; k++) nxt[k] = (yn + k <= H) ? col[(yn + k) * pitch] : 0.0f;
#pragma unroll
        for (int k = 0; k < kColBlk; k++) {
            if (y + k <= H) {
                acc = acc + cur[k];
                col[(y + k) * pitch] = acc;
            }
        }
#pragma unroll
        for (int k = 0; k < kColBlk; k++) cur[k] = nxt[k];
    }
}

}  // namespace

void launch_rowscan(const RowScanArgs &a, int n_frames, hipStream_t s) {
    hipLaunchKernelGGL(rowscan_kernel, dim3(a.g.H, n_frames), dim3(kRowThreads), 0, s, a);
}

void launch_colscan(float4 *table, const TableGeom &g, int n_frames, hipStream_t s) {
    const int n = g.rowp * 4;
    hipLaunchKernelGGL(colscan_kernel, dim3((n + 63) / 64, n_frames), dim3(64), 0, s,
                       reinterpret_cast<float *>(table), g);
}

}  // namespace sc
