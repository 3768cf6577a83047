// sc_kernels.hip -- gfx950 (CDNA4) kernels of the SURF-cascade detect path.
//
//   rowscan  : T2bFilter gradients (DenseSURFFeatureExtractor.cpp:199-349)
//              fused with the exact integer row prefix of cv::integral
//              (:73-76); writes R_y[x] (exact in f32) into table row y+1.
//   colscan  : the f32 column recurrence S[y+1][x] = S[y][x] + R_y[x],
//              sequential in y per (x, channel) -- the association order of
//              OpenCV's scalar integral_.
//   windows  : one workgroup per (frame, level, row y): prefilter
//              (sum(), :351-358 / ObjDetector.cpp:188), then the cascade
//              stage by stage over a compacted survivor list (ballot +
//              prefix), (window, weak) items spread over all lanes k-major so
//              a wave gathers the same corner of consecutive windows; each item
//              is ProjectPatches/CalcFeature/Normalize/LogisticRegression::
//              Predict (:459-484, :379-457, LogisticRegression.cpp:46-68);
//              stage sums in weak order (GentleAdaboost.cpp:247-261); finally
//              the adaptive-stride x walk of ObjDetector.cpp:185-217 over the
//              row's results, emitting detections.
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
constexpr int kWinThreads = 256;
constexpr int kWaves = kWinThreads / 64;

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

// ---------------------------------------------------------------------------
// windows
// ---------------------------------------------------------------------------

// (TL + BR) - (TR + BL) per lane (DenseSURFFeatureExtractor.cpp:385-412).
__device__ __forceinline__ float4 box4(float4 tl, float4 br, float4 tr, float4 bl) {
    float4 r;
    r.x = (tl.x + br.x) - (tr.x + bl.x);
    r.y = (tl.y + br.y) - (tr.y + bl.y);
    r.z = (tl.z + br.z) - (tr.z + bl.z);
    r.w = (tl.w + br.w) - (tr.w + bl.w);
    return r;
}

// c_k = (q0+q1)+(q2+q3); SS = (((eps + c0) + c1) ...) + c7   (:427-433)
__device__ __forceinline__ float ss_hadd(const float (&f)[32]) {
    float ss = FLT_EPSILON;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        float q0 = f[4 * k] * f[4 * k], q1 = f[4 * k + 1] * f[4 * k + 1];
        float q2 = f[4 * k + 2] * f[4 * k + 2], q3 = f[4 * k + 3] * f[4 * k + 3];
        ss = ss + ((q0 + q1) + (q2 + q3));
    }
    return ss;
}

// The 32 box sums of one projected patch: corners deduplicated on the
// (GW+1) x (GH+1) corner grid; cell index = row*GW + col (GetRectsFromPatch).
template <int GW, int GH>
__device__ __forceinline__ void patch_features(const float4 *__restrict__ T, const ProjPatch &pj,
                                               int half_off, float (&f)[32]) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const float4 *Th = T + h * half_off;
        float4 prev[GW + 1], cur[GW + 1];
#pragma unroll
        for (int c = 0; c <= GW; c++) prev[c] = Th[pj.row0 + pj.col[c]];
#pragma unroll
        for (int r = 0; r < GH; r++) {
            const int ro = pj.row0 + (r + 1) * pj.rowstep;
#pragma unroll
            for (int c = 0; c <= GW; c++) cur[c] = Th[ro + pj.col[c]];
#pragma unroll
            for (int c = 0; c < GW; c++) {
                const float4 v = box4(prev[c], cur[c + 1], prev[c + 1], cur[c]);
                const int o = 8 * (r * GW + c) + 4 * h;
                f[o + 0] = v.x;
                f[o + 1] = v.y;
                f[o + 2] = v.z;
                f[o + 3] = v.w;
            }
#pragma unroll
            for (int c = 0; c <= GW; c++) prev[c] = cur[c];
        }
    }
}

// One (window, weak classifier) item: CalcFeature + Normalize + Predict.
// T points at the window's origin cell (row y, window j) in half 0.
__device__ float weak_eval(const float4 *__restrict__ T, int half_off, const ProjPatch &pj,
                           const float4 *__restrict__ w4, double bias, int variant) {
    float f[32];
    if (pj.shape == 0) patch_features<2, 2>(T, pj, half_off, f);
    else if (pj.shape == 1) patch_features<1, 4>(T, pj, half_off, f);
    else patch_features<4, 1>(T, pj, half_off, f);
    if (variant & 1) {  // timing ablation only: gathers without the math
        float sum = 0.0f;
#pragma unroll
        for (int i = 0; i < 32; i++) sum += f[i];
        return sum;
    }
    // Normalize (:417-457): clip at sqrt(SS)*theta, renormalise by 1/sqrt(SS2)
    const float theta = 0.35355338f;  // 2/sqrt(32.f) (.h:36)
    const float t = sqrtf(ss_hadd(f)) * theta, nt = -t;
    // _mm_max_ps(_mm_min_ps(f, t), -t) as one v_med3_f32: identical bits here
    // because f is a finite box sum (never NaN, never -0) and t > 0 (SS >= eps)
#pragma unroll
    for (int i = 0; i < 32; i++) f[i] = __builtin_amdgcn_fmed3f(f[i], nt, t);
    const float r = 1.0f / sqrtf(ss_hadd(f));
#pragma unroll
    for (int i = 0; i < 32; i++) f[i] = f[i] * r;
    // LogisticRegression::Predict (LogisticRegression.cpp:46-68)
    float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f, s3 = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const float4 wv = w4[i];
        s0 = wv.x * f[4 * i + 0] + s0;
        s1 = wv.y * f[4 * i + 1] + s1;
        s2 = wv.z * f[4 * i + 2] + s2;
        s3 = wv.w * f[4 * i + 3] + s3;
    }
    const float z32 = (s0 + s1) + (s2 + s3);
    double prob = (double)z32;
    prob += (double)w4[8].x * bias;
    prob = 1.0 / (1.0 + exp(-prob));
    return (float)prob;
}

struct WinSmem {
    int *cnt;  // [kWaves]
    float *st_s;
    float *sums;
    float *P;  // [kWinThreads]
    int16_t *st_p;
    uint16_t *surv;
};

__device__ __forceinline__ WinSmem carve(unsigned char *smem, int nxa) {
    WinSmem m;
    m.cnt = reinterpret_cast<int *>(smem);
    m.st_s = reinterpret_cast<float *>(smem + 16);
    m.sums = m.st_s + nxa;
    m.P = m.sums + nxa;
    m.st_p = reinterpret_cast<int16_t *>(m.P + kWinThreads);
    m.surv = reinterpret_cast<uint16_t *>(m.st_p + nxa);
    return m;
}

// Order-preserving block compaction: appends j to surv when keep.
__device__ __forceinline__ int compact_append(bool keep, int j, uint16_t *surv, int n, int *cnt) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const unsigned long long m = __ballot(keep);
    const int pre = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) cnt[wv] = __popcll(m);
    __syncthreads();
    int off = n, total = 0;
#pragma unroll
    for (int w = 0; w < kWaves; w++) {
        const int cw = cnt[w];
        if (w < wv) off += cw;
        total += cw;
    }
    if (keep) surv[off + pre] = (uint16_t)j;
    __syncthreads();
    return n + total;
}

template <bool kDebug>
__global__ __launch_bounds__(kWinThreads) void window_kernel(WindowArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    // XCD-aware block order: the dispatcher deals blocks round-robin over the
    // 8 XCDs (b % 8 share one L2); give each XCD a contiguous run of
    // (frame, row) so concurrently resident rows of one XCD are neighbours
    // and share table lines in its L2.  Bijective for any grid size.
    int row, frame;
    {
        const int n = a.n_rows * a.n_frames, b = blockIdx.x;
        const int q = n >> 3, r = n & 7, x = b & 7, idx = b >> 3;
        int lin = b;  // measured: dispatcher order is 7% faster than the XCD-band order
        if (a.variant & 4) lin = x < r ? x * (q + 1) + idx : r * (q + 1) + (x - r) * q + idx;
        frame = lin / a.n_rows;
        row = lin - frame * a.n_rows;
    }
    const int2 rd = a.rows[row];
    const LevelInfo L = a.levels[rd.x];
    const int y = rd.y, nx = L.nx;
    const int step = a.g.step, half_off = a.g.step * a.g.Qp;
    WinSmem sm = carve(smem, a.lds_nx);
    // origin cell of window 0 of this row (phase 0), half 0
    const float4 *T = a.table + (long long)frame * a.g.frame4 + (long long)y * a.g.rowp;

    // 1) prefilter over the whole row; survivors in x order
    int nsurv = 0;
    for (int b = 0; b < nx; b += kWinThreads) {
        const int j = b + tid;
        bool pass = false;
        if (j < nx) {
            const float4 *t0 = T + j;
            const float4 v = box4(t0[0], t0[L.pre_row + L.pre_col], t0[L.pre_col], t0[L.pre_row]);
            const float m = (((v.x + v.y) + v.z) + v.w) / 2.0f;  // sum(), :351-358
            pass = m > L.thr;                                    // ObjDetector.cpp:188
            sm.st_p[j] = pass ? 0 : -1;
            sm.st_s[j] = 0.0f;
        }
        nsurv = compact_append(pass, j, sm.surv, nsurv, sm.cnt);
    }

    // 2) cascade, stage by stage over the compacted survivors
    const ProjPatch *projL = a.proj + (long long)rd.x * a.K;
    for (int s = 0; s < a.n_stages && nsurv > 0; s++) {
        const int off = a.stage_off[s], n = a.stage_off[s + 1] - off;
        for (int i = tid; i < nsurv; i += kWinThreads) sm.sums[i] = 0.0f;
        __syncthreads();
        const int items = nsurv * n;
        const float rcp = 1.0f / (float)nsurv;
        for (int r = 0; r < items; r += kWinThreads) {
            const int t = r + tid;
            if (t < items) {
                // k = t / nsurv without an integer divide (t < 2^24: one correction)
                int k = (int)((float)t * rcp), i = t - k * nsurv;
                if (i < 0) { k--; i += nsurv; }
                else if (i >= nsurv) { k++; i -= nsurv; }
                const int j = sm.surv[i];
                const int gk = off + k;
                const ProjPatch pj = projL[gk];
                if (a.variant & 2) {  // timing ablation only: L1-resident gathers
                    ProjPatch z{};
                    z.shape = pj.shape;
                    sm.P[tid] = weak_eval(T, half_off, z, a.w + (long long)gk * 9, a.bias[gk], a.variant);
                } else {
                    sm.P[tid] = weak_eval(T + j, half_off, pj, a.w + (long long)gk * 9, a.bias[gk],
                                          a.variant);
                }
            }
            __syncthreads();
            const int rend = min(r + kWinThreads, items);
            for (int i = tid; i < nsurv; i += kWinThreads) {
                // items of slot i in [r, rend): t = k*nsurv + i, in increasing k
                const int k = (r > i) ? (r - i + nsurv - 1) / nsurv : 0;
                float acc = sm.sums[i];
                for (int t2 = k * nsurv + i; t2 < rend; t2 += nsurv) acc += sm.P[t2 - r];
                sm.sums[i] = acc;
            }
            __syncthreads();
        }
        // stage decision (GentleAdaboost.cpp:259; ObjDetector.cpp:197)
        const float th = a.theta[s];
        int nn = 0;
        for (int b = 0; b < nsurv; b += kWinThreads) {
            const int i = b + tid;
            bool keep = false;
            int j = 0;
            if (i < nsurv) {
                j = sm.surv[i];
                const float sc = sm.sums[i] / (float)n;
                sm.st_s[j] = sc;
                keep = !((double)sc < (double)th);
                sm.st_p[j] = (int16_t)(keep ? s + 1 : s);
            }
            nn = compact_append(keep, j, sm.surv, nn, sm.cnt);
        }
        nsurv = nn;
    }
    __syncthreads();

    // 3) adaptive-stride walk of the row (ObjDetector.cpp:185-217) by wave 0
    if (tid < 64) {
        const int S = a.n_stages;
        const long long gbase = L.grid_base + (long long)(y / step) * nx;
        int start = 0;
        unsigned long long nvis = 0;
        for (int b = 0; b < nx; b += 64) {
            const int j = b + lane;
            bool skip = true, det = false;
            int p = -1;
            float sl = 0.0f;
            double fin = 0.0;
            if (j < nx) {
                p = sm.st_p[j];
                sl = sm.st_s[j];
                if (p >= 0) {
                    fin = ((double)sl + p + 1) / S;  // ObjDetector.cpp:201
                    skip = fin < a.stride_score;     // :214
                    det = p == S;                    // :203
                }
            }
            const unsigned long long sk = __ballot(skip);
            const int lim = min(64, nx - b);
            unsigned long long vis = 0;
            int pos = start;
            while (pos < lim) {
                vis |= 1ull << pos;
                pos += ((sk >> pos) & 1ull) ? 2 : 1;
            }
            start = pos - 64;
            const bool v = (vis >> lane) & 1ull;
            nvis += __popcll(vis);
            if (kDebug && j < nx) {
                const long long gi = (long long)frame * a.grid_per_frame + gbase + j;
                a.dbg_p[gi] = (int16_t)p;
                a.dbg_s[gi] = sl;
                a.dbg_v[gi] = v ? 1 : 0;
            }
            const bool d = v && det;
            const unsigned long long dm = __ballot(d);
            if (dm) {
                const int cnt = __popcll(dm);
                int slot0 = 0;
                if (lane == 0) {
                    slot0 = atomicAdd(&a.counters[0], cnt);
                    atomicAdd(&a.counters[1 + frame], cnt);
                }
                slot0 = __shfl(slot0, 0, 64);
                if (d) {
                    const int idx = slot0 + __popcll(dm & ((1ull << lane) - 1ull));
                    if (idx < a.capacity) {
                        sc_det_record rec;
                        rec.frame = frame;
                        rec.level = rd.x;
                        rec.x = j * step;
                        rec.y = y;
                        rec.w = L.l;
                        rec.h = L.lh;
                        rec.stage_reached = p;
                        rec._pad = 0;
                        rec.score = fin;
                        a.out[idx] = rec;
                    }
                }
            }
        }
        if (lane == 0 && a.visited) atomicAdd(a.visited, nvis);
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

size_t window_lds_bytes(int nxa) {
    return 16 + (size_t)nxa * 4 * 2 + kWinThreads * 4 + (size_t)nxa * 2 * 2;
}

void launch_windows(const WindowArgs &a, int n_rows, int n_frames, bool debug, hipStream_t s) {
    const size_t lds = window_lds_bytes(a.lds_nx);
    WindowArgs b = a;
    b.n_rows = n_rows;
    b.n_frames = n_frames;
    const dim3 grid(n_rows * n_frames);
    if (debug)
        hipLaunchKernelGGL(window_kernel<true>, grid, dim3(kWinThreads), lds, s, b);
    else
        hipLaunchKernelGGL(window_kernel<false>, grid, dim3(kWinThreads), lds, s, b);
}

}  // namespace sc
