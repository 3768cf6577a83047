// sc_device.hpp -- device building blocks shared by the window kernels
// (sc_windows.hip) and the mining kernels (sc_mine.hip): table views, box
// sums, CalcFeature + Normalize, LogisticRegression::Predict.
//
// Every f32/f64 operation is the one the reference performs, in its order;
// compiled with -ffp-contract=off, IEEE sqrt / division, no fast-math.
#pragma once

#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>

#include "sc_kernels.hpp"

#ifndef SC_SADDR  // 1: corner loads as SGPR base + 32-bit VGPR offset
#define SC_SADDR 1
#endif
#ifndef SC_LOAD_BARRIER  // 1: every corner load issued before the box sums
#define SC_LOAD_BARRIER 1
#endif
#ifndef SC_HALF_BARRIER  // 1: load the second channel half after the first is consumed
#define SC_HALF_BARRIER 0
#endif

namespace sc {

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

// A window's view of the table: uniform base (SGPRs) + the lane's 32-bit
// byte offset of its origin cell, so each corner load is one
// `global_load_dwordx4 v, v_off, s[base]` with a single offset VGPR (frame
// tables are < 4 GiB; host check) instead of a 64-bit per-lane address.
struct TabView {
    const char *base;
    unsigned off;
    __device__ __forceinline__ float4 at(int cell) const {
#if SC_SADDR
        return *reinterpret_cast<const float4 *>(base + (off + ((unsigned)cell << 4)));
#else
        return reinterpret_cast<const float4 *>(base + off)[cell];
#endif
    }
};

// The 32 box sums of one projected patch: corners deduplicated on the
// (GW+1) x (GH+1) corner grid; cell index = row*GW + col (GetRectsFromPatch).
// All 2*(GW+1)*(GH+1) corner loads are issued before any is consumed (a
// scheduling barrier keeps the compiler from interleaving them with the
// math, which would serialise memory round trips within the item).
template <int GW, int GH>
__device__ __forceinline__ void patch_features(const TabView &T, const ProjPatch &pj,
                                               int half_off, float (&f)[32]) {
#if !SC_LOAD_BARRIER  // A/B: rows loaded as they are consumed (compiler schedules)
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int ho = h * half_off;
        float4 prev[GW + 1], cur[GW + 1];
#pragma unroll
        for (int c = 0; c <= GW; c++) prev[c] = T.at(ho + pj.row0 + pj.col[c]);
#pragma unroll
        for (int r = 0; r < GH; r++) {
            const int ro = ho + pj.row0 + (r + 1) * pj.rowstep;
#pragma unroll
            for (int c = 0; c <= GW; c++) cur[c] = T.at(ro + pj.col[c]);
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
    return;
#endif
    float4 cn[2][GH + 1][GW + 1];
#pragma unroll
    for (int h = 0; h < 2; h++) {
#pragma unroll
        for (int r = 0; r <= GH; r++) {
            const int ro = h * half_off + pj.row0 + r * pj.rowstep;
#pragma unroll
            for (int c = 0; c <= GW; c++) cn[h][r][c] = T.at(ro + pj.col[c]);
        }
#if SC_HALF_BARRIER
        __builtin_amdgcn_sched_barrier(0);
#endif
    }
#if !SC_HALF_BARRIER
    __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
        for (int r = 0; r < GH; r++)
#pragma unroll
            for (int c = 0; c < GW; c++) {
                const float4 v = box4(cn[h][r][c], cn[h][r + 1][c + 1], cn[h][r][c + 1], cn[h][r + 1][c]);
                const int o = 8 * (r * GW + c) + 4 * h;
                f[o + 0] = v.x;
                f[o + 1] = v.y;
                f[o + 2] = v.z;
                f[o + 3] = v.w;
            }
}

// A ProjPatch as two 16-B loads issued together (the compiler would
// otherwise fetch col[] only after branching on shape: a second round trip).
__device__ __forceinline__ ProjPatch load_proj(const ProjPatch *p) {
    const int4 *q = reinterpret_cast<const int4 *>(p);
    const int4 a = q[0], b = q[1];
    ProjPatch r;
    r.shape = a.x;
    r.row0 = a.y;
    r.rowstep = a.z;
    r.col[0] = a.w;
    r.col[1] = b.x;
    r.col[2] = b.y;
    r.col[3] = b.z;
    r.col[4] = b.w;
    return r;
}

// CalcFeature + Normalize (DenseSURFFeatureExtractor.cpp:379-457) of one
// projected patch; T views the window's origin cell (half 0).
__device__ __forceinline__ void descriptor(const TabView &T, int half_off, const ProjPatch &pj,
                                           float (&f)[32]) {
    if (pj.shape == 0) patch_features<2, 2>(T, pj, half_off, f);
    else if (pj.shape == 1) patch_features<1, 4>(T, pj, half_off, f);
    else patch_features<4, 1>(T, pj, half_off, f);
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
}

// LogisticRegression::Predict (LogisticRegression.cpp:46-68); w4 = w[0..35].
__device__ __forceinline__ float lr_predict(const float (&f)[32], const float4 *w4, double bias) {
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
#if SC_ABL_EXTRA_EXP  // timing ablation: one more f64 exp per item, result unused
    if (exp(-prob * 1.0000001) == -1.0) prob = 0.0;
#endif
    prob = 1.0 / (1.0 + exp(-prob));
    return (float)prob;
}

// One (window, weak classifier) item.
__device__ __forceinline__ float weak_eval(const TabView &T, int half_off, const ProjPatch &pj,
                                           const float4 *w4, double bias) {
    float f[32];
    descriptor(T, half_off, pj, f);
    return lr_predict(f, w4, bias);
}

}  // namespace sc
