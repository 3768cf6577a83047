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

// The 32 features are kept as 16 float pairs, in the order f[2j], f[2j+1]
// (f index = 8*cell + 4*half + channel): the box sums, the squares, the clip
// output, the final scale and the LR products then stay in aligned register
// pairs and issue as v_pk_* (2 lanes of f32 per instruction, each lane's op
// the reference's own, round-to-nearest) with no re-pairing moves.  Every
// value and every addition order is the reference's.
typedef float f2 __attribute__((ext_vector_type(2)));

// The 32 box sums of one projected patch (CalcFeature :379-415): corners
// deduplicated on the (GW+1) x (GH+1) corner grid; cell index = row*GW + col
// (GetRectsFromPatch).  All 2*(GW+1)*(GH+1) corner loads are issued before
// any is consumed (a scheduling barrier keeps the compiler from interleaving
// them with the math, which would serialise memory round trips within the
// item).  P: ProjPatch (host-projected table) or InlinePatch (projected here).
template <int GW, int GH, class P>
__device__ __forceinline__ void patch_features2(const TabView &T, const P &pj, int half_off,
                                                f2 (&fp)[16]) {
    int col[GW + 1];
#pragma unroll
    for (int c = 0; c <= GW; c++) col[c] = pj.colq(c);
    float4 cn[2][GH + 1][GW + 1];
#pragma unroll
    for (int h = 0; h < 2; h++) {
#pragma unroll
        for (int r = 0; r <= GH; r++) {
            const int ro = h * half_off + pj.row0 + r * pj.rowstep;
#pragma unroll
            for (int c = 0; c <= GW; c++) cn[h][r][c] = T.at(ro + col[c]);
        }
    }
#if SC_LOAD_BARRIER
    __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
        for (int r = 0; r < GH; r++)
#pragma unroll
            for (int c = 0; c < GW; c++) {
                // (TL + BR) - (TR + BL), :385-412
                const float4 tl = cn[h][r][c], br = cn[h][r + 1][c + 1];
                const float4 tr = cn[h][r][c + 1], bl = cn[h][r + 1][c];
                const int o = 4 * (r * GW + c) + 2 * h;
                fp[o] = (f2{tl.x, tl.y} + f2{br.x, br.y}) - (f2{tr.x, tr.y} + f2{bl.x, bl.y});
                fp[o + 1] = (f2{tl.z, tl.w} + f2{br.z, br.w}) - (f2{tr.z, tr.w} + f2{bl.z, bl.w});
            }
}

#ifndef SC_SHAPE_LOADS  // 1: per-shape load branches (A/B only; the default is uniform loads)
#define SC_SHAPE_LOADS 0
#endif

// Uniform corner set: every shape's corners as 10 slots per half, so one
// straight-line sequence of loads serves a wave whatever shapes its lanes
// hold.  Slot m is corner (r, c) = 2x2: (m/3, m%3) (slot 9 repeats (2,2), a
// 2x2 patch has 9 corners); 1x4 (tall): (m/2, m%2); 4x1 (wide): (m/5, m%5).
// Why: the texture addresser costs about the same per vector-memory
// instruction however few lanes are active, and shape-divergent load
// branches issued 2.1x the instructions of one uniform set (measured,
// profiles/r2/itembench.md: item loop -11 %).
template <class P>
__device__ __forceinline__ void corner_offsets(const P &pj, int (&off)[10]) {
    int col[5], ro[5];
#pragma unroll
    for (int c = 0; c < 5; c++) col[c] = pj.colq(c);
#pragma unroll
    for (int r = 0; r < 5; r++) ro[r] = pj.row0 + r * pj.rowstep;
    const bool sq = pj.shape == 0, tall = pj.shape == 1;
#pragma unroll
    for (int m = 0; m < 10; m++) {
        const int o0 = ro[m < 9 ? m / 3 : 2] + col[m < 9 ? m % 3 : 2];
        const int o1 = ro[m / 2] + col[m % 2];
        const int o2 = ro[m / 5] + col[m % 5];
        off[m] = sq ? o0 : (tall ? o1 : o2);
    }
}

// Box sums of one half (4 channels) of the 4 cells from its 10 corner
// slots: fh[2*cell], fh[2*cell+1] = channels (0,1), (2,3) of the half.
template <int GW, int GH>
__device__ __forceinline__ void half_box(const float4 (&cn)[10], f2 (&fh)[8]) {
#pragma unroll
    for (int r = 0; r < GH; r++)
#pragma unroll
        for (int c = 0; c < GW; c++) {
            // (TL + BR) - (TR + BL), :385-412
            const float4 tl = cn[r * (GW + 1) + c], br = cn[(r + 1) * (GW + 1) + c + 1];
            const float4 tr = cn[r * (GW + 1) + c + 1], bl = cn[(r + 1) * (GW + 1) + c];
            const int o = 2 * (r * GW + c);
            fh[o] = (f2{tl.x, tl.y} + f2{br.x, br.y}) - (f2{tr.x, tr.y} + f2{bl.x, bl.y});
            fh[o + 1] = (f2{tl.z, tl.w} + f2{br.z, br.w}) - (f2{tr.z, tr.w} + f2{bl.z, bl.w});
        }
}

__device__ __forceinline__ void half_box(int shape, const float4 (&cn)[10], f2 (&fh)[8]) {
    if (shape == 0) half_box<2, 2>(cn, fh);
    else if (shape == 1) half_box<1, 4>(cn, fh);
    else half_box<4, 1>(cn, fh);
}

// CalcFeature (:379-415) with uniform loads, one half at a time: the 10
// loads of channels 0-3, their box sums, then the 10 loads of channels 4-7
// (40 corner registers live instead of 80; measured as fast as all 20 loads
// in flight at 12 waves per CU).  fp in the 32-feature order f[8 cell + 4 h + ch].
template <class P>
__device__ __forceinline__ void features_uniform(const TabView &T, int half_off, const P &pj, f2 (&fp)[16]) {
    int off[10];
    corner_offsets(pj, off);
    f2 h[2][8];
#pragma unroll
    for (int hh = 0; hh < 2; hh++) {
        float4 cn[10];
#pragma unroll
        for (int m = 0; m < 10; m++) cn[m] = T.at(hh * half_off + off[m]);
#if SC_LOAD_BARRIER
        __builtin_amdgcn_sched_barrier(0);
#endif
        half_box(pj.shape, cn, h[hh]);
    }
#pragma unroll
    for (int c = 0; c < 4; c++) {
        fp[4 * c] = h[0][2 * c];
        fp[4 * c + 1] = h[0][2 * c + 1];
        fp[4 * c + 2] = h[1][2 * c];
        fp[4 * c + 3] = h[1][2 * c + 1];
    }
}

// c_k = (q0+q1)+(q2+q3) of f[4k..4k+3] = fp[2k], fp[2k+1];
// SS = (((eps + c0) + c1) ...) + c7   (:427-433)
__device__ __forceinline__ float ss_hadd2(const f2 (&fp)[16]) {
    float ss = FLT_EPSILON;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const f2 a = fp[2 * k] * fp[2 * k], b = fp[2 * k + 1] * fp[2 * k + 1];
        ss = ss + ((a.x + a.y) + (b.x + b.y));
    }
    return ss;
}

// Normalize (:417-457) of the 32 box sums in place.
__device__ __forceinline__ void normalize2(f2 (&fp)[16]);

// CalcFeature + Normalize (:379-457) of one projected patch.
template <class P>
__device__ __forceinline__ void descriptor2(const TabView &T, int half_off, const P &pj, f2 (&fp)[16]) {
#if SC_SHAPE_LOADS
    if (pj.shape == 0) patch_features2<2, 2>(T, pj, half_off, fp);
    else if (pj.shape == 1) patch_features2<1, 4>(T, pj, half_off, fp);
    else patch_features2<4, 1>(T, pj, half_off, fp);
#else
    features_uniform(T, half_off, pj, fp);
#endif
    normalize2(fp);
}

#ifndef SC_SHORT_RN  // sqrt / reciprocal of Normalize without the range-end steps (same bits in its range)
#define SC_SHORT_RN 1
#endif
// Ranges (the same constants as kRnSqrt* / kRnRcp* in sc_kernels.hpp).
// Normalize's operands for any frame the API accepts: SS, SS2 in
// [FLT_EPSILON, 2^77] (the FLT_EPSILON seed; |box sum| <= 2*255*W*H < 2^36
// with W*H < 2^27, so 32 squares < 2^77), d = sqrt(SS2) in [2^-11.5, 2^38.5]
// (build_geometry checks it: normalize_operand_range).  The sequences below
// are stated for the wider ranges sqrt_rn: x in [2^-96, FLT_MAX] and
// rcp_rn: d in [2^-20, 2^40], and tests/test_gpu_rn.py compares them with
// the full IEEE sequences and the f64 route for EVERY f32 in those ranges
// (sc_selftest_rn).
// sqrt_rn: the compiler's correctly rounded sequence (v_sqrt_f32, then the
// two FMA residual checks one ulp either side) without its scaling of
// x < 2^-96 and its 0 / inf / NaN class select, which never act in its range.
__device__ __forceinline__ float sqrt_rn(float x) {
#if SC_SHORT_RN
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sd = __uint_as_float(__float_as_uint(s) - 1u), su = __uint_as_float(__float_as_uint(s) + 1u);
    float r = fmaf(-sd, s, x) <= 0.0f ? sd : s;
    r = fmaf(-su, s, x) > 0.0f ? su : r;
    return r;
#else
    return sqrtf(x);
#endif
}
// rcp_rn: the compiler's division sequence for 1/d (reciprocal, refinement,
// two FMA corrections) without v_div_scale / v_div_fmas scaling and
// v_div_fixup, which act only for operands near the exponent range's ends or
// special values, never in its range.
__device__ __forceinline__ float rcp_rn(float d) {
#if SC_SHORT_RN
    float r = __builtin_amdgcn_rcpf(d);
    const float e = fmaf(-d, r, 1.0f);
    r = fmaf(e, r, r);
    float q = 1.0f * r;
    const float e2 = fmaf(-d, q, 1.0f);
    q = fmaf(e2, r, q);
    const float e3 = fmaf(-d, q, 1.0f);
    return fmaf(e3, r, q);
#else
    return 1.0f / d;
#endif
}

__device__ __forceinline__ void normalize2(f2 (&fp)[16]) {
    const float theta = 0.35355338f;  // 2/sqrt(32.f) (.h:36)
    const float t = sqrt_rn(ss_hadd2(fp)) * theta, nt = -t;
    // _mm_max_ps(_mm_min_ps(f, t), -t) as one v_med3_f32: identical bits here
    // because f is a finite box sum (never NaN, never -0) and t > 0 (SS >= eps)
#pragma unroll
    for (int j = 0; j < 16; j++) {
        fp[j].x = __builtin_amdgcn_fmed3f(fp[j].x, nt, t);
        fp[j].y = __builtin_amdgcn_fmed3f(fp[j].y, nt, t);
    }
    const float r = rcp_rn(sqrt_rn(ss_hadd2(fp)));
#pragma unroll
    for (int j = 0; j < 16; j++) fp[j] = fp[j] * f2{r, r};
}

// CalcFeature + Normalize as 32 floats (miner descriptors).
template <class P>
__device__ __forceinline__ void descriptor(const TabView &T, int half_off, const P &pj, float (&f)[32]) {
    f2 fp[16];
    descriptor2(T, half_off, pj, fp);
#pragma unroll
    for (int j = 0; j < 16; j++) {
        f[2 * j] = fp[j].x;
        f[2 * j + 1] = fp[j].y;
    }
}

// LogisticRegression::Predict (LogisticRegression.cpp:46-68); w4 = w[0..35]:
// lane sums s0..s3 (s_j += w[4i+j]*f[4i+j], i = 0..7) as the pairs (s0, s1),
// (s2, s3); z = (s0+s1)+(s2+s3); then the f64 bias term and sigmoid.
__device__ __forceinline__ float lr_predict2(const f2 (&fp)[16], const float4 *w4, double bias) {
    f2 s01 = f2{0.0f, 0.0f}, s23 = f2{0.0f, 0.0f};
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const float4 wv = w4[i];
        s01 = f2{wv.x, wv.y} * fp[2 * i] + s01;
        s23 = f2{wv.z, wv.w} * fp[2 * i + 1] + s23;
    }
    const float z32 = (s01.x + s01.y) + (s23.x + s23.y);
    double prob = (double)z32;
    prob += (double)w4[8].x * bias;
#if SC_ABL_EXTRA_EXP  // timing ablation: one more f64 exp per item, result unused
    if (exp(-prob * 1.0000001) == -1.0) prob = 0.0;
#endif
    prob = 1.0 / (1.0 + exp(-prob));
    return (float)prob;
}

#ifndef SC_PAIR  // 1: lane-pair item form on interleaved 32-B cells (pair_z32); 0: one-lane form only
#define SC_PAIR 1
#endif

// ---- lane-pair item form (SC_PAIR) -------------------------------------------
// One item on two lanes: lane 2i + h holds channel half h (channels 4h..4h+3)
// of item i, so one 16-B load instruction reads both halves of 32 items'
// corners from the same 32-B interleaved cells (TableGeom cs 2, hs 1): one
// line per corner instead of one per half for an isolated window, and 16
// descriptor floats per lane instead of 32.  Quad q = 2 cell + h of the
// descriptor (f[4q..4q+3]) lives in lane h; every sequential sum of
// Normalize and LogisticRegression::Predict runs in both lanes, each term
// read from the lane that holds it (DPP quad_perm [0,0,2,2] / [1,1,3,3] as
// the first operand of the add: a + b == b + a bit for bit), so the
// association is the reference's exactly.
__device__ __forceinline__ float from_even(float x) {  // the value of lane 2i (quad_perm [0,0,2,2])
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xA0, 0xF, 0xF, true));
}
__device__ __forceinline__ float from_odd(float x) {  // the value of lane 2i+1 (quad_perm [1,1,3,3])
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xF5, 0xF, 0xF, true));
}

// SS = (((eps + c0) + c1) ...) + c7 (:427-433), c_(2 cell + h) in lane h
__device__ __forceinline__ float ss_pair(const f2 (&fh)[8]) {
    float c[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {  // every c first: the DPP reads then wait on nothing
        const f2 a = fh[2 * k] * fh[2 * k], b = fh[2 * k + 1] * fh[2 * k + 1];
        c[k] = (a.x + a.y) + (b.x + b.y);
    }
    float ss = FLT_EPSILON;
    asm volatile("" : "+v"(ss));  // (in a VGPR: the first add takes the DPP operand too)
#pragma unroll
    for (int k = 0; k < 4; k++) {
        ss = from_even(c[k]) + ss;
        ss = from_odd(c[k]) + ss;
    }
    return ss;
}

// One item of the lane-pair form as its projecting lane computed it: the
// 10 corner offsets (corner_offsets), the origin cell's byte offset, the
// patch shape and the weak index; of_even / of_odd hand a pair the item of
// its even / odd lane.
struct PairItem {
    int off[10];
    unsigned base;
    int shape, gk;
    template <int CTRL>
    __device__ __forceinline__ static int bc(int x) {
        return __builtin_amdgcn_mov_dpp(x, CTRL, 0xF, 0xF, true);
    }
    template <int CTRL>
    __device__ __forceinline__ PairItem of() const {
        PairItem r;
#pragma unroll
        for (int m = 0; m < 10; m++) r.off[m] = bc<CTRL>(off[m]);
        r.base = (unsigned)bc<CTRL>((int)base);
        r.shape = bc<CTRL>(shape);
        r.gk = bc<CTRL>(gk);
        return r;
    }
    __device__ __forceinline__ PairItem of_even() const { return of<0xA0>(); }
    __device__ __forceinline__ PairItem of_odd() const { return of<0xF5>(); }
};

// CalcFeature + Normalize + the f32 part of LogisticRegression::Predict
// (:379-457, LogisticRegression.cpp:46-60) of one item on a lane pair (lane
// half h: +16 B into each 32-B cell).  Returns z32 = (s0 + s1) + (s2 + s3)
// in both lanes.  w4: the item's weights (quad q at w4[q]).
__device__ __forceinline__ float pair_z32(const char *Tb, const PairItem &it, const float4 *w4, int h) {
#if SC_LOAD_BARRIER
    __builtin_amdgcn_sched_barrier(0);  // (the next item's loads stay after this one's math)
#endif
    const TabView T{Tb, it.base + ((unsigned)h << 4)};
    float4 cn[10];
#pragma unroll
    for (int m = 0; m < 10; m++) cn[m] = T.at(it.off[m]);
#if SC_LOAD_BARRIER
    __builtin_amdgcn_sched_barrier(0);
#endif
    f2 fh[8];
    half_box(it.shape, cn, fh);
    const float theta = 0.35355338f;
    const float t = sqrt_rn(ss_pair(fh)) * theta, nt = -t;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        fh[j].x = __builtin_amdgcn_fmed3f(fh[j].x, nt, t);
        fh[j].y = __builtin_amdgcn_fmed3f(fh[j].y, nt, t);
    }
    const float r = rcp_rn(sqrt_rn(ss_pair(fh)));
#pragma unroll
    for (int j = 0; j < 8; j++) fh[j] = fh[j] * f2{r, r};
    // products as single floats: a DPP operand folds into the add only when
    // it is a whole 32-bit register (not half of a v_pk result)
    float p[4][4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const float4 wv = w4[2 * k + h];
        p[k][0] = wv.x * fh[2 * k].x;
        p[k][1] = wv.y * fh[2 * k].y;
        p[k][2] = wv.z * fh[2 * k + 1].x;
        p[k][3] = wv.w * fh[2 * k + 1].y;
    }
    float s[4] = {0.0f, 0.0f, 0.0f, 0.0f};  // lane sums from 0 (LogisticRegression.cpp:51-57)
#pragma unroll
    for (int j = 0; j < 4; j++) asm volatile("" : "+v"(s[j]));
#pragma unroll
    for (int k = 0; k < 4; k++) {
#pragma unroll
        for (int j = 0; j < 4; j++) s[j] = from_even(p[k][j]) + s[j];
#pragma unroll
        for (int j = 0; j < 4; j++) s[j] = from_odd(p[k][j]) + s[j];
    }
    float z = (s[0] + s[1]) + (s[2] + s[3]);
    asm volatile("" : "+v"(z));  // computed here: its DPP reads stay next to their adds
    return z;
}

// The f64 tail of LogisticRegression::Predict (:61-67) from z32.
__device__ __forceinline__ float lr_sigmoid(float z32, float wb, double bias) {
    double prob = (double)z32;
    prob += (double)wb * bias;
    prob = 1.0 / (1.0 + exp(-prob));
    return (float)prob;
}

// One (window, weak classifier) item.
template <class P>
__device__ __forceinline__ float weak_eval(const TabView &T, int half_off, const P &pj, const float4 *w4,
                                           double bias) {
    f2 fp[16];
    descriptor2(T, half_off, pj, fp);
    return lr_predict2(fp, w4, bias);
}

}  // namespace sc
