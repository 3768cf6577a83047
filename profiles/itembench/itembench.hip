// itembench.hip -- microbenchmark of the detect path's inner loop: one
// (window, weak classifier) item = CalcFeature + Normalize + LR::Predict
// (DenseSURFFeatureExtractor.cpp:379-457, LogisticRegression.cpp:46-68) over
// a real item stream (profiles/itembench/run.py builds it from the C2 frame's
// visited windows in the chain kernel's order).  Variants of the item loop
// are timed against each other; every variant's outputs must equal the
// production weak_eval's bit for bit (run.py checks).  Measurement tool only.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../surfcascade_amd/csrc/sc_device.hpp"

using namespace sc;

namespace {

struct Item {
    unsigned origin;  // float4 offset of the window's origin cell in the frame table
    unsigned short k;
    unsigned char level, parity;
};

struct Args {
    const float4 *table;
    TableGeom g;
    const Item *items;      // per XCD queue: items[q * cap + i]
    const int *n_items;     // [8]
    long long cap;
    const float4 *w;        // [K][9]
    const double *bias;     // [K]
    const int4 *rects;      // [K]
    const float *scale;     // [levels]
    int K, n_levels;
    float *out;             // same indexing as items
    int *tickets;           // [8 * 64]
    unsigned omask;         // ablation (k_bcast only): lane offset mask
    unsigned fold;          // ablation (k_fold only): table row &= fold
};

__device__ __forceinline__ unsigned xcc() {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 7;
}

__device__ __forceinline__ InlinePatch project(const Args &a, const int4 *R, const float *Sc, const Item &it) {
    const int4 rc = R[it.k];
    const float s = Sc[it.level];
    const int px = (int)((float)rc.x * s), py = (int)((float)rc.y * s), e = (int)((float)rc.z * s);
    InlinePatch p;
    p.shape = rc.w;
    p.c = rc.w == 0 ? (e >> 1) : e;
    p.row0 = py * a.g.rowp;
    p.rowstep = p.c * a.g.rowp;
    p.x0 = it.parity * a.g.step + px;
    p.cb = a.g.at0((unsigned)(it.parity * a.g.step));
    p.phm = a.g.phm;
    p.ph = a.g.ph;
    p.Qp = a.g.Qp;
    p.cs = a.g.cs;
    return p;
}

constexpr int kChunk = 64;
constexpr int kBlock = 8;  // chunks per ticket

template <int WAVES>
__device__ __forceinline__ void stage(const Args &a, unsigned char *smem, float4 *&Wl, double *&Bl, int4 *&Rl,
                                      float *&Sc) {
    Wl = reinterpret_cast<float4 *>(smem);
    Bl = reinterpret_cast<double *>(Wl + a.K * 9);
    Rl = reinterpret_cast<int4 *>(Bl + a.K);
    Sc = reinterpret_cast<float *>(Rl + a.K);
    for (int i = threadIdx.x; i < a.K * 9; i += WAVES * 64) Wl[i] = a.w[i];
    for (int i = threadIdx.x; i < a.K; i += WAVES * 64) {
        Bl[i] = a.bias[i];
        Rl[i] = a.rects[i];
    }
    for (int i = threadIdx.x; i < a.n_levels; i += WAVES * 64) Sc[i] = a.scale[i];
    __syncthreads();
}

// V0: the production item (weak_eval: uniform loads one half at a time since
// round 2; V11 is round 1's per-shape load branches), one item per lane.
template <int WAVES>
__global__ __launch_bounds__(WAVES * 64, 1) void k_base(Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float4 *Wl; double *Bl; int4 *Rl; float *Sc;
    stage<WAVES>(a, smem, Wl, Bl, Rl, Sc);
    const int lane = threadIdx.x & 63;
    const unsigned q0 = xcc();
    const char *Tb = reinterpret_cast<const char *>(a.table);
    for (unsigned qi = 0; qi < 8; qi++) {  // own XCD's queue first, then steal
      const unsigned q = (q0 + qi) & 7;
      const Item *I = a.items + q * a.cap;
      float *O = a.out + q * a.cap;
      const int n = a.n_items[q];
      for (;;) {
        int b0 = 0;
        if (lane == 0) b0 = atomicAdd(&a.tickets[q * 64], 1);
        b0 = __builtin_amdgcn_readfirstlane(b0) * kChunk * kBlock;
        if (b0 >= n) break;
        const int b1 = min(n, b0 + kChunk * kBlock);
        for (int i = b0 + lane; i < b1; i += 64) {
            Item it = I[i];
            const TabView T{Tb, it.origin << 4};
            O[i] = weak_eval(T, a.g.hs, project(a, Rl, Sc, it), Wl + it.k * 9, Bl[it.k]);
        }
      }
    }
}

// A0 (ablation, wrong results): every lane of a wave evaluates the item of the
// wave's first lane: the same instruction stream with one cache line per
// wave-load -- the issue-bound limit of the item loop.
template <int WAVES>
__global__ __launch_bounds__(WAVES * 64, 1) void k_bcast(Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float4 *Wl; double *Bl; int4 *Rl; float *Sc;
    stage<WAVES>(a, smem, Wl, Bl, Rl, Sc);
    const int lane = threadIdx.x & 63;
    const unsigned q0 = xcc();
    const char *Tb = reinterpret_cast<const char *>(a.table);
    for (unsigned qi = 0; qi < 8; qi++) {
      const unsigned q = (q0 + qi) & 7;
      const Item *I = a.items + q * a.cap;
      float *O = a.out + q * a.cap;
      const int n = a.n_items[q];
      for (;;) {
        int b0 = 0;
        if (lane == 0) b0 = atomicAdd(&a.tickets[q * 64], 1);
        b0 = __builtin_amdgcn_readfirstlane(b0) * kChunk * kBlock;
        if (b0 >= n) break;
        const int b1 = min(n, b0 + kChunk * kBlock);
        for (int i = b0 + lane; i < b1; i += 64) {
            Item it = I[i];
            // the whole item is the first lane's (a window valid for its own
            // level); lane offsets stay inside the first lane's phase-plane row (patch
            // columns reach at most l/6 + 1 <= 106 cells further): no access
            // leaves the table
            const unsigned o0 = __builtin_amdgcn_readfirstlane(it.origin);
            unsigned d = (unsigned)(lane & a.omask);
            if (o0 % (unsigned)a.g.Qp + d + 110u >= (unsigned)a.g.Qp) d = 0;
            it.origin = o0 + d;
            it.k = (unsigned short)__builtin_amdgcn_readfirstlane(it.k);
            it.level = (unsigned char)__builtin_amdgcn_readfirstlane(it.level);
            it.parity = (unsigned char)__builtin_amdgcn_readfirstlane(it.parity);
            const TabView T{Tb, it.origin << 4};
            O[i] = weak_eval(T, a.g.hs, project(a, Rl, Sc, it), Wl + it.k * 9, Bl[it.k]);
        }
      }
    }
}


// Ablations of the item arithmetic (wrong results, timing only): ABL 1 skips
// Normalize, ABL 2 takes the sigmoid in f32, ABL 3 both.
template <int ABL>
__device__ __forceinline__ float item_abl(const TabView &T, int hs, const InlinePatch &pj, const float4 *w4,
                                          double bias) {
    f2 fp[16];
    if (pj.shape == 0) patch_features2<2, 2>(T, pj, hs, fp);
    else if (pj.shape == 1) patch_features2<1, 4>(T, pj, hs, fp);
    else patch_features2<4, 1>(T, pj, hs, fp);
    if (!(ABL & 1)) normalize2(fp);
    if (ABL & 2) {
        f2 s01 = f2{0.0f, 0.0f}, s23 = f2{0.0f, 0.0f};
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const float4 wv = w4[i];
            s01 = f2{wv.x, wv.y} * fp[2 * i] + s01;
            s23 = f2{wv.z, wv.w} * fp[2 * i + 1] + s23;
        }
        const float z = (s01.x + s01.y) + (s23.x + s23.y) + w4[8].x * (float)bias;
        return 1.0f / (1.0f + __expf(-z));
    }
    return lr_predict2(fp, w4, bias);
}

template <int WAVES, int ABL>
__global__ __launch_bounds__(WAVES * 64, 1) void k_abl(Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float4 *Wl; double *Bl; int4 *Rl; float *Sc;
    stage<WAVES>(a, smem, Wl, Bl, Rl, Sc);
    const int lane = threadIdx.x & 63;
    const unsigned q0 = xcc();
    const char *Tb = reinterpret_cast<const char *>(a.table);
    for (unsigned qi = 0; qi < 8; qi++) {
      const unsigned q = (q0 + qi) & 7;
      const Item *I = a.items + q * a.cap;
      float *O = a.out + q * a.cap;
      const int n = a.n_items[q];
      for (;;) {
        int b0 = 0;
        if (lane == 0) b0 = atomicAdd(&a.tickets[q * 64], 1);
        b0 = __builtin_amdgcn_readfirstlane(b0) * kChunk * kBlock;
        if (b0 >= n) break;
        const int b1 = min(n, b0 + kChunk * kBlock);
        for (int i = b0 + lane; i < b1; i += 64) {
            Item it = I[i];
            const TabView T{Tb, it.origin << 4};
            O[i] = item_abl<ABL>(T, a.g.hs, project(a, Rl, Sc, it), Wl + it.k * 9, Bl[it.k]);
        }
      }
    }
}


// V4: two lanes per item on the interleaved 32-B-cell table (TableGeom cs 2):
// lane 2i + h holds half h (channels 4h..4h+3) of item i, so one 16-B load
// instruction reads both halves of 32 items' corners from the same lines
// (half the line touches of the channel-split layout for sparse survivors,
// the same for dense ones).  Normalize's and LR's sequential sums run in
// both lanes of the pair, each term taken from the lane that holds it
// (DPP quad_perm [0,0,2,2] / [1,1,3,3]): the reference's order exactly.
// A trip evaluates 64 items as two 32-item halves, then one f64 sigmoid per
// lane (lane 2i: item i of the first half, lane 2i+1: of the second).
__device__ __forceinline__ float from_even(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xA0, 0xF, 0xF, false));
}
__device__ __forceinline__ float from_odd(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xF5, 0xF, 0xF, false));
}

template <int GW, int GH>
__device__ __forceinline__ void half_feats(const char *Tb, unsigned off, const InlinePatch &pj, f2 (&fh)[8]) {
    int col[GW + 1];
#pragma unroll
    for (int q = 0; q <= GW; q++) col[q] = pj.colq(q);
    float4 cn[GH + 1][GW + 1];
#pragma unroll
    for (int r = 0; r <= GH; r++) {
        const int ro = pj.row0 + r * pj.rowstep;
#pragma unroll
        for (int q = 0; q <= GW; q++)
            cn[r][q] = *reinterpret_cast<const float4 *>(Tb + (off + ((unsigned)(ro + col[q]) << 4)));
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < GH; r++)
#pragma unroll
        for (int q = 0; q < GW; q++) {
            const float4 tl = cn[r][q], br = cn[r + 1][q + 1], tr = cn[r][q + 1], bl = cn[r + 1][q];
            const int o = 2 * (r * GW + q);
            fh[o] = (f2{tl.x, tl.y} + f2{br.x, br.y}) - (f2{tr.x, tr.y} + f2{bl.x, bl.y});
            fh[o + 1] = (f2{tl.z, tl.w} + f2{br.z, br.w}) - (f2{tr.z, tr.w} + f2{bl.z, bl.w});
        }
}

// SS = (((eps + c0) + c1) ... + c7), c_(2 cell + h) in lane h of the pair
__device__ __forceinline__ float ss_pair(const f2 (&fh)[8]) {
    float ss = FLT_EPSILON;
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const f2 a = fh[2 * c] * fh[2 * c], b = fh[2 * c + 1] * fh[2 * c + 1];
        const float cc = (a.x + a.y) + (b.x + b.y);
        ss = ss + from_even(cc);
        ss = ss + from_odd(cc);
    }
    return ss;
}

// z32 of LogisticRegression::Predict: group i = 2 cell + h lives in lane h
__device__ __forceinline__ float z_pair(const f2 (&fh)[8], const float4 *w4, int h) {
    float s[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const float4 wv = w4[2 * c + h];
        const f2 t01 = f2{wv.x, wv.y} * fh[2 * c], t23 = f2{wv.z, wv.w} * fh[2 * c + 1];
        s[0] = s[0] + from_even(t01.x);
        s[1] = s[1] + from_even(t01.y);
        s[2] = s[2] + from_even(t23.x);
        s[3] = s[3] + from_even(t23.y);
        s[0] = s[0] + from_odd(t01.x);
        s[1] = s[1] + from_odd(t01.y);
        s[2] = s[2] + from_odd(t23.x);
        s[3] = s[3] + from_odd(t23.y);
    }
    return (s[0] + s[1]) + (s[2] + s[3]);
}

__device__ __forceinline__ float half_item(const char *Tb, const Item &it, int h, const InlinePatch &pj,
                                           const float4 *w4) {
    f2 fh[8];
    const unsigned off = (it.origin << 4) + (unsigned)h * 16u;
    if (pj.shape == 0) half_feats<2, 2>(Tb, off, pj, fh);
    else if (pj.shape == 1) half_feats<1, 4>(Tb, off, pj, fh);
    else half_feats<4, 1>(Tb, off, pj, fh);
    const float theta = 0.35355338f;
    const float t = sqrtf(ss_pair(fh)) * theta, nt = -t;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        fh[j].x = __builtin_amdgcn_fmed3f(fh[j].x, nt, t);
        fh[j].y = __builtin_amdgcn_fmed3f(fh[j].y, nt, t);
    }
    const float r = 1.0f / sqrtf(ss_pair(fh));
#pragma unroll
    for (int j = 0; j < 8; j++) fh[j] = fh[j] * f2{r, r};
    return z_pair(fh, w4, h);
}

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64, 1) void k_pair(Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float4 *Wl; double *Bl; int4 *Rl; float *Sc;
    stage<WAVES>(a, smem, Wl, Bl, Rl, Sc);
    const int lane = threadIdx.x & 63, h = lane & 1, ii = lane >> 1;
    const unsigned q0 = xcc();
    const char *Tb = reinterpret_cast<const char *>(a.table);
    for (unsigned qi = 0; qi < 8; qi++) {
      const unsigned q = (q0 + qi) & 7;
      const Item *I = a.items + q * a.cap;
      float *O = a.out + q * a.cap;
      const int n = a.n_items[q];
      for (;;) {
        int b0 = 0;
        if (lane == 0) b0 = atomicAdd(&a.tickets[q * 64], 1);
        b0 = __builtin_amdgcn_readfirstlane(b0) * kChunk * kBlock;
        if (b0 >= n) break;
        const int b1 = min(n, b0 + kChunk * kBlock);
        for (int c = b0; c < b1; c += 64) {
            const int iA = c + ii, iB = c + 32 + ii;
            const Item itA = I[iA < b1 ? iA : b0], itB = I[iB < b1 ? iB : b0];
            const float zA = half_item(Tb, itA, h, project(a, Rl, Sc, itA), Wl + itA.k * 9);
            const float zB = half_item(Tb, itB, h, project(a, Rl, Sc, itB), Wl + itB.k * 9);
            const int k = h ? itB.k : itA.k, i = h ? iB : iA;
            double prob = (double)(h ? zB : zA);
            prob += (double)Wl[k * 9 + 8].x * Bl[k];
            prob = 1.0 / (1.0 + exp(-prob));
            if (i < b1) O[i] = (float)prob;
        }
      }
    }
}


// V8: one straight-line set of 20 corner loads for every patch shape (the
// shapes differ only in per-lane offsets; a 2x2 patch's slot 9 repeats its
// corner (2,2)): no shape-divergent load branches, so every vector-memory
// instruction carries all the wave's lanes (the texture addresser costs the
// same per instruction however few lanes are active).
__device__ __forceinline__ void uload(const TabView &T, int half_off, const InlinePatch &pj, float4 (&cn)[20]) {
    int col[5], ro[5];
#pragma unroll
    for (int c = 0; c < 5; c++) col[c] = pj.colq(c);
#pragma unroll
    for (int r = 0; r < 5; r++) ro[r] = pj.row0 + r * pj.rowstep;
    const bool sq = pj.shape == 0, tall = pj.shape == 1;
    int off[10];
#pragma unroll
    for (int m = 0; m < 10; m++) {
        const int o0 = ro[m < 9 ? m / 3 : 2] + col[m < 9 ? m % 3 : 2];
        const int o1 = ro[m / 2] + col[m % 2];
        const int o2 = ro[m / 5] + col[m % 5];
        off[m] = sq ? o0 : (tall ? o1 : o2);
    }
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
        for (int m = 0; m < 10; m++) cn[h * 10 + m] = T.at(h * half_off + off[m]);
}

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64, 1) void k_uload(Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float4 *Wl; double *Bl; int4 *Rl; float *Sc;
    stage<WAVES>(a, smem, Wl, Bl, Rl, Sc);
    const int lane = threadIdx.x & 63;
    const unsigned q0 = xcc();
    const char *Tb = reinterpret_cast<const char *>(a.table);
    for (unsigned qi = 0; qi < 8; qi++) {
      const unsigned q = (q0 + qi) & 7;
      const Item *I = a.items + q * a.cap;
      float *O = a.out + q * a.cap;
      const int n = a.n_items[q];
      for (;;) {
        int b0 = 0;
        if (lane == 0) b0 = atomicAdd(&a.tickets[q * 64], 1);
        b0 = __builtin_amdgcn_readfirstlane(b0) * kChunk * kBlock;
        if (b0 >= n) break;
        const int b1 = min(n, b0 + kChunk * kBlock);
        for (int c = b0; c < b1; c += 64) {
            const int i = c + lane;
            const Item it = I[i < b1 ? i : b0];
            const InlinePatch pj = project(a, Rl, Sc, it);
            float4 cn[20];
            uload(TabView{Tb, it.origin << 4}, a.g.hs, pj, cn);
            __builtin_amdgcn_sched_barrier(0);
            f2 fp[16];
            {
                float4 c0[10], c1[10];
#pragma unroll
                for (int m = 0; m < 10; m++) { c0[m] = cn[m]; c1[m] = cn[10 + m]; }
                f2 h0[8], h1[8];
                half_box(pj.shape, c0, h0);
                half_box(pj.shape, c1, h1);
#pragma unroll
                for (int cl = 0; cl < 4; cl++) {
                    fp[4 * cl] = h0[2 * cl]; fp[4 * cl + 1] = h0[2 * cl + 1];
                    fp[4 * cl + 2] = h1[2 * cl]; fp[4 * cl + 3] = h1[2 * cl + 1];
                }
            }
            normalize2(fp);
            const float p = lr_predict2(fp, Wl + it.k * 9, Bl[it.k]);
            if (i < b1) O[i] = p;
        }
      }
    }
}


// V9: V4's two lanes per item with V8's uniform load set: each lane issues
// the 10 corner loads of its half, straight-line for every shape.
template <int GW, int GH>
__device__ __forceinline__ void ib_half_box(const float4 (&cn)[10], f2 (&fh)[8]) {
#pragma unroll
    for (int r = 0; r < GH; r++)
#pragma unroll
        for (int q = 0; q < GW; q++) {
            const float4 tl = cn[r * (GW + 1) + q], br = cn[(r + 1) * (GW + 1) + q + 1];
            const float4 tr = cn[r * (GW + 1) + q + 1], bl = cn[(r + 1) * (GW + 1) + q];
            const int o = 2 * (r * GW + q);
            fh[o] = (f2{tl.x, tl.y} + f2{br.x, br.y}) - (f2{tr.x, tr.y} + f2{bl.x, bl.y});
            fh[o + 1] = (f2{tl.z, tl.w} + f2{br.z, br.w}) - (f2{tr.z, tr.w} + f2{bl.z, bl.w});
        }
}

__device__ __forceinline__ float half_item_u(const char *Tb, const Item &it, int h, const InlinePatch &pj,
                                             const float4 *w4) {
    int col[5], ro[5];
#pragma unroll
    for (int c = 0; c < 5; c++) col[c] = pj.colq(c);
#pragma unroll
    for (int r = 0; r < 5; r++) ro[r] = pj.row0 + r * pj.rowstep;
    const bool sq = pj.shape == 0, tall = pj.shape == 1;
    const unsigned base = (it.origin << 4) + (unsigned)h * 16u;
    float4 cn[10];
#pragma unroll
    for (int m = 0; m < 10; m++) {
        const int o0 = ro[m < 9 ? m / 3 : 2] + col[m < 9 ? m % 3 : 2];
        const int o1 = ro[m / 2] + col[m % 2];
        const int o2 = ro[m / 5] + col[m % 5];
        const int off = sq ? o0 : (tall ? o1 : o2);
        cn[m] = *reinterpret_cast<const float4 *>(Tb + (base + ((unsigned)off << 4)));
    }
    __builtin_amdgcn_sched_barrier(0);
    f2 fh[8];
    if (sq) ib_half_box<2, 2>(cn, fh);
    else if (tall) ib_half_box<1, 4>(cn, fh);
    else ib_half_box<4, 1>(cn, fh);
    const float theta = 0.35355338f;
    const float t = sqrtf(ss_pair(fh)) * theta, nt = -t;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        fh[j].x = __builtin_amdgcn_fmed3f(fh[j].x, nt, t);
        fh[j].y = __builtin_amdgcn_fmed3f(fh[j].y, nt, t);
    }
    const float r = 1.0f / sqrtf(ss_pair(fh));
#pragma unroll
    for (int j = 0; j < 8; j++) fh[j] = fh[j] * f2{r, r};
    return z_pair(fh, w4, h);
}

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64, 1) void k_pairu(Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float4 *Wl; double *Bl; int4 *Rl; float *Sc;
    stage<WAVES>(a, smem, Wl, Bl, Rl, Sc);
    const int lane = threadIdx.x & 63, h = lane & 1, ii = lane >> 1;
    const unsigned q0 = xcc();
    const char *Tb = reinterpret_cast<const char *>(a.table);
    for (unsigned qi = 0; qi < 8; qi++) {
      const unsigned q = (q0 + qi) & 7;
      const Item *I = a.items + q * a.cap;
      float *O = a.out + q * a.cap;
      const int n = a.n_items[q];
      for (;;) {
        int b0 = 0;
        if (lane == 0) b0 = atomicAdd(&a.tickets[q * 64], 1);
        b0 = __builtin_amdgcn_readfirstlane(b0) * kChunk * kBlock;
        if (b0 >= n) break;
        const int b1 = min(n, b0 + kChunk * kBlock);
        for (int c = b0; c < b1; c += 64) {
            const int iA = c + ii, iB = c + 32 + ii;
            const Item itA = I[iA < b1 ? iA : b0], itB = I[iB < b1 ? iB : b0];
            const float zA = half_item_u(Tb, itA, h, project(a, Rl, Sc, itA), Wl + itA.k * 9);
            const float zB = half_item_u(Tb, itB, h, project(a, Rl, Sc, itB), Wl + itB.k * 9);
            const int k = h ? itB.k : itA.k, i = h ? iB : iA;
            double prob = (double)(h ? zB : zA);
            prob += (double)Wl[k * 9 + 8].x * Bl[k];
            prob = 1.0 / (1.0 + exp(-prob));
            if (i < b1) O[i] = (float)prob;
        }
      }
    }
}


// V10: V8's uniform loads one half at a time (10 loads, box sums of that
// half, then the other half's 10 loads): half the corner registers, two
// memory round trips per item.
__device__ __forceinline__ void uload_half(const TabView &T, int hoff, const int (&off)[10], float4 (&cn)[10]) {
#pragma unroll
    for (int m = 0; m < 10; m++) cn[m] = T.at(hoff + off[m]);
}
__device__ __forceinline__ void box_half(int shape, const float4 (&cn)[10], f2 *fh) {
    if (shape == 0) ib_half_box<2, 2>(cn, *reinterpret_cast<f2(*)[8]>(fh));
    else if (shape == 1) ib_half_box<1, 4>(cn, *reinterpret_cast<f2(*)[8]>(fh));
    else ib_half_box<4, 1>(cn, *reinterpret_cast<f2(*)[8]>(fh));
}

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64, 1) void k_uhalf(Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float4 *Wl; double *Bl; int4 *Rl; float *Sc;
    stage<WAVES>(a, smem, Wl, Bl, Rl, Sc);
    const int lane = threadIdx.x & 63;
    const unsigned q0 = xcc();
    const char *Tb = reinterpret_cast<const char *>(a.table);
    for (unsigned qi = 0; qi < 8; qi++) {
      const unsigned q = (q0 + qi) & 7;
      const Item *I = a.items + q * a.cap;
      float *O = a.out + q * a.cap;
      const int n = a.n_items[q];
      for (;;) {
        int b0 = 0;
        if (lane == 0) b0 = atomicAdd(&a.tickets[q * 64], 1);
        b0 = __builtin_amdgcn_readfirstlane(b0) * kChunk * kBlock;
        if (b0 >= n) break;
        const int b1 = min(n, b0 + kChunk * kBlock);
        for (int c = b0; c < b1; c += 64) {
            const int i = c + lane;
            const Item it = I[i < b1 ? i : b0];
            const InlinePatch pj = project(a, Rl, Sc, it);
            int col[5], ro[5], off[10];
#pragma unroll
            for (int q2 = 0; q2 < 5; q2++) col[q2] = pj.colq(q2);
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
            const TabView T{Tb, it.origin << 4};
            f2 h0[8], h1[8];
            {
                float4 cn[10];
                uload_half(T, 0, off, cn);
                __builtin_amdgcn_sched_barrier(0);
                box_half(pj.shape, cn, h0);
            }
            {
                float4 cn[10];
                uload_half(T, a.g.hs, off, cn);
                __builtin_amdgcn_sched_barrier(0);
                box_half(pj.shape, cn, h1);
            }
            // interleave the halves back into the 32-feature order: f[8 cell + 4 h + ch]
            f2 fp[16];
#pragma unroll
            for (int cl = 0; cl < 4; cl++) {
                fp[4 * cl] = h0[2 * cl];
                fp[4 * cl + 1] = h0[2 * cl + 1];
                fp[4 * cl + 2] = h1[2 * cl];
                fp[4 * cl + 3] = h1[2 * cl + 1];
            }
            normalize2(fp);
            const float p = lr_predict2(fp, Wl + it.k * 9, Bl[it.k]);
            if (i < b1) O[i] = p;
        }
      }
    }
}

// V12: one item per lane on the interleaved 32-B-cell table (TableGeom cs 2),
// loads paired across the wave's halves: for each corner slot, instruction X
// reads cell(A).h0 in lane i < 32 and cell(A).h1 in lane i + 32 (A = lane
// i's item), instruction Y reads cell(B).h0 in lane i and cell(B).h1 in lane
// i + 32 (B = lane i + 32's item): each instruction's lane pair touches one
// 32-B cell, i.e. one cache line, instead of the channel-split layout's two
// lines per lane in sparse stages (dense stages: the same 8 lines per 1 KiB).
// One v_permlane32_swap per dword then gives every lane both halves of its
// own item (X' = own h0, Y' = own h1).  All 20 loads in flight.
template <int SW>
__device__ __forceinline__ auto swp(unsigned a, unsigned b) {
    if constexpr (SW == 32) return __builtin_amdgcn_permlane32_swap(a, b, false, false);
    else return __builtin_amdgcn_permlane16_swap(a, b, false, false);
}

// V13: V12 with the pairs (i, i + 16) of v_permlane16_swap (rows 0/1, 2/3)
template <int WAVES, int SW>
__global__ __launch_bounds__(WAVES * 64, 1) void k_xswap(Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float4 *Wl; double *Bl; int4 *Rl; float *Sc;
    stage<WAVES>(a, smem, Wl, Bl, Rl, Sc);
    const int lane = threadIdx.x & 63;
    const unsigned hoff = (lane & SW) ? 16u : 0u;  // SW 32: pairs (i, i+32); 16: (i, i+16)
    const unsigned q0 = xcc();
    const char *Tb = reinterpret_cast<const char *>(a.table);
    for (unsigned qi = 0; qi < 8; qi++) {
      const unsigned q = (q0 + qi) & 7;
      const Item *I = a.items + q * a.cap;
      float *O = a.out + q * a.cap;
      const int n = a.n_items[q];
      for (;;) {
        int b0 = 0;
        if (lane == 0) b0 = atomicAdd(&a.tickets[q * 64], 1);
        b0 = __builtin_amdgcn_readfirstlane(b0) * kChunk * kBlock;
        if (b0 >= n) break;
        const int b1 = min(n, b0 + kChunk * kBlock);
        for (int c = b0; c < b1; c += 64) {
            const int i = c + lane;
            const Item it = I[i < b1 ? i : b0];
            const InlinePatch pj = project(a, Rl, Sc, it);
            int off[10];
            corner_offsets(pj, off);
            float4 X[10], Y[10];
#pragma unroll
            for (int m = 0; m < 10; m++) {
                const unsigned own = (it.origin + (unsigned)off[m]) << 4;
                const auto pa = swp<SW>(own, own);
                X[m] = *reinterpret_cast<const float4 *>(Tb + (pa[0] + hoff));
                Y[m] = *reinterpret_cast<const float4 *>(Tb + (pa[1] + hoff));
            }
            __builtin_amdgcn_sched_barrier(0);
            float4 c0[10], c1[10];
#pragma unroll
            for (int m = 0; m < 10; m++) {
                const auto sx = swp<SW>(__float_as_uint(X[m].x), __float_as_uint(Y[m].x)); 
                const auto sy = swp<SW>(__float_as_uint(X[m].y), __float_as_uint(Y[m].y));
                const auto sz = swp<SW>(__float_as_uint(X[m].z), __float_as_uint(Y[m].z));
                const auto sw = swp<SW>(__float_as_uint(X[m].w), __float_as_uint(Y[m].w));
                c0[m] = make_float4(__uint_as_float(sx[0]), __uint_as_float(sy[0]), __uint_as_float(sz[0]), __uint_as_float(sw[0]));
                c1[m] = make_float4(__uint_as_float(sx[1]), __uint_as_float(sy[1]), __uint_as_float(sz[1]), __uint_as_float(sw[1]));
            }
            f2 h0[8], h1[8], fp[16];
            half_box(pj.shape, c0, h0);
            half_box(pj.shape, c1, h1);
#pragma unroll
            for (int cl = 0; cl < 4; cl++) {
                fp[4 * cl] = h0[2 * cl]; fp[4 * cl + 1] = h0[2 * cl + 1];
                fp[4 * cl + 2] = h1[2 * cl]; fp[4 * cl + 3] = h1[2 * cl + 1];
            }
            normalize2(fp);
            const float p = lr_predict2(fp, Wl + it.k * 9, Bl[it.k]);
            if (i < b1) O[i] = p;
        }
      }
    }
}

// A3 (ablation, wrong results): the production item with every corner's
// table row folded into a band of (fold+1) rows (row & fold): the same
// lanes->lines pattern per wave-instruction, a table footprint the XCD's L2
// holds -- isolates the cost of the gathers that go beyond L2.
template <int GW, int GH>
__device__ __forceinline__ void feat_fold(const char *Tb, unsigned colpart, int y, int py, int c, int x0, int cb,
                                          const TableGeom &g, unsigned fold, f2 (&fp)[16]) {
    int col[GW + 1];
#pragma unroll
    for (int q = 0; q <= GW; q++) {
        const unsigned x = (unsigned)(x0 + q * c), qq = __umulhi(x, g.phm);
        col[q] = (int)(x - qq * (unsigned)g.ph) * g.Qp + (int)qq - cb;
    }
    float4 cn[2][GH + 1][GW + 1];
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
        for (int r = 0; r <= GH; r++) {
            const unsigned ro = ((unsigned)(y + py + r * c) & fold) * (unsigned)g.rowp + colpart + h * g.hs;
#pragma unroll
            for (int q = 0; q <= GW; q++)
                cn[h][r][q] = *reinterpret_cast<const float4 *>(Tb + ((ro + col[q]) << 4));
        }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
        for (int r = 0; r < GH; r++)
#pragma unroll
            for (int q = 0; q < GW; q++) {
                const float4 tl = cn[h][r][q], br = cn[h][r + 1][q + 1];
                const float4 tr = cn[h][r][q + 1], bl = cn[h][r + 1][q];
                const int o = 4 * (r * GW + q) + 2 * h;
                fp[o] = (f2{tl.x, tl.y} + f2{br.x, br.y}) - (f2{tr.x, tr.y} + f2{bl.x, bl.y});
                fp[o + 1] = (f2{tl.z, tl.w} + f2{br.z, br.w}) - (f2{tr.z, tr.w} + f2{bl.z, bl.w});
            }
}

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64, 1) void k_fold(Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float4 *Wl; double *Bl; int4 *Rl; float *Sc;
    stage<WAVES>(a, smem, Wl, Bl, Rl, Sc);
    const int lane = threadIdx.x & 63;
    const unsigned q0 = xcc();
    const char *Tb = reinterpret_cast<const char *>(a.table);
    for (unsigned qi = 0; qi < 8; qi++) {
      const unsigned q = (q0 + qi) & 7;
      const Item *I = a.items + q * a.cap;
      float *O = a.out + q * a.cap;
      const int n = a.n_items[q];
      for (;;) {
        int b0 = 0;
        if (lane == 0) b0 = atomicAdd(&a.tickets[q * 64], 1);
        b0 = __builtin_amdgcn_readfirstlane(b0) * kChunk * kBlock;
        if (b0 >= n) break;
        const int b1 = min(n, b0 + kChunk * kBlock);
        for (int i = b0 + lane; i < b1; i += 64) {
            const Item it = I[i];
            const int y = (int)(it.origin / (unsigned)a.g.rowp);
            const unsigned colpart = it.origin - (unsigned)y * (unsigned)a.g.rowp;
            const int4 rc = Rl[it.k];
            const float s = Sc[it.level];
            const int px = (int)((float)rc.x * s), py = (int)((float)rc.y * s), e = (int)((float)rc.z * s);
            const int c = rc.w == 0 ? (e >> 1) : e;
            const int x0 = it.parity * a.g.step + px;
            const int cb = a.g.at0((unsigned)(it.parity * a.g.step));
            f2 fp[16];
            if (rc.w == 0) feat_fold<2, 2>(Tb, colpart, y, py, c, x0, cb, a.g, a.fold, fp);
            else if (rc.w == 1) feat_fold<1, 4>(Tb, colpart, y, py, c, x0, cb, a.g, a.fold, fp);
            else feat_fold<4, 1>(Tb, colpart, y, py, c, x0, cb, a.g, a.fold, fp);
            normalize2(fp);
            O[i] = lr_predict2(fp, Wl + it.k * 9, Bl[it.k]);
        }
      }
    }
}

// V14 (round 4 ablation, wrong results, timing only): the LDS-path ceiling of
// the item loop.  Every corner is read from a 64 KiB table tile in the
// workgroup's LDS (ds_read_b128 at the global cell offset mod 4096, so the
// lanes of a wave instruction keep the production access pattern: consecutive
// windows -> consecutive 16-B cells, same bank spread) instead of through
// the texture path; the tile is staged once per workgroup (no staging cost
// in the loop).  Same corner slots, box sums, Normalize, LR, sigmoid: the
// time an item loop would take if every gather were an LDS hit for free.
constexpr int kTileCells = 4096;  // 64 KiB of float4
template <class P>
__device__ __forceinline__ void features_lds(const float4 *tile, unsigned org, int half_off, const P &pj,
                                             f2 (&fp)[16]) {
    int off[10];
    corner_offsets(pj, off);
    f2 h[2][8];
#pragma unroll
    for (int hh = 0; hh < 2; hh++) {
        float4 cn[10];
#pragma unroll
        for (int m = 0; m < 10; m++) cn[m] = tile[(org + (unsigned)(hh * half_off + off[m])) & (kTileCells - 1)];
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

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64, 1) void k_ldsgather(Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float4 *Wl; double *Bl; int4 *Rl; float *Sc;
    stage<WAVES>(a, smem, Wl, Bl, Rl, Sc);
    float4 *tile = reinterpret_cast<float4 *>(smem + (((size_t)a.K * (144 + 8 + 16) + a.n_levels * 4 + 63) & ~(size_t)63));
    for (int i = threadIdx.x; i < kTileCells; i += WAVES * 64) tile[i] = a.table[(size_t)a.g.rowp * 400 + i];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const unsigned q0 = xcc();
    for (unsigned qi = 0; qi < 8; qi++) {
      const unsigned q = (q0 + qi) & 7;
      const Item *I = a.items + q * a.cap;
      float *O = a.out + q * a.cap;
      const int n = a.n_items[q];
      for (;;) {
        int b0 = 0;
        if (lane == 0) b0 = atomicAdd(&a.tickets[q * 64], 1);
        b0 = __builtin_amdgcn_readfirstlane(b0) * kChunk * kBlock;
        if (b0 >= n) break;
        const int b1 = min(n, b0 + kChunk * kBlock);
        for (int i = b0 + lane; i < b1; i += 64) {
            const Item it = I[i];
            f2 fp[16];
            features_lds(tile, it.origin, a.g.hs, project(a, Rl, Sc, it), fp);
            normalize2(fp);
            O[i] = lr_predict2(fp, Wl + it.k * 9, Bl[it.k]);
        }
      }
    }
}

// V15 (round 4): the production item with every corner fetched by LDS DMA
// (global_load_lds_dwordx4: per-lane source, the wave's 1 KiB lands
// lane-linear in its LDS slot) and read back with a conflict-free
// ds_read_b128 at lane*16: does routing the gathers' data into LDS instead of
// VGPRs relieve the texture data path (TD ~97 % busy in the chain kernel)?
// Same corners, same arithmetic: bit-exact with V0.
template <class P>
__device__ __forceinline__ void features_dma(const char *Tb, unsigned off, int half_off, const P &pj,
                                             float4 *slot, f2 (&fp)[16]) {
    int co[10];
    corner_offsets(pj, co);
    const int lane = threadIdx.x & 63;
    f2 h[2][8];
#pragma unroll
    for (int hh = 0; hh < 2; hh++) {
#pragma unroll
        for (int m = 0; m < 10; m++)
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(Tb + (off + ((unsigned)(hh * half_off + co[m]) << 4))),
                (__attribute__((address_space(3))) void *)(slot + m * 64), 16, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        float4 cn[10];
#pragma unroll
        for (int m = 0; m < 10; m++) cn[m] = slot[m * 64 + lane];
        half_box(pj.shape, cn, h[hh]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot reads done before the next half's DMA
    }
#pragma unroll
    for (int c = 0; c < 4; c++) {
        fp[4 * c] = h[0][2 * c];
        fp[4 * c + 1] = h[0][2 * c + 1];
        fp[4 * c + 2] = h[1][2 * c];
        fp[4 * c + 3] = h[1][2 * c + 1];
    }
}

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64, 1) void k_dma(Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float4 *Wl; double *Bl; int4 *Rl; float *Sc;
    stage<WAVES>(a, smem, Wl, Bl, Rl, Sc);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float4 *slot = reinterpret_cast<float4 *>(smem + (((size_t)a.K * (144 + 8 + 16) + a.n_levels * 4 + 63) & ~(size_t)63)) +
                   (size_t)wv * 10 * 64;
    const int lane = threadIdx.x & 63;
    const unsigned q0 = xcc();
    const char *Tb = reinterpret_cast<const char *>(a.table);
    for (unsigned qi = 0; qi < 8; qi++) {
      const unsigned q = (q0 + qi) & 7;
      const Item *I = a.items + q * a.cap;
      float *O = a.out + q * a.cap;
      const int n = a.n_items[q];
      for (;;) {
        int b0 = 0;
        if (lane == 0) b0 = atomicAdd(&a.tickets[q * 64], 1);
        b0 = __builtin_amdgcn_readfirstlane(b0) * kChunk * kBlock;
        if (b0 >= n) break;
        const int b1 = min(n, b0 + kChunk * kBlock);
        for (int i0 = b0; i0 < b1; i0 += 64) {  // (the whole wave runs every iteration: the DMA needs it)
            const int i = i0 + lane;
            const bool live = i < b1;
            const Item it = I[live ? i : b0];
            f2 fp[16];
            features_dma(Tb, it.origin << 4, a.g.hs, project(a, Rl, Sc, it), slot, fp);
            normalize2(fp);
            const float o = lr_predict2(fp, Wl + it.k * 9, Bl[it.k]);
            if (live) O[i] = o;
        }
      }
    }
}

// V16 (round 5): V15's LDS DMA, software-pipelined.
// Each wave holds two 10-KiB slot sets (corner slots of half 0 and half 1 of
// one 64-item chunk).  While chunk c runs Normalize + LR + the f64 sigmoid
// (the item's long dependent VALU tail), the DMAs of BOTH halves of chunk
// c+1 are in flight into the slots chunk c's box sums have just freed.  No
// corner VGPRs are held across the tail (the register form spilled:
// profiles/r3/pipe2), at the price of 20 KiB of LDS per wave: 6 waves per
// CU next to the model.
// The DMAs are issued as inline asm (global_load_lds_dwordx4, M0 = the slot's
// LDS address): the compiler then inserts no "wait for every outstanding LDS
// DMA" before each LDS read (the builtin made it wait vmcnt(0) before the LR
// weight reads, which serialised the pipeline); its own waits for the
// VMEM ops it knows stay conservative (the DMAs only add younger ops).
// vmcnt bookkeeping (in-order vector-memory counter): at the top of chunk c
// the outstanding VMEM ops are, oldest first, DMA(c).h0 [10], DMA(c).h1
// [10], STORE(c-1) [1, not on a ticket's first chunk], ITEM(c+1) [1].
// Same corners, same arithmetic: bit-exact with V0.
__device__ __forceinline__ void dma16(unsigned lds, unsigned voff, const char *base) {
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
                 :: "s"(lds), "v"(voff), "s"(base) : "memory", "m0");
}
template <class P>
__device__ __forceinline__ void dma_corners(const char *Tb, unsigned off, int half_off, const P &pj,
                                            unsigned ldsA) {
    int co[10];
    corner_offsets(pj, co);
#pragma unroll
    for (int hh = 0; hh < 2; hh++)
#pragma unroll
        for (int m = 0; m < 10; m++)
            dma16(ldsA + (unsigned)(hh * 10 + m) * 1024u, off + ((unsigned)(hh * half_off + co[m]) << 4), Tb);
}

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64, 1) void k_dmap(Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float4 *Wl; double *Bl; int4 *Rl; float *Sc;
    stage<WAVES>(a, smem, Wl, Bl, Rl, Sc);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float4 *slotA = reinterpret_cast<float4 *>(smem + (((size_t)a.K * (144 + 8 + 16) + a.n_levels * 4 + 63) & ~(size_t)63)) +
                    (size_t)wv * 20 * 64;
    const float4 *slotB = slotA + 10 * 64;
    const unsigned ldsA = __builtin_amdgcn_readfirstlane(
        (unsigned)(size_t)(__attribute__((address_space(3))) float4 *)slotA);
    const int lane = threadIdx.x & 63;
    const unsigned q0 = xcc();
    const char *Tb = reinterpret_cast<const char *>(a.table);
    for (unsigned qi = 0; qi < 8; qi++) {
      const unsigned q = (q0 + qi) & 7;
      const Item *I = a.items + q * a.cap;
      float *O = a.out + q * a.cap;
      const int n = a.n_items[q];
      for (;;) {
        int b0 = 0;
        if (lane == 0) b0 = atomicAdd(&a.tickets[q * 64], 1);
        b0 = __builtin_amdgcn_readfirstlane(b0) * kChunk * kBlock;
        if (b0 >= n) break;
        const int b1 = min(n, b0 + kChunk * kBlock);
        auto item_at = [&](int c0) { const int i = c0 + lane; return I[i < b1 ? i : b0]; };
        // prologue: chunk b0's corners in flight
        Item it = item_at(b0);
        InlinePatch pj = project(a, Rl, Sc, it);
        dma_corners(Tb, it.origin << 4, a.g.hs, pj, ldsA);
        for (int c = b0; c < b1; c += 64) {
            const bool more = c + 64 < b1;
            const Item itn = item_at(more ? c + 64 : c);  // ITEM(c+1): the youngest VMEM op
            f2 h[2][8];
            if (c == b0) asm volatile("s_waitcnt vmcnt(11)" ::: "memory");  // DMA(c).h0 landed
            else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
            {
                float4 cn[10];
#pragma unroll
                for (int m = 0; m < 10; m++) cn[m] = slotA[m * 64 + lane];
                half_box(pj.shape, cn, h[0]);
            }
            if (c == b0) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");   // DMA(c).h1 landed
            else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            {
                float4 cn[10];
#pragma unroll
                for (int m = 0; m < 10; m++) cn[m] = slotB[m * 64 + lane];
                half_box(pj.shape, cn, h[1]);
            }
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // slots read; ITEM(c+1), STORE(c-1) done
            {   // ITEM(c+1) consumed on every path: otherwise the compiler sees its
                // load still pending past the branch and waits vmcnt(0) in the
                // tail (which, unknown to it, would also wait for DMA(c+1))
                const uint2 raw = __builtin_bit_cast(uint2, itn);
                asm volatile("" :: "v"(raw.x), "v"(raw.y));
            }
            const int k = it.k;
            if (more) {  // chunk c+1's corners into the freed slots
                it = itn;
                pj = project(a, Rl, Sc, it);
                dma_corners(Tb, it.origin << 4, a.g.hs, pj, ldsA);
            }
            f2 fp[16];
#pragma unroll
            for (int cl = 0; cl < 4; cl++) {
                fp[4 * cl] = h[0][2 * cl];
                fp[4 * cl + 1] = h[0][2 * cl + 1];
                fp[4 * cl + 2] = h[1][2 * cl];
                fp[4 * cl + 3] = h[1][2 * cl + 1];
            }
            normalize2(fp);
            const float o = lr_predict2(fp, Wl + k * 9, Bl[k]);
            const int i = c + lane;
            if (i < b1) O[i] = o;  // (lane 0 always stores: one VMEM op per chunk)
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
}

}  // namespace

extern "C" int ib_run(int variant, int waves, const Args *a, void *stream) {
    const size_t lds = (size_t)a->K * (144 + 8 + 16) + a->n_levels * 4 + 64;
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipStream_t s = (hipStream_t)stream;
    hipMemsetAsync(a->tickets, 0, 8 * 64 * 4, s);
#define L(KER, WV) hipLaunchKernelGGL((KER<WV>), dim3(cus), dim3(WV * 64), lds, s, *a)
    if (variant == 0) {
        if (waves == 4) L(k_base, 4); else if (waves == 6) L(k_base, 6);
        else if (waves == 8) L(k_base, 8); else if (waves == 12) L(k_base, 12); else if (waves == 16) L(k_base, 16); else return -1;
    } else if (variant == 1) {
        return -1;  // (V1, the software-pipelined item, retired: slower, profiles/r2/itembench.md)
    } else if (variant == 2) {
        if (waves == 8) L(k_bcast, 8); else if (waves == 12) L(k_bcast, 12); else if (waves == 16) L(k_bcast, 16); else return -1;
    } else if (variant == 9) {
        if (waves == 8) L(k_pairu, 8); else if (waves == 12) L(k_pairu, 12); else if (waves == 16) L(k_pairu, 16); else return -1;
    } else if (variant == 10) {
        if (waves == 8) L(k_uhalf, 8); else if (waves == 12) L(k_uhalf, 12); else if (waves == 16) L(k_uhalf, 16); else return -1;
    } else if (variant == 8) {
        if (waves == 8) L(k_uload, 8); else if (waves == 12) L(k_uload, 12); else if (waves == 16) L(k_uload, 16); else return -1;
    } else if (variant == 4) {
        if (waves == 8) L(k_pair, 8); else if (waves == 12) L(k_pair, 12); else if (waves == 16) L(k_pair, 16); else return -1;
    } else if (variant == 11) {  // the round-1 production item: per-shape load branches
        if (waves != 12) return -1;
        hipLaunchKernelGGL((k_abl<12, 0>), dim3(cus), dim3(768), lds, s, *a);
    } else if (variant >= 5 && variant <= 7) {
        if (waves != 12) return -1;
        if (variant == 5) hipLaunchKernelGGL((k_abl<12, 1>), dim3(cus), dim3(768), lds, s, *a);
        else if (variant == 6) hipLaunchKernelGGL((k_abl<12, 2>), dim3(cus), dim3(768), lds, s, *a);
        else hipLaunchKernelGGL((k_abl<12, 3>), dim3(cus), dim3(768), lds, s, *a);
    } else if (variant == 12) {
        if (waves == 12) hipLaunchKernelGGL((k_xswap<12, 32>), dim3(cus), dim3(768), lds, s, *a);
        else if (waves == 16) hipLaunchKernelGGL((k_xswap<16, 32>), dim3(cus), dim3(1024), lds, s, *a);
        else return -1;
    } else if (variant == 13) {
        if (waves == 12) hipLaunchKernelGGL((k_xswap<12, 16>), dim3(cus), dim3(768), lds, s, *a);
        else if (waves == 16) hipLaunchKernelGGL((k_xswap<16, 16>), dim3(cus), dim3(1024), lds, s, *a);
        else return -1;
    } else if (variant == 14) {  // LDS-path ceiling: + the 64 KiB tile
        const size_t lt = ((lds + 63) & ~(size_t)63) + kTileCells * 16;
        if (waves == 12) hipLaunchKernelGGL((k_ldsgather<12>), dim3(cus), dim3(768), lt, s, *a);
        else if (waves == 16) hipLaunchKernelGGL((k_ldsgather<16>), dim3(cus), dim3(1024), lt, s, *a);
        else return -1;
    } else if (variant == 15) {  // corners by LDS DMA: + 10 KiB per wave
        const size_t lt = ((lds + 63) & ~(size_t)63) + (size_t)waves * 10 * 1024;
        if (waves == 8) hipLaunchKernelGGL((k_dma<8>), dim3(cus), dim3(512), lt, s, *a);
        else if (waves == 12) hipLaunchKernelGGL((k_dma<12>), dim3(cus), dim3(768), lt, s, *a);
        else return -1;
    } else if (variant == 16) {  // pipelined LDS DMA: + 20 KiB per wave
        const size_t lt = ((lds + 63) & ~(size_t)63) + (size_t)waves * 20 * 1024;
        if (waves == 4) hipLaunchKernelGGL((k_dmap<4>), dim3(cus), dim3(256), lt, s, *a);
        else if (waves == 6) hipLaunchKernelGGL((k_dmap<6>), dim3(cus), dim3(384), lt, s, *a);
        else return -1;
    } else if (variant == 3) {
        if (waves == 8) L(k_fold, 8); else if (waves == 12) L(k_fold, 12); else if (waves == 16) L(k_fold, 16); else return -1;
    } else {
        return -1;
    }
#undef L
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int ib_args_size() { return (int)sizeof(Args); }
