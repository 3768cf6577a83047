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

// V0: the production item (weak_eval), one item per lane per iteration.
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

// V1: software pipelined: the next item's corner loads are issued right
// after this item's box sums (uniform 20-load set), so they are in flight
// during this item's normalise + LR + sigmoid.
template <int WAVES>
__global__ __launch_bounds__(WAVES * 64, 1) void k_pipe(Args a) {
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
        float4 cn[20];
        int i = b0 + lane;
        Item it{};
        int shape = 0;
        if (i < b1) {
            it = I[i];
            const InlinePatch p = project(a, Rl, Sc, it);
            shape = p.shape;
            corners_load(TabView{Tb, it.origin << 4}, a.g.hs, p, cn);
        }
        for (int c = b0; c < b1; c += 64) {
            f2 fp[16];
            corners_box(shape, cn, fp);
            const int ic = i;
            const Item itc = it;
            i = c + 64 + lane;
            if (i < b1) {
                it = I[i];
                    const InlinePatch p = project(a, Rl, Sc, it);
                shape = p.shape;
                corners_load(TabView{Tb, it.origin << 4}, a.g.hs, p, cn);
            }
            __builtin_amdgcn_sched_barrier(0);
            if (ic < b1) {
                normalize2(fp);
                O[ic] = lr_predict2(fp, Wl + itc.k * 9, Bl[itc.k]);
            }
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

}  // namespace

extern "C" int ib_run(int variant, int waves, const Args *a, void *stream) {
    const size_t lds = (size_t)a->K * (144 + 8 + 16) + a->n_levels * 4 + 64;
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipStream_t s = (hipStream_t)stream;
    hipMemsetAsync(a->tickets, 0, 8 * 64 * 4, s);
#define L(KER, WV) hipLaunchKernelGGL((KER<WV>), dim3(cus), dim3(WV * 64), lds, s, *a)
    if (variant == 0) {
        if (waves == 8) L(k_base, 8); else if (waves == 12) L(k_base, 12); else if (waves == 16) L(k_base, 16); else return -1;
    } else if (variant == 1) {
        if (waves == 8) L(k_pipe, 8); else if (waves == 12) L(k_pipe, 12); else if (waves == 16) L(k_pipe, 16); else return -1;
    } else if (variant == 2) {
        if (waves == 8) L(k_bcast, 8); else if (waves == 12) L(k_bcast, 12); else if (waves == 16) L(k_bcast, 16); else return -1;
    } else if (variant == 3) {
        if (waves == 8) L(k_fold, 8); else if (waves == 12) L(k_fold, 12); else if (waves == 16) L(k_fold, 16); else return -1;
    } else {
        return -1;
    }
#undef L
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int ib_args_size() { return (int)sizeof(Args); }
