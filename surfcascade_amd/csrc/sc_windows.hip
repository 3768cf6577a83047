// sc_windows.hip -- gfx950 (CDNA4) window kernels of the detect path.
//
// cascade_kernel: persistent workgroups of 4 independent waves.  Each wave
// pulls tasks from its XCD's queue; a task is one strip of one (frame, level,
// row y) row of the stride-`step` window grid (ObjDetector.cpp:178-186).
// XCD x owns the same column band of every row (sc_kernels.hpp), which keeps
// the table rows its L2 sees narrow: measured on MI355X, 1080p x 24 levels,
// L2 hit rate 13% -> 48-71% and beyond-L2 read requests -37..-55% against
// row-per-wave tasks, where the gathers were capped by fabric bandwidth.
//   1) prefilter: sum(win) > area*6 (DenseSURFFeatureExtractor.cpp:351-358,
//      ObjDetector.cpp:188); survivors compacted in x order (__ballot + popc).
//   2) cascade, stage by stage (ObjDetector.cpp:193-199).  Many survivors:
//      one lane per survivor, the weak index k wave-uniform, the lane sums its
//      window's results in weak order in a register (GentleAdaboost.cpp:
//      255-258).  Few survivors: (survivor, weak) items packed k-major over
//      the lanes, results through LDS, each survivor's lane adds them in k
//      order.  Each item is ProjectPatches/GetRectsFromPatch/CalcFeature/
//      Normalize/LogisticRegression::Predict (:459-484, :360-457,
//      LogisticRegression.cpp:46-68).  The theta test rejects (:197), the
//      survivors are compacted again.
//   3) per-window results (stage reached, last stage score) go to HBM.
// walk_kernel: one wave per row, the adaptive-stride x walk
// (ObjDetector.cpp:185-217) over the row's results; visited windows that
// passed every stage are emitted with score (s + p + 1)/S (:201-212).
//
// Every f32/f64 operation is the one the reference performs, in its order;
// compiled with -ffp-contract=off, IEEE sqrt / division, no fast-math.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cfloat>
#include <cstdint>

#include "sc_device.hpp"
#include "sc_integral_dev.hpp"
#include "sc_kernels.hpp"

namespace sc {

namespace {

#ifndef SC_CASCADE_MIN_WGS  // workgroups per CU the register budget must allow
#define SC_CASCADE_MIN_WGS 1
#endif


#ifndef SC_TEST_HOOKS  // 1: test-hook library (lib/testhooks): SC_OPT_TEST_DROP_HANDOFF acts
#define SC_TEST_HOOKS 0
#endif

#ifndef SC_ABL_NOWAIT  // timing ablation only: segments start without the hand-off (wrong results)
#define SC_ABL_NOWAIT 0
#endif

#ifndef SC_ITEM_BUF  // per-wave LDS results of the (survivor, weak) item path
#define SC_ITEM_BUF 640
#endif

constexpr int kWavesPerWg = 4;
constexpr int kItemBuf = SC_ITEM_BUF;
constexpr int kWalkMaxChunks = 64;  // windows per row <= 4096 (host check)
constexpr int kCascadeThreads = 64 * kWavesPerWg;
// chain kernel: one workgroup of NW waves per CU (the model is staged in LDS
// once per workgroup): 16 (4 per SIMD, 128 VGPRs) or 12 (3 per SIMD), chosen
// per launch (launch_chain).


__device__ __forceinline__ unsigned long long lanes_below() {
    return (1ull << (threadIdx.x & 63)) - 1ull;
}

// This lane's index.  RM: recomputed at each use (v_mbcnt, no input
// register) and opaque to the optimiser, so per-lane LDS addresses derived
// from it are rematerialised where they are used instead of being hoisted out
// of the persistent loop and held in VGPRs for the kernel's whole life: the
// chain kernel then fits 128 VGPRs (16 waves per CU; 156 -> 134 VGPRs at 12).
template <bool RM>
__device__ __forceinline__ int lane_id() {
    if constexpr (RM) {
        int l = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        asm volatile("" : "+v"(l));
        return l;
    } else {
        return threadIdx.x & 63;
    }
}

// The wave's lead lane: the first ACTIVE lane (v_mbcnt over the current exec
// mask).  Every "one lane does it, readfirstlane broadcasts it" site of the
// chain kernel uses it, so the lane that performs the atomic / load / store
// is by construction the lane readfirstlane reads, whatever the exec mask.
// The earlier form (lane_id() == 0, with the 12-wave kernel's lane-0 mask
// hoisted into an SGPR pair before the walker loop) is correct only while
// lane 0 is active at every such site; a dequeue whose atomic lane is
// inactive returns task 0 forever (readfirstlane then reads a lane that
// never did the atomic): the livelock shape of round 3's hang (DESIGN.md
// section 6a).
__device__ __forceinline__ bool lead_lane() {
    const unsigned long long ex = __ballot(1);
    return __builtin_amdgcn_mbcnt_hi((unsigned)(ex >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)ex, 0u)) == 0u;
}

// A row descriptor read through the scalar cache: the row list is written by
// the host before the launch and only read here, and the scalar path keeps
// this dependent round trip out of the vector-memory pipe, which the item
// gathers keep busy (TD ~96 %): a vector load queues behind them.
__device__ __forceinline__ int2 row_desc(const int2 *rows, int i) {
    // the constant address space: a wave-uniform address becomes an s_load
    typedef __attribute__((address_space(4))) const unsigned long long cu64;
    const unsigned long long v = ((cu64 *)(unsigned long long)rows)[i];
    return make_int2((int)(unsigned)v, (int)(unsigned)(v >> 32));
}

// Bit i of m -> bit base + 2i of the bit array w (i < 64: the positions
// k = r + 2u of a batch chunk's windows): the 32-bit halves of m spread to
// every second bit of a 64-bit word, each ORed in at its offset.
__device__ __forceinline__ unsigned long long spread32(unsigned long long x) {
    x &= 0xffffffffull;
    x = (x | (x << 16)) & 0x0000ffff0000ffffull;
    x = (x | (x << 8)) & 0x00ff00ff00ff00ffull;
    x = (x | (x << 4)) & 0x0f0f0f0f0f0f0f0full;
    x = (x | (x << 2)) & 0x3333333333333333ull;
    x = (x | (x << 1)) & 0x5555555555555555ull;
    return x;
}
__device__ __forceinline__ void or_word(unsigned long long *w, int bit, unsigned long long e) {
    if (!e) return;
    const int wd = bit >> 6, sh = bit & 63;
    atomicOr(&w[wd], e << sh);
    if (sh && (e >> (64 - sh))) atomicOr(&w[wd + 1], e >> (64 - sh));
}
__device__ __forceinline__ void or_spread(unsigned long long *w, int base, unsigned long long m) {
    or_word(w, base, spread32(m));
    or_word(w, base + 64, spread32(m >> 32));
}

// popcount of the bits of m below this lane (v_mbcnt: no 64-bit lane mask held)
__device__ __forceinline__ int popc_below(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// Orders LDS traffic between the lanes of ONE wave (a wave's DS instructions
// execute in order; this only stops the compiler from moving them).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// A wave-uniform 64-bit value (read by every lane) into SGPRs.
__device__ __forceinline__ unsigned long long uniform64(unsigned long long v) {
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return ((unsigned long long)hi << 32) | lo;
}

__device__ __forceinline__ unsigned xcc_id() {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & (kXcds - 1);
}

// LDS: weights [K][36] f32 | bias [K] f64 | order [K] i16 | per wave:
// P f32[kItemBuf], st_s f32[SA], surv u32[SA], st_p i8[SA]
// (SA = strip_max * band_rows rounded to 64)
__host__ __device__ inline size_t wave_scratch_bytes(int SA) {
    return (size_t)SA * 9 + (size_t)kItemBuf * 4;
}
// LW: weights and biases staged in LDS (else read through the caches: models
// whose weights do not fit the LDS)
__host__ __device__ inline size_t model_lds_bytes(int K, bool LW) {
    return (LW ? (size_t)K * 144 + (size_t)K * 8 : 0) + (((size_t)K * 2 + 15) & ~(size_t)15) +
           (size_t)K * 16;  // + template rect records (InlinePatch)
}

#ifndef SC_PROJ_INLINE  // chain kernel: project patches per item from LDS rects (0: ProjPatch table)
#define SC_PROJ_INLINE 1
#endif

// A set of windows of one level: nr rows of nw windows; window (r, u) has
// its origin cell (phase 0, half 0) at t_off + r*row_cells + u*wstep.
// Row-set policies of eval_windows.  A survivor is (r << 16 | u): window u
// of row r; its LDS slot r*stride() + u.
struct BandRows {  // full grid: nr rows of one level, windows j0 + u of row r
    unsigned t_off;   // row 0's table row
    int nw, nr, row_cells, j0, K;
    float thr;  // prefilter threshold (ObjDetector.cpp:188)
    int pre_row, pre_col0, pre_col1;
    const ProjPatch *projL;  // the level's projected fitted patches [2 parities][K]
    TableGeom g;
    __device__ int rows() const { return nr; }
    __device__ int stride() const { return nw; }
    __device__ int width(int) const { return nw; }
    __device__ unsigned origin(int r, int u) const {
        return t_off + r * row_cells + g.win_cell(j0 + u);
    }
    __device__ float thr_of(int) const { return thr; }
    __device__ int pre_row_of(int) const { return pre_row; }
    __device__ int pre_col_of(int, int u) const { return ((j0 + u) & 1) ? pre_col1 : pre_col0; }
    __device__ ProjPatch patch(int, int u, int gk) const { return load_proj(projL + ((j0 + u) & 1) * K + gk); }
};

// chain kernel: one row per task slot, each with its own frame, level and
// chain position; descriptors in LDS (t_off counts from frame 0's table)
struct SlotDesc {
    unsigned t_off;  // origin cell of the slot's first batch window
    int nw;          // windows in the batch (0: slot idle), all of one parity
    float thr;
    int pre_row, pre_col;
    int proj;        // (level * 2 + parity) * K
    int r;           // the batch's first window, relative to the segment
    float scale;     // the level's ProjectPatches scale
    int xb;          // the parity's base column: step * parity
    int cb;          // its table column: at(xb, 0)
    int pad;
};
struct SlotRows {
    const SlotDesc *d;
    int nr, bstride, wstep;
    const ProjPatch *proj;
    const int4 *R;  // template rect records in LDS
    TableGeom g;
    __device__ int rows() const { return nr; }
    __device__ int stride() const { return bstride; }
    __device__ int width(int r) const { return d[r].nw; }
    __device__ unsigned origin(int r, int u) const { return d[r].t_off + u * wstep; }
    __device__ float thr_of(int r) const { return d[r].thr; }
    __device__ int pre_row_of(int r) const { return d[r].pre_row; }
    __device__ int pre_col_of(int r, int) const { return d[r].pre_col; }
#if SC_PROJ_INLINE
    // ProjectPatches (DenseSURFFeatureExtractor.cpp:459-484): x' = (int)(px*scale),
    // y' likewise, the scaled side e = (int)(side*scale); GetRectsFromPatch
    // (:360-377): square -> c = e/2 (2x2 cells), otherwise c = e (1x4 / 4x1).
    // The host's ProjPatch table holds the same values (build_geometry).
    __device__ InlinePatch patch(int r, int, int gk) const {
        const int4 rc = R[gk];
        const float s = d[r].scale;
        const int px = (int)((float)rc.x * s), py = (int)((float)rc.y * s), e = (int)((float)rc.z * s);
        InlinePatch p;
        p.shape = rc.w;
        p.c = rc.w == 0 ? (e >> 1) : e;
        p.row0 = py * g.rowp;
        p.rowstep = p.c * g.rowp;
        p.x0 = d[r].xb + px;
        p.cb = d[r].cb;
        p.phm = g.phm;
        p.ph = g.ph;
        p.Qp = g.Qp;
        p.cs = g.cs;
        return p;
    }
#else
    __device__ ProjPatch patch(int r, int, int gk) const { return load_proj(proj + d[r].proj + gk); }
#endif
};

// The per-window work of the detect loop for the windows `need(slot)`
// selects: prefilter, then the cascade stage by stage over compacted
// survivors.  Results in LDS: st_p[slot] = stage reached (-1: prefilter
// reject), st_s[slot] = last stage score, slot = r*nw + u.
//   1) prefilter: sum(win) > area*6 (DenseSURFFeatureExtractor.cpp:351-358,
//      ObjDetector.cpp:188); survivors compacted in order (__ballot + popc).
//   2) each stage (ObjDetector.cpp:193-199): (survivor, weak) items over the
//      lanes in shape-sorted weak order, results through LDS, each survivor's
//      lane adds them in the model's k order (GentleAdaboost.cpp:255-258);
//      the theta test (:197) and order-preserving compaction.
// Item-schedule counters of profiling builds (SC_PROF_CHAIN): wave-uniform.
struct NoStats {
    [[maybe_unused]] static constexpr bool on = false;
    __device__ void iter(int) {}
    __device__ void stage(int) {}
    __device__ void pre(int, int) {}
};
struct ItemStats {
    [[maybe_unused]] static constexpr bool on = true;
    unsigned long long iters = 0, lanes = 0, pre_cyc = 0, thin32 = 0, stages = 0, surv = 0, need = 0, pass = 0;
    __device__ void iter(int active) {  // one item iteration (a gather round trip)
        iters++;
        lanes += (unsigned)active;
        thin32 += active <= 32;
    }
    __device__ void stage(int nsurv) {
        stages++;
        surv += (unsigned)nsurv;
    }
    __device__ void pre(int n_need, int n_pass) {
        need += (unsigned)n_need;
        pass += (unsigned)n_pass;
    }
};

template <bool LW, bool RM, class Rows, class Need, class Stats = NoStats>
__device__ __forceinline__ void eval_windows(const CascadeArgs &a, const Rows &B, const char *Tb,
                                             const float4 *Wl, const double *Bl, const int16_t *Ol,
                                             float *P, float *st_s, unsigned *surv, int8_t *st_p,
                                             int /*lane*/, Need need, Stats &&stats = Stats{}) {
    const int half_off = a.g.hs, stride = B.stride();
    const float4 *T = reinterpret_cast<const float4 *>(Tb);
    auto cell = [&](unsigned sv) { return B.origin((int)(sv >> 16), (int)(sv & 0xffffu)); };
    auto slot = [&](unsigned sv) { return (int)(sv >> 16) * stride + (int)(sv & 0xffffu); };

    // 1) prefilter; survivors in (row, x) order
    [[maybe_unused]] unsigned long long t_pre0 = 0;
    if constexpr (std::remove_reference_t<Stats>::on) t_pre0 = __builtin_amdgcn_s_memtime();
    // The rows' windows flattened into one list of 64-lane chunks (the chain
    // kernel's two slots hold ~35 windows each: one set of 4 corner loads
    // instead of one per slot)
    int nsurv = 0, tot = 0;
    for (int r = 0; r < B.rows(); r++) tot += B.width(r);
    for (int b = 0; b < tot; b += 64) {
        int u = b + lane_id<RM>(), r = 0;
        while (r + 1 < B.rows() && u >= B.width(r)) {
            u -= B.width(r);
            r++;
        }
        const bool act = b + lane_id<RM>() < tot && need(r * stride + u);
        bool pass = false;
        if (act) {
            const int pre_row = B.pre_row_of(r), pre_col = B.pre_col_of(r, u);
            const float4 *t0 = T + B.origin(r, u);
            const float4 v = box4(t0[0], t0[pre_row + pre_col], t0[pre_col], t0[pre_row]);
            const float m = (((v.x + v.y) + v.z) + v.w) / 2.0f;  // sum(), :351-358
            pass = m > B.thr_of(r);                              // ObjDetector.cpp:188
            st_p[r * stride + u] = pass ? 0 : -1;
            st_s[r * stride + u] = 0.0f;
        }
        const unsigned long long mk = __ballot(pass);
        if (pass) surv[nsurv + popc_below(mk)] = ((unsigned)r << 16) | (unsigned)u;
        nsurv += __popcll(mk);
        if constexpr (std::remove_reference_t<Stats>::on) stats.pre(__popcll(__ballot(act)), __popcll(mk));
    }
    wave_sync();
    if constexpr (std::remove_reference_t<Stats>::on) stats.pre_cyc += __builtin_amdgcn_s_memtime() - t_pre0;

    // 2) cascade, stage by stage over the compacted survivors
    for (int s = 0; s < a.n_stages && nsurv > 0; s++) {
        const int off = a.stage_off[s], n = a.stage_off[s + 1] - off;
        const float th = a.theta[s];
        int nn = 0;
        stats.stage(nsurv);
        // stage decision of one survivor (GentleAdaboost.cpp:259;
        // ObjDetector.cpp:197) and in-place order-preserving compaction:
        // kept survivors move to [nn, ...), never past the group just read
        auto decide = [&](bool valid, unsigned sv, float sum) {
            bool keep = false;
            if (valid) {
                const float sc = sum / (float)n;
                const int li = slot(sv);
                st_s[li] = sc;
                keep = !((double)sc < (double)th);
                st_p[li] = (int8_t)(keep ? s + 1 : s);
            }
            const unsigned long long mk = __ballot(keep);
            wave_sync();
            if (keep) surv[nn + popc_below(mk)] = sv;
            nn += __popcll(mk);
            wave_sync();
        };
        if (nsurv >= a.chunk_min || n > kItemBuf) {
            // one lane per survivor, k wave-uniform: parameters via scalar loads
            for (int c = 0; c < nsurv; c += 64) {
                stats.iter(min(64, nsurv - c));
                const int i = c + lane_id<RM>();
                unsigned sv = 0;
                float sum = 0.0f;
                if (i < nsurv) {
                    sv = surv[i];
                    const TabView Tj{Tb, cell(sv) << 4};
                    const int sr = (int)(sv >> 16), su = (int)(sv & 0xffffu);
                    for (int k = 0; k < n; k++) {
                        const int gk = off + k;
                        sum += weak_eval(Tj, half_off, B.patch(sr, su, gk), a.w + gk * 9, a.bias[gk]);
                    }
                }
                decide(i < nsurv, sv, sum);
            }
        } else {
            // (survivor, weak) items over the lanes, groups of G survivors
            // whose n*G results fit the wave's LDS buffer.  Items run in
            // shape-sorted weak order (Ol: few patch shapes per wave
            // instruction, so little divergence); each survivor's lane then
            // adds its results in the reference's k order.
            const int gcap = min(64, kItemBuf / n);
            for (int c = 0; c < nsurv; c += gcap) {
                const int G = min(gcap, nsurv - c), items = G * n;
                const float rcp = 1.0f / (float)G;
                auto decode = [&](int t2, int &k, int &i) {  // item -> (weak k, survivor i)
                    int kk = (int)((float)t2 * rcp);                // kk = t2 / G
                    i = t2 - kk * G;
                    if (i < 0) { kk--; i += G; }
                    else if (i >= G) { kk++; i -= G; }
                    k = Ol[off + kk];
                };
                for (int b2 = 0; b2 < items; b2 += 64) stats.iter(min(64, items - b2));
#if SC_PAIR
                // lane-pair form (sc_device.hpp pair_z32) on the interleaved
                // cells (hs == 1; the split layout keeps the one-lane form):
                // lane 2i + h decodes and projects item b2 + 32 h + i (the one
                // whose f64 sigmoid it runs at the end), pass h of the pair
                // reads those offsets from lane 2i + h (DPP), so each item is
                // projected once; 32 items per pass on all 64 lanes (lanes past
                // the items repeat item 0: the cross-lane reads need every lane)
                if (half_off == 1) {
                    for (int b2 = 0; b2 < items; b2 += 64) {
                        const int ln = lane_id<RM>(), h = ln & 1, ii = ln >> 1;
                        const int t2 = b2 + h * 32 + ii;
                        int k, i;
                        decode(t2 < items ? t2 : 0, k, i);
                        const int gk = off + k;
                        const unsigned sv = surv[c + i];
                        const auto pj = B.patch((int)(sv >> 16), (int)(sv & 0xffffu), gk);
                        PairItem it;
                        corner_offsets(pj, it.off);
                        it.base = cell(sv) << 4;
                        it.shape = pj.shape;
                        it.gk = gk;
                        float z[2];
#pragma unroll
                        for (int ps = 0; ps < 2; ps++) {
                            z[ps] = 0.0f;
                            if (ps == 1 && b2 + 32 >= items) break;  // (wave-uniform)
                            const PairItem q = ps == 0 ? it.of_even() : it.of_odd();
                            z[ps] = pair_z32(Tb, q, LW ? Wl + q.gk * 9 : a.w + q.gk * 9, h);
                        }
                        if (t2 < items)
                            P[k * G + i] = LW ? lr_sigmoid(h ? z[1] : z[0], Wl[gk * 9 + 8].x, Bl[gk])
                                              : lr_sigmoid(h ? z[1] : z[0], a.w[gk * 9 + 8].x, a.bias[gk]);
                    }
                } else
#endif
                for (int t2 = lane_id<RM>(); t2 < items; t2 += 64) {
                    int k, i;
                    decode(t2, k, i);
                    const int gk = off + k;
                    const unsigned sv = surv[c + i];
                    const TabView Tj{Tb, cell(sv) << 4};
                    const auto pj = B.patch((int)(sv >> 16), (int)(sv & 0xffffu), gk);
                    P[k * G + i] = LW ? weak_eval(Tj, half_off, pj, Wl + gk * 9, Bl[gk])
                                      : weak_eval(Tj, half_off, pj, a.w + gk * 9, a.bias[gk]);
                }
                wave_sync();
                unsigned sv = 0;
                float acc = 0.0f;  // GentleAdaboost.cpp:255-258 order
                const int ln = lane_id<RM>();
                if (ln < G) {
                    sv = surv[c + ln];
                    for (int k = 0; k < n; k++) acc += P[k * G + ln];
                }
                decide(ln < G, sv, acc);
            }
        }
        nsurv = nn;
    }
}

// The model staged in LDS once per persistent workgroup (the only
// workgroup barrier: the waves are independent afterwards).
template <bool LW, int NT = kCascadeThreads>
__device__ __forceinline__ void stage_model(const CascadeArgs &a, unsigned char *smem, float4 *&Wl,
                                            double *&Bl, int16_t *&Ol, int4 *&Rl) {
    const int K = a.K, tid = threadIdx.x;
    Wl = reinterpret_cast<float4 *>(smem);
    Bl = reinterpret_cast<double *>(smem + (LW ? (size_t)K * 144 : 0));
    Ol = reinterpret_cast<int16_t *>(Bl + (LW ? K : 0));
    Rl = reinterpret_cast<int4 *>(reinterpret_cast<unsigned char *>(Ol) + (((size_t)K * 2 + 15) & ~(size_t)15));
    if (LW)
        for (int i = tid; i < K * 9; i += NT) Wl[i] = a.w[i];
    for (int i = tid; i < K; i += NT) {
        if (LW) Bl[i] = a.bias[i];
        Ol[i] = a.order[i];
        Rl[i] = a.rects[i];
    }
    __syncthreads();
}

// Full-grid cascade: every window of the stride-`step` grid is evaluated
// (parity dumps, FillNegSamples' scan).  Persistent workgroups of 4
// independent waves; a task is one strip of a band of rows (sc_kernels.hpp),
// XCD x serving the strips [x*n_sub, (x+1)*n_sub) of every band from its own
// queue (steals from the others when empty): the table rows its L2 sees stay
// in a narrow column band.
template <bool LW>
__global__ __launch_bounds__(kCascadeThreads, SC_CASCADE_MIN_WGS) void cascade_kernel(CascadeArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // (uniform: per-wave LDS bases in SGPRs)
    float4 *Wl;
    double *Bl;
    int16_t *Ol;
    int4 *Rl;
    stage_model<LW>(a, smem, Wl, Bl, Ol, Rl);

    const int SA = (a.strip_max * a.band_rows + 63) & ~63;
    unsigned char *ws = smem + model_lds_bytes(a.K, LW) + (size_t)wv * wave_scratch_bytes(SA);
    float *P = reinterpret_cast<float *>(ws);
    float *st_s = P + kItemBuf;
    unsigned *surv = reinterpret_cast<unsigned *>(st_s + SA);
    int8_t *st_p = reinterpret_cast<int8_t *>(surv + SA);

    const TableGeom g = a.g;
    const int n_tasks = a.n_frames * a.n_bands * a.n_sub, nseg = kXcds * a.n_sub;
    int q = (int)xcc_id(), empty = 0;
    // dequeue: one atomic per task on this XCD's queue word; the next task's
    // index and descriptor are fetched while the current task runs
    auto task_index = [&](int t) {  // queue position -> descriptor slot, frame
        const int rt = t / a.n_sub, sub = t - rt * a.n_sub;
        const int frame = rt / a.n_bands, band = rt - frame * a.n_bands;
        return make_int2(band * nseg + q * a.n_sub + sub, frame);
    };
    int t = 0;
    if (lead_lane()) t = atomicAdd(&a.queues[q * kQueueStride], 1);
    t = __builtin_amdgcn_readfirstlane(t);
    TaskDesc D{};
    int2 tf = make_int2(0, 0);
    if (t < n_tasks) {
        tf = task_index(t);
        D = a.tasks[tf.x];
    }
    for (;;) {
        if (t >= n_tasks) {  // this queue is drained: steal from the next XCD's
            if (++empty == kXcds) break;
            q = (q + 1) & (kXcds - 1);
            t = 0;
            if (lead_lane()) t = atomicAdd(&a.queues[q * kQueueStride], 1);
            t = __builtin_amdgcn_readfirstlane(t);
            if (t < n_tasks) {
                tf = task_index(t);
                D = a.tasks[tf.x];
            }
            continue;
        }
        int tn = 0;  // prefetch the next task index
        if (lead_lane()) tn = atomicAdd(&a.queues[q * kQueueStride], 1);
        const int frame = tf.y;
        if (D.nw > 0) {  // (empty strips of narrow rows: nothing to do)
            const char *Tb = reinterpret_cast<const char *>(a.table + (long long)frame * g.frame4);
            const BandRows B{(unsigned)D.t_off, D.nw, D.nr, g.step * g.rowp, D.j0, a.K, D.thr,
                             D.pre_row, D.pre_col[0], D.pre_col[1],
                             a.proj + (long long)D.level * 2 * a.K, g};
            eval_windows<LW, false>(a, B, Tb, Wl, Bl, Ol, P, st_s, surv, st_p, lane,
                             [](int) { return true; });
            // 3) per-window results to HBM (coalesced per row)
            const long long gi = (long long)frame * a.grid_per_frame + D.g_off;
            for (int r = 0; r < D.nr; r++) {
                for (int u = lane; u < D.nw; u += 64) {
                    a.st_p[gi + (long long)r * D.g_row + u] = st_p[r * D.nw + u];
                    a.st_s[gi + (long long)r * D.g_row + u] = st_s[r * D.nw + u];
                }
            }
            wave_sync();
        }
        t = __builtin_amdgcn_readfirstlane(tn);
        if (t < n_tasks) {
            tf = task_index(t);
            D = a.tasks[tf.x];
        }
    }
}

__global__ __launch_bounds__(64) void walk_kernel(WalkArgs a) {
    __shared__ uint8_t s_flag[kWalkMaxChunks * 64];  // bit0 skip, bit1 detection
    const int lane = threadIdx.x;
    const int frame = blockIdx.x / a.n_rows, row = blockIdx.x - frame * a.n_rows;
    const int2 rd = a.rows[row];
    const LevelInfo L = a.levels[rd.x];
    const int y = rd.y, nx = L.nx, S = a.n_stages;
    const long long gbase = (long long)frame * a.grid_per_frame + L.grid_base +
                            (long long)(y / a.step) * nx;
    const int nch = (nx + 63) >> 6;
    // pass 1: per-window decisions (independent, unrolled: loads in flight together)
#pragma unroll 4
    for (int j = lane; j < nch * 64; j += 64) {
        uint8_t fl = 1;
        if (j < nx) {
            const int p = a.st_p[gbase + j];
            if (p >= 0) {
                const double fin = ((double)a.st_s[gbase + j] + p + 1) / S;  // ObjDetector.cpp:201
                fl = (fin < a.stride_score ? 1 : 0) | (p == S ? 2 : 0);        // :214, :203
            }
        }
        s_flag[j] = fl;
    }
    __syncthreads();
    // pass 2: the x chain, +1 after a good window, +2 after a skip (bad /
    // prefilter reject / past the row end).  From a landing position p it
    // visits p, p+2, ... until it lands on a good window q (first q >= p of
    // p's parity with skip == 0), then continues at q+1: one step per good
    // window instead of one per visited window.
    const unsigned long long kEven = 0x5555555555555555ull;
    int start = 0;
    unsigned long long nvis = 0;
    for (int c = 0; c < nch; c++) {
        const uint8_t fl = s_flag[(c << 6) + lane];
        const unsigned long long sk = __ballot(fl & 1), dt = __ballot(fl & 2);
        unsigned long long vis = 0;
        int pos = start;
        while (pos < 64) {
            const unsigned long long par = (pos & 1) ? ~kEven : kEven;
            const unsigned long long from = ~0ull << pos;
            const unsigned long long good = ~sk & par & from;
            if (!good) {
                vis |= par & from;
                pos = 64 + (pos & 1);
                break;
            }
            const int q = __builtin_ctzll(good);
            vis |= par & from & (q == 63 ? ~0ull : ((2ull << q) - 1ull));
            pos = q + 1;
        }
        const int lim = min(64, nx - (c << 6));
        if (lim < 64) vis &= (1ull << lim) - 1ull;
        start = pos - 64;
        nvis += __popcll(vis);
        const int j = (c << 6) + lane;
        const bool v = (vis >> lane) & 1ull;
        if (a.dbg_v && j < nx) a.dbg_v[gbase + j] = v ? 1 : 0;
        const unsigned long long dm = vis & dt;
        if (dm) {
            const int cnt = __popcll(dm);
            int slot0 = 0;
            if (lane == 0) {
                slot0 = atomicAdd(&a.counters[0], cnt);
                atomicAdd(&a.counters[1 + frame], cnt);
            }
            slot0 = __shfl(slot0, 0, 64);
            if ((dm >> lane) & 1ull) {
                const int idx = slot0 + __popcll(dm & lanes_below());
                if (idx < a.capacity) {
                    sc_det_record rec;
                    rec.frame = frame;
                    rec.level = rd.x;
                    rec.x = j * a.step;
                    rec.y = y;
                    rec.w = L.l;
                    rec.h = L.lh;
                    rec.stage_reached = S;
                    rec._pad = 0;
                    rec.score = ((double)a.st_s[gbase + j] + S + 1) / S;
                    a.out[idx] = rec;
                }
            }
        }
    }
    // per-row count, summed on the host on request: one atomic word hit by
    // every row (~10^4 per frame) serialises at ~90 adds/us
    if (lane == 0) a.row_visited[blockIdx.x] = (unsigned)nvis;
}

#ifndef SC_PROF_CHAIN  // profiling builds: per-phase s_memtime totals into WalkArgs::prof
#define SC_PROF_CHAIN 0
#endif
#if SC_PROF_CHAIN
#define SC_PROF(acc)                                               \
    do {                                                           \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
        acc += t_ - t_last;                                        \
        t_last = t_;                                               \
    } while (0)
#else
#define SC_PROF(acc) \
    do {             \
    } while (0)
#endif

#ifndef SC_ABL_EXTRA_RT
#define SC_ABL_EXTRA_RT 0
#endif
#ifndef SC_WIDECAP  // A/B: cap on a CU's task slots holding a wide-level row (0: one row list)
#define SC_WIDECAP 0
#endif
#ifndef SC_CHAIN_SLOTS  // chain kernel: rows (tasks) a wave advances together
#define SC_CHAIN_SLOTS 2
#endif
constexpr int kSlots = SC_CHAIN_SLOTS;
#ifndef SC_CHAIN_BATCH
#define SC_CHAIN_BATCH 128
#endif
constexpr int kBatch = SC_CHAIN_BATCH;  // chain kernel: windows of one parity per slot and round
constexpr int kBatchChunks = (kBatch + 63) / 64;
static_assert(kBatch % 4 == 0 && kItemBuf % 4 == 0, "chain LDS carve: keep the u64 bit arrays aligned");

// chain kernel LDS per wave: P f32[kItemBuf] | st_s f32[kSlots*kBatch] |
// surv u32[kSlots*kBatch] | per slot: segment scores f32[SEGA], evaluated /
// good / detection bits u64[SEGA/64] x 3 | SlotDesc[kSlots] | st_p i8[kSlots*kBatch]
__host__ __device__ inline size_t chain_wave_bytes(int seg_max) {
    const size_t sa = (size_t)((seg_max + 63) & ~63);
    const size_t b = (size_t)kItemBuf * 4 + (size_t)kSlots * kBatch * 9 +
                     (size_t)kSlots * (sa * 4 + sa / 64 * 24) + kSlots * sizeof(SlotDesc) +
                     (size_t)kSlots * 10 * 4 + 64;
    return (b + 15) & ~(size_t)15;  // every wave's block 16-B aligned (64-bit LDS atomics)
}

// Fused integral: colstrip_kernel's column walk (sc_integral.hip) as a task
// of the chain kernel.  One wave per (frame, 64-column strip, channel half),
// lane = column; the f32 column recurrence S[y+1] = S[y] + R_y in colstrip's
// order, so the table is bit-identical.  In the chain kernel's 128-VGPR
// budget: two blocks of kWalkRows rows of pixel loads in flight, each
// block's strip carries loaded one row per lane and read back with
// v_readlane.  Cells are stored write-through (buffer store with sc1: the
// line leaves this XCD's L2), then every store is drained (vmcnt 0) before
// lane 0 counts the walk done for its frame -- the in-launch hand-off of
// cdna_hip_programming.md Guideline 16 (R1); the reading waves poll that
// count and take an agent-scope acquire (chain_kernel, frame_ready).
constexpr int kWalkRows = 8;
#if SC_PROF_CHAIN
constexpr long long kTraceTasks = 65536;  // task trace capacity (tasks of the last launch)
#endif
static_assert((kWalkRows & (kWalkRows - 1)) == 0 && kWalkRows <= 64, "walk block");
// SC_WALK_STORE: 1 sc1 (write-through) stores; 2 plain stores + release fence
// at the walk's end (+0.5 % kernel time); 0 none, the tables built by the
// separate kernels (timing ablation: the walks' cost without their stores)
#ifndef SC_WALK_STORE
#define SC_WALK_STORE 1
#endif

// INTER (interleaved 32-B cells, TableGeom cs 2): one wave per (frame,
// 32-column strip), lanes 0-31 channel half 0 and lanes 32-63 half 1 of the
// same columns, so each store instruction writes whole 32-B cells (with a
// wave per half, two waves wrote the two halves of every cell: a C2 launch
// with interleaved cells took 13.61 vs 12.84 ms unfused, profiles/r6/h);
// two 32-lane scans, each half's carries read from its own lanes.
template <bool INTER>
__device__ __forceinline__ void fused_walk(const CascadeArgs &a, const WalkArgs &w, int t) {
    using namespace idev;
    const int fi = t / w.walks_per_frame, rem = t - fi * w.walks_per_frame;
    const TableGeom g = a.g;
    const int W = g.W, H = g.H, ns = (W + kStrip - 1) / kStrip;
    const int lane = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    const int f = w.int_f0 + fi;
    const int s = INTER ? rem : rem >> 1;              // 32-px strip (INTER) / 64-px strip
    const int h = INTER ? lane >> 5 : rem & 1;         // channel half: per lane (INTER) / per wave
    const int x = INTER ? s * kStrip + (lane & 31) : s * 2 * kStrip + lane;
    const bool live = x < W;
    const int xs = live ? x : W - 1;  // dead lanes still join the scan with zeros
    const uint8_t *img = w.frames + (long long)f * w.frame_bytes;
    // the frame's table through a buffer descriptor (wave-uniform), so the
    // 16-B stores can carry sc1 (aux 16)
    const float4 *tab = a.table + (long long)f * g.frame4;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float4 *>(tab), (short)0, (int)(g.frame4 * 16), 0x00020000);
    const unsigned rowb = (unsigned)g.rowp * 16u;
    unsigned off = (unsigned)g.at(x + 1, h) * 16u + rowb;  // table row 1 of the column
    // the exclusive carry at column 64*s is the 32-px strip 2*s's
    const uint4 *cin = reinterpret_cast<const uint4 *>(w.carry) + (long long)f * H * ns * 2 +
                       (long long)(INTER ? s : 2 * s) * 2 + h;
    auto load_block = [&](int y0, Px4 (&px)[kWalkRows], uint4 &cr) {
#pragma unroll
        for (int k = 0; k < kWalkRows; k++)
            px[k] = INTER ? load_px_lanes(img, w.stride, W, H, min(y0 + k, H - 1), xs, h)
                          : load_px(img, w.stride, W, H, min(y0 + k, H - 1), xs, h);
        cr = cin[(long long)min(y0 + (lane & (kWalkRows - 1)), H - 1) * ns * 2];  // lane k (32 + k): row y0 + k
    };
    Px4 pa[kWalkRows];
    uint4 ca;
    load_block(0, pa, ca);
    float S0 = 0.0f, S1 = 0.0f, S2 = 0.0f, S3 = 0.0f;  // table row 0
    for (int y0 = 0; y0 < H; y0 += kWalkRows) {
        Px4 pb[kWalkRows];
        uint4 cb;
        load_block(y0 + kWalkRows < H ? y0 + kWalkRows : y0, pb, cb);
#pragma unroll
        for (int k = 0; k < kWalkRows; k++) {
            uint2 p = live ? grad_packed(pa[k]) : make_uint2(0u, 0u);
            if (INTER) {
                p.x = half_scan(p.x);
                p.y = half_scan(p.y);
            } else {
                p.x = wave_scan(p.x);  // 16-bit channel pairs: 64 px x 255 < 2^16
                p.y = wave_scan(p.y);
            }
            // this row's strip carry: lane k's (half 0) or lane 32 + k's (half 1)
            auto carry = [&](uint32_t c) -> uint32_t {
                const uint32_t c0 = (uint32_t)__builtin_amdgcn_readlane((int)c, k);
                if (!INTER) return c0;
                const uint32_t c1 = (uint32_t)__builtin_amdgcn_readlane((int)c, 32 + k);
                return h ? c1 : c0;
            };
            S0 = S0 + (float)(carry(ca.x) + (p.x & 0xffffu));
            S1 = S1 + (float)(carry(ca.y) + (p.x >> 16));
            S2 = S2 + (float)(carry(ca.z) + (p.y & 0xffffu));
            S3 = S3 + (float)(carry(ca.w) + (p.y >> 16));
            if (live && y0 + k < H) {  // rows past H: harmless extra steps, not stored
                typedef unsigned v4u __attribute__((ext_vector_type(4)));
                const v4u v = {__float_as_uint(S0), __float_as_uint(S1), __float_as_uint(S2), __float_as_uint(S3)};
#if SC_WALK_STORE == 1
                __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)off, 0, 16);  // sc1
#elif SC_WALK_STORE == 2
                __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)off, 0, 0);
#else
                if (S0 == -1.0f) __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)off, 0, 16);
#endif
            }
            off += rowb;
        }
#pragma unroll
        for (int k = 0; k < kWalkRows; k++) pa[k] = pb[k];
        ca = cb;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every store of this wave drained
#if SC_WALK_STORE == 2
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
#if SC_TEST_HOOKS  // test builds only: a lost walk count (the frame's readers must time out)
    if (t + 1 == w.drop_walk1) return;
#endif
    if (lead_lane()) __hip_atomic_fetch_add(&w.int_ctl[1 + f], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Lazy grid (the default detect path).  The reference evaluates only the
// windows its adaptive-stride x chain visits (ObjDetector.cpp:185-217): after
// a window with final score < 0.5 (or a prefilter reject) the chain skips one
// window, after a good one it steps to the next.  Here the chain drives the
// cascade.  Each row is cut into kXcds segments and XCD x owns segment x of
// every row (the table columns its L2 sees stay in one band, as in the
// full-grid kernel).  A task (row, segment) starts from the chain's entry
// position, published by the task of the previous segment (one 4-B
// agent-scope word: the payload is the flag), then alternates
//   - evaluate the next kBatch not-yet-evaluated windows of the chain's
//     parity (p, p+2, ... up to the segment end): prefilter + cascade,
//   - advance the chain over evaluated windows (64-bit parity masks, one
//     step per good window) until it reaches an unevaluated one,
// and publishes where the chain leaves the segment.  A wave carries kSlots
// tasks at once and evaluates their batches together (one prefilter pass,
// one set of stage rounds), so the stage-by-stage round trips serve twice
// the windows.  One workgroup of kChainWaves independent waves per CU (the
// model staged in LDS once per CU).  On the C2 frames the lazy grid
// evaluates ~55 % of the grid's weak items (the visited windows alone are
// 53 %).  Visited windows that
// passed every stage are emitted with score (s + S + 1)/S (:201-212).
template <bool LW, int NW>
__global__ __launch_bounds__(64 * NW, 1) void chain_kernel(CascadeArgs a, WalkArgs w) {
    constexpr int kChainWaves = NW, kChainThreads = 64 * NW;
    constexpr bool RM = NW > 12;  // rematerialised lane values (128-VGPR budget)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // (uniform: per-wave LDS bases in SGPRs)
    float4 *Wl;
    double *Bl;
    int16_t *Ol;
    int4 *Rl;
    // the level table in LDS: slot descriptors and merges read it every round
    LevelInfo *Lv = reinterpret_cast<LevelInfo *>(smem + model_lds_bytes(a.K, LW) +
                                                  kChainWaves * chain_wave_bytes(w.row_max));
    for (int i = threadIdx.x; i < w.n_levels; i += kChainThreads) Lv[i] = w.levels[i];
    // fused integral: frames below *cu_rdy have complete tables this CU may
    // read (the launch's prebuilt frames; then each frame after an sc1 poll
    // of its walk count and an agent-scope acquire by a wave of this CU)
    int *cu_rdy = reinterpret_cast<int *>(Lv + w.n_levels);
    if (threadIdx.x == 0) *cu_rdy = w.int_walks > 0 ? w.int_f0 : a.n_frames;
#if SC_WIDECAP
    int *cu_wide = cu_rdy + 1;  // this CU's slots holding a wide-level row
    if (threadIdx.x == 0) *cu_wide = 0;
#endif
    stage_model<LW, kChainThreads>(a, smem, Wl, Bl, Ol, Rl);  // (its barrier covers Lv, cu_rdy)

    const int sa = (w.row_max + 63) & ~63, nwords = sa >> 6;  // row_max: widest segment
    unsigned char *ws = smem + model_lds_bytes(a.K, LW) + (size_t)wv * chain_wave_bytes(w.row_max);
    float *P = reinterpret_cast<float *>(ws);
    float *st_s = P + kItemBuf;
    unsigned *surv = reinterpret_cast<unsigned *>(st_s + kSlots * kBatch);
    float *s_seg0 = reinterpret_cast<float *>(surv + kSlots * kBatch);
    unsigned long long *bits0 = reinterpret_cast<unsigned long long *>(s_seg0 + kSlots * sa);
    SlotDesc *desc = reinterpret_cast<SlotDesc *>(bits0 + kSlots * 3 * nwords);
    int *park = reinterpret_cast<int *>(desc + kSlots);  // slot state parked across a round
    int8_t *st_p = reinterpret_cast<int8_t *>(park + kSlots * 10);
    auto s_seg = [&](int sl) { return s_seg0 + sl * sa; };
    auto evb = [&](int sl) { return bits0 + (sl * 3 + 0) * nwords; };
    auto gdb = [&](int sl) { return bits0 + (sl * 3 + 1) * nwords; };
    auto dtb = [&](int sl) { return bits0 + (sl * 3 + 2) * nwords; };

    const TableGeom g = a.g;
    const int S = a.n_stages, cs = g.cs;
#if SC_WIDECAP
    // two row lists: the narrow levels' rows [0, nN) and the wide levels'
    // [nN, n_rows), each dealt in its own order from its own queue; task ids
    // t < n_tasks narrow (frame t / nN), t >= n_tasks wide
    const int nW = w.n_wide, nN = w.n_rows - nW;
    const int n_tasks = nN * a.n_frames, nt_w = nW * a.n_frames;
    const int pszw = (nt_w + (1 << w.seg_shift) - 1) >> w.seg_shift;
    int qw = (int)xcc_id(), emptyw = 0;
    bool wdrained = nt_w == 0, ndrained = false;
#else
    const int n_tasks = w.n_rows * a.n_frames;  // per segment queue, in row order
#endif
    const unsigned long long kEven = 0x5555555555555555ull;
    // queue of XCD q: its part of segment q >> sh of every row, in row order,
    // dealt through nsq counters on separate lines (sub-queue u: tasks u,
    // u + nsq, ...).  A drained sub-queue sends the wave on to the next one,
    // then to the other XCDs' queues.  nsq is per launch (WalkArgs::subq):
    // one-frame launches use 8 (their ~400 waves per XCD otherwise serialise
    // on one atomic word's line: chain kernel 0.589 vs 0.606 ms with 4,
    // profiles/r4/subq; 0.573 vs 0.582 with 8 over contiguous parts,
    // profiles/r5/l/split), batches 1 (sub-queues deal the row blocks out of
    // order and cost their L2 locality: C2 +25 %)
    const int nsg = w.nseg, sh = w.seg_shift;  // segments per row; XCDs per segment = 1 << sh
    const int nsq = w.subq;
    int q = (int)xcc_id(), empty = 0;
    int u = (int)((blockIdx.x / kXcds * kChainWaves + wv) % nsq);
    bool drained = false;
    unsigned idle = 0;  // rounds with every task waiting for its entry
    unsigned long long idle_t0 = 0;  // when the current wait began (s_memrealtime)
#if SC_PROF_CHAIN
    unsigned long long c_idle = 0, c_setup = 0, c_eval = 0, c_merge = 0, n_rounds = 0, n_slots = 0;
    unsigned long long c_deq = 0, c_poll = 0;
    ItemStats istats;
    unsigned long long t_last = __builtin_amdgcn_s_memtime();
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();  // (chip-wide clock: per-XCD memtime counters differ)
#endif

    // Fused integral: the last wave of every workgroup first runs column
    // walks (fused_walk) until none is left, then joins the chain work.  One
    // walker per workgroup: whichever workgroups are resident, the walks of
    // every frame progress, so no wave waits on a frame forever.
#ifndef SC_WALKERS  // walking waves per workgroup (1 measured best of 1/8, 1/4, 1/2, 1, 2: profiles/r3/g18-19)
#define SC_WALKERS 1
#endif
    if (w.int_walks > 0 && wv >= kChainWaves - SC_WALKERS) {
#ifndef SC_WALK_PRIO
#define SC_WALK_PRIO 2
#endif
        __builtin_amdgcn_s_setprio(SC_WALK_PRIO);  // latency-bound: issue ahead of the gathers
        for (;;) {
            int t = 0;
            if (lead_lane()) t = atomicAdd(&w.int_ctl[0], 1);
            t = __builtin_amdgcn_readfirstlane(t);
            if (t >= w.int_walks) break;
#ifndef SC_NO_WALK
            if (a.g.cs == 2) fused_walk<true>(a, w, t);
            else fused_walk<false>(a, w, t);
#endif
        }
        __builtin_amdgcn_s_setprio(0);
    }
    // Frame fr's table is complete and this CU may read it (Guideline 16:
    // the acquire invalidates the CU's L1; the LDS word, raised after the
    // acquire's wait, orders the CU's other waves after it)
    auto frame_ready = [&](int fr) -> bool {
        int c = __builtin_amdgcn_readfirstlane(__hip_atomic_load(cu_rdy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        if (fr < c) return true;
        const int c0 = c;
        while (c < a.n_frames) {
            int v = 0;
            if (lead_lane())
                v = __hip_atomic_load(&w.int_ctl[1 + c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__builtin_amdgcn_readfirstlane(v) < w.walks_per_frame) break;
            c++;
        }
        if (c > c0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lead_lane()) __hip_atomic_fetch_max(cu_rdy, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        return fr < c;
    };

    // per-slot task state (wave-uniform)
    int st[kSlots], tq[kSlots], tt[kSlots], r[kSlots], j0[kSlots], nseg[kSlots];
    int frame[kSlots], level[kSlots], ys[kSlots];
    unsigned vtot = 0;  // windows this wave's chains visited (summed into row_visited at the end)
    unsigned nspec = 0;  // speculative rounds this wave ran (summed into *w.spec at the end)
#pragma unroll
    for (int sl = 0; sl < kSlots; sl++) st[sl] = 0;  // 0 empty, 1 waiting for entry, 2 active, 3 waiting for the frame's table

#ifndef SC_FILL_K  // launch fill: segment-0 tasks per wave = SC_FILL_K * s / SC_FILL_DEN
#define SC_FILL_K 1
#endif
#ifndef SC_FILL_DEN
#define SC_FILL_DEN 2
#endif
    // Launch fill: a task of segment s cannot start before s hand-offs, so at
    // the start of a launch the XCDs of the later segments would only wait.
    // A wave on the XCDs of segment s first takes s/2 tasks of segment 0
    // (always ready; their hand-offs feed the other queues sooner), then its
    // own queue.  s/2 measured best of 0, s/2, s, 3s/2, 2s, 4s (-1.0 % at 32
    // frames per launch, -8.5 % at one frame; profiles/r2/fill).
    int pre = SC_FILL_K * (q >> sh) / SC_FILL_DEN;
    // queue position k of XCD sub-index q0 (of the 1 << sh XCDs serving a
    // segment) -> task k of part q0 of the row list: the XCDs sharing a
    // segment (one-frame launches: 2) take contiguous parts, so an XCD's tasks
    // in flight are neighbouring rows; dealt alternately (task (k << sh) + q0)
    // they spanned twice the rows and the one-frame chain kernel took
    // 0.5875 vs 0.5823 ms, 0.573 with 8 sub-queues (profiles/r5/l/split)
    const int psz = (n_tasks + (1 << sh) - 1) >> sh;
    auto task_of = [&](int k, int q0) -> int { return k < psz ? q0 * psz + k : n_tasks; };
    auto dequeue = [&](int &t, int &qq, int2 &rd) -> bool {
        while (pre > 0) {
            pre--;
            const int q0 = q & ((1 << sh) - 1);  // an XCD of segment 0
            int v = 0;
            if (lead_lane()) v = atomicAdd(&a.queues[(q0 * kMaxSubQ + u) * kQueueStride], 1);
            v = task_of(__builtin_amdgcn_readfirstlane(v) * nsq + u, q0);
            if (v < n_tasks) {
                t = v;
                qq = 0;
#if SC_WIDECAP
                rd = row_desc(w.rows, v % nN);
#else
                rd = row_desc(w.rows, v % w.n_rows);
#endif
                return true;
            }
            pre = 0;
        }
#if SC_WIDECAP
        for (;;) {
            // a wide row while this CU holds fewer than wide_cap (any once the
            // narrow rows are gone); the count is raised first, returned if
            // no wide row is taken
            while (!wdrained) {
                int old = 0;
                if (lead_lane()) old = __hip_atomic_fetch_add(cu_wide, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                old = __builtin_amdgcn_readfirstlane(old);
                bool took = false;
                if (old < w.wide_cap || ndrained) {
                    int v = 0;
                    if (lead_lane()) v = atomicAdd(&a.queues[(qw * kMaxSubQ + kMaxSubQ - 1) * kQueueStride], 1);
                    v = __builtin_amdgcn_readfirstlane(v);
                    v = v < pszw ? (qw & ((1 << sh) - 1)) * pszw + v : nt_w;
                    if (v < nt_w) {
                        t = n_tasks + v;
                        qq = qw >> sh;
                        rd = row_desc(w.rows, nN + v % nW);
                        took = true;
                    } else if (++emptyw == kXcds) {
                        wdrained = true;
                    } else {
                        qw = (qw + 1) & (kXcds - 1);
                    }
                }
                if (took) return true;
                if (lead_lane()) __hip_atomic_fetch_add(cu_wide, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (!(old < w.wide_cap || ndrained) || wdrained) break;
            }
            if (ndrained) {
                drained = wdrained;
                if (drained) return false;
                continue;
            }
#else
        {
#endif
        while (!drained) {
            int v = 0;
            if (lead_lane()) v = atomicAdd(&a.queues[(q * kMaxSubQ + u) * kQueueStride], 1);
            v = task_of(__builtin_amdgcn_readfirstlane(v) * nsq + u, q & ((1 << sh) - 1));
            if (v < n_tasks) {
                t = v;
                qq = q >> sh;  // the segment
#if SC_WIDECAP
                rd = row_desc(w.rows, v % nN);
#else
                rd = row_desc(w.rows, v % w.n_rows);
#endif
                return true;
            }
            if (++empty == kXcds * nsq) {  // every sub-queue drained
                drained = true;
            } else if (++u == nsq) {
                u = 0;
                q = (q + 1) & (kXcds - 1);
            }
        }
#if SC_WIDECAP
            ndrained = true;
            drained = wdrained;
            if (drained) return false;
#endif
        }
        return false;
    };
    int spec = -1;      // this round: speculative evaluation of waiting slot `spec` (both parities)
    // bit sl: slot sl's task was evaluated speculatively; bits 8 + 8 sl: its
    // speculative rounds so far, each 2*kBatch windows (both parities) on
    // from the segment start (at most w.spec_max rounds per task)
    unsigned spd = 0;
    auto spec_cur = [&](int sl) -> int { return (int)((spd >> (8 + 8 * sl)) & 0xFFu); };
    // the chain leaves slot sl's segment at absolute position pos: hand it on
#if SC_PROF_CHAIN  // task trace (profiling builds): realtime stamps per task at dequeue / start / finish
    auto stamp = [&](int sl, int which) {
        const long long ti = (long long)tt[sl] * nsg + tq[sl];
        if (w.prof && lead_lane() && ti < kTraceTasks)
            w.prof[16 + 2 * 8192 + 3 * ti + which] = __builtin_amdgcn_s_memrealtime();
    };
#else
    auto stamp = [&](int, int) {};
#endif
    auto finish = [&](int sl, int pos) {
        stamp(sl, 2);
        if (lead_lane()) {
#if SC_TEST_HOOKS  // test builds only (a lost hand-off for the watchdog test): the check spills in the 16-wave kernel
            if (tq[sl] + 1 < nsg && !(tq[sl] == 0 && tt[sl] + 1 == w.drop_task1))
#else
            if (tq[sl] + 1 < nsg)
#endif
                __hip_atomic_store(&w.entry[(long long)tt[sl] * nsg + tq[sl] + 1], pos + 1,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#if SC_WIDECAP
            if (tt[sl] >= n_tasks) __hip_atomic_fetch_add(cu_wide, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
        }
        st[sl] = 0;
    };
    auto start = [&](int sl, int pos) {  // the chain entered the segment at pos
        stamp(sl, 1);
        const int rel = pos - j0[sl];
        if (rel >= nseg[sl]) {
            finish(sl, pos);
            return;
        }
        if (!((spd >> sl) & 1u))  // (a speculated task's bits hold its evaluated windows)
            for (int i = lane_id<RM>(); i < 3 * nwords; i += 64) bits0[sl * 3 * nwords + i] = 0ull;
        r[sl] = rel;
        st[sl] = 2;
    };
#ifndef SC_SPEC_IDLE  // a wave with no active slot evaluates a waiting task's windows ahead of its entry
#define SC_SPEC_IDLE 1
#endif
    static_assert(!SC_SPEC_IDLE || kSlots == 2, "speculative rounds use the two slots' descriptors");
    // (one-frame launches, in the 12-wave kernel they use: their tails are
    // the hand-off chains' latency; a bandwidth-bound launch pays for the
    // extra windows -- C4 +3.9 % -- and the 16-wave kernel would spill)
#ifndef SC_SPEC16
#define SC_SPEC16 0
#endif
    constexpr bool kSpec = SC_SPEC_IDLE && (NW == 12 || SC_SPEC16);

    for (;;) {
        // 1) refill empty slots, poll the entries of waiting ones
        int n_active = 0, n_wait = 0;
#pragma unroll
        for (int sl = 0; sl < kSlots; sl++) {
            if (st[sl] == 0 && sl < w.slots) {  // (w.slots 1: the second slot stays empty)
                int t, qq;
                int2 rd;
                if (dequeue(t, qq, rd)) {
                    const int nx = Lv[rd.x].nx, nxs = (nx + nsg - 1) / nsg;
                    tt[sl] = t;
                    tq[sl] = qq;
#if SC_WIDECAP
                    frame[sl] = t < n_tasks ? t / nN : (t - n_tasks) / nW;
#else
                    frame[sl] = t / w.n_rows;
#endif
                    level[sl] = rd.x;
                    ys[sl] = rd.y;
                    j0[sl] = min(nx, qq * nxs);
                    nseg[sl] = min(nx, j0[sl] + nxs) - j0[sl];
                    st[sl] = 3;  // the poll below checks the frame, then starts segment 0
                    spd &= ~((1u << sl) | (0xFFu << (8 + 8 * sl)));
                    stamp(sl, 0);
                }
                SC_PROF(c_deq);
            }
        }
        {   // poll every waiting slot once, the loads in flight together; a lost
            // hand-off must not hang the GPU (watchdog below)
            int e[kSlots];
#pragma unroll
            for (int sl = 0; sl < kSlots; sl++)
                if (st[sl] == 3 && frame_ready(frame[sl])) {
                    st[sl] = 1;
                    if (tq[sl] == 0 || SC_ABL_NOWAIT) start(sl, j0[sl]);  // (segment 0 enters at 0)
                }
#pragma unroll
            for (int sl = 0; sl < kSlots; sl++) {
                e[sl] = 0;
                if (st[sl] == 1 && lead_lane())
                    e[sl] = __hip_atomic_load(&w.entry[(long long)tt[sl] * nsg + tq[sl]], __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
            }
#pragma unroll
            for (int sl = 0; sl < kSlots; sl++) {
                const int es = __builtin_amdgcn_readfirstlane(e[sl]);
                if (st[sl] == 1 && es) start(sl, es - 1);
                n_active += st[sl] == 2;
                n_wait += st[sl] == 1 || st[sl] == 3;
            }
            SC_PROF(c_poll);
        }
        spec = -1;
        if (n_active == 0 && kSpec && a.n_frames == 1) {  // (one-frame launches: latency-bound)
            // nothing to evaluate: the first waiting task with speculative
            // rounds left gets both parities of its next 2*kBatch windows
            // evaluated now, so its chain runs through them when its entry
            // arrives (the hand-off chain's latency, not the work, sets a
            // one-frame launch's tail).  w.spec_max rounds per task: 1 for a
            // whole frame (more cost the windows the chain skips), all of the
            // segment for a grid shard (few tasks per wave: the idle waves
            // are free)
#pragma unroll
            for (int sl = 0; sl < kSlots; sl++)
                if (spec < 0 && st[sl] == 1 && spec_cur(sl) < w.spec_max && spec_cur(sl) * 2 * kBatch < nseg[sl])
                    spec = sl;
            if (spec >= 0) {
                if (!((spd >> spec) & 1u))  // the task's first speculative round: its bits from zero
                    for (int i = lane_id<RM>(); i < 3 * nwords; i += 64) bits0[spec * 3 * nwords + i] = 0ull;
                spd |= 1u << spec;
                nspec++;
            }
        }
        if (n_active == 0 && spec < 0) {
            SC_PROF(c_idle);
            if (n_wait == 0) {
                if (drained) break;
                continue;
            }
            __builtin_amdgcn_s_sleep(4);
            // a lost hand-off or walk count must not hang the GPU: after 0.5 s
            // of waiting (the chip-wide 100 MHz clock) the waiting tasks start
            // anyway, each counted in the sticky error word; once any wave's
            // watchdog has fired in this launch (the per-launch flag), every
            // waiting task -- for an entry or for its frame's table -- starts
            // at once, uncounted (the call raises already; its results are
            // discarded), so a failed launch drains in about one timeout.
            // The wait's clock restarts only when a slot did start.
            if (idle++ == 0) idle_t0 = __builtin_amdgcn_s_memrealtime();
            if ((idle & 255u) == 0u) {
                int e = 0;
                if (lead_lane()) e = __hip_atomic_load(w.fired, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const bool own = __builtin_amdgcn_s_memrealtime() - idle_t0 > 50000000ull;
                if (__builtin_amdgcn_readfirstlane(e) != 0 || own) {
                    bool started = false;
#pragma unroll
                    for (int sl = 0; sl < kSlots; sl++)
                        if (st[sl] == 1 || st[sl] == 3) {
                            if (own && lead_lane()) {
                                atomicAdd(w.err, 1);
                                __hip_atomic_store(w.err_host, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                                __hip_atomic_store(w.fired, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            }
                            start(sl, j0[sl]);
                            started = true;
                        }
                    if (started) idle = 0;
                }
            }
            continue;
        }
        idle = 0;

        // 2) one evaluation round over every active slot's next batch
#if SC_ABL_EXTRA_RT  // timing ablation: SC_ABL_EXTRA_RT dependent round trips to L2 per round
#pragma unroll
        for (int i = 0; i < SC_ABL_EXTRA_RT; i++) {
            int v = 0;  // (word 1 of this XCD's queue line: unused, stays 0)
            if (lead_lane()) v = atomicAdd(&a.queues[(q * kMaxSubQ + u) * kQueueStride + 1], 0);
            v = __builtin_amdgcn_readfirstlane(v);
            if (v == 0x7fffffff) drained = true;
        }
#endif
        // descriptor sl's task: slot sl's own, or in a speculative round the
        // waiting task `spec` at parity offset sl (selects, no dynamic index
        // into the per-slot registers)
#define SC_OF(v, sl) (spec < 0 ? (v)[sl] : (spec == 0 ? (v)[0] : (v)[1]))
#define SC_ACT(sl) (spec < 0 ? st[sl] == 2 : (sl) < 2)
#pragma unroll
        for (int sl = 0; sl < kSlots; sl++) {
            if (lead_lane()) {
                SlotDesc dd{};
                if (SC_ACT(sl)) {
                    const int lv = SC_OF(level, sl), ns_ = SC_OF(nseg, sl);
                    const int rr = spec < 0 ? r[sl] : sl + 2 * kBatch * spec_cur(spec == 0 ? 0 : 1);
                    const LevelInfo &L = Lv[lv];
                    const int jb = SC_OF(j0, sl) + rr;  // the batch: jb, jb + 2, ...
                    dd.t_off = (unsigned)((long long)SC_OF(frame, sl) * g.frame4 + SC_OF(ys, sl) * g.rowp + g.win_cell(jb));
                    dd.nw = min(kBatch, (ns_ - rr + 1) >> 1);
                    dd.thr = L.thr;
                    dd.pre_row = L.pre_row;
                    dd.pre_col = (jb & 1) ? L.pre_col[1] : L.pre_col[0];  // (no dynamic index: scratch)
                    dd.proj = (lv * 2 + (jb & 1)) * a.K;
                    dd.r = rr;
                    dd.scale = L.scale;
                    dd.xb = (jb & 1) * g.step;
                    dd.cb = g.at0((unsigned)dd.xb);
                }
                desc[sl] = dd;
            }
        }
        wave_sync();
        const SlotRows B{desc, kSlots, kBatch, g.ph == g.step ? 2 * cs : cs, a.proj, Rl, g};
        auto need = [&](int slot) {  // window not evaluated yet (an earlier batch may have)
            const int sl = slot / kBatch, u = slot - sl * kBatch;
            const int k = desc[sl].r + 2 * u;
            return ((evb(spec < 0 ? sl : spec)[k >> 6] >> (k & 63)) & 1ull) == 0ull;
        };
        // the windows this round evaluates, window c*64 + lane of each slot's batch
        unsigned long long mine[kSlots][kBatchChunks];
#pragma unroll
        for (int sl = 0; sl < kSlots; sl++)
#pragma unroll
            for (int c = 0; c < kBatchChunks; c++) {
                const int u = c * 64 + lane_id<RM>();
                mine[sl][c] = __ballot(SC_ACT(sl) && u < desc[sl].nw && need(sl * kBatch + u));
            }
        // park the slot state in LDS across the evaluation: it would otherwise
        // stay live in SGPRs / VGPR lanes through the register-heavy item loop
        if (lead_lane()) {
#pragma unroll
            for (int sl = 0; sl < kSlots; sl++) {
                int *pk = park + sl * 10;
                pk[0] = st[sl]; pk[1] = tq[sl]; pk[2] = tt[sl]; pk[3] = r[sl]; pk[4] = j0[sl];
                pk[5] = nseg[sl]; pk[6] = frame[sl]; pk[7] = level[sl];
                pk[8] = sl == 0 ? spec : (int)spd;
                pk[9] = ys[sl];
            }
        }
        wave_sync();
        SC_PROF(c_setup);
#if SC_PROF_CHAIN
        eval_windows<LW, RM>(a, B, reinterpret_cast<const char *>(a.table), Wl, Bl, Ol, P, st_s, surv,
                         st_p, 0, need, istats);
#else
        eval_windows<LW, RM>(a, B, reinterpret_cast<const char *>(a.table), Wl, Bl, Ol, P, st_s, surv,
                         st_p, 0, need);
#endif
        wave_sync();
        SC_PROF(c_eval);
#if SC_PROF_CHAIN
        n_rounds++;
        n_slots += n_active;
#endif
#pragma unroll
        for (int sl = 0; sl < kSlots; sl++) {
            const int *pk = park + sl * 10;
            st[sl] = __builtin_amdgcn_readfirstlane(pk[0]);
            tq[sl] = __builtin_amdgcn_readfirstlane(pk[1]);
            tt[sl] = __builtin_amdgcn_readfirstlane(pk[2]);
            r[sl] = __builtin_amdgcn_readfirstlane(pk[3]);
            j0[sl] = __builtin_amdgcn_readfirstlane(pk[4]);
            nseg[sl] = __builtin_amdgcn_readfirstlane(pk[5]);
            frame[sl] = __builtin_amdgcn_readfirstlane(pk[6]);
            level[sl] = __builtin_amdgcn_readfirstlane(pk[7]);
            ys[sl] = __builtin_amdgcn_readfirstlane(pk[9]);
        }
        spec = __builtin_amdgcn_readfirstlane(park[8]);
        spd = (unsigned)__builtin_amdgcn_readfirstlane(park[10 + 8]);
        if (kSpec && spec >= 0) {  // a speculative round: results and bits into task `spec`'s arrays, no chain step
            const int fr = spec == 0 ? frame[0] : frame[1], y = spec == 0 ? ys[0] : ys[1], jj = spec == 0 ? j0[0] : j0[1];
            const LevelInfo &L = Lv[spec == 0 ? level[0] : level[1]];
            const long long gi0 = (long long)fr * w.grid_per_frame + L.grid_base +
                                  (long long)(y / w.step) * L.nx + jj;
            unsigned long long *ev_ = evb(spec), *gd_ = gdb(spec), *dt_ = dtb(spec);
            float *sg = s_seg(spec);
            const int k0 = 2 * kBatch * spec_cur(spec == 0 ? 0 : 1);  // the round's first window
#pragma unroll
            for (int d = 0; d < 2; d++)
#pragma unroll
                for (int c = 0; c < kBatchChunks; c++) {
                    const unsigned long long mk = mine[d][c];
                    if (!mk) continue;
                    const bool in = (mk >> lane_id<RM>()) & 1ull;
                    const int u = c * 64 + lane_id<RM>();
                    const int k = k0 + d + 2 * u;
                    bool good = false, det = false;
                    if (in) {
                        const int p = st_p[d * kBatch + u];
                        const float sc = st_s[d * kBatch + u];
                        if (p >= 0) {
                            const double fin = ((double)sc + p + 1) / S;  // ObjDetector.cpp:201
                            good = !(fin < w.stride_score);               // :214
                        }
                        det = p == S;
                        sg[k] = sc;
                        if (a.st_p) {
                            a.st_p[gi0 + k] = (int8_t)p;
                            a.st_s[gi0 + k] = sc;
                        }
                    }
                    const unsigned long long gm = __ballot(good), dm = __ballot(det);
                    if (lead_lane()) {
                        const int base = k0 + d + 128 * c;
                        or_spread(ev_, base, mk);
                        if (gm) or_spread(gd_, base, gm);
                        if (dm) or_spread(dt_, base, dm);
                    }
                }
            wave_sync();
            spd += 1u << (8 + 8 * (spec == 0 ? 0 : 1));  // the task's next round starts 2*kBatch on
            SC_PROF(c_merge);
            continue;
        }

        // 3) per slot: merge the batch, advance the chain
#pragma unroll
        for (int sl = 0; sl < kSlots; sl++) {
            if (st[sl] != 2) continue;
            const int fr = frame[sl], y = ys[sl];
            const LevelInfo &L = Lv[level[sl]];
            const long long gi0 = (long long)fr * w.grid_per_frame + L.grid_base +
                                  (long long)(y / w.step) * L.nx + j0[sl];
            unsigned long long *ev_ = evb(sl), *gd_ = gdb(sl), *dt_ = dtb(sl);
            float *sg = s_seg(sl);
#pragma unroll
            for (int c = 0; c < kBatchChunks; c++) {
                const unsigned long long mk = mine[sl][c];
                if (!mk) continue;
                const bool in = (mk >> lane_id<RM>()) & 1ull;
                const int u = c * 64 + lane_id<RM>();
                const int k = r[sl] + 2 * u;
                bool good = false, det = false;
                if (in) {
                    const int p = st_p[sl * kBatch + u];
                    const float sc = st_s[sl * kBatch + u];
                    if (p >= 0) {
                        const double fin = ((double)sc + p + 1) / S;  // ObjDetector.cpp:201
                        good = !(fin < w.stride_score);               // :214
                    }
                    det = p == S;  // passed every stage
                    sg[k] = sc;
                    if (a.st_p) {  // debug: per-window results for the parity dumps
                        a.st_p[gi0 + k] = (int8_t)p;
                        a.st_s[gi0 + k] = sc;
                    }
                }
                // the chunk's windows sit at k = r + 2u: their evaluated / good /
                // detection bits, spread to every second bit, written by one
                // lane (per-lane 64-bit LDS atomics on one or two words were
                // the kernel's LDS bank conflicts)
                const unsigned long long gm = __ballot(good), dm = __ballot(det);
                if (lead_lane()) {
                    const int base = r[sl] + 128 * c;
                    or_spread(ev_, base, mk);
                    if (gm) or_spread(gd_, base, gm);
                    if (dm) or_spread(dt_, base, dm);
                }
            }
            wave_sync();
            int rr = r[sl];
            const int ns = nseg[sl];
            // the segment's bit words, read once per word into SGPRs (the
            // chain lands on a good window many times per word)
            int cw = -1;
            unsigned long long evw = 0, gdw = 0, dtw = 0;
            for (;;) {  // from a landing position: every second window until a good one
                const int c = rr >> 6, b = rr & 63;
                if (c != cw) {
                    evw = uniform64(ev_[c]);
                    gdw = uniform64(gd_[c]);
                    dtw = uniform64(dt_[c]);
                    cw = c;
                }
                const unsigned long long par = (b & 1) ? ~kEven : kEven;
                const int lim = min(64, ns - (c << 6));  // bits past the segment
                const unsigned long long inseg = lim == 64 ? ~0ull : ((1ull << lim) - 1ull);
                const unsigned long long path = par & (~0ull << b) & inseg;
                const unsigned long long unev = path & ~evw, good = path & evw & gdw;
                const int f = unev ? __builtin_ctzll(unev) : 64;
                const int qg = good ? __builtin_ctzll(good) : 64;
                unsigned long long vis;
                if (f < qg) {  // an unevaluated window: next batch from there
                    vis = path & ((1ull << f) - 1ull);
                    rr = (c << 6) + f;
                } else if (qg < 64) {  // lands on good window qg, continues at qg + 1
                    vis = path & (qg == 63 ? ~0ull : ((2ull << qg) - 1ull));
                    const int k = (c << 6) + qg;
                    if (lead_lane() && ((dtw >> qg) & 1ull)) {  // detection (:203)
                        const int slot = atomicAdd(&w.counters[0], 1);
                        atomicAdd(&w.counters[1 + w.frame0 + fr], 1);
                        if (slot < w.capacity) {
                            sc_det_record rec;
                            rec.frame = w.frame0 + fr;
                            rec.level = level[sl];
                            rec.x = (j0[sl] + k) * w.step;
                            rec.y = y;
                            rec.w = L.l;
                            rec.h = L.lh;
                            rec.stage_reached = S;
                            rec._pad = 0;
                            rec.score = ((double)sg[k] + S + 1) / S;  // :201
                            w.out[slot] = rec;
                        }
                    }
                    rr = k + 1;
                } else {  // every path bit of this word visited
                    vis = path;
                    if (lim < 64) rr = (c << 6) + (63 - __builtin_clzll(path)) + 2;
                    else rr = ((c + 1) << 6) + (b & 1);
                }
                vtot += __popcll(vis);
                if (w.dbg_v && ((vis >> lane_id<RM>()) & 1ull)) w.dbg_v[gi0 + (c << 6) + lane_id<RM>()] = 1;
                if (f < qg || rr >= ns) break;
            }
            r[sl] = rr;
            if (rr >= ns) finish(sl, j0[sl] + rr);
        }
        wave_sync();
        SC_PROF(c_merge);
    }
    // the visited count: only its sum is read (SC_INFO_VISITED), so one add
    // per wave instead of one returning-free atomic per task, spread over the
    // launch's words (the poll after a task's end waits for its atomics)
    if (vtot && lead_lane())
        atomicAdd(&w.row_visited[(blockIdx.x * kChainWaves + wv) % (w.n_rows * a.n_frames)], vtot);
    if (nspec && lead_lane()) atomicAdd(w.spec, (int)nspec);
#undef SC_OF
#undef SC_ACT
#if SC_PROF_CHAIN
    if (w.prof && lead_lane()) {  // this wave's start and exit times (launch timeline)
        const int gw = blockIdx.x * kChainWaves + wv;
        if (gw < 8192) {
            w.prof[16 + 2 * gw] = t_start;
            w.prof[17 + 2 * gw] = __builtin_amdgcn_s_memrealtime();
        }
    }
    if (w.prof && lead_lane()) {
        atomicAdd(&w.prof[0], c_idle);
        atomicAdd(&w.prof[1], c_setup);
        atomicAdd(&w.prof[2], c_eval);
        atomicAdd(&w.prof[3], c_merge);
        atomicAdd(&w.prof[4], n_rounds);
        atomicAdd(&w.prof[5], n_slots);
        atomicAdd(&w.prof[6], c_deq);
        atomicAdd(&w.prof[7], c_poll);
        atomicAdd(&w.prof[8], istats.iters);
        atomicAdd(&w.prof[9], istats.lanes);
        atomicAdd(&w.prof[10], istats.pre_cyc);
        atomicAdd(&w.prof[11], istats.thin32);
        atomicAdd(&w.prof[12], istats.stages);
        atomicAdd(&w.prof[13], istats.surv);
        atomicAdd(&w.prof[14], istats.need);
        atomicAdd(&w.prof[15], istats.pass);
    }
#endif
}

}  // namespace

int launch_cascade(const CascadeArgs &a, const LaunchCfg &c, hipStream_t s) {
    const int SA = (a.strip_max * a.band_rows + 63) & ~63;
    const size_t scratch = kWavesPerWg * wave_scratch_bytes(SA);
    // weights in LDS whenever they fit: measured faster even where it costs
    // occupancy (64x128 model, K = 380: 2 instead of 3 workgroups per CU, -2.5%)
    bool lw = model_lds_bytes(a.K, true) + scratch <= 160 * 1024;
    if (c.lds_weights >= 0) lw = lw && c.lds_weights != 0;  // SC_OPT_LDS_WEIGHTS
    const size_t lds = model_lds_bytes(a.K, lw) + scratch;
    int per_cu = 0;
    if (lw)
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, cascade_kernel<true>, kCascadeThreads, lds);
    else
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, cascade_kernel<false>, kCascadeThreads, lds);
    per_cu = std::max(1, std::min(per_cu, 4));
    if (c.wgs_per_cu > 0) per_cu = std::min(per_cu, c.wgs_per_cu);  // SC_OPT_WGS_PER_CU
    const int grid = std::max(1, c.cus) * per_cu;
    if (lw)
        hipLaunchKernelGGL(cascade_kernel<true>, dim3(grid), dim3(kCascadeThreads), lds, s, a);
    else
        hipLaunchKernelGGL(cascade_kernel<false>, dim3(grid), dim3(kCascadeThreads), lds, s, a);
    return grid;
}

void launch_walk(const WalkArgs &a, int n_frames, hipStream_t s) {
    hipLaunchKernelGGL(walk_kernel, dim3(a.n_rows * n_frames), dim3(64), 0, s, a);
}

bool chain_batch_waves16(int K, int row_max, int n_levels, long long frame4) {
    return frame4 * 16 <= (128ll << 20) &&
           model_lds_bytes(K, true) + 16 * chain_wave_bytes(row_max) + n_levels * sizeof(LevelInfo) + 16 <=
               160 * 1024;
}

int launch_chain(const CascadeArgs &a, const WalkArgs &w, const LaunchCfg &c, hipStream_t s, int *waves_out) {
    auto scratch = [&](int nw) { return nw * chain_wave_bytes(w.row_max) + w.n_levels * sizeof(LevelInfo) + 16; };
    const size_t kLds = 160 * 1024;
    // 16 waves with the weights in LDS when they fit and a frame's table sits
    // comfortably in the 256 MiB Infinity Cache; else 12 (weights in LDS when
    // they fit: measured faster even where it costs occupancy).  More waves
    // help the latency-bound narrow levels (C2 levels 0-12: -3 %) and hurt the
    // wide ones, whose gathers already saturate the Infinity-Cache fabric
    // (levels 13-23 alone: 106 % of the measured gather ceiling, +12 % at 16
    // waves); a 4K frame's 265 MB table leaves the Infinity Cache (C4: +8 %
    // at 16 waves).  C2 as a whole: -2.7 % (profiles/r3/g3).
    // One-frame launches (the latency path): 12 (0.656 vs 0.673 ms per 1080p
    // frame, profiles/r3/g12), the hand-off fill and drain dominate them.
    // Tables beyond the Infinity Cache (a 4K frame's 265 MB) with 2+ frames
    // per launch: 10 (fewer rows in flight per XCD: C4 24.70 ms per launch vs
    // 24.92 at 8 and 25.22 at 12, profiles/r5/f; at 8 its widest levels 24-31
    // alone 7.58 vs 7.85 ms, levels 0-23 19.30 vs 18.45, profiles/r5/e).
    // With the lane-pair item form (interleaved cells, cs 2: §3 of DESIGN.md)
    // such tables run 12 waves again: C4 21.80 vs 22.52 ms at 10, 22.10 at
    // 14, 24.39 at 8 (profiles/r6/n); 10 stays for the one-lane form.
    const bool fabric_bound = a.g.frame4 * 16 > (128ll << 20);
    int nw = a.n_frames > 1 && chain_batch_waves16(a.K, w.row_max, w.n_levels, a.g.frame4) ? 16
             : fabric_bound && a.n_frames > 1 && a.g.cs == 1                                 ? 10
                                                                                             : 12;
    if (c.chain_waves == 8 || c.chain_waves == 10 || c.chain_waves == 12 ||
        ((c.chain_waves == 14 || c.chain_waves == 16) &&
         model_lds_bytes(a.K, false) + scratch(c.chain_waves) <= kLds))
        nw = c.chain_waves;  // SC_OPT_CHAIN_WAVES (8 / 14: A/B only)
    bool lw = model_lds_bytes(a.K, true) + scratch(nw) <= kLds;
    if (c.lds_weights >= 0) lw = lw && c.lds_weights != 0;  // SC_OPT_LDS_WEIGHTS
    const size_t lds = model_lds_bytes(a.K, lw) + scratch(nw);
    const int nt = 64 * nw;
    int per_cu = 0;
    if (nw == 8)
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lw ? chain_kernel<true, 8> : chain_kernel<false, 8>,
                                                           nt, lds);
    else if (nw == 10)
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lw ? chain_kernel<true, 10> : chain_kernel<false, 10>,
                                                           nt, lds);
    else if (nw == 14)
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lw ? chain_kernel<true, 14> : chain_kernel<false, 14>,
                                                           nt, lds);
    else if (nw == 16 && lw)
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, chain_kernel<true, 16>, nt, lds);
    else if (nw == 16)
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, chain_kernel<false, 16>, nt, lds);
    else if (lw)
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, chain_kernel<true, 12>, nt, lds);
    else
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, chain_kernel<false, 12>, nt, lds);
    per_cu = std::max(1, std::min(per_cu, 4));
    if (c.wgs_per_cu > 0) per_cu = std::min(per_cu, c.wgs_per_cu);  // SC_OPT_WGS_PER_CU
    const int grid = std::max(1, c.cus) * per_cu;
    if (waves_out) *waves_out = nw;
    if (nw == 10 && lw)
        hipLaunchKernelGGL((chain_kernel<true, 10>), dim3(grid), dim3(nt), lds, s, a, w);
    else if (nw == 10)
        hipLaunchKernelGGL((chain_kernel<false, 10>), dim3(grid), dim3(nt), lds, s, a, w);
    else if (nw == 14 && lw)
        hipLaunchKernelGGL((chain_kernel<true, 14>), dim3(grid), dim3(nt), lds, s, a, w);
    else if (nw == 14)
        hipLaunchKernelGGL((chain_kernel<false, 14>), dim3(grid), dim3(nt), lds, s, a, w);
    else if (nw == 8 && lw)
        hipLaunchKernelGGL((chain_kernel<true, 8>), dim3(grid), dim3(nt), lds, s, a, w);
    else if (nw == 8)
        hipLaunchKernelGGL((chain_kernel<false, 8>), dim3(grid), dim3(nt), lds, s, a, w);
    else if (nw == 16 && lw)
        hipLaunchKernelGGL((chain_kernel<true, 16>), dim3(grid), dim3(nt), lds, s, a, w);
    else if (nw == 16)
        hipLaunchKernelGGL((chain_kernel<false, 16>), dim3(grid), dim3(nt), lds, s, a, w);
    else if (lw)
        hipLaunchKernelGGL((chain_kernel<true, 12>), dim3(grid), dim3(nt), lds, s, a, w);
    else
        hipLaunchKernelGGL((chain_kernel<false, 12>), dim3(grid), dim3(nt), lds, s, a, w);
    return grid;
}

size_t chain_lds_bytes(int K, int row_max, int n_levels) {  // smallest variant (12 waves, weights via caches)
    return model_lds_bytes(K, false) + 12 * chain_wave_bytes(row_max) + n_levels * sizeof(LevelInfo) + 16;
}

size_t cascade_lds_bytes(int K, int strip_max, int band_rows) {  // smallest variant
    return model_lds_bytes(K, false) +
           kWavesPerWg * wave_scratch_bytes((strip_max * band_rows + 63) & ~63);
}

}  // namespace sc
