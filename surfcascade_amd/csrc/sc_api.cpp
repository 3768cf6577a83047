// sc_api.cpp -- the C ABI (include/surfcascade.h): model I/O, detector
// lifecycle, geometry tables, launches, result gathering.
//
// Host-side precomputation mirrors the reference's per-image setup:
//   levels     l_i = (int)(70*pow(1.1,i)), count (int)min(log..)+1  ObjDetector.cpp:174,180
//   step       win.width>20 ? win.width/20 : 1                      ObjDetector.cpp:139
//   fitted patch table per stage (GetFittedPatchIndexes)            ObjDetector.cpp:119-130
//   ProjectPatches per level (depends on l only; the window origin is an
//   additive offset)                                                DenseSURFFeatureExtractor.cpp:459-484
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <sstream>
#include <string>
#include <vector>

#include "sc_kernels.hpp"
#include "sc_group.hpp"
#include "sc_jpeg.hpp"
#include "sc_model.hpp"
#include "surfcascade.h"

using sc::Error;

struct sc_model {
    sc::Cascade c;
};

namespace {

constexpr int kBandRows = 1;  // grid rows per cascade task (SC_BAND_ROWS overrides)
constexpr bool kSplitLayout = true;  // table cell format (SC_OPT_TABLE_LAYOUT 1: interleaved)
#ifndef SC_PAIR
#define SC_PAIR 1
#endif
#if SC_PAIR
// the lane-pair item form (sc_device.hpp) runs on interleaved cells: chosen
// per frame size and model (build_geometry); SC_OPT_TABLE_LAYOUT 1 forces it
constexpr bool kPairBigTables = true;
#ifndef SC_PAIR_MIN_MIB  // (A/B: 0 puts every lazy-grid frame on the lane-pair form)
#define SC_PAIR_MIN_MIB 128
#endif
#else
#define SC_PAIR_MIN_MIB 128
constexpr bool kPairBigTables = false;
#endif

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            throw Error{SC_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)}; \
    } while (0)

template <class T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    void ensure(size_t want) {
        if (want <= n) return;
        release();
        HIPCHK(hipMalloc(&p, std::max<size_t>(want, 1) * sizeof(T)));
        n = want;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

// Pinned host staging for frames handed over in pageable host memory: the
// DMA engine reads pinned pages directly, while a pageable 2-D copy is
// staged by the runtime in small pieces (measured on MI355X: 16 x 1080p
// frames through hipMemcpy2DAsync from pageable memory took ~21 ms).
struct PinnedBuf {
    uint8_t *p = nullptr;
    size_t n = 0;
    void ensure(size_t want) {
        if (want <= n) return;
        release();
        HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&p), std::max<size_t>(want, 1), hipHostMallocDefault));
        n = want;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
    }
};

struct Geometry {
    int W = 0, H = 0;
    int n_levels = 0, step = 1, nx_max = 0;
    int n_sub = 1, strip_max = 1;  // cascade tasks: 8*n_sub strips per band
    int band_rows = 1, n_bands = 0;
    sc::TableGeom tg{};
    long long grid = 0;
    std::vector<sc::LevelInfo> levels;
    std::vector<int2> rows;   // chain kernel task order (rows1: one-frame launches)
    std::vector<int2> rows1;
    int n_wide = 0;           // SC_WIDECAP builds: the wide levels' rows at the end of `rows`
    std::vector<sc::ProjPatch> proj;
    std::vector<sc::ProjPatch> proj_all;  // miner: every template patch per level
    std::vector<sc::TaskDesc> tasks;
};

}  // namespace

struct sc_detector {
    int device = 0;
    hipStream_t stream = nullptr;      // where launches go: own_stream, or the caller's (sc_detector_set_stream)
    hipStream_t own_stream = nullptr;  // created with the detector, destroyed with it
    sc_scan_params prm{};
    sc::Cascade casc;
    int K = 0, S = 0;
    std::vector<int32_t> patch_rects;  // fitted template rect per global weak
    // model on device
    DevBuf<float> d_w;
    DevBuf<double> d_bias;
    DevBuf<float> d_theta;
    DevBuf<int> d_stage_off;
    DevBuf<int16_t> d_order;      // per stage: weak indices sorted by patch shape
    DevBuf<int4> d_rects;         // per weak: template rect record (sc::InlinePatch)
    int chunk_min = 1 << 30;  // one-lane-per-window stages only when n > item buffer
    bool lazy = true;         // chain kernel: only windows the x chain reaches are evaluated
    int cus = 0;              // compute units of `device` (queried once at creation)
    // tuning / test options (sc_detector_set_option; never read from the environment)
    struct Options {
        int full_grid = 0, chunk_min = 0, table_layout = 0, phases = 0, substrips = 0;
        int band_rows = 0, row_order = 2, row_block = 32, chain_chunk = 0;
        bool order_set = false;  // ROW_ORDER / ROW_BLOCK set: one-frame launches use them too
        int lds_weights = -1, wgs_per_cu = 0, profile = 0, chain_segs = 0, integral_passes = 0;
        int level_lo = 0, level_hi = 0;  // scan only levels [lo, hi) (hi 0: all)
        int chain_waves = 0;             // chain kernel waves per workgroup (0 auto)
        int integral_fuse = 0;           // column walks inside the chain kernel: 0 auto, 1 never, 2 from 2 frames
        int integral_pre = 0;            // fused: frames integrated before the chain kernel (0: 2)
        int drop_handoff = -1;           // test only: task whose segment-0 hand-off is dropped (watchdog)
        int drop_walk = -1;              // test only: fused column walk whose completion count is dropped
        int chain_subq = 0;              // chain kernel dequeue sub-queues per XCD (0 auto: 4 one frame, else 1)
        int chain_spec = 0;              // speculative rounds per waiting task of a one-frame launch (0 auto)
        int chain_slots = 0;             // task slots per wave of the chain kernel (0 auto: 1 one frame, 2 batches)
    } opt;
    int shard_rank = 0, shard_world = 1;  // grid sharding: rows i with i % world == rank
    // geometry on device
    Geometry geo;
    DevBuf<sc::LevelInfo> d_levels;
    DevBuf<int2> d_rows;
    DevBuf<sc::ProjPatch> d_proj;
    // hard-negative miner (FillNegSamples): stride 10, no prefilter, no walk
    bool miner = false;
    std::vector<int32_t> all_rects;  // every template patch (ExtractPatches)
    DevBuf<sc::ProjPatch> d_proj_all;
    DevBuf<int> d_mine_cnt, d_mine_off;
    DevBuf<sc::MineWindow> d_mine_win;
    DevBuf<int> d_mine_fc;  // [1 + n]: candidates of the batch, per frame
    DevBuf<float> d_feat;
    DevBuf<sc::TaskDesc> d_tasks;
    // working buffers
    DevBuf<uint8_t> d_frames;
    PinnedBuf h_stage;           // host frames -> pinned -> d_frames (upload_frames)
    DevBuf<float4> d_table;
    DevBuf<uint32_t> d_carry;    // integral pass 1 -> pass 2: per-strip row prefixes
    DevBuf<uint32_t> d_colblk;   // one-frame column pass: exact column-block sums (colseg)
    int table_frames = 0;
    DevBuf<sc_det_record> d_out;
    DevBuf<int> d_counters;
    DevBuf<unsigned> d_visited;  // [frame][row] words whose sum is the windows the x chain visited
    DevBuf<int> d_queues;       // per-XCD task counters of the cascade kernel
    DevBuf<int> d_entry;        // chain kernel: per (row, segment) chain entry + 1
    DevBuf<unsigned long long> d_prof;  // chain kernel phase cycles (SC_PROF_CHAIN builds)
    long long err_word = -1;    // chain kernel: index of the launch's watchdog-fired flag in d_entry
    long long spec_word = -1;   // ... and of its speculative-round count (SC_INFO_SPEC_ROUNDS)
    // chain kernel: hand-offs that timed out, summed over every launch since
    // the last check_chain (sticky: rowcarry's per-call zeroing does not
    // touch it, so a timeout in any pipelined step is still raised at the
    // next synchronisation); zeroed once at allocation and after each read
    DevBuf<int> d_err;
    int *h_err = nullptr;  // its raised flag, mapped host memory the kernel writes (check_chain)
    bool chain_launched = false;  // a chain launch since the last check_chain
    DevBuf<int8_t> d_st_p;      // per grid window: stage reached (-1 prefilter reject)
    DevBuf<float> d_st_s;       // per grid window: last stage score
    // debug
    bool debug = false;
    DevBuf<uint8_t> d_dbg_v;    // per grid window: visited by the x chain
    int last_frames = 0;
    int last_fused = 0;  // frames of the last call integrated inside the chain kernel
    int last_nseg = 8;   // segments per row of the last chain launch (profiling readout)
    int last_waves = 0;  // waves per workgroup of the last chain launch (SC_INFO_CHAIN_WAVES)
    int last_subq = 0;   // dequeue sub-queues of the last chain launch (SC_INFO_CHAIN_SUBQ)
    int last_colpass = 0;  // column pass of the last call's prebuilt frames (SC_INFO_COLUMN_PASS)
    // timing
    bool timing = false;
    struct Pending {
        int kind;
        hipEvent_t a, b;
    };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> event_pool;
    double t_ms[SC_KERNEL_COUNT] = {};
    long long t_n[SC_KERNEL_COUNT] = {};

    ~sc_detector() {
        (void)hipSetDevice(device);
        (void)hipStreamSynchronize(stream);  // (also the null stream, sc_detector_set_stream(d, NULL, 0))
        if (own_stream && own_stream != stream) (void)hipStreamSynchronize(own_stream);
        for (auto &p : pending) {
            event_pool.push_back(p.a);
            event_pool.push_back(p.b);
        }
        for (hipEvent_t e : event_pool) (void)hipEventDestroy(e);
        d_w.release(); d_bias.release(); d_theta.release(); d_stage_off.release(); d_order.release();
        d_rects.release();
        d_levels.release(); d_rows.release(); d_proj.release(); d_tasks.release();
        d_proj_all.release(); d_mine_cnt.release(); d_mine_off.release(); d_mine_win.release();
        d_feat.release();
        d_frames.release(); d_table.release(); d_carry.release(); d_colblk.release(); d_out.release(); d_counters.release();
        d_visited.release(); d_queues.release(); d_entry.release(); d_err.release(); d_st_p.release(); d_st_s.release();
        d_dbg_v.release(); d_prof.release();
        h_stage.release();
        if (h_err) (void)hipHostFree(h_err);
        if (own_stream) (void)hipStreamDestroy(own_stream);
    }

    hipEvent_t ev() {
        if (!event_pool.empty()) {
            hipEvent_t e = event_pool.back();
            event_pool.pop_back();
            return e;
        }
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        return e;
    }
};

namespace {

int ref_step(const sc_scan_params &p) {
    if (p.step > 0) return p.step;
    return p.base_len > 20 ? p.base_len / 20 : 1;  // ObjDetector.cpp:139
}

// ObjDetector.cpp:174 (float log of W/(float)70, f64 division by log(1.1)) + 1.
int ref_levels(int W, int H, const sc_scan_params &p) {
    if (p.n_levels >= 0) return p.n_levels;
    double a = std::log((float)W / (float)p.base_len) / std::log(p.scale_factor);
    double b = std::log((float)H / (float)(p.base_len * p.aspect_h)) / std::log(p.scale_factor);
    return (int)std::min(a, b) + 1;
}

// Operand ranges of Normalize's sqrt / reciprocal (DenseSURFFeatureExtractor.cpp:
// 427-457) for a W x H frame: a channel's table value is at most 255*W*H (the
// f32 sums round to at most that bound's next representable value), a box
// sum (TL + BR) - (TR + BL) at most twice that, so SS = eps + sum of 32
// squares <= eps + 32 * (2 * 255 * W * H)^2 (with a 1e-6 relative margin for
// the f32 roundings); SS >= eps (FLT_EPSILON seed, non-negative terms); the
// clipped SS2 lies between eps and SS.  d = sqrt(SS2).
void normalize_operand_range(int W, int H, double ss[2], double d[2]) {
    const double fmax = 2.0 * 255.0 * (double)W * (double)H * (1.0 + 1e-6);
    ss[0] = (double)FLT_EPSILON;
    ss[1] = ((double)FLT_EPSILON + 32.0 * fmax * fmax) * (1.0 + 1e-6);
    d[0] = std::sqrt(ss[0]) * (1.0 - 1e-6);
    d[1] = std::sqrt(ss[1]);
}

void build_geometry(sc_detector *d, int W, int H) {
    Geometry &g = d->geo;
    if (g.W == W && g.H == H) return;
    if (W < 2 || H < 2) throw Error{SC_ERR_INVALID, "frame must be at least 2x2"};
    if (W > 32767 || H > 32767) throw Error{SC_ERR_INVALID, "frame dimension above 32767"};
    const sc_scan_params &p = d->prm;
    Geometry ng;
    ng.W = W;
    ng.H = H;
    ng.step = ref_step(p);
    // a frame smaller than the base window gives a negative count from the
    // formula: the reference's inclusive level loop (ObjDetector.cpp:178)
    // then runs no level, and so does the scan here
    ng.n_levels = std::max(0, ref_levels(W, H, p));
    if (ng.n_levels > 256) throw Error{SC_ERR_INVALID, "bad level count"};
    {   // phase-split table geometry (sc_kernels.hpp)
        sc::TableGeom &t = ng.tg;
        t.W = W;
        t.H = H;
        t.step = ng.step;
        // parity-split phase planes: the lazy grid's batches (one parity,
        // windows 2 apart) then read consecutive cells
        // (the full grid -- dumps, the miner -- reads consecutive windows: step planes)
        const int mult = d->opt.phases ? d->opt.phases : (d->lazy ? 2 : 1);  // SC_OPT_PHASES
        t.ph = mult * ng.step;
        const int Q = (W + 1 + t.ph - 1) / t.ph;
        t.Qp = (Q + 15) & ~15;
        t.rowp = 2 * t.ph * t.Qp;
        t.frame4 = (long long)(H + 1) * t.rowp;
        // the lane-pair item form (interleaved cells) wherever a batch's chain
        // kernel is not the 16-wave one: tables beyond 128 MiB (C4: chain
        // 23.02 vs 24.75 ms) and models whose LDS copy leaves 12 waves (C5:
        // 21.41 vs 23.08 ms); the 16-wave kernel ties with it (C2 13.52 vs
        // 13.48 ms), one-frame launches lose (0.588 vs 0.569 ms): split cells
        // there (profiles/r6/e, f)
        bool pair = kPairBigTables && d->lazy;
        if (pair) {
            const int l0 = (int)p.base_len, nx0 = l0 >= 1 && l0 <= W ? (W - l0) / ng.step + 1 : 1;
            pair = t.frame4 * 16 > ((long long)SC_PAIR_MIN_MIB << 20) ||
                   !sc::chain_batch_waves16(d->K, (nx0 + sc::kXcds - 1) / sc::kXcds, ng.n_levels, t.frame4);
        }
        const bool split = d->opt.table_layout ? false : kSplitLayout && !pair;
        t.cs = split ? 1 : 2;  // SC_OPT_TABLE_LAYOUT
        t.hs = split ? t.ph * t.Qp : 1;
        if ((long long)(H + 1) * t.rowp > (1ll << 28))  // byte offsets within a frame table: u32
            throw Error{SC_ERR_INVALID, "frame too large for 32-bit table offsets"};
        {   // Normalize's operands stay inside the ranges the short sqrt /
            // reciprocal were checked over exhaustively (sc_device.hpp,
            // tests/test_gpu_rn.py); never fires for a frame the offset check admits
            double ss[2], dd[2];
            normalize_operand_range(W, H, ss, dd);
            if (ss[0] < sc::kRnSqrtLo || ss[1] > sc::kRnSqrtHi || dd[0] < sc::kRnRcpLo || dd[1] > sc::kRnRcpHi)
                throw Error{SC_ERR_INVALID, "frame too large for Normalize's checked operand range"};
        }
        // x / ph as umulhi(x, ceil(2^32/ph)) in the chain kernel's per-item
        // projection: exact for every column a patch corner can take
        t.phm = t.ph > 1 ? (unsigned)((0x100000000ull + (unsigned)t.ph - 1) / (unsigned)t.ph) : 0u;
        bool exact = t.ph > 1;
        for (unsigned x = 0; exact && x <= (unsigned)(W + 2 * t.ph); x++)
            exact = (unsigned)(((unsigned long long)x * t.phm) >> 32) == x / (unsigned)t.ph;
        if (!exact && d->lazy)
            throw Error{SC_ERR_INVALID, "phase-plane count unsupported by the chain kernel"};
    }
    const sc::TableGeom &tg = ng.tg;
    // cell of column cx relative to the window origin, for windows of parity
    // par (x = step*j, j % 2 == par): at(x + cx) - at(x) depends on x only
    // through that parity
    auto col_off = [&](int par, int cx) { return tg.at(ng.step * par + cx, 0) - tg.at(ng.step * par, 0); };
    ng.proj.resize((size_t)ng.n_levels * 2 * d->K);
    long long gb = 0;
    for (int i = 0; i < ng.n_levels; i++) {
        sc::LevelInfo L{};
        L.l = (int)(p.base_len * std::pow(p.scale_factor, i));  // ObjDetector.cpp:180
        L.lh = L.l * p.aspect_h;
        L.grid_base = gb;
        L.thr = (float)(L.l * L.lh) * p.prefilter_k;
        L.scale = (float)L.l / (float)p.tmpl_w;  // ProjectPatches (DenseSURFFeatureExtractor.cpp:463)
        if (L.l >= 1 && L.l <= W && L.lh <= H) {
            L.nx = (W - L.l) / ng.step + 1;
            L.ny = (H - L.lh) / ng.step + 1;
            L.pre_col[0] = col_off(0, L.l);
            L.pre_col[1] = col_off(1, L.l);
            L.pre_row = L.lh * tg.rowp;
            if (L.nx > 4096)  // walk kernel: one wave, 64 chunks of 64 windows per row
                throw Error{SC_ERR_INVALID, "more than 4096 windows per row (frame too wide)"};
            const bool scanned = i >= d->opt.level_lo && (d->opt.level_hi == 0 || i < d->opt.level_hi);
            if (scanned)  // SC_OPT_LEVEL_LO / _HI (level-group profiling); grid indices stay the frame's
                for (int r = 0; r < L.ny; r++) ng.rows.push_back(make_int2(i, r * ng.step));
            gb += (long long)L.nx * L.ny;
            ng.nx_max = std::max(ng.nx_max, L.nx);
        }
        // ProjectPatches (DenseSURFFeatureExtractor.cpp:459-484) + cell split
        // (GetRectsFromPatch :360-377) for every fitted patch at this level.
        const float scale = L.scale;
        auto project = [&](const int32_t *r, int par) {
            int px = (int)((float)r[0] * scale), py = (int)((float)r[1] * scale), pw, ph;
            if (r[2] >= r[3]) {
                int ratio = r[2] / r[3];
                ph = (int)((float)r[3] * scale);
                pw = ph * ratio;
            } else {
                int ratio = r[3] / r[2];
                pw = (int)((float)r[2] * scale);
                ph = pw * ratio;
            }
            sc::ProjPatch pp{};
            int gw, gh, c;
            if (pw == ph) {
                c = pw / 2;
                pp.shape = 0;
                gw = gh = 2;
            } else {
                c = std::min(pw, ph);
                pp.shape = pw < ph ? 1 : 2;
                gw = pw / std::max(c, 1);
                gh = ph / std::max(c, 1);
            }
            if (c <= 0)
                throw Error{SC_ERR_INVALID, "projected cell edge is 0 at level " + std::to_string(i)};
            if (L.nx > 0 && (px + gw * c > L.l || py + gh * c > L.lh))
                throw Error{SC_ERR_INVALID, "projected patch leaves the window at level " +
                                                std::to_string(i)};
            pp.row0 = py * tg.rowp;
            pp.rowstep = c * tg.rowp;
            for (int q = 0; q <= gw; q++) pp.col[q] = col_off(par, px + q * c);
            return pp;
        };
        for (int par = 0; par < 2; par++) {
            for (int k = 0; k < d->K; k++)
                ng.proj[((size_t)i * 2 + par) * d->K + k] = project(&d->patch_rects[4 * k], par);
            if (d->miner)  // ExtractFeatures over every template patch (:88-93)
                for (size_t j = 0; j < d->all_rects.size() / 4; j++)
                    ng.proj_all.push_back(project(&d->all_rects[4 * j], par));
        }
        ng.levels.push_back(L);
    }
    ng.grid = gb;  // may be 0: no window fits (the reference loop runs 0 times)
    if (d->shard_world > 1) {
        // single-frame window-grid sharding: this rank keeps
        // the (level, y) rows i of the canonical row list with i % world ==
        // rank -- every rank gets ny/world (+-1) rows of every level, so the
        // grid windows balance, and spatially clustered work spreads over the
        // ranks.  The adaptive-stride chain never leaves its row
        // (ObjDetector.cpp:185-217), so the rows are independent; grid
        // indices (dumps) stay those of the whole frame.
        std::vector<int2> mine;
        for (size_t i = 0; i < ng.rows.size(); i++)
            if ((int)(i % (size_t)d->shard_world) == d->shard_rank) mine.push_back(ng.rows[i]);
        ng.rows.swap(mine);
    }
    {   // cascade tasks: one strip (~72 windows wide at the widest level) of a
        // band of band_rows consecutive grid rows of one level
        ng.n_sub = d->opt.substrips ? d->opt.substrips  // SC_OPT_SUBSTRIPS
                                    : std::max(1, (ng.nx_max + sc::kXcds * 72 / 2) / (sc::kXcds * 72));
        ng.band_rows = d->opt.band_rows ? d->opt.band_rows : kBandRows;  // SC_OPT_BAND_ROWS
        if (d->shard_world > 1) ng.band_rows = 1;  // a rank's rows are not consecutive
        const int nseg = sc::kXcds * ng.n_sub;
        ng.strip_max = std::max(1, (ng.nx_max + nseg - 1) / nseg);
        if (ng.strip_max > 0xffff) throw Error{SC_ERR_INVALID, "strip too wide"};
        const size_t lds = sc::cascade_lds_bytes(d->K, ng.strip_max, ng.band_rows);
        if (lds > 160 * 1024)
            throw Error{SC_ERR_INVALID, "cascade with " + std::to_string(d->K) +
                                            " weak classifiers does not fit the kernel's LDS (" +
                                            std::to_string(lds) + " B)"};
        // one descriptor per (band, strip); rows are level-major, y ascending
        ng.tasks.clear();
        for (size_t r0 = 0; r0 < ng.rows.size();) {
            const int lv = ng.rows[r0].x;
            size_t r1 = r0;
            while (r1 < ng.rows.size() && ng.rows[r1].x == lv && (int)(r1 - r0) < ng.band_rows) r1++;
            const sc::LevelInfo &L = ng.levels[lv];
            const int y = ng.rows[r0].y, nxs = (L.nx + nseg - 1) / nseg;
            for (int sgi = 0; sgi < nseg; sgi++) {
                sc::TaskDesc t{};
                const int j0 = sgi * nxs;
                t.nw = std::max(0, std::min(L.nx, j0 + nxs) - j0);
                t.nr = (int)(r1 - r0);
                t.g_row = L.nx;
                t.t_off = y * tg.rowp;
                t.j0 = j0;
                t.g_off = (int)(L.grid_base + (long long)(y / ng.step) * L.nx + j0);
                t.level = lv;
                t.thr = L.thr;
                t.pre_row = L.pre_row;
                t.pre_col[0] = L.pre_col[0];
                t.pre_col[1] = L.pre_col[1];
                ng.tasks.push_back(t);
            }
            r0 = r1;
        }
        ng.n_bands = (int)(ng.tasks.size() / nseg);
    }
    {   // the chain kernel's task order (its queues deal rows in this order):
        // 2 (default): blocks of 32 grid rows (96 px at step 3), level-major
        // inside -- the rows in flight on an XCD then read a band of table
        // rows that fits its L2: 14 % less kernel time than plain level-major
        // order (0) on the C2 frames; blocks of 64 rows 1 % and of 128 rows
        // 3 % slower than 32 (profiles/r1/sweep); 1: y-major.
        // One-frame launches deal a second list (rows1): blocks of 4 grid rows
        // bottom-up (3), so the last block dealt holds every level's top rows
        // and the wide levels' short rows end the launch: chain kernel 0.606
        // vs 0.614 ms with blocks of 8 (profiles/r4/order/), 0.5822 vs 0.5854
        // with 4 (4 sub-queues, profiles/r5/e); SC_OPT_ROW_ORDER / _ROW_BLOCK
        // set explicitly apply to both lists.
        // (The full-grid tasks above are built from the level-major list.)
        auto order = [&](std::vector<int2> rows, int mode, int blk) {
            if (mode == 1)
                std::stable_sort(rows.begin(), rows.end(),
                                 [](const int2 &a, const int2 &b) { return a.y < b.y; });
            else if (mode == 2)
                std::stable_sort(rows.begin(), rows.end(),
                                 [blk](const int2 &a, const int2 &b) { return a.y / blk < b.y / blk; });
            else if (mode == 3)
                std::stable_sort(rows.begin(), rows.end(),
                                 [blk](const int2 &a, const int2 &b) { return a.y / blk > b.y / blk; });
            return rows;
        };
        ng.rows1 = d->opt.order_set ? order(ng.rows, d->opt.row_order, d->opt.row_block * ng.step)
                                    : order(ng.rows, 3, 4 * ng.step);
        ng.rows = order(ng.rows, d->opt.row_order, d->opt.row_block * ng.step);
#if defined(SC_WIDECAP) && SC_WIDECAP
        // A/B (SC_WIDECAP): the rows of levels with l >= SC_WIDE_L dealt from
        // a list of their own, each list in the order above
#ifndef SC_WIDE_L
#define SC_WIDE_L 690
#endif
        auto narrow = std::stable_partition(ng.rows.begin(), ng.rows.end(),
                                             [&](const int2 &r) { return ng.levels[r.x].l < SC_WIDE_L; });
        ng.n_wide = (int)(ng.rows.end() - narrow);
#endif
    }
    d->d_tasks.ensure(std::max<size_t>(ng.tasks.size(), 1));
    if (!ng.tasks.empty())
        HIPCHK(hipMemcpyAsync(d->d_tasks.p, ng.tasks.data(), ng.tasks.size() * sizeof(sc::TaskDesc),
                              hipMemcpyHostToDevice, d->stream));
    d->d_levels.ensure(std::max<size_t>(ng.levels.size(), 1));
    d->d_rows.ensure(std::max<size_t>(2 * ng.rows.size(), 1));  // [rows | rows1]
    d->d_proj.ensure(std::max<size_t>(ng.proj.size(), 1));
    if (!ng.levels.empty())
        HIPCHK(hipMemcpyAsync(d->d_levels.p, ng.levels.data(),
                              ng.levels.size() * sizeof(sc::LevelInfo), hipMemcpyHostToDevice,
                              d->stream));
    if (!ng.rows.empty()) {
        HIPCHK(hipMemcpyAsync(d->d_rows.p, ng.rows.data(), ng.rows.size() * sizeof(int2),
                              hipMemcpyHostToDevice, d->stream));
        HIPCHK(hipMemcpyAsync(d->d_rows.p + ng.rows.size(), ng.rows1.data(), ng.rows1.size() * sizeof(int2),
                              hipMemcpyHostToDevice, d->stream));
    }
    if (!ng.proj.empty())
        HIPCHK(hipMemcpyAsync(d->d_proj.p, ng.proj.data(), ng.proj.size() * sizeof(sc::ProjPatch),
                              hipMemcpyHostToDevice, d->stream));
    if (!ng.proj_all.empty()) {
        d->d_proj_all.ensure(ng.proj_all.size());
        HIPCHK(hipMemcpyAsync(d->d_proj_all.p, ng.proj_all.data(),
                              ng.proj_all.size() * sizeof(sc::ProjPatch), hipMemcpyHostToDevice,
                              d->stream));
    }
    HIPCHK(hipStreamSynchronize(d->stream));  // host vectors are re-assigned below
    d->geo = std::move(ng);
}

void upload_model(sc_detector *d) {
    const sc::Cascade &c = d->casc;
    d->S = (int)c.stages.size();
    d->K = c.total_weak();
    std::vector<int32_t> all = sc::extract_patches(d->prm.tmpl_w, d->prm.tmpl_h);
    if (!(d->miner && c.stages.empty()))  // a miner may run before the first stage
        sc::validate_for_detect(c, (int)all.size() / 4);
    std::vector<float> w((size_t)d->K * 36, 0.0f);
    std::vector<double> bias(d->K);
    std::vector<float> theta(d->S);
    std::vector<int> off(d->S + 1, 0);
    d->patch_rects.assign((size_t)d->K * 4, 0);
    int g = 0;
    for (int s = 0; s < d->S; s++) {
        theta[s] = c.stages[s].theta;
        off[s] = g;
        for (const sc::WeakLR &wk : c.stages[s].weak) {
            std::copy(wk.w.begin(), wk.w.end(), w.begin() + (size_t)g * 36);
            bias[g] = wk.bias;
            std::copy(all.begin() + 4 * wk.patch_index, all.begin() + 4 * wk.patch_index + 4,
                      d->patch_rects.begin() + 4 * g);
            g++;
        }
    }
    off[d->S] = g;
    // Evaluation order of the item path: within each stage, weak classifiers
    // grouped by patch shape (square / tall / wide, as GetRectsFromPatch splits
    // them) so a wave instruction mostly sees one shape.  Sums still follow
    // the model's order.
    std::vector<int16_t> order(std::max(d->K, 1));
    auto shape = [&](int k) {
        const int32_t *r = &d->patch_rects[4 * k];
        return r[2] == r[3] ? 0 : (r[2] < r[3] ? 1 : 2);
    };
    for (int s = 0; s < d->S; s++) {
        std::vector<int> ks;
        for (int k = off[s]; k < off[s + 1]; k++) ks.push_back(k - off[s]);
        std::stable_sort(ks.begin(), ks.end(),
                         [&](int x, int y) { return shape(off[s] + x) < shape(off[s] + y); });
        for (size_t j = 0; j < ks.size(); j++) order[off[s] + j] = (int16_t)ks[j];
    }
    if (d->K > 32767) throw Error{SC_ERR_MODEL, "more than 32767 weak classifiers"};
    // template rect records for the chain kernel's per-item projection
    // (sc::InlinePatch): ProjectPatches scales ph for square / wide rects and
    // pw for tall ones (DenseSURFFeatureExtractor.cpp:466-478), then
    // GetRectsFromPatch splits square rects 2x2 and the others 1x4 / 4x1
    std::vector<int4> rects(std::max(d->K, 1), make_int4(0, 0, 0, 0));
    for (int k = 0; k < d->K; k++) {
        const int32_t *r = &d->patch_rects[4 * k];
        if (r[2] <= 0 || r[3] <= 0) throw Error{SC_ERR_MODEL, "empty template patch"};
        const bool wide = r[2] >= r[3];
        const int ratio = wide ? r[2] / r[3] : r[3] / r[2];
        if (ratio != 1 && ratio != 4)  // the kernels' cell grids: 2x2, 1x4, 4x1
            throw Error{SC_ERR_MODEL, "template patch is not 2x2, 1x4 or 4x1 cells"};
        rects[k] = make_int4(r[0], r[1], wide ? r[3] : r[2], ratio == 1 ? 0 : (wide ? 2 : 1));
    }
    d->chunk_min = d->opt.chunk_min > 0 ? d->opt.chunk_min : 1 << 30;  // SC_OPT_CHUNK_MIN
    d->lazy = !d->opt.full_grid && !d->miner;  // FillNegSamples evaluates every window
    d->d_w.ensure(w.size());
    d->d_bias.ensure(bias.size());
    d->d_theta.ensure(theta.size());
    d->d_stage_off.ensure(off.size());
    HIPCHK(hipMemcpy(d->d_w.p, w.data(), w.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d->d_bias.p, bias.data(), bias.size() * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d->d_theta.p, theta.data(), theta.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d->d_stage_off.p, off.data(), off.size() * 4, hipMemcpyHostToDevice));
    d->d_order.ensure(order.size());
    HIPCHK(hipMemcpy(d->d_order.p, order.data(), order.size() * 2, hipMemcpyHostToDevice));
    d->d_rects.ensure(rects.size());
    HIPCHK(hipMemcpy(d->d_rects.p, rects.data(), rects.size() * sizeof(int4), hipMemcpyHostToDevice));
}

void check_params(const sc_scan_params &p) {
    if (p.base_len < 1 || p.tmpl_w < 2 || p.tmpl_h < 2 || p.aspect_h < 1 ||
        !(p.scale_factor > 1.0) || p.step < 0)
        throw Error{SC_ERR_INVALID, "invalid scan parameters"};
}

sc_detector *make_detector(const sc::Cascade &c, const sc_scan_params *p, int device,
                           bool miner = false) {
    // host-side validation first: a bad model / parameter set is reported as
    // such even on a machine without a GPU
    sc_scan_params prm;
    if (p) prm = *p;
    else sc_scan_params_default(&prm);
    check_params(prm);
    if (!(miner && c.stages.empty()))
        sc::validate_for_detect(c, (int)sc::extract_patches(prm.tmpl_w, prm.tmpl_h).size() / 4);
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev)
        throw Error{SC_ERR_DEVICE, "device " + std::to_string(device) + " not present (" +
                                       std::to_string(ndev) + " visible)"};
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        throw Error{SC_ERR_DEVICE, std::string("kernels are built for gfx950, device is ") +
                                       prop.gcnArchName};
    HIPCHK(hipSetDevice(device));
    auto *d = new sc_detector();
    try {
        d->device = device;
        d->prm = prm;
        d->casc = c;
        d->miner = miner;
        if (miner) d->all_rects = sc::extract_patches(prm.tmpl_w, prm.tmpl_h);
        HIPCHK(hipDeviceGetAttribute(&d->cus, hipDeviceAttributeMultiprocessorCount, device));
        HIPCHK(hipStreamCreateWithFlags(&d->own_stream, hipStreamNonBlocking));
        d->stream = d->own_stream;
        upload_model(d);
    } catch (...) {
        delete d;
        throw;
    }
    return d;
}

void ensure_buffers(sc_detector *d, int n) {
    const Geometry &g = d->geo;
    d->d_table.ensure((size_t)g.tg.frame4 * n);
    d->d_carry.ensure((size_t)n * g.H * ((g.W + sc::kStrip - 1) / sc::kStrip) * 8);
    d->d_counters.ensure((size_t)n + 1);
    d->d_visited.ensure(std::max<size_t>(g.rows.size() * n, 1));
    d->d_queues.ensure(sc::kQueueWords);
    d->d_st_p.ensure(std::max<size_t>((size_t)g.grid * n, 1));
    d->d_st_s.ensure(std::max<size_t>((size_t)g.grid * n, 1));
    if (d->debug) d->d_dbg_v.ensure(std::max<size_t>((size_t)g.grid * n, 1));
}

sc::LaunchCfg launch_cfg(const sc_detector *d) {
    return sc::LaunchCfg{d->cus, d->opt.lds_weights, d->opt.wgs_per_cu, d->opt.chain_waves};
}

void timed_begin(sc_detector *d, hipEvent_t *a) {
    if (!d->timing) return;
    *a = d->ev();
    HIPCHK(hipEventRecord(*a, d->stream));
}
void timed_end(sc_detector *d, int kind, hipEvent_t a) {
    if (!d->timing) return;
    hipEvent_t b = d->ev();
    HIPCHK(hipEventRecord(b, d->stream));
    d->pending.push_back({kind, a, b});
}

// rowscan -> colscan -> windows on the detector's stream.
void enqueue(sc_detector *d, const uint8_t *d_frames, int n, int W, int H, int stride,
             sc_det_record *d_out, int capacity, int *d_counts) {
    build_geometry(d, W, H);
    ensure_buffers(d, n);
    const Geometry &g = d->geo;
    // chain kernel launches: chunks of frames whose tables span < 4 GiB (32-bit
    // byte offsets); rows cut into 8 segments (one per XCD), or 4 for a
    // one-frame launch, whose time the segment hand-off chain's fill and
    // drain dominate (0.73 vs 0.83 ms per 1080p frame; 8 win from 2 frames
    // on) and for a one-frame grid shard of 8 or more
    // ranks, whose few rows make the segment-0 evaluation the serial floor
    // (C2 W = 8 chain 0.239 vs 0.253 ms, profiles/r6/o)
    int chunk = (int)std::max<long long>(1, (1ll << 28) / g.tg.frame4);
    if (d->opt.chain_chunk > 0) chunk = std::min(chunk, d->opt.chain_chunk);  // SC_OPT_CHAIN_CHUNK
    auto segs_for = [&](int frames) {  // SC_OPT_CHAIN_SEGS overrides
        return d->opt.chain_segs ? d->opt.chain_segs : (frames == 1 && d->shard_world < 8 ? sc::kXcds / 2 : sc::kXcds);
    };
    auto seg_max_for = [&](int s) { return (g.nx_max + s - 1) / s; };
    const int last = n % chunk ? n % chunk : std::min(chunk, n);
    const int smin = std::min(segs_for(std::min(chunk, n)), segs_for(last));  // widest segment of the call
    const int seg_max = seg_max_for(smin);
    const bool lazy = d->lazy && sc::chain_lds_bytes(d->K, seg_max, g.n_levels) <= 160 * 1024;
    const size_t n_rows = g.rows.size();
    const bool chain = n_rows > 0 && lazy && !d->miner;
    // hand-off words of a chain launch: [rows x frames x kXcds] entries, the
    // watchdog-fired flag, the fused integral's walk counter and per-frame
    // walk counts (WalkArgs::int_ctl), the speculative-round count; sized
    // for the largest launch
    auto entry_words = [&](int frames) { return (long long)n_rows * frames * sc::kXcds + 3 + frames; };
    if (chain) {
        d->d_entry.ensure((size_t)entry_words(std::min(chunk, n)));
        if (!d->d_err.p) {
            if (!d->h_err) {
                HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&d->h_err), sizeof(int),
                                     hipHostMallocMapped | hipHostMallocCoherent));
                *d->h_err = 0;
            }
            d->d_err.ensure(1);
            HIPCHK(hipMemsetAsync(d->d_err.p, 0, sizeof(int), d->stream));
        }
    }
    // Fused integral (SC_OPT_INTEGRAL_FUSE): the first `pre` frames of every
    // launch are integrated by their own kernels, the column walks of the
    // others run inside the chain kernel as a second task type, overlapping
    // the gathers.  Auto: from 4 frames per launch,
    // where colstrip would be the integral's column pass.  `pre` is 2 for
    // tables that fit the Infinity Cache (a frame's 60 walks inside the chain
    // kernel take longer than the chain takes over frame 0: 13.63 vs 13.74 ms
    // at C2, profiles/r3/g10) and 1 for larger ones (a 4K frame: C4 25.55 vs
    // 25.77 ms per step unfused, 25.69 with 2, 25.82 with 3, profiles/r4/c4fuse;
    // round 3's fused 4K kernel was slower than unfused, profiles/r3/g21).
    const bool big_table = g.tg.frame4 * 16 > (128ll << 20);
    const int pre = d->opt.integral_pre > 0 ? d->opt.integral_pre : big_table ? 1 : 2;
    const int fuse_from = d->opt.integral_fuse == 2 ? 2 : 4;
    const bool fuse = chain && d->opt.integral_fuse != 1 && std::min(chunk, n) >= fuse_from &&
                      std::min(chunk, n) > pre;

    sc::RowScanArgs ra{d_frames, (long long)H * stride, stride, d->d_table.p, g.tg, d->d_carry.p, {}, {}};
    // zeroed by rowcarry (stream order: before every kernel that uses them):
    // the output counters, the task queues, the visited counts and the first
    // chunk's hand-off words
    ra.zero[0] = d_counts;
    ra.zero_n[0] = n + 1;
    if (n_rows > 0) {
        ra.zero[1] = d->d_queues.p;
        ra.zero_n[1] = sc::kQueueWords;
    }
    if (chain) {
        ra.zero[2] = reinterpret_cast<int *>(d->d_visited.p);
        ra.zero_n[2] = (long long)n_rows * n;
        ra.zero[3] = d->d_entry.p;
        ra.zero_n[3] = entry_words(std::min(chunk, n));
    }
    // the frames whose column pass is two-pass (the first launch's `pre`
    // frames when fused, else all of a 1-3-frame call): rowcarry4 writes
    // their R rows too, so rowfull does not run for them
    const bool two_pass_all = d->opt.integral_passes ? d->opt.integral_passes == 2 : n <= 3;
    const bool two_pass_pre = d->opt.integral_passes ? d->opt.integral_passes == 2 : pre <= 3;
    ra.rfull_n = fuse ? (two_pass_pre ? std::min(pre, n) : 0) : (two_pass_all ? n : 0);
    if (n == 1 && two_pass_all && sc::colseg_segments() > 1) {
        d->d_colblk.ensure((size_t)(g.H + sc::colblk_rows() - 1) / sc::colblk_rows() * g.tg.rowp * 4);
        ra.colblk = d->d_colblk.p;
    }
    d->spec_word = -1;  // (set by a chain launch below: SC_INFO_SPEC_ROUNDS reads 0 otherwise)
    hipEvent_t e0 = nullptr;
    timed_begin(d, &e0);
    bool colblk_done = false;
    const bool have_r = sc::launch_rowscan(ra, n, d->stream, &colblk_done);
    HIPCHK(hipGetLastError());
    timed_end(d, SC_KERNEL_ROWSCAN, e0);

    timed_begin(d, &e0);
    // colstrip's 60 waves per frame walk every row: for up to three frames the
    // row-parallel two-pass form is shorter (SC_OPT_INTEGRAL_PASSES overrides)
    const long long carry_frame = (long long)H * ((W + sc::kStrip - 1) / sc::kStrip) * 8;  // u32 per frame
#if defined(SC_WALK_STORE) && SC_WALK_STORE == 0  // timing ablation: walks store nothing, tables built here
    if (false) {
#else
    if (fuse) {  // only the first `pre` frames of each launch here
#endif
        for (int f0 = 0; f0 < n; f0 += chunk) {
            sc::RowScanArgs rc = ra;
            rc.frames = d_frames + (long long)f0 * H * stride;
            rc.table = d->d_table.p + (size_t)f0 * g.tg.frame4;
            rc.carry = d->d_carry.p + f0 * carry_frame;
            sc::launch_colscan(rc, std::min(pre, n - f0), two_pass_pre, d->stream, have_r && f0 == 0);
        }
    } else {
        sc::launch_colscan(ra, n, two_pass_all, d->stream, have_r, colblk_done);
    }
    d->last_colpass = (fuse ? two_pass_pre : two_pass_all) ? (ra.colblk ? 3 : 1) : 2;
    HIPCHK(hipGetLastError());
    timed_end(d, SC_KERNEL_COLSCAN, e0);

    d->last_frames = n;
    d->last_fused = 0;
    if (g.rows.empty()) return;

    sc::CascadeArgs ca{};
    ca.table = d->d_table.p;
    ca.g = g.tg;
    ca.tasks = d->d_tasks.p;
    ca.proj = d->d_proj.p;
    ca.rects = d->d_rects.p;
    ca.w = reinterpret_cast<const float4 *>(d->d_w.p);
    ca.bias = d->d_bias.p;
    ca.theta = d->d_theta.p;
    ca.stage_off = d->d_stage_off.p;
    ca.order = d->d_order.p;
    ca.chunk_min = d->chunk_min;
    ca.K = d->K;
    ca.n_stages = d->S;
    ca.n_bands = g.n_bands;
    ca.band_rows = g.band_rows;
    ca.n_frames = n;
    ca.n_sub = g.n_sub;
    ca.strip_max = g.strip_max;
    ca.grid_per_frame = g.grid;
    ca.queues = d->d_queues.p;
    ca.st_p = d->d_st_p.p;
    ca.st_s = d->d_st_s.p;
    if (!lazy) {
        timed_begin(d, &e0);
        sc::launch_cascade(ca, launch_cfg(d), d->stream);
        HIPCHK(hipGetLastError());
        timed_end(d, SC_KERNEL_WINDOWS, e0);
    }
    if (d->miner) return;  // FillNegSamples visits every window: no walk

    sc::WalkArgs wk{};
    wk.rows = d->d_rows.p;
    wk.levels = d->d_levels.p;
    wk.n_rows = (int)g.rows.size();
    wk.n_levels = g.n_levels;
    wk.n_stages = d->S;
    wk.step = g.step;
    wk.stride_score = d->prm.stride_score;
    wk.grid_per_frame = g.grid;
    wk.st_p = d->d_st_p.p;
    wk.st_s = d->d_st_s.p;
    wk.out = d_out;
    wk.capacity = capacity;
    wk.counters = d_counts;
    wk.row_visited = d->d_visited.p;
    wk.dbg_v = d->debug ? d->d_dbg_v.p : nullptr;
    wk.row_max = seg_max;
    if (lazy) {  // the walk drives the cascade: one chain kernel per chunk of frames
        if (d->debug) {  // dumps: unevaluated windows read -2, unvisited 0
            HIPCHK(hipMemsetAsync(d->d_st_p.p, 0xFE, (size_t)g.grid * n, d->stream));
            HIPCHK(hipMemsetAsync(d->d_st_s.p, 0, sizeof(float) * (size_t)g.grid * n, d->stream));
            HIPCHK(hipMemsetAsync(d->d_dbg_v.p, 0, (size_t)g.grid * n, d->stream));
        }
        timed_begin(d, &e0);
        for (int f0 = 0; f0 < n; f0 += chunk) {
            const int nc = std::min(chunk, n - f0);
            sc::CascadeArgs cc = ca;
            sc::WalkArgs wc = wk;
            cc.table = d->d_table.p + (size_t)f0 * g.tg.frame4;
            cc.n_frames = nc;
            cc.st_p = d->debug ? d->d_st_p.p + (size_t)f0 * g.grid : nullptr;
            cc.st_s = d->debug ? d->d_st_s.p + (size_t)f0 * g.grid : nullptr;
            wc.dbg_v = d->debug ? d->d_dbg_v.p + (size_t)f0 * g.grid : nullptr;
            wc.row_visited = d->d_visited.p + (size_t)f0 * n_rows;
            if (nc == 1) wc.rows = d->d_rows.p + n_rows;  // the one-frame order
            wc.entry = d->d_entry.p;
            d->err_word = (long long)(n_rows * std::min(chunk, n) * sc::kXcds);
            wc.fired = d->d_entry.p + d->err_word;  // per launch: zeroed with the entries
            wc.err = d->d_err.p;                    // sticky over launches and calls
            HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void **>(&wc.err_host), d->h_err, 0));
            wc.int_ctl = wc.fired + 1;
            wc.spec = wc.int_ctl + 1 + std::min(chunk, n);
            d->spec_word = wc.spec - d->d_entry.p;
            d->chain_launched = true;
            if (fuse && nc > pre) {
                wc.frames = d_frames + (long long)f0 * H * stride;
                wc.frame_bytes = (long long)H * stride;
                wc.stride = stride;
                wc.carry = d->d_carry.p + f0 * carry_frame;
                wc.int_f0 = pre;
                // a wave per (64-column strip, channel half); interleaved cells:
                // per 32-column strip, both halves (sc_windows.hip fused_walk)
                wc.walks_per_frame = g.tg.cs == 2 ? (W + sc::kStrip - 1) / sc::kStrip
                                                  : 2 * ((W + 2 * sc::kStrip - 1) / (2 * sc::kStrip));
                wc.int_walks = (nc - pre) * wc.walks_per_frame;
                d->last_fused += nc - pre;
            }
            wc.frame0 = f0;
            wc.drop_task1 = d->opt.drop_handoff + 1;  // SC_OPT_TEST_DROP_HANDOFF (0: none)
            wc.drop_walk1 = d->opt.drop_walk + 1;     // SC_OPT_TEST_DROP_WALK (0: none)
            // task slots per wave (SC_OPT_CHAIN_SLOTS): a one-frame launch is
            // latency-bound by its rows' hand-off chains, and one task per wave
            // runs each task at the wave's full speed (one frame: chain 0.532
            // vs 0.574 ms with 2); a batch wants two tasks sharing each round
            // (C2 14.12 vs 13.53 ms with 1) (profiles/r6/p)
            wc.slots = d->opt.chain_slots ? d->opt.chain_slots : (nc == 1 ? 1 : 2);
            // dequeue sub-queues (SC_OPT_CHAIN_SUBQ): for a one-frame launch 4
            // with one task per wave (chain 0.5249 vs 0.5324 ms with 8, 0.5310
            // with 1, profiles/r6/r), 8 with two (0.573 vs 0.582 ms with 4,
            // profiles/r5/l/split); 1 for batches (C2 with 4: 17.0 vs 13.6 ms)
            wc.subq = d->opt.chain_subq ? d->opt.chain_subq : (nc == 1 ? (wc.slots == 1 ? 4 : 8) : 1);
            // speculative rounds per waiting task (one-frame launches): 1 for
            // a whole frame; a grid shard's launch has a fraction of the rows
            // on the same waves, whose idle rounds then evaluate whole
            // segments ahead of their entries (profiles/r6)
            wc.spec_max = d->opt.chain_spec ? d->opt.chain_spec : (d->shard_world > 1 ? 64 : 1);
#if defined(SC_WIDECAP) && SC_WIDECAP
            if (nc > 1 && wc.subq < sc::kMaxSubQ) {  // (the wide list's counter is sub-queue word kMaxSubQ - 1)
                wc.n_wide = g.n_wide;
                wc.wide_cap = SC_WIDECAP;
            }
#endif
            d->last_subq = wc.subq;
            wc.nseg = segs_for(nc);
            d->last_nseg = wc.nseg;
            wc.seg_shift = wc.nseg == 8 ? 0 : wc.nseg == 4 ? 1 : wc.nseg == 2 ? 2 : 3;
            wc.row_max = seg_max_for(wc.nseg);  // (<= seg_max: the LDS check above)
            if (d->opt.profile) {  // SC_OPT_PROFILE (SC_PROF_CHAIN builds): cumulative phase cycles
                if (!d->d_prof.p) {  // 16 phase totals, per wave (start, exit), per task (dequeue, start, finish)
                    d->d_prof.ensure(16 + 2 * 8192 + 3 * 65536);
                    HIPCHK(hipMemsetAsync(d->d_prof.p, 0, (16 + 2 * 8192 + 3 * 65536) * sizeof(unsigned long long),
                                          d->stream));
                }
                wc.prof = d->d_prof.p;
            }
            if (f0 > 0) {  // (the first chunk's were cleared by rowcarry)
                HIPCHK(hipMemsetAsync(d->d_entry.p, 0, sizeof(int) * n_rows * nc * sc::kXcds, d->stream));
                HIPCHK(hipMemsetAsync(wc.fired, 0, sizeof(int) * (size_t)(3 + std::min(chunk, n)), d->stream));  // + int_ctl, spec
                HIPCHK(hipMemsetAsync(d->d_queues.p, 0, sizeof(int) * sc::kQueueWords, d->stream));
            }
            sc::launch_chain(cc, wc, launch_cfg(d), d->stream, &d->last_waves);
            HIPCHK(hipGetLastError());
        }
        timed_end(d, SC_KERNEL_WINDOWS, e0);
        return;
    }
    timed_begin(d, &e0);
    sc::launch_walk(wk, n, d->stream);
    HIPCHK(hipGetLastError());
    timed_end(d, SC_KERNEL_WALK, e0);
}

// The chain kernel's hand-off watchdog (reads after the stream has drained):
// every launch since the last check, pipelined steps included.
void check_chain(sc_detector *d) {
    if (!d->lazy || !d->chain_launched || !d->d_err.p) return;
    d->chain_launched = false;
    int err = 0;
    // the common case costs no device copy: the kernel raised the host flag
    // with its first count (the stream has drained, so the flag is final)
    if (*static_cast<volatile int *>(d->h_err)) {
        HIPCHK(hipMemcpy(&err, d->d_err.p, sizeof(int), hipMemcpyDeviceToHost));
        // (stream-ordered: the detector's stream is non-blocking, so a null-stream
        // clear would not be ordered before the next call's kernels)
        HIPCHK(hipMemsetAsync(d->d_err.p, 0, sizeof(int), d->stream));
        *d->h_err = 0;
        if (!err) err = 1;
    }
    if (err) {
        throw Error{SC_ERR_DEVICE, "chain kernel: " + std::to_string(err) + " segment hand-off or table wait(s) timed out"};
    }
    if (d->d_prof.p) {
        unsigned long long pc[16];
        HIPCHK(hipMemcpy(pc, d->d_prof.p, sizeof(pc), hipMemcpyDeviceToHost));
        std::fprintf(stderr, "SC_PROF_CHAIN idle %llu setup %llu eval %llu merge %llu rounds %llu slots %llu "
                     "deq %llu poll %llu iters %llu lanes %llu prefilter %llu thin32 %llu stages %llu "
                     "surv %llu need %llu pass %llu\n", pc[0], pc[1], pc[2], pc[3], pc[4], pc[5], pc[6],
                     pc[7], pc[8], pc[9], pc[10], pc[11], pc[12], pc[13], pc[14], pc[15]);
        // the last launch's wave exits, as fractions of its span (first start -> last exit)
        std::vector<unsigned long long> tw(2 * 8192);
        HIPCHK(hipMemcpy(tw.data(), d->d_prof.p + 16, tw.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        std::vector<double> ex;
        unsigned long long t0 = ~0ull, t1 = 0;
        for (int i = 0; i < 8192; i++)
            if (tw[2 * i]) {
                t0 = std::min(t0, tw[2 * i]);
                t1 = std::max(t1, tw[2 * i + 1]);
            }
        for (int i = 0; i < 8192; i++)
            if (tw[2 * i] && t1 > t0) ex.push_back((double)(tw[2 * i + 1] - t0) / (double)(t1 - t0));
        std::sort(ex.begin(), ex.end());
        if (!ex.empty()) {
            double mean = 0;
            for (double v : ex) mean += v;
            auto q = [&](double f) { return ex[std::min(ex.size() - 1, (size_t)(f * ex.size()))]; };
            std::fprintf(stderr, "SC_PROF_WAVES waves %zu span %llu exit p10 %.3f p50 %.3f p90 %.3f p99 %.3f mean %.3f\n",
                         ex.size(), t1 - t0, q(0.1), q(0.5), q(0.9), q(0.99), mean / ex.size());
            // task trace of the last launch, per segment: mean wait for the entry
            // (dequeue -> start) and evaluation (start -> finish), in launch-span
            // fractions; and the share of tasks finishing in the last 10 / 25 %
            const int nsg = (int)d->last_nseg;
            const size_t ntk = std::min<size_t>(65536, (size_t)d->last_frames * d->geo.rows.size() * nsg);
            std::vector<unsigned long long> tr(3 * ntk);
            HIPCHK(hipMemcpy(tr.data(), d->d_prof.p + 16 + 2 * 8192, tr.size() * sizeof(unsigned long long),
                             hipMemcpyDeviceToHost));
            const double span = (double)(t1 - t0);
            for (int sg = 0; sg < nsg; sg++) {
                double wsum = 0, esum = 0, dsum = 0;
                size_t n = 0, late10 = 0, late25 = 0;
                for (size_t i = sg; i < ntk; i += nsg) {
                    const unsigned long long a = tr[3 * i], b = tr[3 * i + 1], c = tr[3 * i + 2];
                    if (!a || !b || !c || a < t0 || c < b || b < a) continue;
                    n++;
                    dsum += (double)(a - t0) / span;
                    wsum += (double)(b - a) / span;
                    esum += (double)(c - b) / span;
                    late10 += (double)(c - t0) / span > 0.9;
                    late25 += (double)(c - t0) / span > 0.75;
                }
                if (n)
                    std::fprintf(stderr, "SC_PROF_TASKS seg %d tasks %zu dequeue %.3f wait %.4f eval %.4f finish>0.75 %zu >0.9 %zu\n",
                                 sg, n, dsum / n, wsum / n, esum / n, late25, late10);
            }
        }
    }
}

// A caller's device pointer must be device memory of this detector's GPU: a
// host pointer or another GPU's memory would fault in a kernel instead of
// returning SC_ERR_INVALID.
void check_device_ptr(const sc_detector *d, const void *p, const char *what) {
    if (!p) return;
    hipPointerAttribute_t at{};
    const hipError_t e = hipPointerGetAttributes(&at, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();  // an unregistered host pointer: clear the error
        throw Error{SC_ERR_INVALID, std::string(what) + " is not device memory"};
    }
    if (at.type != hipMemoryTypeDevice && at.type != hipMemoryTypeManaged)
        throw Error{SC_ERR_INVALID, std::string(what) + " is not device memory"};
    if (at.device != d->device)
        throw Error{SC_ERR_INVALID, std::string(what) + " is on device " + std::to_string(at.device) +
                                        ", the detector on device " + std::to_string(d->device)};
}

bool rec_less(const sc_det_record &a, const sc_det_record &b) {
    if (a.frame != b.frame) return a.frame < b.frame;
    if (a.level != b.level) return a.level < b.level;
    if (a.y != b.y) return a.y < b.y;
    return a.x < b.x;
}

// Synchronous device-frame detection with host output.
int detect_device_sync(sc_detector *d, const uint8_t *d_frames, int n, int W, int H, int stride,
                       sc_window *out, int capacity, int *n_out) {
    if (d->miner) throw Error{SC_ERR_INVALID, "a miner scans with sc_mine, not sc_detect*"};
    if (n <= 0 || !d_frames || !n_out || (capacity > 0 && !out) || capacity < 0)
        throw Error{SC_ERR_INVALID, "bad arguments"};
    if (stride < W) throw Error{SC_ERR_INVALID, "stride smaller than width"};
    size_t cap_dev = std::max<size_t>(d->d_out.n, 4096);
    std::vector<int> counts(n + 1);
    for (int attempt = 0; attempt < 2; attempt++) {
        d->d_out.ensure(cap_dev);
        d->d_counters.ensure((size_t)n + 1);
        enqueue(d, d_frames, n, W, H, stride, d->d_out.p, (int)cap_dev, d->d_counters.p);
        HIPCHK(hipMemcpyAsync(counts.data(), d->d_counters.p, sizeof(int) * (n + 1),
                              hipMemcpyDeviceToHost, d->stream));
        HIPCHK(hipStreamSynchronize(d->stream));
        if ((size_t)counts[0] <= cap_dev) break;
        cap_dev = (size_t)counts[0];
    }
    check_chain(d);
    const int total = counts[0];
    std::vector<sc_det_record> recs(total);
    if (total > 0)
        HIPCHK(hipMemcpy(recs.data(), d->d_out.p, sizeof(sc_det_record) * total, hipMemcpyDeviceToHost));
    std::sort(recs.begin(), recs.end(), rec_less);
    for (int f = 0; f < n; f++) n_out[f] = counts[1 + f];
    const int m = std::min(total, capacity);
    for (int i = 0; i < m; i++) {
        const sc_det_record &r = recs[i];
        out[i] = sc_window{r.level, r.x, r.y, r.w, r.h, r.stage_reached, r.score};
    }
    if (total > capacity) {
        g_err = "output capacity " + std::to_string(capacity) + " < " + std::to_string(total);
        return SC_ERR_CAPACITY;
    }
    return SC_OK;
}

// FillNegSamples' scan of n device frames of one size (frame f at
// d_frames + f*H*stride): the shared integral + cascade kernels on the
// stride-10 grid, then candidate selection -- block counts, a device scan,
// the scatter -- and descriptors, with one host synchronisation at the end.
// Candidates in (frame, level, y, x) order; the first `capacity` are kept;
// n_out[f] = frame f's candidates (all of them).
int mine_sync(sc_detector *d, const uint8_t *d_frames, int n, int W, int H, int stride, sc_window *wins,
              float *feat, int capacity, int *n_out, bool feat_device = false) {
    if (!d->miner) throw Error{SC_ERR_INVALID, "not a miner (sc_miner_create)"};
    if (!d_frames || !n_out || n <= 0 || capacity < 0 || (capacity > 0 && !wins))
        throw Error{SC_ERR_INVALID, "bad arguments"};
    if (stride < W) throw Error{SC_ERR_INVALID, "stride smaller than width"};
    d->d_counters.ensure((size_t)n + 1);
    enqueue(d, d_frames, n, W, H, stride, nullptr, 0, d->d_counters.p);
    const Geometry &g = d->geo;
    for (int f = 0; f < n; f++) n_out[f] = 0;
    if (g.grid == 0) {
        HIPCHK(hipStreamSynchronize(d->stream));
        return SC_OK;
    }
    const int bpf = (int)((g.grid + sc::kMineBlock - 1) / sc::kMineBlock);
    if ((long long)bpf * n > INT32_MAX / 2) throw Error{SC_ERR_INVALID, "batch too large"};
    const int nb = bpf * n;
    d->d_mine_cnt.ensure(nb);
    d->d_mine_off.ensure(nb);
    d->d_mine_fc.ensure((size_t)n + 1);
    d->d_mine_win.ensure(std::max(capacity, 1));
    sc::MineArgs ma{};
    ma.st_p = d->d_st_p.p;
    ma.st_s = d->d_st_s.p;
    ma.grid = g.grid;
    ma.n_frames = n;
    ma.bpf = bpf;
    ma.n_stages = d->S;
    ma.step = g.step;
    ma.n_levels = g.n_levels;
    ma.levels = d->d_levels.p;
    ma.block_count = d->d_mine_cnt.p;
    ma.block_offset = d->d_mine_off.p;
    ma.frame_count = d->d_mine_fc.p;
    ma.out = d->d_mine_win.p;
    ma.capacity = capacity;
    sc::launch_mine_count(ma, d->stream);
    HIPCHK(hipGetLastError());
    sc::launch_mine_scan(ma, d->stream);
    HIPCHK(hipGetLastError());
    sc::launch_mine_scatter(ma, d->stream);
    HIPCHK(hipGetLastError());
    // descriptors of every kept window, kept = min(total, capacity).  Host
    // output: read the scan's total first (the call ends in a host sync
    // anyway) and size the descriptor buffer and launch to the kept windows
    // -- a trainer-style capacity (FillNegSamples' n_total) far above the
    // candidates found then costs nothing.  Device output: kept is only known
    // on the device, so the feature kernel covers `capacity` windows and its
    // threads past the device-side total exit (no host round trip).
    const int P = (int)d->all_rects.size() / 4;
    std::vector<int> fc((size_t)n + 1);
    auto read_counts = [&] {
        HIPCHK(hipMemcpyAsync(fc.data(), d->d_mine_fc.p, sizeof(int) * (n + 1), hipMemcpyDeviceToHost,
                              d->stream));
        HIPCHK(hipStreamSynchronize(d->stream));
    };
    long long total = -1;
    auto launch_desc = [&](int n_win, float *out) {
        sc::FeatureArgs fa{};
        fa.table = d->d_table.p;
        fa.g = g.tg;
        fa.windows = d->d_mine_win.p;
        fa.n_windows = n_win;
        fa.n_valid = d->d_mine_fc.p;
        fa.n_patches = P;
        fa.proj_all = d->d_proj_all.p;
        fa.out = out;
        sc::launch_features(fa, d->stream);
        HIPCHK(hipGetLastError());
    };
    if (feat && capacity > 0 && feat_device) {
        launch_desc(capacity, feat);
    } else if (feat && capacity > 0) {
        read_counts();
        total = 0;
        for (int f = 0; f < n; f++) total += fc[1 + f];
        const int kept0 = (int)std::min<long long>(total, capacity);
        if (kept0 > 0) {
            d->d_feat.ensure((size_t)kept0 * P * 32);
            launch_desc(kept0, d->d_feat.p);
        }
    }
    if (total < 0) {
        read_counts();
        total = 0;
        for (int f = 0; f < n; f++) total += fc[1 + f];
    }
    const int kept = (int)std::min<long long>(total, capacity);
    HIPCHK(hipStreamSynchronize(d->stream));  // the descriptor kernel (the copies below are synchronous)
    if (feat && kept > 0 && !feat_device)
        HIPCHK(hipMemcpy(feat, d->d_feat.p, sizeof(float) * (size_t)kept * P * 32, hipMemcpyDeviceToHost));
    std::vector<sc::MineWindow> mw(kept);
    if (kept > 0)
        HIPCHK(hipMemcpy(mw.data(), d->d_mine_win.p, sizeof(sc::MineWindow) * kept, hipMemcpyDeviceToHost));
    for (int i = 0; i < kept; i++)
        wins[i] = sc_window{mw[i].level, mw[i].x, mw[i].y, mw[i].l, mw[i].l, d->S, (double)mw[i].score};
    for (int f = 0; f < n; f++) n_out[f] = fc[1 + f];
    if (total > capacity) {
        g_err = "capacity " + std::to_string(capacity) + " < " + std::to_string(total) +
                " candidates (the first " + std::to_string(capacity) + " were returned)";
        return SC_ERR_CAPACITY;
    }
    return SC_OK;
}

template <class F>
int guarded(F &&f) {
    try {
        return f();
    } catch (const Error &e) {
        return fail(e.code, e.msg);
    } catch (const std::bad_alloc &) {
        return fail(SC_ERR_NOMEM, "out of host memory");
    } catch (const std::exception &e) {
        return fail(SC_ERR_INVALID, e.what());
    }
}

}  // namespace

// =========================================================================
// C ABI
// =========================================================================
// Host frames (any row stride) -> d->d_frames, w x h per frame at a row
// pitch rounded up to 4 bytes (rowcarry4's dword loads; the pad bytes are
// never part of a result), returned: each frame is copied into the pinned
// staging buffer and its DMA queued at once, so the host copy of frame f+1
// overlaps the transfer of frame f.  The caller's stream synchronisation at
// the end of the call covers the staging buffer's reuse by the next call.
static int upload_frames(sc_detector *d, const uint8_t *const *frames, int n, int w, int h, int stride) {
    const int pitch = (w + 3) & ~3;
    const size_t fb = (size_t)pitch * h;
    HIPCHK(hipStreamSynchronize(d->stream));  // no earlier transfer still reads the staging buffer
    d->d_frames.ensure(fb * n);
    d->h_stage.ensure(fb * n);
    for (int f = 0; f < n; f++) {
        if (!frames[f]) throw Error{SC_ERR_INVALID, "null frame pointer"};
        uint8_t *dst = d->h_stage.p + fb * f;
        if (stride == w && w == pitch) {  // (a caller's last row may end at w: copy no pad)
            std::memcpy(dst, frames[f], fb);
        } else {
            for (int y = 0; y < h; y++) {
                std::memcpy(dst + (size_t)y * pitch, frames[f] + (size_t)y * stride, w);
                if (pitch > w) std::memset(dst + (size_t)y * pitch + w, 0, pitch - w);
            }
        }
        HIPCHK(hipMemcpyAsync(d->d_frames.p + fb * f, dst, fb, hipMemcpyHostToDevice, d->stream));
    }
    return pitch;
}

extern "C" {

void sc_scan_params_default(sc_scan_params *p) {
    if (!p) return;
    p->base_len = 70;
    p->scale_factor = 1.1;
    p->n_levels = -1;
    p->step = 0;
    p->prefilter_k = 6.0f;
    p->stride_score = 0.5;
    p->tmpl_w = 40;
    p->tmpl_h = 40;
    p->aspect_h = 1;
}

const char *sc_last_error(void) { return g_err.c_str(); }
const char *sc_version(void) { return "surfcascade-mi355x 0.1 (gfx950)"; }

int sc_model_parse(const char *text, size_t len, sc_model **out) {
    return guarded([&] {
        if (!text || !out) throw Error{SC_ERR_INVALID, "null argument"};
        sc::CfgValue root = sc::cfg_parse(std::string(text, len));
        auto *m = new sc_model{sc::cascade_from_cfg(root)};
        *out = m;
        return SC_OK;
    });
}

int sc_model_load(const char *path, sc_model **out) {
    return guarded([&] {
        if (!path || !out) throw Error{SC_ERR_INVALID, "null argument"};
        std::ifstream f(path, std::ios::binary);
        if (!f) throw Error{SC_ERR_IO, std::string("I/O error while reading file: ") + path};
        std::stringstream ss;
        ss << f.rdbuf();
        std::string t = ss.str();
        sc::CfgValue root = sc::cfg_parse(t);
        *out = new sc_model{sc::cascade_from_cfg(root)};
        return SC_OK;
    });
}

int sc_model_save(const sc_model *m, const char *path) {
    return guarded([&] {
        if (!m || !path) throw Error{SC_ERR_INVALID, "null argument"};
        std::string t = sc::cfg_write(sc::cascade_to_cfg(m->c));
        std::ofstream f(path, std::ios::binary);
        if (!f) throw Error{SC_ERR_IO, std::string("I/O error while writing file: ") + path};
        f << t;
        if (!f) throw Error{SC_ERR_IO, std::string("I/O error while writing file: ") + path};
        return SC_OK;
    });
}

int sc_model_num_stages(const sc_model *m) { return m ? (int)m->c.stages.size() : SC_ERR_INVALID; }

int sc_model_stage(const sc_model *m, int s, float *theta, int *n_weak) {
    if (!m || s < 0 || s >= (int)m->c.stages.size()) return fail(SC_ERR_INVALID, "bad stage index");
    if (theta) *theta = m->c.stages[s].theta;
    if (n_weak) *n_weak = (int)m->c.stages[s].weak.size();
    return SC_OK;
}

int sc_model_weak(const sc_model *m, int s, int k, int *patch_index, float w33[33], double *bias) {
    if (!m || s < 0 || s >= (int)m->c.stages.size() || k < 0 ||
        k >= (int)m->c.stages[s].weak.size())
        return fail(SC_ERR_INVALID, "bad weak index");
    const sc::WeakLR &wk = m->c.stages[s].weak[k];
    if (patch_index) *patch_index = wk.patch_index;
    if (bias) *bias = wk.bias;
    if (w33)
        for (int i = 0; i < 33; i++) w33[i] = i < (int)wk.w.size() ? wk.w[i] : 0.0f;
    return SC_OK;
}

void sc_model_free(sc_model *m) { delete m; }

int sc_group_rectangles(const sc_scored_rect *in, int n, int group_threshold, double eps,
                        sc_scored_rect *out, int capacity, int *n_out) {
    return guarded([&] {
        if ((n > 0 && !in) || n < 0 || !n_out) throw Error{SC_ERR_INVALID, "null argument"};
        const std::vector<sc_scored_rect> g = sc::group_rectangles(in, n, group_threshold, eps);
        *n_out = (int)g.size();
        if (out) std::copy(g.begin(), g.begin() + std::min<size_t>(g.size(), std::max(capacity, 0)), out);
        if ((int)g.size() > capacity) throw Error{SC_ERR_CAPACITY, "output capacity too small"};
        return SC_OK;
    });
}

int sc_group_detections(const sc_det_record *rec, int n, int n_frames, int group_threshold,
                        double eps, sc_scored_rect *out, int capacity, int32_t *frame_counts,
                        int *n_out) {
    return guarded([&] {
        if ((n > 0 && !rec) || n < 0 || n_frames < 0 || !n_out || (n_frames > 0 && !frame_counts))
            throw Error{SC_ERR_INVALID, "null argument"};
        std::vector<int> idx(n);
        for (int i = 0; i < n; i++) {
            if (rec[i].frame < 0 || rec[i].frame >= n_frames)
                throw Error{SC_ERR_INVALID, "record frame index out of range"};
            idx[i] = i;
        }
        std::sort(idx.begin(), idx.end(), [&](int a, int b) {
            const sc_det_record &p = rec[a], &q = rec[b];
            if (p.frame != q.frame) return p.frame < q.frame;
            if (p.level != q.level) return p.level < q.level;
            if (p.y != q.y) return p.y < q.y;
            return p.x < q.x;
        });
        int total = 0;
        std::vector<sc_scored_rect> rects;
        for (int f = 0, i = 0; f < n_frames; f++) {
            rects.clear();
            for (; i < n && rec[idx[i]].frame == f; i++) {
                const sc_det_record &r = rec[idx[i]];
                rects.push_back(sc_scored_rect{r.x, r.y, r.w, r.h, r.score});
            }
            const std::vector<sc_scored_rect> g =
                sc::group_rectangles(rects.data(), (int)rects.size(), group_threshold, eps);
            frame_counts[f] = (int)g.size();
            for (const sc_scored_rect &r : g) {
                if (out && total < capacity) out[total] = r;
                total++;
            }
        }
        *n_out = total;
        if (total > capacity) throw Error{SC_ERR_CAPACITY, "output capacity too small"};
        return SC_OK;
    });
}

int sc_fddb_format(const char *name, const sc_scored_rect *r, int n, char *buf, size_t cap,
                   size_t *len) {
    return guarded([&] {
        if (!name || (n > 0 && !r) || n < 0 || !len) throw Error{SC_ERR_INVALID, "null argument"};
        const std::string s = sc::fddb_block(name, r, n);
        *len = s.size();
        if (!buf || cap <= s.size()) throw Error{SC_ERR_CAPACITY, "buffer too small"};
        std::memcpy(buf, s.c_str(), s.size() + 1);
        return SC_OK;
    });
}

int sc_fast_nms(const sc_scored_rect *in, int n, double overlap_th, sc_scored_rect *out,
                int capacity, int *n_out) {
    return guarded([&] {
        if ((n > 0 && !in) || n < 0 || !n_out || capacity < 0 || (capacity > 0 && !out))
            throw Error{SC_ERR_INVALID, "bad arguments"};
        const std::vector<sc_scored_rect> r = sc::fast_nms(in, n, overlap_th);
        *n_out = (int)r.size();
        std::copy(r.begin(), r.begin() + std::min<size_t>(r.size(), (size_t)capacity), out);
        if ((int)r.size() > capacity) throw Error{SC_ERR_CAPACITY, "output capacity too small"};
        return SC_OK;
    });
}

namespace {
int decode_into(const uint8_t *data, size_t len, uint8_t *out, size_t cap, int *w, int *h) {
    if (!data || !w || !h) throw Error{SC_ERR_INVALID, "null argument"};
    std::string err;
    int W = 0, H = 0;
    if (sc::jpeg_gray(data, len, nullptr, &W, &H, &err) != 0) throw Error{SC_ERR_PARSE, err};
    *w = W;
    *h = H;
    if (!out || cap < (size_t)W * H)
        throw Error{SC_ERR_CAPACITY, "gray plane needs " + std::to_string((size_t)W * H) + " bytes"};
    std::vector<uint8_t> img;
    if (sc::jpeg_gray(data, len, &img, &W, &H, &err) != 0) throw Error{SC_ERR_PARSE, err};
    std::memcpy(out, img.data(), img.size());
    return SC_OK;
}
}  // namespace

int sc_decode_jpeg_gray(const uint8_t *data, size_t len, uint8_t *out, size_t cap, int *w, int *h) {
    return guarded([&] { return decode_into(data, len, out, cap, w, h); });
}

int sc_imread_gray(const char *path, uint8_t *out, size_t cap, int *w, int *h) {
    return guarded([&] {
        if (!path) throw Error{SC_ERR_INVALID, "null path"};
        std::ifstream f(path, std::ios::binary);
        if (!f) throw Error{SC_ERR_IO, std::string("cannot open ") + path};
        std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
        return decode_into(buf.data(), buf.size(), out, cap, w, h);
    });
}

int sc_extract_patches(int tw, int th, int32_t *rects, int cap) {
    if (tw < 1 || th < 1) return fail(SC_ERR_INVALID, "bad template size");
    std::vector<int32_t> r = sc::extract_patches(tw, th);
    const int n = (int)r.size() / 4;
    if (rects) std::copy(r.begin(), r.begin() + 4 * std::min(n, std::max(cap, 0)), rects);
    return n;
}

int sc_detector_create_from_model(const sc_model *m, const sc_scan_params *p, int device,
                                  sc_detector **out) {
    return guarded([&] {
        if (!m || !out) throw Error{SC_ERR_INVALID, "null argument"};
        *out = make_detector(m->c, p, device);
        return SC_OK;
    });
}

int sc_detector_create(const char *path, const sc_scan_params *p, int device, sc_detector **out) {
    sc_model *m = nullptr;
    int rc = sc_model_load(path, &m);
    if (rc != SC_OK) return rc;
    rc = sc_detector_create_from_model(m, p, device, out);
    sc_model_free(m);
    return rc;
}

void sc_detector_destroy(sc_detector *d) { delete d; }

void *sc_detector_stream(sc_detector *d) { return d ? (void *)d->stream : nullptr; }

int sc_detector_wait_stream(sc_detector *d, void *stream) {
    return guarded([&] {
        if (!d) throw Error{SC_ERR_INVALID, "null detector"};
        HIPCHK(hipSetDevice(d->device));
        hipEvent_t e = d->ev();
        HIPCHK(hipEventRecord(e, static_cast<hipStream_t>(stream)));
        HIPCHK(hipStreamWaitEvent(d->stream, e, 0));
        d->event_pool.push_back(e);  // reusable once recorded and waited on
        return SC_OK;
    });
}

int sc_detector_set_stream(sc_detector *d, void *stream, int use_own) {
    return guarded([&] {
        if (!d) throw Error{SC_ERR_INVALID, "null detector"};
        HIPCHK(hipSetDevice(d->device));
        hipStream_t s = use_own ? d->own_stream : static_cast<hipStream_t>(stream);
        if (s == d->stream) return SC_OK;
        if (s && !use_own) {
            int dev = -1;
            HIPCHK(hipStreamGetDevice(s, &dev));
            if (dev != d->device)
                throw Error{SC_ERR_INVALID, "stream of device " + std::to_string(dev) + ", detector on " +
                                                std::to_string(d->device)};
        }
        hipEvent_t e = d->ev();
        HIPCHK(hipEventRecord(e, d->stream));
        HIPCHK(hipStreamWaitEvent(s, e, 0));
        d->event_pool.push_back(e);
        d->stream = s;
        return SC_OK;
    });
}

int sc_stream_wait_detector(sc_detector *d, void *stream) {
    return guarded([&] {
        if (!d) throw Error{SC_ERR_INVALID, "null detector"};
        HIPCHK(hipSetDevice(d->device));
        hipEvent_t e = d->ev();
        HIPCHK(hipEventRecord(e, d->stream));
        HIPCHK(hipStreamWaitEvent(static_cast<hipStream_t>(stream), e, 0));
        d->event_pool.push_back(e);
        return SC_OK;
    });
}

int sc_detect_device(sc_detector *d, const uint8_t *d_frames, int n, int w, int h, int stride,
                     sc_window *out, int capacity, int *n_out) {
    return guarded([&] {
        if (!d) throw Error{SC_ERR_INVALID, "null detector"};
        HIPCHK(hipSetDevice(d->device));
        check_device_ptr(d, d_frames, "d_frames");
        return detect_device_sync(d, d_frames, n, w, h, stride, out, capacity, n_out);
    });
}

int sc_miner_create(const sc_model *m, int tmpl_w, int tmpl_h, int device, sc_detector **out) {
    return guarded([&] {
        if (!out) throw Error{SC_ERR_INVALID, "null argument"};
        sc_scan_params prm;
        sc_scan_params_default(&prm);
        prm.base_len = tmpl_w;  // l_k = (int)(size.width * 1.1^k)  (:153)
        prm.step = 10;          // win.x/y += 10  (:155, :161)
        prm.prefilter_k = -INFINITY;  // no prefilter: every grid window is scanned
        prm.tmpl_w = tmpl_w;
        prm.tmpl_h = tmpl_h;
        prm.aspect_h = 1;       // Rect win(0, 0, l, l)  (:154)
        *out = make_detector(m ? m->c : sc::Cascade{}, &prm, device, true);
        return SC_OK;
    });
}

int sc_mine_batch(sc_detector *d, const uint8_t *const *frames, int n, int w, int h, int stride,
                  sc_window *wins, float *features, int capacity, int *n_out) {
    return guarded([&] {
        if (!d || !frames || n <= 0) throw Error{SC_ERR_INVALID, "bad arguments"};
        if (w < 2 || h < 2 || stride < w) throw Error{SC_ERR_INVALID, "bad frame geometry"};
        HIPCHK(hipSetDevice(d->device));
        const int pitch = upload_frames(d, frames, n, w, h, stride);
        return mine_sync(d, d->d_frames.p, n, w, h, pitch, wins, features, capacity, n_out);
    });
}

int sc_mine_batch_device(sc_detector *d, const uint8_t *d_frames, int n, int w, int h, int stride,
                         sc_window *wins, float *d_features, int capacity, int *n_out) {
    return guarded([&] {
        if (!d || !d_frames || n <= 0) throw Error{SC_ERR_INVALID, "bad arguments"};
        if (w < 2 || h < 2 || stride < w) throw Error{SC_ERR_INVALID, "bad frame geometry"};
        HIPCHK(hipSetDevice(d->device));
        check_device_ptr(d, d_frames, "d_frames");
        check_device_ptr(d, d_features, "d_features");
        return mine_sync(d, d_frames, n, w, h, stride, wins, d_features, capacity, n_out, true);
    });
}

int sc_mine(sc_detector *d, const uint8_t *gray, int w, int h, int stride, sc_window *wins,
            float *features, int capacity, int *n_out) {
    const uint8_t *fr[1] = {gray};
    return sc_mine_batch(d, fr, 1, w, h, stride, wins, features, capacity, n_out);
}

int sc_mine_device(sc_detector *d, const uint8_t *d_gray, int w, int h, int stride, sc_window *wins,
                   float *d_features, int capacity, int *n_out) {
    return sc_mine_batch_device(d, d_gray, 1, w, h, stride, wins, d_features, capacity, n_out);
}

int sc_detect_batch(sc_detector *d, const uint8_t *const *frames, int n, int w, int h, int stride,
                    sc_window *out, int capacity, int *n_out) {
    return guarded([&] {
        if (!d || !frames || n <= 0) throw Error{SC_ERR_INVALID, "bad arguments"};
        if (w < 2 || h < 2 || stride < w) throw Error{SC_ERR_INVALID, "bad frame geometry"};
        HIPCHK(hipSetDevice(d->device));
        const int pitch = upload_frames(d, frames, n, w, h, stride);
        return detect_device_sync(d, d->d_frames.p, n, w, h, pitch, out, capacity, n_out);
    });
}

int sc_detect(sc_detector *d, const uint8_t *gray, int w, int h, int stride, sc_window *out,
              int capacity, int *n_out) {
    const uint8_t *fr[1] = {gray};
    return sc_detect_batch(d, fr, 1, w, h, stride, out, capacity, n_out);
}

int sc_enqueue_device(sc_detector *d, const uint8_t *d_frames, int n, int w, int h, int stride,
                      sc_det_record *d_out, int capacity, int32_t *d_counts) {
    return guarded([&] {
        if (!d || !d_frames || n <= 0 || !d_counts || capacity < 0 || (capacity > 0 && !d_out))
            throw Error{SC_ERR_INVALID, "bad arguments"};
        if (w < 2 || h < 2 || stride < w) throw Error{SC_ERR_INVALID, "bad frame geometry"};
        if (d->miner) throw Error{SC_ERR_INVALID, "a miner scans with sc_mine, not sc_enqueue_device"};
        HIPCHK(hipSetDevice(d->device));
        check_device_ptr(d, d_frames, "d_frames");
        check_device_ptr(d, d_out, "d_out");
        check_device_ptr(d, d_counts, "d_counts");
        enqueue(d, d_frames, n, w, h, stride, d_out, capacity, d_counts);
        return SC_OK;
    });
}

int sc_synchronize(sc_detector *d) {
    return guarded([&] {
        if (!d) throw Error{SC_ERR_INVALID, "null detector"};
        HIPCHK(hipStreamSynchronize(d->stream));
        check_chain(d);
        return SC_OK;
    });
}

int sc_detector_info(sc_detector *d, int what, int64_t *value) {
    if (!d || !value) return fail(SC_ERR_INVALID, "null argument");
    switch (what) {
        case SC_INFO_LEVELS: *value = d->geo.n_levels; break;
        case SC_INFO_GRID_WINDOWS: *value = d->geo.grid; break;
        case SC_INFO_ROWS: *value = (int64_t)d->geo.rows.size(); break;
        case SC_INFO_TABLE_PITCH: *value = d->geo.tg.rowp; break;
        case SC_INFO_FUSED_FRAMES: *value = d->last_fused; break;
        case SC_INFO_CHAIN_WAVES: *value = d->last_waves; break;
        case SC_INFO_CHAIN_SUBQ: *value = d->last_subq; break;
        case SC_INFO_ITEM_FORM: *value = d->geo.tg.cs; break;
        case SC_INFO_COLUMN_PASS: *value = d->last_colpass; break;
        case SC_INFO_SPEC_ROUNDS:  // the last chain launch's speculative rounds
            return guarded([&] {
                int v = 0;
                if (d->spec_word >= 0) {
                    HIPCHK(hipSetDevice(d->device));
                    HIPCHK(hipStreamSynchronize(d->stream));
                    HIPCHK(hipMemcpy(&v, d->d_entry.p + d->spec_word, sizeof(int), hipMemcpyDeviceToHost));
                }
                *value = v;
                return SC_OK;
            });
        case SC_INFO_VISITED: {  // sum of the walk kernel's per-row counts
            return guarded([&] {
                HIPCHK(hipSetDevice(d->device));
                HIPCHK(hipStreamSynchronize(d->stream));
                const size_t n = (size_t)d->last_frames * d->geo.rows.size();
                std::vector<unsigned> rv(n);
                if (n) HIPCHK(hipMemcpy(rv.data(), d->d_visited.p, n * sizeof(unsigned),
                                        hipMemcpyDeviceToHost));
                long long s = 0;
                for (unsigned v : rv) s += v;
                *value = s;
                return SC_OK;
            });
        }
        default: return fail(SC_ERR_INVALID, "unknown info key");
    }
    return SC_OK;
}

int sc_detector_set_shard(sc_detector *d, int rank, int world) {
    if (!d) return fail(SC_ERR_INVALID, "null detector");
    if (world < 1 || rank < 0 || rank >= world) return fail(SC_ERR_INVALID, "bad shard rank/world");
    if (d->miner) return fail(SC_ERR_INVALID, "a miner scans whole images");
    if (d->shard_rank != rank || d->shard_world != world) {
        d->shard_rank = rank;
        d->shard_world = world;
        d->geo.W = d->geo.H = 0;  // rebuild the row list at the next detect
    }
    return SC_OK;
}

int sc_detector_set_option(sc_detector *d, int option, int64_t value) {
    if (!d) return fail(SC_ERR_INVALID, "null detector");
    auto range = [&](int64_t lo, int64_t hi) {
        if (value < lo || value > hi)
            throw Error{SC_ERR_INVALID, "option " + std::to_string(option) + " value " +
                                            std::to_string(value) + " out of range"};
        return (int)value;
    };
    return guarded([&] {
        sc_detector::Options &o = d->opt;
        bool regeo = true;  // the geometry / task tables depend on the option
        switch (option) {
            case SC_OPT_FULL_GRID: o.full_grid = range(0, 1); break;
            case SC_OPT_CHUNK_MIN: o.chunk_min = range(0, 1 << 30); regeo = false; break;
            case SC_OPT_TABLE_LAYOUT: o.table_layout = range(0, 1); break;
            case SC_OPT_PHASES: o.phases = range(0, 2); break;
            case SC_OPT_SUBSTRIPS: o.substrips = range(0, 64); break;
            case SC_OPT_BAND_ROWS: o.band_rows = range(0, 64); break;
            case SC_OPT_ROW_ORDER: o.row_order = range(0, 3); o.order_set = true; break;
            case SC_OPT_ROW_BLOCK: o.row_block = range(1, 1 << 16); o.order_set = true; break;
            case SC_OPT_CHAIN_CHUNK: o.chain_chunk = range(0, 1 << 20); regeo = false; break;
            case SC_OPT_LDS_WEIGHTS: o.lds_weights = range(-1, 1); regeo = false; break;
            case SC_OPT_WGS_PER_CU: o.wgs_per_cu = range(0, 4); regeo = false; break;
            case SC_OPT_PROFILE: o.profile = range(0, 1); regeo = false; break;
            case SC_OPT_INTEGRAL_PASSES: o.integral_passes = range(0, 2); regeo = false; break;
            case SC_OPT_INTEGRAL_FUSE: o.integral_fuse = range(0, 2); regeo = false; break;
            case SC_OPT_INTEGRAL_PRE: o.integral_pre = range(0, 64); regeo = false; break;
            case SC_OPT_TEST_DROP_HANDOFF:
#if !defined(SC_TEST_HOOKS) || !SC_TEST_HOOKS
                if (value != -1) throw Error{SC_ERR_INVALID, "test_drop_handoff needs the test-hook build (lib/testhooks)"};
#endif
                o.drop_handoff = range(-1, INT32_MAX - 1);
                regeo = false;
                break;
            case SC_OPT_TEST_DROP_WALK:
#if !defined(SC_TEST_HOOKS) || !SC_TEST_HOOKS
                if (value != -1) throw Error{SC_ERR_INVALID, "test_drop_walk needs the test-hook build (lib/testhooks)"};
#endif
                o.drop_walk = range(-1, INT32_MAX - 1);
                regeo = false;
                break;
            case SC_OPT_CHAIN_SUBQ: o.chain_subq = range(0, sc::kMaxSubQ); regeo = false; break;
            case SC_OPT_CHAIN_SPEC: o.chain_spec = range(0, 64); regeo = false; break;
            case SC_OPT_CHAIN_SLOTS: o.chain_slots = range(0, 2); regeo = false; break;
            case SC_OPT_CHAIN_WAVES:
                o.chain_waves = range(0, 16);
                if (o.chain_waves != 0 && o.chain_waves != 8 && o.chain_waves != 10 && o.chain_waves != 12 &&
                    o.chain_waves != 14 && o.chain_waves != 16)
                    throw Error{SC_ERR_INVALID, "chain_waves: 0, 8, 10, 12, 14 or 16"};
                regeo = false;
                break;
            case SC_OPT_LEVEL_LO: o.level_lo = range(0, 256); break;
            case SC_OPT_LEVEL_HI: o.level_hi = range(0, 256); break;
            case SC_OPT_CHAIN_SEGS:
                o.chain_segs = range(0, sc::kXcds);
                if (o.chain_segs & (o.chain_segs - 1)) throw Error{SC_ERR_INVALID, "chain_segs: 0, 1, 2, 4 or 8"};
                regeo = false;
                break;
            default: throw Error{SC_ERR_INVALID, "unknown option " + std::to_string(option)};
        }
        d->chunk_min = o.chunk_min > 0 ? o.chunk_min : 1 << 30;
        d->lazy = !o.full_grid && !d->miner;
        if (regeo) d->geo.W = d->geo.H = 0;  // rebuilt at the next detect
        return SC_OK;
    });
}

int sc_detector_set_debug(sc_detector *d, int on) {
    if (!d) return fail(SC_ERR_INVALID, "null detector");
    d->debug = on != 0;
    return SC_OK;
}

int sc_debug_dump(sc_detector *d, int what, int frame, void *dst, size_t bytes) {
    return guarded([&] {
        if (!d || !dst) throw Error{SC_ERR_INVALID, "null argument"};
        if (frame < 0 || frame >= d->last_frames) throw Error{SC_ERR_INVALID, "bad frame index"};
        HIPCHK(hipSetDevice(d->device));
        HIPCHK(hipStreamSynchronize(d->stream));
        const Geometry &g = d->geo;
        if (what == SC_DUMP_INTEGRAL) {
            // back to the reference's interleaved S[y][x][8] layout
            const size_t need = (size_t)(g.W + 1) * 32 * (g.H + 1);
            if (bytes < need) throw Error{SC_ERR_CAPACITY, "dump buffer too small"};
            const sc::TableGeom &t = g.tg;
            std::vector<float4> tab((size_t)t.frame4);
            HIPCHK(hipMemcpy(tab.data(), d->d_table.p + (size_t)frame * t.frame4,
                             tab.size() * sizeof(float4), hipMemcpyDeviceToHost));
            float *o = static_cast<float *>(dst);
            for (int y = 0; y <= g.H; y++)
                for (int x = 0; x <= g.W; x++) {
                    const size_t base = (size_t)y * t.rowp + t.at(x, 0);
                    const float4 lo = tab[base];
                    const float4 hi = tab[base + t.hs];
                    float *c = o + ((size_t)y * (g.W + 1) + x) * 8;
                    c[0] = lo.x; c[1] = lo.y; c[2] = lo.z; c[3] = lo.w;
                    c[4] = hi.x; c[5] = hi.y; c[6] = hi.z; c[7] = hi.w;
                }
            return SC_OK;
        }
        const size_t n = (size_t)g.grid;
        if (n == 0) return SC_OK;
        if (what == SC_DUMP_GRID_STAGE) {  // the cascade kernel's per-window records
            if (bytes < n * 2) throw Error{SC_ERR_CAPACITY, "dump buffer too small"};
            std::vector<int8_t> tmp(n);
            HIPCHK(hipMemcpy(tmp.data(), d->d_st_p.p + n * frame, n, hipMemcpyDeviceToHost));
            int16_t *o = static_cast<int16_t *>(dst);
            for (size_t i = 0; i < n; i++) o[i] = tmp[i];
        } else if (what == SC_DUMP_GRID_SCORE) {
            if (bytes < n * 4) throw Error{SC_ERR_CAPACITY, "dump buffer too small"};
            HIPCHK(hipMemcpy(dst, d->d_st_s.p + n * frame, n * 4, hipMemcpyDeviceToHost));
        } else if (what == SC_DUMP_GRID_VISIT) {
            if (!d->debug)
                throw Error{SC_ERR_INVALID, "visited flags need sc_detector_set_debug before detect"};
            if (bytes < n) throw Error{SC_ERR_CAPACITY, "dump buffer too small"};
            HIPCHK(hipMemcpy(dst, d->d_dbg_v.p + n * frame, n, hipMemcpyDeviceToHost));
        } else {
            throw Error{SC_ERR_INVALID, "unknown dump kind"};
        }
        return SC_OK;
    });
}

int sc_set_timing(sc_detector *d, int on) {
    if (!d) return fail(SC_ERR_INVALID, "null detector");
    d->timing = on != 0;
    return SC_OK;
}

int sc_get_timing(sc_detector *d, double ms[SC_KERNEL_COUNT], int64_t n[SC_KERNEL_COUNT]) {
    return guarded([&] {
        if (!d) throw Error{SC_ERR_INVALID, "null detector"};
        HIPCHK(hipStreamSynchronize(d->stream));
        for (auto &p : d->pending) {
            float t = 0;
            HIPCHK(hipEventElapsedTime(&t, p.a, p.b));
            d->t_ms[p.kind] += t;
            d->t_n[p.kind] += 1;
            d->event_pool.push_back(p.a);
            d->event_pool.push_back(p.b);
        }
        d->pending.clear();
        for (int k = 0; k < SC_KERNEL_COUNT; k++) {
            if (ms) ms[k] = d->t_ms[k];
            if (n) n[k] = d->t_n[k];
            d->t_ms[k] = 0;
            d->t_n[k] = 0;
        }
        return SC_OK;
    });
}

int sc_selftest_rn(int device, int op, uint32_t lo, uint32_t hi, uint64_t out[4]) {
    return guarded([&] {
        if (!out || (op != 0 && op != 1) || hi < lo) throw Error{SC_ERR_INVALID, "bad self-test arguments"};
        int ndev = 0;
        HIPCHK(hipGetDeviceCount(&ndev));
        if (device < 0 || device >= ndev) throw Error{SC_ERR_DEVICE, "device not present"};
        HIPCHK(hipSetDevice(device));
        int cus = 0;
        HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
        unsigned long long *d_out = nullptr;
        HIPCHK(hipMalloc(&d_out, 4 * sizeof(unsigned long long)));
        const unsigned long long init[4] = {0, 0, 0, ~0ull};
        int rc = SC_OK;
        if (hipMemcpy(d_out, init, sizeof(init), hipMemcpyHostToDevice) != hipSuccess) rc = SC_ERR_DEVICE;
        if (rc == SC_OK) {
            sc::launch_rn_check(op, lo, hi, d_out, cus, nullptr);
            if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
                hipMemcpy(out, d_out, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess)
                rc = SC_ERR_DEVICE;
        }
        (void)hipFree(d_out);
        if (rc != SC_OK) throw Error{rc, "self-test kernel failed"};
        return SC_OK;
    });
}

void sc_normalize_operand_range(int max_w, int max_h, double ss[2], double d[2]) {
    normalize_operand_range(max_w, max_h, ss, d);
}

}  // extern "C"
