// sc_mine.hip -- gfx950 kernels of the hard-negative mining scan
// (DenseSURFFeatureExtractor::FillNegSamples, DenseSURFFeatureExtractor.cpp:
// 124-195), after the shared integral + cascade kernels have run on the
// stride-10, no-prefilter window grid:
//   mine_count   : candidates (stage reached == number of stages) per block
//                  of kMineBlock grid windows of one frame
//   mine_scan    : exclusive prefix of the block counts and per-frame totals
//                  (one workgroup; no host round trip)
//   mine_scatter : candidate windows in (frame, level, y, x) order, the
//                  first `capacity` of them
//   features     : ExtractFeatures (:88-93) of each kept window over every
//                  template patch: ProjectPatches + CalcFeature + Normalize,
//                  one (window, patch) item per lane, 128 B stored per item
#include <hip/hip_runtime.h>

#include "sc_device.hpp"
#include "sc_kernels.hpp"

namespace sc {

namespace {

constexpr int kMineThreads = 256;
constexpr int kMinePer = kMineBlock / kMineThreads;  // windows per thread
constexpr int kMaxLevels = 256;                      // host check

// global block b: frame b / bpf, windows [(b % bpf) * kMineBlock, ...) of it
__device__ __forceinline__ long long block_frame_base(const MineArgs &a, int b, long long &lim) {
    const int f = b / a.bpf;
    const long long w0 = (long long)(b - f * a.bpf) * kMineBlock;
    lim = a.grid - w0;  // windows of this block inside the frame
    return (long long)f * a.grid + w0;
}

__global__ __launch_bounds__(kMineThreads) void mine_count_kernel(MineArgs a) {
    __shared__ int s_cnt;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    long long lim;
    const long long b0 = block_frame_base(a, blockIdx.x, lim);
    int c = 0;
#pragma unroll
    for (int k = 0; k < kMinePer; k++) {
        const int i = k * kMineThreads + threadIdx.x;
        c += i < lim && a.st_p[b0 + i] == a.n_stages;
    }
    c += __shfl_xor(c, 32, 64);
    c += __shfl_xor(c, 16, 64);
    c += __shfl_xor(c, 8, 64);
    c += __shfl_xor(c, 4, 64);
    c += __shfl_xor(c, 2, 64);
    c += __shfl_xor(c, 1, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(&s_cnt, c);
    __syncthreads();
    if (threadIdx.x == 0) a.block_count[blockIdx.x] = s_cnt;
}

// Exclusive prefix of the block counts (64-bit running total, offsets
// saturated at INT32_MAX) and the per-frame totals: one workgroup, chunks of
// kScanThreads blocks, a wave scan (shuffles) + the waves' totals in LDS.
constexpr int kScanThreads = 1024;
__global__ __launch_bounds__(kScanThreads) void mine_scan_kernel(MineArgs a) {
    __shared__ long long s_wave[kScanThreads / 64];
    __shared__ long long s_carry;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int nb = a.n_frames * a.bpf;
    if (threadIdx.x == 0) s_carry = 0;
    for (int f = threadIdx.x; f <= a.n_frames; f += kScanThreads) a.frame_count[f] = 0;
    __syncthreads();
    for (int c0 = 0; c0 < nb; c0 += kScanThreads) {
        const int b = c0 + (int)threadIdx.x;
        const long long v = b < nb ? a.block_count[b] : 0;
        long long x = v;  // inclusive wave scan
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const long long o = __shfl_up(x, d, 64);
            if (lane >= d) x += o;
        }
        if (lane == 63) s_wave[wv] = x;
        __syncthreads();
        long long before = s_carry;
        for (int w = 0; w < wv; w++) before += s_wave[w];
        if (b < nb) {
            const long long ex = before + x - v;
            a.block_offset[b] = (int)(ex < 0x7fffffffll ? ex : 0x7fffffffll);
            if (v) atomicAdd(&a.frame_count[1 + b / a.bpf], (int)v);
        }
        __syncthreads();
        if (threadIdx.x == kScanThreads - 1) s_carry = before + x;
        __syncthreads();
    }
    if (threadIdx.x == 0) a.frame_count[0] = (int)(s_carry < 0x7fffffffll ? s_carry : 0x7fffffffll);
}

__global__ __launch_bounds__(kMineThreads) void mine_scatter_kernel(MineArgs a) {
    __shared__ LevelInfo s_lv[kMaxLevels];
    __shared__ int s_wave[kMineThreads / 64];
    for (int i = threadIdx.x; i < a.n_levels; i += kMineThreads) s_lv[i] = a.levels[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    long long lim;
    const long long b0 = block_frame_base(a, blockIdx.x, lim);
    const int frame = blockIdx.x / a.bpf;
    const long long w0 = b0 - (long long)frame * a.grid;  // the block's first window in its frame
    long long base = a.block_offset[blockIdx.x];
    for (int k = 0; k < kMinePer; k++) {  // chunks of kMineThreads windows, in order
        const int i = k * kMineThreads + threadIdx.x;
        const bool hit = i < lim && a.st_p[b0 + i] == a.n_stages;
        const unsigned long long m = __ballot(hit);
        if (lane == 0) s_wave[wv] = __popcll(m);
        __syncthreads();
        int before = 0, total = 0;
        for (int w = 0; w < kMineThreads / 64; w++) {
            before += w < wv ? s_wave[w] : 0;
            total += s_wave[w];
        }
        const long long rank = base + before + __popcll(m & ((1ull << lane) - 1ull));
        if (hit && rank < a.capacity) {
            const long long gi = w0 + i;  // window within the frame's grid
            int lv = 0;  // last level whose grid range starts at or before gi
            for (int q = 1; q < a.n_levels; q++)
                if (s_lv[q].nx > 0 && s_lv[q].grid_base <= gi) lv = q;
            const LevelInfo &L = s_lv[lv];
            const int local = (int)(gi - L.grid_base), row = local / L.nx, col = local - row * L.nx;
            MineWindow w;
            w.frame = frame;
            w.level = lv;
            w.x = col * a.step;
            w.y = row * a.step;
            w.l = L.l;
            w.score = a.st_s[b0 + i];
            a.out[rank] = w;
        }
        base += total;
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void features_kernel(FeatureArgs a) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
    if (t >= (long long)a.n_windows * a.n_patches) return;
    const int i = (int)(t / a.n_patches), j = (int)(t - (long long)i * a.n_patches);
    if (a.n_valid && i >= *a.n_valid) return;  // past the candidates found (capacity-sized launch)
    const MineWindow w = a.windows[i];
    const int par = (w.x / a.g.step) & 1;
    const ProjPatch pj = load_proj(a.proj_all + ((long long)w.level * 2 + par) * a.n_patches + j);
    const TabView T{reinterpret_cast<const char *>(a.table + (long long)w.frame * a.g.frame4),
                    (unsigned)(w.y * a.g.rowp + a.g.at(w.x, 0)) << 4};
    float f[32];
    descriptor(T, a.g.hs, pj, f);
    float4 *o = reinterpret_cast<float4 *>(a.out + t * 32);
#pragma unroll
    for (int q = 0; q < 8; q++) o[q] = make_float4(f[4 * q], f[4 * q + 1], f[4 * q + 2], f[4 * q + 3]);
}

}  // namespace

void launch_mine_count(const MineArgs &a, hipStream_t s) {
    hipLaunchKernelGGL(mine_count_kernel, dim3(a.n_frames * a.bpf), dim3(kMineThreads), 0, s, a);
}

void launch_mine_scan(const MineArgs &a, hipStream_t s) {
    hipLaunchKernelGGL(mine_scan_kernel, dim3(1), dim3(kScanThreads), 0, s, a);
}

void launch_mine_scatter(const MineArgs &a, hipStream_t s) {
    hipLaunchKernelGGL(mine_scatter_kernel, dim3(a.n_frames * a.bpf), dim3(kMineThreads), 0, s, a);
}

void launch_features(const FeatureArgs &a, hipStream_t s) {
    const long long n = (long long)a.n_windows * a.n_patches;
    hipLaunchKernelGGL(features_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
}

}  // namespace sc
