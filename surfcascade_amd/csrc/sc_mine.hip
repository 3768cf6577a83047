// sc_mine.hip -- gfx950 kernels of the hard-negative mining scan
// (DenseSURFFeatureExtractor::FillNegSamples, DenseSURFFeatureExtractor.cpp:
// 124-195), after the shared integral + cascade kernels have run on the
// stride-10, no-prefilter window grid:
//   mine_count   : candidates (stage reached == number of stages) per block
//                  of kMineBlock grid windows
//   mine_scatter : candidate windows in grid order = (level, y, x), the
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

__global__ __launch_bounds__(kMineThreads) void mine_count_kernel(MineArgs a) {
    __shared__ int s_cnt;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    const long long b0 = (long long)blockIdx.x * kMineBlock;
    int c = 0;
#pragma unroll
    for (int k = 0; k < kMinePer; k++) {
        const long long gi = b0 + k * kMineThreads + threadIdx.x;
        c += gi < a.grid && a.st_p[gi] == a.n_stages;
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

__global__ __launch_bounds__(kMineThreads) void mine_scatter_kernel(MineArgs a) {
    __shared__ LevelInfo s_lv[kMaxLevels];
    __shared__ int s_wave[kMineThreads / 64];
    for (int i = threadIdx.x; i < a.n_levels; i += kMineThreads) s_lv[i] = a.levels[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long b0 = (long long)blockIdx.x * kMineBlock;
    int base = a.block_offset[blockIdx.x];
    for (int k = 0; k < kMinePer; k++) {  // chunks of kMineThreads windows, in order
        const long long gi = b0 + k * kMineThreads + threadIdx.x;
        const bool hit = gi < a.grid && a.st_p[gi] == a.n_stages;
        const unsigned long long m = __ballot(hit);
        if (lane == 0) s_wave[wv] = __popcll(m);
        __syncthreads();
        int before = 0, total = 0;
        for (int w = 0; w < kMineThreads / 64; w++) {
            before += w < wv ? s_wave[w] : 0;
            total += s_wave[w];
        }
        const int rank = base + before + __popcll(m & ((1ull << lane) - 1ull));
        if (hit && rank < a.capacity) {
            int lv = 0;  // last level whose grid range starts at or before gi
            for (int i = 1; i < a.n_levels; i++)
                if (s_lv[i].nx > 0 && s_lv[i].grid_base <= gi) lv = i;
            const LevelInfo &L = s_lv[lv];
            const int local = (int)(gi - L.grid_base), row = local / L.nx, col = local - row * L.nx;
            MineWindow w;
            w.level = lv;
            w.x = col * a.step;
            w.y = row * a.step;
            w.l = L.l;
            w.score = a.st_s[gi];
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
    const MineWindow w = a.windows[i];
    const int par = (w.x / a.g.step) & 1;
    const ProjPatch pj = load_proj(a.proj_all + ((long long)w.level * 2 + par) * a.n_patches + j);
    const TabView T{reinterpret_cast<const char *>(a.table),
                    (unsigned)(w.y * a.g.rowp + a.g.at(w.x, 0)) << 4};
    float f[32];
    descriptor(T, a.g.hs, pj, f);
    float4 *o = reinterpret_cast<float4 *>(a.out + t * 32);
#pragma unroll
    for (int q = 0; q < 8; q++) o[q] = make_float4(f[4 * q], f[4 * q + 1], f[4 * q + 2], f[4 * q + 3]);
}

}  // namespace

void launch_mine_count(const MineArgs &a, hipStream_t s) {
    const int nb = (int)((a.grid + kMineBlock - 1) / kMineBlock);
    hipLaunchKernelGGL(mine_count_kernel, dim3(nb), dim3(kMineThreads), 0, s, a);
}

void launch_mine_scatter(const MineArgs &a, hipStream_t s) {
    const int nb = (int)((a.grid + kMineBlock - 1) / kMineBlock);
    hipLaunchKernelGGL(mine_scatter_kernel, dim3(nb), dim3(kMineThreads), 0, s, a);
}

void launch_features(const FeatureArgs &a, hipStream_t s) {
    const long long n = (long long)a.n_windows * a.n_patches;
    hipLaunchKernelGGL(features_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
}

}  // namespace sc
