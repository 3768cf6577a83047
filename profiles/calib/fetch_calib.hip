// fetch_calib.hip -- calibrates rocprofv3's FETCH_SIZE / TCC_MISS for the
// chain kernel's access shape (16 B per lane, float4 gathers) against known
// byte counts, and measures the gather ceilings of that shape from the
// Infinity Cache and from HBM ("Next" 1: calibrate the counter,
// add a fabric roofline fraction).
//
// Kernels (one dispatch each per pass; names are what rocprofv3 reports):
//   k_stream      16-B-per-lane coalesced read of the whole big buffer
//                 (1 GiB, beyond the 256 MiB Infinity Cache): known bytes =
//                 the buffer (MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 here)
//   k_sparse      one 16-B load per 128-B line, every line of the big buffer
//                 exactly once, lines in a scattered order (odd-multiplier
//                 permutation): known = lines x 128 B if the fabric moves
//                 whole lines, lines x 64 B if it moves 64-B sectors
//   k_dense8      8 consecutive lanes read the 8 16-B cells of one line
//                 (the phase-split table's coalesced case), lines scattered
//   k_mall_sparse the k_sparse shape over a 64 MiB table (the size of one
//                 C2 frame's integral table: fits the Infinity Cache, not an
//                 XCD's 4 MiB L2), 32 passes per launch, after a warming
//                 stream: its L2 misses are Infinity-Cache hits -> the
//                 gather ceiling of this shape
//   k_mall_dense8 the k_dense8 shape over the 64 MiB table, 32 passes
//   k_rows_<T>    (round 4) MI355X_MICROARCH.md's best gather form: whole
//                 1-KiB pieces (64 lanes x 16 B, the chain kernel's dense
//                 batch load) of random rows, staged through LDS
//                 (global_load_dwordx4 + ds_write_b128, the guide's
//                 register-staging form), one 4-wave workgroup per CU, 16
//                 pieces per wave in flight (64 KiB per CU); k_rows_dma_<T>
//                 the same pieces by LDS DMA (global_load_lds_dwordx4);
//                 tables of 32 / 64 / 256 MiB (~ one C4 table) / 1 GiB:
//                 the beyond-L2
//                 ceiling the chain kernel's fabric_frac is reported against
// Each kernel: 256 CUs x 16 waves, every lane keeps 8 independent loads in
// flight; a sum of the loaded words goes to `sink` so nothing is dead.
//
//   hipcc --offload-arch=gfx950 -O3 -o fetch_calib fetch_calib.hip
//   ./fetch_calib            (prints one JSON line per kernel: bytes, ms, GB/s)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#define CHK(x)                                                                         \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

constexpr int kThreads = 256;
constexpr int kUnroll = 8;
constexpr unsigned kMul = 0x9E3779B1u;  // odd: i -> (i * kMul) mod 2^n is a permutation

// 16-B-per-lane coalesced stream: thread t reads float4 t, t + T, ...
__global__ __launch_bounds__(kThreads) void k_stream(const float4 *__restrict__ p, size_t n4,
                                                     float *sink) {
    const size_t T = (size_t)gridDim.x * kThreads;
    float acc = 0.0f;
    for (size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x; i < n4; i += T * kUnroll) {
        float4 v[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; u++) {
            const size_t j = i + (size_t)u * T;
            v[u] = j < n4 ? p[j] : make_float4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < kUnroll; u++) acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    if (acc == 1234.5f) sink[0] = acc;
}

// `lanes_per_line` lanes share one 128-B line (1: sparse, 8: the whole line);
// the line of group g is perm(g) = (g * kMul) & (lines - 1), lines a power
// of 2, so each line is read exactly once per pass.
template <int LPL>
__device__ __forceinline__ float gather_pass(const float4 *__restrict__ p, unsigned lines) {
    const unsigned T = gridDim.x * kThreads;
    const unsigned groups = lines;  // one group of LPL lanes per line
    const unsigned n = groups * LPL;
    float acc = 0.0f;
    for (unsigned i = blockIdx.x * kThreads + threadIdx.x; i < n; i += T * kUnroll) {
        float4 v[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; u++) {
            const unsigned j = i + u * T;
            const unsigned g = j / LPL, c = j % LPL;
            const unsigned line = (g * kMul) & (lines - 1);
            v[u] = j < n ? p[(size_t)line * 8 + c] : make_float4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < kUnroll; u++) acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    return acc;
}

__global__ __launch_bounds__(kThreads) void k_sparse(const float4 *p, unsigned lines, float *sink) {
    const float a = gather_pass<1>(p, lines);
    if (a == 1234.5f) sink[0] = a;
}
__global__ __launch_bounds__(kThreads) void k_dense8(const float4 *p, unsigned lines, float *sink) {
    const float a = gather_pass<8>(p, lines);
    if (a == 1234.5f) sink[0] = a;
}
// Infinity-Cache-resident table: `passes` passes per launch (a launch of a
// single 64 MiB pass is ~14 us, too short to time against its launch cost)
__global__ __launch_bounds__(kThreads) void k_mall_sparse(const float4 *p, unsigned lines, float *sink,
                                                          int passes) {
    float a = 0.0f;
    for (int q = 0; q < passes; q++) a += gather_pass<1>(p, lines);
    if (a == 1234.5f) sink[0] = a;
}
__global__ __launch_bounds__(kThreads) void k_mall_dense8(const float4 *p, unsigned lines, float *sink,
                                                          int passes) {
    float a = 0.0f;
    for (int q = 0; q < passes; q++) a += gather_pass<8>(p, lines);
    if (a == 1234.5f) sink[0] = a;
}

// Random 1-KiB pieces staged through LDS: each wave loads kPieces pieces
// (lane l: 16 B at piece + 16 l), writes them to its LDS tile, repeats
// `steps` times; the rows (pieces) are a permutation of the table's pieces.
constexpr int kPieces = 16;
__global__ __launch_bounds__(256) void k_rows(const float4 *__restrict__ p, unsigned pieces, int steps,
                                              float *sink) {
    __shared__ float4 tile[4][kPieces][64];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const unsigned W = gridDim.x * 4, gw = blockIdx.x * 4 + wv;
    float acc = 0.0f;
    for (int st = 0; st < steps; st++) {
        float4 v[kPieces];
#pragma unroll
        for (int u = 0; u < kPieces; u++) {
            const unsigned g = (unsigned)st * W * kPieces + gw * kPieces + u;
            const unsigned piece = (g * kMul) & (pieces - 1);
            v[u] = p[(size_t)piece * 64 + lane];
        }
#pragma unroll
        for (int u = 0; u < kPieces; u++) tile[wv][u][lane] = v[u];
        acc += tile[wv][(lane + st) & (kPieces - 1)][lane ^ 1].x;
    }
    if (acc == 1234.5f) sink[0] = acc;
}

// The same pieces by LDS DMA (global_load_lds_dwordx4: per-lane source,
// the wave's 1 KiB lands contiguous in its LDS ring), nothing read back
// until the end: as many pieces in flight as the vector-memory counter
// allows (the guide's gather-into-LDS form without a consumer)
__global__ __launch_bounds__(256) void k_rows_dma(const float4 *__restrict__ p, unsigned pieces, int steps,
                                                  float *sink) {
    __shared__ float4 ring[4][kPieces][64];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const unsigned W = gridDim.x * 4, gw = blockIdx.x * 4 + wv;
    for (int st = 0; st < steps; st++) {
#pragma unroll
        for (int u = 0; u < kPieces; u++) {
            const unsigned g = (unsigned)st * W * kPieces + gw * kPieces + u;
            const unsigned piece = (g * kMul) & (pieces - 1);
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(p + (size_t)piece * 64 + lane),
                (__attribute__((address_space(3))) void *)&ring[wv][u][0], 16, 0, 0);
        }
    }
    __syncthreads();
    if (ring[wv][lane & (kPieces - 1)][lane].x == 1234.5f) sink[0] = 1.0f;
}

__global__ void k_fill(float4 *p, size_t n4, unsigned seed) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const unsigned h = (unsigned)i * 2654435761u ^ seed;
        p[i] = make_float4((float)(h & 255), 1.0f, 2.0f, 3.0f);
    }
}

int main() {
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = cus * 4;  // 4 blocks of 4 waves per CU = 16 waves per CU
    const size_t big = 1ull << 30, small = 64ull << 20, flush = 512ull << 20;
    float4 *pb, *ps, *pf;
    float *sink;
    CHK(hipMalloc(&pb, big));
    CHK(hipMalloc(&ps, small));
    CHK(hipMalloc(&pf, flush));
    CHK(hipMalloc(&sink, 64));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, pb, big / 16, 1u);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, ps, small / 16, 2u);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, pf, flush / 16, 3u);
    CHK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    // evict the big buffer from the Infinity Cache: stream the flush buffer
    auto evict = [&] {
        hipLaunchKernelGGL(k_stream, dim3(grid), dim3(kThreads), 0, 0, pf, flush / 16, sink);
        CHK(hipDeviceSynchronize());
    };
    auto timed = [&](const char *name, auto launch, double bytes, size_t lines, int reps) {
        double best = 1e30, sum = 0;
        for (int r = 0; r < reps; r++) {
            CHK(hipEventRecord(a, 0));
            launch();
            CHK(hipEventRecord(b, 0));
            CHK(hipEventSynchronize(b));
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, a, b));
            best = ms < best ? ms : best;
            sum += ms;
        }
        std::printf("{\"kernel\": \"%s\", \"reps\": %d, \"lines\": %zu, \"requested_bytes\": %.0f, "
                    "\"ms_min\": %.4f, \"ms_mean\": %.4f, \"lines_per_s\": %.4g, \"line_GBps\": %.1f}\n",
                    name, reps, lines, bytes, best, sum / reps, lines / (best * 1e-3),
                    lines * 128.0 / (best * 1e-3) / 1e9);
        std::fflush(stdout);
    };
    const unsigned big_lines = (unsigned)(big / 128), small_lines = (unsigned)(small / 128);
    // cold, each kernel once after an eviction (rocprofv3 sees one dispatch per
    // kernel name from these legs)
    evict();
    timed("k_stream", [&] { hipLaunchKernelGGL(k_stream, dim3(grid), dim3(kThreads), 0, 0, pb, big / 16, sink); },
          (double)big, big_lines, 1);
    evict();
    timed("k_sparse", [&] { hipLaunchKernelGGL(k_sparse, dim3(grid), dim3(kThreads), 0, 0, pb, big_lines, sink); },
          16.0 * big_lines, big_lines, 1);
    evict();
    timed("k_dense8", [&] { hipLaunchKernelGGL(k_dense8, dim3(grid), dim3(kThreads), 0, 0, pb, big_lines, sink); },
          128.0 * big_lines, big_lines, 1);
    // Infinity-Cache-resident table: 1 warm pass, then 8 timed passes each
    hipLaunchKernelGGL(k_stream, dim3(grid), dim3(kThreads), 0, 0, ps, small / 16, sink);
    CHK(hipDeviceSynchronize());
    const int passes = 32;
    timed("k_mall_sparse",
          [&] { hipLaunchKernelGGL(k_mall_sparse, dim3(grid), dim3(kThreads), 0, 0, ps, small_lines, sink, passes); },
          16.0 * small_lines * passes, (size_t)small_lines * passes, 4);
    timed("k_mall_dense8",
          [&] { hipLaunchKernelGGL(k_mall_dense8, dim3(grid), dim3(kThreads), 0, 0, ps, small_lines, sink, passes); },
          128.0 * small_lines * passes, (size_t)small_lines * passes, 4);
    // round 4: 1-KiB row pieces through LDS (the guide's gather-into-LDS
    // form) from 64 MiB, 265 MiB and 1 GiB tables; each table warmed by one
    // untimed launch, then timed launches of the same permutation order
    for (size_t tb : {32ull << 20, 64ull << 20, 256ull << 20, 1ull << 30}) {
        float4 *pt = tb == big ? pb : nullptr;
        if (!pt) {
            CHK(hipMalloc(&pt, tb));
            hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, pt, tb / 16, 4u);
        }
        const unsigned pcs = (unsigned)(tb / 1024);
        const int steps = (int)std::max<size_t>(1, (size_t)pcs * 4 / ((size_t)cus * 4 * kPieces));  // ~4 table passes
        const size_t n_lines = (size_t)cus * 4 * kPieces * steps * 8;
        for (int dma = 0; dma < 2; dma++) {
            auto go = [&] {
                if (dma) hipLaunchKernelGGL(k_rows_dma, dim3(cus), dim3(256), 0, 0, pt, pcs, steps, sink);
                else hipLaunchKernelGGL(k_rows, dim3(cus), dim3(256), 0, 0, pt, pcs, steps, sink);
            };
            go();
            CHK(hipDeviceSynchronize());
            char name[64];
            std::snprintf(name, sizeof name, "k_rows%s_%zuMiB", dma ? "_dma" : "", tb >> 20);
            timed(name, go, 128.0 * n_lines, n_lines, 4);
        }
        if (pt != pb) CHK(hipFree(pt));
    }
    CHK(hipFree(pb));
    CHK(hipFree(ps));
    CHK(hipFree(pf));
    CHK(hipFree(sink));
    return 0;
}
