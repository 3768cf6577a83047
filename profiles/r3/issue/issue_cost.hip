// Issue cost of the item chain's instruction classes on gfx950 (profiling tool):
// a dependent chain of N ops per lane, one workgroup of W waves on one CU,
// cycles per op from s_memtime.  Also: a chain with half the lanes active.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int KIND>
__global__ void chain(float *o, double *od, unsigned long long *t, int n, int active) {
    const int lane = threadIdx.x & 63;
    float x = (float)threadIdx.x * 1e-3f, y = 1.0001f;
    double xd = (double)threadIdx.x * 1e-3, yd = 1.0001;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (lane < active) {
        for (int i = 0; i < n; i++) {
            if (KIND == 0) { x = x * y + 0.5f; }                       // v_fma_f32 (contracted below)
            if (KIND == 1) { xd = xd * yd + 0.5; }                     // v_fma_f64
            if (KIND == 2) { x = sqrtf(x + 1.0f); }                    // IEEE sqrt sequence
            if (KIND == 3) { xd = exp(-xd) * 0.5; }                    // OCML exp f64
            if (KIND == 4) { xd = 1.0 / (1.0 + xd); }                  // IEEE f64 division
            if (KIND == 5) { x = 1.0f / (x + 1.0f); }                  // IEEE f32 division
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    o[blockIdx.x * blockDim.x + threadIdx.x] = x;
    od[blockIdx.x * blockDim.x + threadIdx.x] = xd;
    if (lane == 0) t[blockIdx.x * 64 + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
    float *o; double *od; unsigned long long *t;
    hipMalloc(&o, 1 << 20); hipMalloc(&od, 1 << 21); hipMalloc(&t, 1 << 16);
    const int n = 4096;
    const char *names[] = {"fma_f32", "fma_f64", "sqrt_f32(ieee)", "exp_f64", "div_f64", "div_f32"};
    for (int kind = 0; kind < 6; kind++)
        for (int waves : {1, 4, 16})
            for (int active : {64, 32}) {
                auto k = kind == 0 ? chain<0> : kind == 1 ? chain<1> : kind == 2 ? chain<2> : kind == 3 ? chain<3> : kind == 4 ? chain<4> : chain<5>;
                hipLaunchKernelGGL(k, dim3(1), dim3(64 * waves), 0, 0, o, od, t, n, active);
                hipLaunchKernelGGL(k, dim3(1), dim3(64 * waves), 0, 0, o, od, t, n, active);
                hipDeviceSynchronize();
                std::vector<unsigned long long> h(64);
                hipMemcpy(h.data(), t, 64 * 8, hipMemcpyDeviceToHost);
                unsigned long long mx = 0;
                for (int w = 0; w < waves; w++) mx = h[w] > mx ? h[w] : mx;
                printf("%-16s waves %2d active %2d: %.2f cycles per op per wave\n", names[kind], waves, active, (double)mx / n);
            }
    return 0;
}
