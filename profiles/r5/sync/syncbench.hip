// Round 5: where a one-frame call's ~12 us of round trip goes.  Per
// iteration: launch K tiny kernels on one stream, then wait for them by
//   stream  hipStreamSynchronize
//   event   hipEventRecord + hipEventSynchronize
//   flag    the last workgroup of the last kernel stores the iteration number
//           to mapped host memory (system scope); the host spins on it (one
//           hipStreamSynchronize after all iterations)
//   queued  N iterations' launches back to back, one hipStreamSynchronize
// hipcc --offload-arch=gfx950 -O2 syncbench.hip -o syncbench
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1); } } while (0)

__global__ void spin_kernel(int *scratch, long long cycles, int *flag, int v) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {}
    if (threadIdx.x == 0) atomicAdd(scratch, 1);
    // the last workgroup to finish raises the host flag (system scope)
    if (flag && threadIdx.x == 0 && atomicAdd(scratch + 1, 1) == (int)gridDim.x - 1) {
        scratch[1] = 0;
        __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const int N = 300, K = argc > 1 ? std::atoi(argv[1]) : 3;
    const long long cyc = argc > 2 ? std::atoll(argv[2]) : 20000;  // per kernel (~10 us at 2 GHz)
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int *scratch, *hflag, *dflag;
    CK(hipMalloc(&scratch, 64));
    CK(hipMemset(scratch, 0, 64));
    CK(hipHostMalloc(&hflag, 64, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void **)&dflag, hflag, 0));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    auto launch = [&](int it, bool flag) {
        for (int k = 0; k < K; k++)
            hipLaunchKernelGGL(spin_kernel, dim3(256), dim3(64), 0, s, scratch, cyc, flag && k == K - 1 ? dflag : nullptr, it);
    };
    for (int i = 0; i < 50; i++) launch(0, false);
    CK(hipStreamSynchronize(s));
    std::vector<double> r[4];
    int seq = 1;
    for (int rep = 0; rep < 5; rep++) {
        double t0 = now_us();
        for (int i = 0; i < N; i++) { launch(0, false); CK(hipStreamSynchronize(s)); }
        r[0].push_back((now_us() - t0) / N);
        t0 = now_us();
        for (int i = 0; i < N; i++) { launch(0, false); CK(hipEventRecord(ev, s)); CK(hipEventSynchronize(ev)); }
        r[1].push_back((now_us() - t0) / N);
        t0 = now_us();
        for (int i = 0; i < N; i++) {
            const int v = ++seq;
            launch(v, true);
            while (__atomic_load_n(static_cast<volatile int *>(hflag), __ATOMIC_ACQUIRE) != v) {}
        }
        CK(hipStreamSynchronize(s));
        r[2].push_back((now_us() - t0) / N);
        t0 = now_us();
        for (int i = 0; i < N; i++) launch(0, false);
        CK(hipStreamSynchronize(s));
        r[3].push_back((now_us() - t0) / N);
    }
    const char *names[4] = {"stream", "event", "flag", "queued"};
    std::printf("{\"kernels_per_call\": %d, \"spin_cycles\": %lld", K, cyc);
    for (int j = 0; j < 4; j++) {
        std::sort(r[j].begin(), r[j].end());
        std::printf(", \"%s_us\": %.2f", names[j], r[j][r[j].size() / 2]);
    }
    std::printf("}\n");
    return 0;
}
