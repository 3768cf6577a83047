// sc_integral_dev.hpp -- device helpers of the integral passes, shared by
// sc_integral.hip (rowcarry / colstrip / two-pass kernels) and the chain
// kernel's fused column walks (sc_windows.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace sc {
namespace idev {

__device__ __forceinline__ uint32_t sat_sub(uint32_t a, uint32_t b) { return a > b ? a - b : 0u; }

// The 4 gradient values of pixel (y, x) in this lane's half (T2bFilter,
// DenseSURFFeatureExtractor.cpp:224-347), borders clamped.  Returned packed:
// p0 = g0 | g1 << 16, p1 = g2 | g3 << 16 (strip sums stay < 2^16).
struct Px4 {
    uint32_t a, b, c, d;  // the four source bytes this half needs
};

__device__ __forceinline__ Px4 load_px(const uint8_t *img, int stride, int W, int H, int y, int x,
                                       int h) {
    const int xp = x > 0 ? x - 1 : 0, xn = x < W - 1 ? x + 1 : W - 1;
    const uint8_t *rc = img + (long long)y * stride;
    const uint8_t *ru = img + (long long)(y > 0 ? y - 1 : 0) * stride;
    const uint8_t *rd = img + (long long)(y < H - 1 ? y + 1 : H - 1) * stride;
    Px4 v;
    if (h == 0) {  // dx: I[y][x-1], I[y][x+1]; dy: I[y-1][x], I[y+1][x]
        v.a = rc[xp]; v.b = rc[xn]; v.c = ru[x]; v.d = rd[x];
    } else {       // du: I[y-1][x-1], I[y+1][x+1]; dv: I[y+1][x-1], I[y-1][x+1]
        v.a = ru[xp]; v.b = rd[xn]; v.c = rd[xp]; v.d = ru[xn];
    }
    return v;
}

// load_px with h per lane (the interleaved-cell walk: both halves in one
// wave): the same four bytes through selected addresses, no divergent branch
__device__ __forceinline__ Px4 load_px_lanes(const uint8_t *img, int stride, int W, int H, int y, int x,
                                             int h) {
    const int xp = x > 0 ? x - 1 : 0, xn = x < W - 1 ? x + 1 : W - 1;
    const uint8_t *rc = img + (long long)y * stride;
    const uint8_t *ru = img + (long long)(y > 0 ? y - 1 : 0) * stride;
    const uint8_t *rd = img + (long long)(y < H - 1 ? y + 1 : H - 1) * stride;
    Px4 v;
    v.a = (h ? ru : rc)[xp];
    v.b = (h ? rd : rc)[xn];
    v.c = (h ? rd : ru)[h ? xp : x];
    v.d = (h ? ru : rd)[h ? xn : x];
    return v;
}

// plane 2k = sat(Ip - In), plane 2k+1 = sat(In - Ip)  
__device__ __forceinline__ uint2 grad_packed(const Px4 &v) {
    // half 0: (Ip, In) = (I[y][x-1], I[y][x+1]) and (I[y-1][x], I[y+1][x])
    // half 1: (Ip, In) = (I[y-1][x-1], I[y+1][x+1]) and (I[y+1][x-1], I[y-1][x+1])
    const uint32_t g0 = sat_sub(v.a, v.b), g1 = sat_sub(v.b, v.a);
    const uint32_t g2 = sat_sub(v.c, v.d), g3 = sat_sub(v.d, v.c);
    return make_uint2(g0 | (g1 << 16), g2 | (g3 << 16));
}

// inclusive prefix sum within each 32-lane half: DPP row shifts (Hillis-
// Steele in 16-lane rows), then row 0's / row 2's last lane broadcast into
// rows 1 / 3 -- VALU only, no LDS round trips
__device__ __forceinline__ uint32_t half_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    return v;
}

// inclusive prefix sum over the whole wave: the half scan, then row 1's last
// lane broadcast into rows 2 and 3
__device__ __forceinline__ uint32_t wave_scan(uint32_t v) {
    v = half_scan(v);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

}  // namespace idev
}  // namespace sc
