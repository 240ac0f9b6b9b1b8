// Shared device helpers for the Rad-NeRF MI355X (gfx950) hot path.
//
// Floating-point contraction policy (DESIGN.md §"Contraction policy"): every
// translation unit is compiled under `#pragma clang fp contract(off)`; the
// multiply-add sites that nvcc fuses in the reference (raymarching.cu:197,205,
// 215,225,229) are written as explicit fmaf() calls.  The CPU oracle
// (oracle/vren_oracle.c) uses the identical explicit-fmaf policy, which is what
// makes per-ray sample counts and sample positions bit-exact between the two.
#pragma once
#include <hip/hip_runtime.h>
#include <type_traits>
#include <stdint.h>
#include "radnerf.h"   // the C ABI: definitions below must match these declarations

#pragma clang fp contract(off)

#define RN_SQRT3 1.73205080757f
#define RN_WAVE 64

// Timing studies (tools/ablate.py, bin_probe.py, march_probe.py) switch parts
// of kernels off or swap in variants through rn_set_debug_flags.  Only the
// ablation build reads those switches: librn_abl.so (-DRN_ABLATION, tools
// only).  In librn.so RN_ABL is 0, rn_dbg() folds every switch to 0 at compile
// time, the variant kernels are not instantiated, and each kernel has exactly
// one code path.
#ifdef RN_ABLATION
#define RN_ABL 1
#else
#define RN_ABL 0
#endif
__host__ __device__ constexpr int rn_dbg(int flags) { return RN_ABL ? flags : 0; }

// ---------------------------------------------------------------------------
// status / error plumbing shared by every C-ABI entry point
// ---------------------------------------------------------------------------
extern "C" void rn_set_error(const char* fmt, ...);

#define RN_CHECK_ARG(cond, msg)                                   \
    do {                                                          \
        if (!(cond)) { rn_set_error("%s: %s", __func__, msg);     \
                       return 1; }                                \
    } while (0)

#define RN_CHECK_LAUNCH()                                                  \
    do {                                                                   \
        hipError_t _e = hipGetLastError();                                 \
        if (_e != hipSuccess) {                                            \
            rn_set_error("%s: launch failed: %s", __func__,                \
                         hipGetErrorString(_e));                           \
            return 2;                                                      \
        }                                                                  \
    } while (0)

// ---------------------------------------------------------------------------
// reference math helpers (raymarching.cu:7-60, helper_math.h:280-283)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float rn_signf(float x) { return copysignf(1.0f, x); }

// helper_math.h:280  clamp(f,a,b) = fmaxf(a, fminf(f, b))
__device__ __forceinline__ float rn_clampf(float f, float a, float b) {
    return fmaxf(a, fminf(f, b));
}

// raymarching.cu:11-13 (calc_dt).  `scale` is a float parameter; the test-time
// kernel passes `cascades` there (raymarching.cu:370,399) and so do we.
__device__ __forceinline__ float rn_calc_dt(float t, float esf, int max_samples,
                                            int grid_size, float scale) {
    return rn_clampf(t * esf, RN_SQRT3 / max_samples,
                     RN_SQRT3 * 2 * scale / grid_size);
}

// raymarching.cu:19-23
__device__ __forceinline__ int rn_mip_from_pos(float x, float y, float z, int cascades) {
    const float mx = fmaxf(fabsf(x), fmaxf(fabsf(y), fabsf(z)));
    int e;
    frexpf(mx, &e);
    return min(cascades - 1, max(0, e + 1));
}

// raymarching.cu:29-32
__device__ __forceinline__ int rn_mip_from_dt(float dt, int grid_size, int cascades) {
    int e;
    frexpf(dt * grid_size, &e);
    return min(cascades - 1, max(0, e));
}

// raymarching.cu:35-60 (Morton coding, 10 bits per axis)
__host__ __device__ __forceinline__ uint32_t rn_expand_bits(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}
__host__ __device__ __forceinline__ uint32_t rn_morton3d(uint32_t x, uint32_t y, uint32_t z) {
    return rn_expand_bits(x) | (rn_expand_bits(y) << 1) | (rn_expand_bits(z) << 2);
}
__host__ __device__ __forceinline__ uint32_t rn_morton3d_invert(uint32_t x) {
    x = x & 0x49249249u;
    x = (x | (x >> 2)) & 0xc30c30c3u;
    x = (x | (x >> 4)) & 0x0f00f00fu;
    x = (x | (x >> 8)) & 0xff0000ffu;
    x = (x | (x >> 16)) & 0x0000ffffu;
    return x;
}

// ---------------------------------------------------------------------------
// wave64 collectives
// ---------------------------------------------------------------------------
__device__ __forceinline__ int rn_lane() { return threadIdx.x & (RN_WAVE - 1); }

__device__ __forceinline__ float rn_wave_max(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
    return v;
}

__device__ __forceinline__ uint32_t rn_wave_max_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off));
    return v;
}

__device__ __forceinline__ float rn_wave_sum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// DPP move of v with control CTRL (row_shr:n = 0x110 + n, wave_shr:1 = 0x138):
// lanes whose source lane is outside the row / wave get `ident`
template <int CTRL>
__device__ __forceinline__ float rn_dpp(float ident, float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(ident), __float_as_int(v),
                                                      CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ int rn_dpp_i(int ident, int v) {
    return __builtin_amdgcn_update_dpp(ident, v, CTRL, 0xf, 0xf, false);
}

// Inclusive wave64 scan: Hillis-Steele inside each 16-lane row with DPP
// row shifts (no LDS crossbar), then the row totals (lanes 15, 31, 47) are
// carried in.  `op` must be commutative (+, *).
template <typename T, typename Op, typename Dpp>
__device__ __forceinline__ T rn_wave_incl_scan(T v, T ident, Op op, Dpp dpp) {
    v = op(v, dpp(ident, v, std::integral_constant<int, 0x111>{}));
    v = op(v, dpp(ident, v, std::integral_constant<int, 0x112>{}));
    v = op(v, dpp(ident, v, std::integral_constant<int, 0x114>{}));
    v = op(v, dpp(ident, v, std::integral_constant<int, 0x118>{}));
    const int row = rn_lane() >> 4;
    const T r0 = __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 15));
    const T r1 = __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 31));
    const T r2 = __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 47));
    const T c01 = op(r0, r1);
    const T carry = row == 1 ? r0 : (row == 2 ? c01 : op(c01, r2));
    return row == 0 ? v : op(carry, v);
}

struct RnDppF {
    template <int C>
    __device__ float operator()(float id, float v, std::integral_constant<int, C>) const {
        return rn_dpp<C>(id, v);
    }
};
struct RnDppI {
    template <int C>
    __device__ int operator()(int id, int v, std::integral_constant<int, C>) const {
        return rn_dpp_i<C>(id, v);
    }
};

// inclusive prefix sum across the 64 lanes of a wave
__device__ __forceinline__ float rn_wave_incl_sum(float v) {
    return rn_wave_incl_scan(v, 0.0f, [](float a, float b) { return a + b; }, RnDppF{});
}

// inclusive prefix product across the 64 lanes of a wave
__device__ __forceinline__ float rn_wave_incl_prod(float v) {
    return rn_wave_incl_scan(v, 1.0f, [](float a, float b) { return a * b; }, RnDppF{});
}

// v of lane l - 1 (lane 0: first)
__device__ __forceinline__ float rn_wave_shr1(float v, float first) { return rn_dpp<0x138>(first, v); }

// v of lane 63, in every lane
__device__ __forceinline__ float rn_wave_last(float v) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), RN_WAVE - 1));
}

__device__ __forceinline__ int rn_wave_incl_sum_i(int v) {
    return rn_wave_incl_scan(v, 0, [](int a, int b) { return a + b; }, RnDppI{});
}

// ---------------------------------------------------------------------------
// compositing arithmetic shared bit-for-bit with the CPU oracle
// ---------------------------------------------------------------------------
// exp(x) as one fixed sequence of IEEE-754 single operations (round to
// nearest, fused fmaf, exact ldexpf), so that the GPU and the oracle
// (vren_oracle.c det_expf) produce identical bits.  The reference uses CUDA's
// __expf (ex2.approx, up to ~2 ulp); this is within 1 ulp of exp on the
// compositing range x = -sigma*delta <= 0.  Range reduction x = k ln2 + r
// (Cody-Waite, ln2 split in a 15-bit head and a tail), |r| <= ln2/2, then a
// degree-7 Taylor polynomial (truncation < 6e-9 relative).
__device__ __forceinline__ float rn_exp_det(float x) {
    if (!(x >= -87.0f)) return x != x ? x : 0.0f;     // exp(-87) > FLT_MIN: no denormals
    if (x > 88.0f) return __builtin_inff();
    const float k = rintf(x * 1.44269502162933349609375f);          // log2(e) in f32
    float r = fmaf(k, -0.693145751953125f, x);                      // ln2 head (exact product)
    r = fmaf(k, -1.428606765330187045037746429443359375e-06f, r);   // ln2 tail
    float p = 1.98412701138295233249664306640625e-04f;              // 1/5040
    p = fmaf(p, r, 1.388888922519981861114501953125e-03f);          // 1/720
    p = fmaf(p, r, 8.333333767950534820556640625e-03f);             // 1/120
    p = fmaf(p, r, 4.16666679084300994873046875000e-02f);           // 1/24
    p = fmaf(p, r, 1.66666671633720397949218750000e-01f);           // 1/6
    p = fmaf(p, r, 0.5f);
    p = fmaf(p, r, 1.0f);
    p = fmaf(p, r, 1.0f);
    return ldexpf(p, (int)k);
}

// Early termination, bit-exact against the reference's serial fold
// (volumerendering.cu:39-44: `T *= 1.0f - a; if (T <= T_threshold) break;`,
// one sample after the other).  The wave forms T with a prefix product
// (`pin`, tree order), which differs from the serial fold by at most one
// rounding per factor on each side: |pin / T_serial - 1| <= 2 (pos+1) 2^-24
// for the sample at segment position pos.  With that margin a lane is
// "surely past" (pin (1+m) <= thr), "surely not" (pin (1-m) > thr) or
// ambiguous.  rn_chunk_break returns the first lane that is not surely-not if
// it is surely past, -1 if every valid lane is surely-not, and -2 if the first
// candidate is ambiguous (T within ~1e-5 of T_threshold: rare), where the
// caller folds the segment serially (rn_serial_break).  The weights keep the
// tree-order T (within the 1e-4 tolerance); only the integer break is exact.
__device__ __forceinline__ int rn_chunk_break(float pin, bool valid, int pos, float thr) {
    const float m = (float)(pos + 2) * 2.384185791015625e-07f;     // 4 ulps per factor
    const bool cand = valid && pin * (1.0f - m) <= thr;
    const unsigned long long cb = __ballot(cand);
    if (!cb) return -1;
    const int l = __ffsll((long long)cb) - 1;
    const unsigned long long sure = __ballot(cand && pin * (1.0f + m) <= thr);
    return ((sure >> l) & 1ull) ? l : -2;
}

// Serial fold of a whole segment (the reference's order, same exponent):
// index of the sample whose product first reaches <= thr, or n if none.
// Lane j of a chunk folds after lanes < j (readlane chain); only called for
// the ambiguous chunks of rn_chunk_break.
__device__ __noinline__ int rn_serial_break(const float* __restrict__ sig,
                                            const float* __restrict__ dl, int64_t start, int n,
                                            float thr) {
    const int lane = rn_lane();
    float t = 1.0f;
    for (int base = 0; base < n; base += RN_WAVE) {
        const int i = base + lane;
        float om = 1.0f;
        if (i < n) om = 1.0f - (1.0f - rn_exp_det(-sig[start + i] * dl[start + i]));
        const int cnt = min(RN_WAVE, n - base);
        for (int j = 0; j < cnt; ++j) {
            t = t * __int_as_float(__builtin_amdgcn_readlane(__float_as_int(om), j));
            if (t <= thr) return base + j;
        }
    }
    return n;
}
