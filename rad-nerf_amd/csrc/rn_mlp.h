// MFMA building blocks for the tiny fp16 MLPs of the Rad-NeRF field and gate.
//
// Orientation: activations are kept TRANSPOSED, features x samples, so one
// wave holds a 32-sample tile.  A layer computes  Y^T = W . X^T  with
// v_mfma_f32_32x32x16_f16 (A = weight fragment, B = activation fragment,
// fp32 accumulate).  Lane maps on gfx950 (cdna_hip_programming.md §3):
//   A: lane l (r=l&31, h=l>>5) holds A[r][8h+j]        j = 0..7
//   B: lane l holds B[8h+j][r]
//   C: reg i of lane l holds C[(i&3) + 8(i>>2) + 4h][l&31]
// so an accumulator tile is ALREADY the B operand of the next layer once its
// regs 8s..8s+7 are packed to f16 (k-step s).  The k index inside such a step
// is permuted: element j of lane half h is row  16s + 8(j>>2) + 4h + (j&3).
// Weight fragments are pre-permuted to match (host tables, see
// radnerf_amd/layout.py), so no lane shuffles or LDS round-trips are
// needed between layers.  A fragment = 64 lanes x 8 halfs = 1 KiB, stored
// lane-linear so one ds_read_b128 per lane fetches it conflict-free.
#pragma once
#include "rn_common.h"

typedef _Float16 rn_half;
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define RN_FRAG_HALFS 512   // 64 lanes x 8 halfs
#define RN_FRAG_BYTES 1024

__device__ __forceinline__ f32x16 rn_zero16() {
    f32x16 z;
#pragma unroll
    for (int i = 0; i < 16; ++i) z[i] = 0.f;
    return z;
}

__device__ __forceinline__ half8 rn_zero8() {
    half8 z;
#pragma unroll
    for (int i = 0; i < 8; ++i) z[i] = (rn_half)0.f;
    return z;
}

__device__ __forceinline__ f32x16 rn_mfma(const half8& a, const half8& b, const f32x16& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// fragment `f` of a lane-linear fragment array (LDS or global)
__device__ __forceinline__ half8 rn_frag(const rn_half* base, int f) {
    return *reinterpret_cast<const half8*>(base + f * RN_FRAG_HALFS + rn_lane() * 8);
}

// accumulator tile -> two B-operand fragments (k-steps 0 and 1), optional ReLU
template <bool RELU>
__device__ __forceinline__ void rn_acc_to_frags(const f32x16& acc, half8& f0, half8& f1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        float a = acc[j], b = acc[8 + j];
        if (RELU) { a = fmaxf(a, 0.f); b = fmaxf(b, 0.f); }
        f0[j] = (rn_half)a;
        f1[j] = (rn_half)b;
    }
}

// backward ReLU: keep gradient where the forward activation (f16) was > 0
__device__ __forceinline__ void rn_acc_to_frags_masked(const f32x16& acc, const half8& m0,
                                                       const half8& m1, half8& f0, half8& f1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        f0[j] = (float)m0[j] > 0.f ? (rn_half)acc[j] : (rn_half)0.f;
        f1[j] = (float)m1[j] > 0.f ? (rn_half)acc[8 + j] : (rn_half)0.f;
    }
}

// cooperative copy of n_bytes (multiple of 16) global -> LDS by a whole block
__device__ __forceinline__ void rn_block_copy16(void* lds, const void* g, int n_bytes) {
    const int4* src = reinterpret_cast<const int4*>(g);
    int4* dst = reinterpret_cast<int4*>(lds);
    for (int i = threadIdx.x; i < n_bytes / 16; i += blockDim.x) dst[i] = src[i];
}

// ---------------------------------------------------------------------------
// dW staging: an activation fragment (B-operand form, k-step q of a tile
// whose rows start at row0) is written into a wave-private LDS image
// [row][32 samples] (f16, row stride RN_STG_STRIDE halfs) so that the
// samples become the contraction index of the weight-gradient MFMA.
// ---------------------------------------------------------------------------
#define RN_STG_STRIDE 40   // 32 samples + 8 pad halfs (80 B rows)

__device__ __forceinline__ void rn_stage_frag(rn_half* stg, int row0, int q, const half8& f) {
    const int lane = rn_lane(), c = lane & 31, h = lane >> 5;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int row = row0 + 16 * (q & 1) + 8 * (j >> 2) + 4 * h + (j & 3) + 32 * (q >> 1);
        stg[row * RN_STG_STRIDE + c] = f[j];
    }
}

// operand fragment for the dW MFMA: rows (row_base + lane&31), samples 16s+8h..+7
__device__ __forceinline__ half8 rn_stage_read(const rn_half* stg, int row_base, int s) {
    const int lane = rn_lane(), r = lane & 31, h = lane >> 5;
    return *reinterpret_cast<const half8*>(stg + (row_base + r) * RN_STG_STRIDE + 16 * s + 8 * h);
}

// dW tile (rows of dY image at ya, rows of X image at xa) over the 32 samples
// of the staged tile, accumulated into the block's LDS fp32 gradient through
// the (tile, reg, lane) -> parameter map.  map < 0 = padding.
__device__ __forceinline__ void rn_dw_tile(const rn_half* stg_y, int ya, const rn_half* stg_x,
                                           int xa, const int16_t* __restrict__ map,
                                           float* dw_lds, float inv_scale) {
    f32x16 acc = rn_zero16();
    acc = rn_mfma(rn_stage_read(stg_y, ya, 0), rn_stage_read(stg_x, xa, 0), acc);
    acc = rn_mfma(rn_stage_read(stg_y, ya, 1), rn_stage_read(stg_x, xa, 1), acc);
    const int lane = rn_lane();
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int p = map[i * 64 + lane];
        if (p >= 0) atomicAdd(&dw_lds[p], acc[i] * inv_scale);
    }
}

// Per-wave power-of-two gradient scale for the f16 backward chain: maps the
// wave's largest seed magnitude into [8, 16) so small loss gradients stay in
// the f16 normal range (tcnn relies on a global GradScaler for the same).
// Power-of-two scaling is exact; results are unscaled in fp32.
__device__ __forceinline__ float rn_wave_grad_scale(float local_absmax) {
    float m = local_absmax;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
    if (!(m > 0.f) || !isfinite(m)) return 1.0f;
    int e;
    frexpf(m, &e);                 // m = f * 2^e, f in [0.5, 1)
    e = max(-100, min(100, 4 - e));
    return scalbnf(1.0f, e);
}
