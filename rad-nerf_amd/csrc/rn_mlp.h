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
        f0[j] = (rn_half)acc[j];
        f1[j] = (rn_half)acc[8 + j];
    }
    // ReLU after the f16 rounding (same values: rounding is monotone and keeps
    // the sign): packed maxes on canonical operands, 1 op per 2 elements
    // instead of canonicalize + max per element
    if (RELU) {
        f0 = __builtin_elementwise_max(f0, rn_zero8());
        f1 = __builtin_elementwise_max(f1, rn_zero8());
    }
}

// backward ReLU: keep gradient where the forward activation (f16) was > 0.
// The activations are ReLU outputs (>= 0, or -0), so "> 0" is "not +-0": per
// f16 pair, (m & 0x7fff) -> min(., 1) -> 0 - . gives a 0 / 0xffff mask that
// is ANDed onto the RNE-converted pair (packed u16 ops, 2 elements each; the
// per-element compare + select + repack took ~3.5 VALU per element plus
// hazard nops).  Bit-identical to the select form (masked lanes are +0).
__device__ __forceinline__ uint32_t rn_relu_mask2(uint32_t mbits) {
    // (written as u16x2 min / subtract, the compiler turned it back into two
    // compares + selects + a permute per pair: packed ops are spelled out)
    uint32_t t, r;
    // (op_sel_hi:[1,0]: the inline constant 1 is a 32-bit 0x00000001, so the
    // high lane reads its low half too)
    asm("v_pk_min_u16 %0, %1, 1 op_sel_hi:[1,0]" : "=v"(t) : "v"(mbits & 0x7fff7fffu));
    asm("v_pk_sub_u16 %0, 0, %1" : "=v"(r) : "v"(t));
    return r;
}
__device__ __forceinline__ void rn_acc_to_frags_masked(const f32x16& acc, const half8& m0,
                                                       const half8& m1, half8& f0, half8& f1) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const u4 mb0 = __builtin_bit_cast(u4, m0), mb1 = __builtin_bit_cast(u4, m1);
    u4 r0, r1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const h2 a = h2{(rn_half)acc[2 * j], (rn_half)acc[2 * j + 1]};
        const h2 b = h2{(rn_half)acc[8 + 2 * j], (rn_half)acc[8 + 2 * j + 1]};
        r0[j] = __builtin_bit_cast(uint32_t, a) & rn_relu_mask2(mb0[j]);
        r1[j] = __builtin_bit_cast(uint32_t, b) & rn_relu_mask2(mb1[j]);
    }
    f0 = __builtin_bit_cast(half8, r0);
    f1 = __builtin_bit_cast(half8, r1);
}

// cooperative copy of n_bytes (multiple of 16) global -> LDS by a whole block
__device__ __forceinline__ void rn_block_copy16(void* lds, const void* g, int n_bytes) {
    const int4* src = reinterpret_cast<const int4*>(g);
    int4* dst = reinterpret_cast<int4*>(lds);
    for (int i = threadIdx.x; i < n_bytes / 16; i += blockDim.x) dst[i] = src[i];
}

// ---------------------------------------------------------------------------
// dW staging.  The weight gradient dW = dY . X^T contracts over the samples,
// which live on the lanes of the accumulator layout, so (dY, X) go through a
// wave-private LDS image in SAMPLE-major order img[sample][feature] (row
// stride RN_IMG_STRIDE halfs): each lane stores its fragment with two 8-byte
// ds_write_b64 (4 consecutive features each), and the MFMA operands
// [feature][8 consecutive samples] come back with two ds_read_b64_tr_b16
// (gfx950 transposed read, cdna_hip_programming.md §5.5 T10).
// Row stride 68 halfs: conflict-free b64 writes (16 rows -> 16 bank pairs).
// ---------------------------------------------------------------------------
#define RN_IMG_STRIDE 68
#define RN_IMG_HALFS (32 * RN_IMG_STRIDE)

typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef short rn_s4 __attribute__((__vector_size__(4 * sizeof(short))));
typedef __attribute__((address_space(3))) rn_s4 rn_lds_s4;

// fragment q (B-operand form, k-step q of a multi-tile activation) -> image
__device__ __forceinline__ void rn_img_write(rn_half* img, int q, const half8& f) {
    const int lane = rn_lane(), c = lane & 31, h = lane >> 5;
    const int f0 = 32 * (q >> 1) + 16 * (q & 1) + 4 * h;
    half4 lo, hi;
#pragma unroll
    for (int j = 0; j < 4; ++j) { lo[j] = f[j]; hi[j] = f[4 + j]; }
    *reinterpret_cast<half4*>(img + c * RN_IMG_STRIDE + f0) = lo;
    *reinterpret_cast<half4*>(img + c * RN_IMG_STRIDE + f0 + 8) = hi;
}

__device__ __forceinline__ half4 rn_tr_read(const rn_half* p) {
    rn_s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((rn_lds_s4*)(p));
    return __builtin_bit_cast(half4, v);
}

// dW MFMA operand: features fbase + (lane&31), samples 16s + 8h + 0..7
__device__ __forceinline__ half8 rn_img_read(const rn_half* img, int fbase, int s) {
    const int l = rn_lane(), g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
    const int col = fbase + 16 * (g & 1) + 4 * p;
    const int sb = 16 * s + 8 * (g >> 1);
    const half4 a = rn_tr_read(img + (sb + q) * RN_IMG_STRIDE + col);
    const half4 b = rn_tr_read(img + (sb + 4 + q) * RN_IMG_STRIDE + col);
    half8 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) { r[j] = a[j]; r[4 + j] = b[j]; }
    return r;
}

// compiler-only ordering point between LDS image writes and reads of one
// wave (a wave's LDS operations execute in order; nothing to wait for)
__device__ __forceinline__ void rn_lds_order() { asm volatile("" ::: "memory"); }

// dW tile: dY features [ya, ya+32) x X features [xa, xa+32) over the 32
// samples of the staged tile, accumulated (x inv_scale) into the block's LDS
// fp32 gradient (row-major [out][in] master layout at `off`, `ncols` inputs).
// Output row i of the tile is dY feature ya+i -> weight row out_base + i
// (DW_PLAIN), only rows < 3 exist (DW_ROWS_LT3: rgb output layer), or the
// geo-net remap rows 0..15 -> outputs 1..16, row 16 -> output 0 (DW_GEO).
#define DW_PLAIN 0
#define DW_ROWS_LT3 1
#define DW_GEO 2
template <int MODE>
__device__ __forceinline__ void rn_dw_tile(const rn_half* img_y, int ya, const rn_half* img_x,
                                           int xa, float* dw_lds, int off, int ncols,
                                           int out_base, int in_base, float inv_scale,
                                           int dbg = 0) {
    f32x16 acc = rn_zero16();
    acc = rn_mfma(rn_img_read(img_y, ya, 0), rn_img_read(img_x, xa, 0), acc);
    acc = rn_mfma(rn_img_read(img_y, ya, 1), rn_img_read(img_x, xa, 1), acc);
    if (rn_dbg(dbg) & 8) { asm volatile("" :: "v"(acc)); return; }
    const int lane = rn_lane(), col = lane & 31, h = lane >> 5;
    float* base = dw_lds + off + in_base + col;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
        int out;
        if (MODE == DW_PLAIN) out = out_base + row;
        else if (MODE == DW_ROWS_LT3) out = row < 3 ? row : -1;
        else out = row < 16 ? row + 1 : (row == 16 ? 0 : -1);
        if (out >= 0) atomicAdd(base + out * ncols, acc[i] * inv_scale);
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
