// Ray gate of Rad-NeRF on gfx950: MLP 6 -> 64 -> 64 -> 64 -> 64 -> K (ReLU,
// no bias, f16 weights and input like tcnn FullyFusedMLP; hidden activations
// and logits kept at ~fp32, see gate_split) + softmax, forward and backward.
//
// Reference: models/networks.py:1070-1093 (Ray_Gate), call site
// models/ml_rendering.py:31-36 (input cat(rays_o, rays_d) or cat(rays_o, imgs_d)).
// Same MFMA orientation and fragment conventions as field.hip (rn_mlp.h).
#include "rn_mlp.h"
#pragma clang fp contract(off)

#define GATE_FWD_FRAGS 30
#define GATE_FRAGS 56
#define GATE_DW_TILES 16
#define GATE_WAVES 4
#define GATE_MAX_PARAMS (12672 + 64 * 16)

struct GateArgs {
    const float* in0; const float* in1;         // input cols 0..2 / 3..5, row stride `stride`
    int stride;
    int64_t n_rays; int K;
    const rn_half* frags;                        // [GATE_FRAGS][512]
    float* gate;                                 // (B,K) softmax
    float* importance;                           // (K) gate.sum(0), may be null
    const float* dgate;                          // (B,K) dL/dgate
    float* dw;                                   // (n_params)
    int n_params;
    const rn_half* dfrags;                       // [4][512] W0^T (input gradient), or null
    float* dx;                                   // (B,6) dL/dinput, or null
};

namespace {

// h: hidden activations (ReLU, f16 head); the forward carries each layer's
// f16 tail alongside (split precision, below)
struct GateState { half8 x; half8 h[4][4]; f32x16 logit; };

// fp32 accumulator tile -> ReLU -> head + tail f16 fragments (v = hi + lo to
// ~2^-22 relative): the next layer runs W.hi + W.lo on MFMA, i.e. fp32
// activations with f16 weights.  tcnn rounds every hidden activation to f16;
// at scale 16 (|rays_o| up to 24) the rounding points flip against any
// other accumulation order and move the gate by ~2e-3, so the gate is
// evaluated wider than tcnn (north_star allows wider).
__device__ __forceinline__ void gate_split(const f32x16& acc, half8& h0, half8& h1, half8& l0,
                                           half8& l1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float v0 = fmaxf(acc[j], 0.f), v1 = fmaxf(acc[8 + j], 0.f);
        h0[j] = (rn_half)v0; h1[j] = (rn_half)v1;
        l0[j] = (rn_half)(v0 - (float)h0[j]); l1[j] = (rn_half)(v1 - (float)h1[j]);
    }
}

__device__ __forceinline__ void gate_input(const GateArgs& a, int64_t r, bool valid, half8& x) {
    const int lane = rn_lane(), h = lane >> 5;
    x = rn_zero8();
    if (!valid) return;
    // element j <-> input 8(j>>2) + 4h + (j&3); inputs 0..5 = (o, d)
    const float* p0 = a.in0 + r * a.stride;
    const float* p1 = a.in1 + r * a.stride;
    if (h == 0) {
        x[0] = (rn_half)p0[0]; x[1] = (rn_half)p0[1]; x[2] = (rn_half)p0[2]; x[3] = (rn_half)p1[0];
    } else {
        x[0] = (rn_half)p1[1]; x[1] = (rn_half)p1[2];
    }
}

__device__ __forceinline__ void gate_forward(const rn_half* W, GateState& st) {
    f32x16 a0 = rn_zero16(), a1 = rn_zero16();
    a0 = rn_mfma(rn_frag(W, 0), st.x, a0);
    a1 = rn_mfma(rn_frag(W, 1), st.x, a1);
    half8 lo[4];
    gate_split(a0, st.h[0][0], st.h[0][1], lo[0], lo[1]);
    gate_split(a1, st.h[0][2], st.h[0][3], lo[2], lo[3]);
#pragma unroll
    for (int L = 1; L < 4; ++L) {
        a0 = rn_zero16(); a1 = rn_zero16();
        const int fb = 2 + 8 * (L - 1);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            a0 = rn_mfma(rn_frag(W, fb + q), st.h[L - 1][q], a0);
            a0 = rn_mfma(rn_frag(W, fb + q), lo[q], a0);
            a1 = rn_mfma(rn_frag(W, fb + 4 + q), st.h[L - 1][q], a1);
            a1 = rn_mfma(rn_frag(W, fb + 4 + q), lo[q], a1);
        }
        gate_split(a0, st.h[L][0], st.h[L][1], lo[0], lo[1]);
        gate_split(a1, st.h[L][2], st.h[L][3], lo[2], lo[3]);
    }
    st.logit = rn_zero16();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        st.logit = rn_mfma(rn_frag(W, 26 + q), st.h[3][q], st.logit);
        st.logit = rn_mfma(rn_frag(W, 26 + q), lo[q], st.logit);
    }
}

// softmax over the K logit rows of this lane's sample (rows spread over the
// two lane halves: reg i <-> row (i&3) + 8(i>>2) + 4h).  Returns probs in the
// same register positions (0 for rows >= K).
__device__ __forceinline__ f32x16 gate_softmax(const f32x16& logit, int K) {
    const int h = rn_lane() >> 5;
    float z[16];
    float m = -INFINITY;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
        z[i] = logit[i];   // fp32 logits (tcnn rounds them to f16: wider here), softmax in f32
        if (row < K) m = fmaxf(m, z[i]);
    }
    m = fmaxf(m, __shfl_xor(m, 32));
    float sum = 0.f;
    float e[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
        e[i] = row < K ? expf(z[i] - m) : 0.f;
        sum += e[i];
    }
    sum += __shfl_xor(sum, 32);
    f32x16 p;
#pragma unroll
    for (int i = 0; i < 16; ++i) p[i] = e[i] / sum;
    return p;
}

__global__ void __launch_bounds__(GATE_WAVES * 64)
k_gate_fwd(GateArgs a) {
    __shared__ __attribute__((aligned(16))) rn_half sW[GATE_FWD_FRAGS * RN_FRAG_HALFS];
    rn_block_copy16(sW, a.frags, GATE_FWD_FRAGS * RN_FRAG_BYTES);
    __syncthreads();
    const int lane = rn_lane(), c = lane & 31, h = lane >> 5;
    const int64_t n_tiles = (a.n_rays + 31) / 32;
    for (int64_t tile = (int64_t)blockIdx.x * GATE_WAVES + threadIdx.x / RN_WAVE; tile < n_tiles;
         tile += (int64_t)gridDim.x * GATE_WAVES) {
        rn_lds_order();   // weights stay in LDS: no hoisting of fragment reads
        const int64_t r = tile * 32 + c;
        const bool valid = r < a.n_rays;
        GateState st;
        gate_input(a, r, valid, st.x);
        gate_forward(sW, st);
        const f32x16 p = gate_softmax(st.logit, a.K);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
            if (row < a.K) {
                if (valid) a.gate[r * a.K + row] = p[i];
                if (a.importance) {
                    // per-wave column sum over the 32 samples of this half
                    float v = valid ? p[i] : 0.f;
#pragma unroll
                    for (int off = 16; off > 0; off >>= 1) v += __shfl_xor(v, off);
                    if (c == 0) atomicAdd(&a.importance[row], v);
                }
            }
        }
    }
}


// gate output layer dW: rows < K of dz x H3 (W4 at 12672, 64 inputs)
__device__ __forceinline__ void rn_dw_tile_gate_out(const rn_half* img_y, int ya, const rn_half* img_x,
                                                    int xa, float* dw_lds, int K, float inv_scale) {
    f32x16 acc = rn_zero16();
    acc = rn_mfma(rn_img_read(img_y, ya, 0), rn_img_read(img_x, xa, 0), acc);
    acc = rn_mfma(rn_img_read(img_y, ya, 1), rn_img_read(img_x, xa, 1), acc);
    const int lane = rn_lane(), col = lane & 31, h = lane >> 5;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
        if (row < K) atomicAdd(dw_lds + 12672 + row * 64 + xa + col, acc[i] * inv_scale);
    }
}

// gate input layer dW: dH0 rows x 6 inputs (W0 at 0, [64][6])
__device__ __forceinline__ void rn_dw_tile_gate_in(const rn_half* img_y, int ya, const rn_half* img_x,
                                                   float* dw_lds, int out_base, float inv_scale) {
    f32x16 acc = rn_zero16();
    acc = rn_mfma(rn_img_read(img_y, ya, 0), rn_img_read(img_x, 0, 0), acc);
    acc = rn_mfma(rn_img_read(img_y, ya, 1), rn_img_read(img_x, 0, 1), acc);
    const int lane = rn_lane(), col = lane & 31, h = lane >> 5;
    if (col >= 6) return;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
        atomicAdd(dw_lds + (out_base + row) * 6 + col, acc[i] * inv_scale);
    }
}

__global__ void __launch_bounds__(GATE_WAVES * 64)
k_gate_bwd(GateArgs a) {
    __shared__ __attribute__((aligned(16))) rn_half sW[GATE_FRAGS * RN_FRAG_HALFS];
    __shared__ __attribute__((aligned(16))) rn_half sImg[GATE_WAVES * 2 * RN_IMG_HALFS];
    __shared__ __attribute__((aligned(16))) float sDW[GATE_MAX_PARAMS];
    rn_block_copy16(sW, a.frags, GATE_FRAGS * RN_FRAG_BYTES);
    for (int i = threadIdx.x; i < a.n_params; i += blockDim.x) sDW[i] = 0.f;
    __syncthreads();
    const int wid = threadIdx.x / RN_WAVE;
    const int lane = rn_lane(), c = lane & 31, h = lane >> 5;
    rn_half* imgY = sImg + wid * 2 * RN_IMG_HALFS;
    rn_half* imgX = imgY + RN_IMG_HALFS;
    const half8 z8 = rn_zero8();
    const int64_t n_tiles = (a.n_rays + 31) / 32;
    for (int64_t tile = (int64_t)blockIdx.x * GATE_WAVES + wid; tile < n_tiles;
         tile += (int64_t)gridDim.x * GATE_WAVES) {
        rn_lds_order();   // weights stay in LDS: no hoisting of fragment reads
        const int64_t r = tile * 32 + c;
        const bool valid = r < a.n_rays;
        GateState st;
        gate_input(a, r, valid, st.x);
        gate_forward(sW, st);
        const f32x16 p = gate_softmax(st.logit, a.K);
        // softmax backward: dz = p * (dg - sum_j p_j dg_j)
        float dg[16];
        float dot = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
            dg[i] = (valid && row < a.K) ? a.dgate[r * a.K + row] : 0.f;
            dot += p[i] * dg[i];
        }
        dot += __shfl_xor(dot, 32);
        f32x16 dz;
        float dmax = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) { dz[i] = p[i] * (dg[i] - dot); dmax = fmaxf(dmax, fabsf(dz[i])); }
        const float gscale = rn_wave_grad_scale(dmax);
        const float ginv = 1.0f / gscale;
#pragma unroll
        for (int i = 0; i < 16; ++i) dz[i] *= gscale;
        half8 dz0, dz1;
        rn_acc_to_frags<false>(dz, dz0, dz1);   // rows 0..15 in dz0 (K <= 16)
        // dH3 = W4^T dz ; dH2 = W3^T dH3 ; dH1 = W2^T dH2 ; dH0 = W1^T dH1
        half8 dh[4][4];
        {
            f32x16 b0 = rn_zero16(), b1 = rn_zero16();
            b0 = rn_mfma(rn_frag(sW, 30), dz0, b0);
            b1 = rn_mfma(rn_frag(sW, 31), dz0, b1);
            rn_acc_to_frags_masked(b0, st.h[3][0], st.h[3][1], dh[3][0], dh[3][1]);
            rn_acc_to_frags_masked(b1, st.h[3][2], st.h[3][3], dh[3][2], dh[3][3]);
        }
#pragma unroll
        for (int L = 3; L >= 1; --L) {
            const int fb = 32 + 8 * (3 - L);
            f32x16 b0 = rn_zero16(), b1 = rn_zero16();
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                b0 = rn_mfma(rn_frag(sW, fb + q), dh[L][q], b0);
                b1 = rn_mfma(rn_frag(sW, fb + 4 + q), dh[L][q], b1);
            }
            rn_acc_to_frags_masked(b0, st.h[L - 1][0], st.h[L - 1][1], dh[L - 1][0], dh[L - 1][1]);
            rn_acc_to_frags_masked(b1, st.h[L - 1][2], st.h[L - 1][3], dh[L - 1][2], dh[L - 1][3]);
        }
        // input gradient (tcnn Network backward into its input, when the rays
        // require grad): dX = W0^T dH0, rows 0..5 = (in0, in1)
        if (a.dx) {
            f32x16 b = rn_zero16();
#pragma unroll
            for (int q = 0; q < 4; ++q) b = rn_mfma(rn_frag(a.dfrags, q), dh[0][q], b);
            if (valid) {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
                    if (row < 6) a.dx[r * 6 + row] = b[i] * ginv;
                }
            }
        }
        // W4: dY = dz (features 0..15, 16..31 zero), X = H3
        rn_img_write(imgY, 0, dz0); rn_img_write(imgY, 1, z8);
#pragma unroll
        for (int q = 0; q < 4; ++q) rn_img_write(imgX, q, st.h[3][q]);
        rn_lds_order();
        rn_dw_tile_gate_out(imgY, 0, imgX, 0, sDW, a.K, ginv);
        rn_dw_tile_gate_out(imgY, 0, imgX, 32, sDW, a.K, ginv);
        rn_lds_order();
        // W1..W3: dY = dH_L, X = H_{L-1}
#pragma unroll
        for (int L = 1; L <= 3; ++L) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                rn_img_write(imgY, q, dh[L][q]);
                rn_img_write(imgX, q, st.h[L - 1][q]);
            }
            rn_lds_order();
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int nn = 0; nn < 2; ++nn)
                    rn_dw_tile<DW_PLAIN>(imgY, 32 * m, imgX, 32 * nn, sDW, 384 + 4096 * (L - 1),
                                         64, 32 * m, 32 * nn, ginv);
            rn_lds_order();
        }
        // W0: dY = dH0, X = input (features 0..15; 16..31 zero)
#pragma unroll
        for (int q = 0; q < 4; ++q) rn_img_write(imgY, q, dh[0][q]);
        rn_img_write(imgX, 0, st.x); rn_img_write(imgX, 1, z8);
        rn_lds_order();
        rn_dw_tile_gate_in(imgY, 0, imgX, sDW, 0, ginv);
        rn_dw_tile_gate_in(imgY, 32, imgX, sDW, 32, ginv);
        rn_lds_order();
    }
    __syncthreads();
    for (int i = threadIdx.x; i < a.n_params; i += blockDim.x) {
        const float v = sDW[i];
        if (v != 0.f) atomicAdd(&a.dw[i], v);
    }
}

}  // namespace

extern "C" {

int rn_gate_fwd(const float* in0, const float* in1, int32_t stride, int64_t n_rays, int32_t n_models,
                const void* frags, float* gate, float* importance, int32_t n_blocks,
                void* stream) {
    RN_CHECK_ARG(n_rays >= 0 && n_models >= 1 && n_models <= 16 && n_blocks >= 1, "bad sizes");
    if (n_rays == 0) return 0;
    RN_CHECK_ARG(in0 && in1 && frags && gate && stride >= 3, "null pointer / bad stride");
    GateArgs a{};
    a.in0 = in0; a.in1 = in1; a.stride = stride; a.n_rays = n_rays; a.K = n_models;
    a.frags = (const rn_half*)frags; a.gate = gate; a.importance = importance;
    k_gate_fwd<<<n_blocks, GATE_WAVES * 64, 0, (hipStream_t)stream>>>(a);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_gate_bwd(const float* in0, const float* in1, int32_t stride, int64_t n_rays, int32_t n_models,
                const void* frags, const float* dL_dgate, float* dw, int32_t n_params,
                const void* dinput_frags, float* dL_dinput, int32_t n_blocks, void* stream) {
    RN_CHECK_ARG(n_rays >= 0 && n_models >= 1 && n_models <= 16 && n_blocks >= 1, "bad sizes");
    RN_CHECK_ARG(n_params == 12672 + 64 * n_models, "n_params mismatch");
    if (n_rays == 0) return 0;
    RN_CHECK_ARG(in0 && in1 && frags && dL_dgate && dw && stride >= 3,
                 "null pointer / bad stride");
    GateArgs a{};
    a.in0 = in0; a.in1 = in1; a.stride = stride; a.n_rays = n_rays; a.K = n_models;
    a.frags = (const rn_half*)frags; a.dgate = dL_dgate; a.dw = dw;
    a.n_params = n_params;
    RN_CHECK_ARG(!dL_dinput || dinput_frags, "the input gradient needs dinput_frags");
    a.dfrags = (const rn_half*)dinput_frags; a.dx = dL_dinput;
    k_gate_bwd<<<n_blocks, GATE_WAVES * 64, 0, (hipStream_t)stream>>>(a);
    RN_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
