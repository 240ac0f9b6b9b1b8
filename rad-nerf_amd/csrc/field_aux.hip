// Field kernels off the training step's main chain, for gfx950:
//  * k_field_dinput: gradients w.r.t. the field's INPUTS (sample positions and
//    directions).  tcnn's Encoding / Network modules back-propagate into their
//    inputs when those require grad; with --optimize_ext (train_ml.py:90-93)
//    the poses' dR / dT make rays_o / rays_d require grad, and the chain is
//    MNGP.forward (models/networks.py:300-328: clip, hash grid, d / |d|, SH)
//    -> RayMarcher.backward (custom_functions.py:102-112).
//  * k_field_density: MNGP.density(x, ind, return_feat) (networks.py:291-309):
//    hash grid + geo MLP only (no SH / rgb net), sigma and optionally the 16
//    geo features; used by the occupancy-grid update (networks.py:393-394).
//
// dinput, one wave per 32-sample tile (the forward's lane map, rn_field.h):
//  1. forward recompute (encoding cache or gathers) and the dX chain of the
//     MLPs on MFMA (as field.hip's bwd_window, without dW): dL/dencoding and,
//     with four extra transposed fragments of the rgb net's SH columns,
//     dL/dSH;
//  2. dL/dx: the lane re-gathers the 4 corners of its x-half for every level
//     and sums  dE_l . v_c * dw_c/dpos * grid_scale_l  (the trilinear weight
//     derivative; the cell index is piecewise constant), / extent, masked by
//     the clip (torch's clamp passes the gradient on [0, 1] inclusive);
//  3. dL/ddir: the SH degree-4 Jacobian times dL/dSH on (d/|d| + 1)/2 -> x2-1,
//     then through the normalisation: (g - d^ (d^ . g)) / |d|.
#include "rn_field.h"
#pragma clang fp contract(off)

#define DIN_WAVES 4
#define DIN_FRAGS 4        // Wr1[:, 0:16]^T: rows = SH inputs, k = rgb hidden (4 steps)

namespace {

// encoding feature row n (MFMA input order of geo layer 1) of level L, feature f
__device__ __forceinline__ int enc_row(int L, int f) {
    const int q = (L & 1) + 2 * (L >> 2), s = q >> 2, j = 2 * (q & 3) + f, hh = (L >> 1) & 1;
    return 16 * s + 8 * (j >> 2) + 4 * hh + (j & 3);
}

struct Seeds { float o0, o1, o2, gsig; };

__device__ __forceinline__ Seeds field_seeds(const FieldArgs& a, const FwdState& st, bool valid,
                                             int64_t s) {
    Seeds z = {0.f, 0.f, 0.f, 0.f};
    if (valid && (rn_lane() >> 5) == 0) {
        const float y0 = sigmoidf(st.out[0]), y1 = sigmoidf(st.out[1]), y2 = sigmoidf(st.out[2]);
        z.o0 = a.drgb[3 * s] * (y0 * (1.0f - y0));
        z.o1 = a.drgb[3 * s + 1] * (y1 * (1.0f - y1));
        z.o2 = a.drgb[3 * s + 2] * (y2 * (1.0f - y2));
        z.gsig = a.dsigma[s] * expf(fminf(fmaxf(st.g0, -15.f), 15.f));
    }
    return z;
}

// dX chain of one wave's tile: dE (dL/dencoding, accumulator rows) at 1/ginv,
// dSH (rows 0..15 = SH inputs) at 1/rinv.  Wave-local power-of-two scales:
// the rgb chain by its own seeds, the geo chain by all seeds (bwd_window).
__device__ __forceinline__ void dx_chain(const rn_half* sW, const rn_half* sWd, const FwdState& st,
                                         const Seeds& z, f32x16& dE, float& ginv, f32x16& dSH,
                                         float& rinv) {
    const int h = rn_lane() >> 5;
    const half8 z8 = rn_zero8();
    const float mr = rn_wave_max(fmaxf(fmaxf(fabsf(z.o0), fabsf(z.o1)), fabsf(z.o2)));
    const float mg = rn_wave_max(fabsf(z.gsig));
    const float gscale = rn_wave_grad_scale(fmaxf(mr, mg));
    const float rscale = rn_wave_grad_scale(mr);
    half8 dO = z8;
    if (h == 0) {
        dO[0] = (rn_half)(z.o0 * rscale);
        dO[1] = (rn_half)(z.o1 * rscale);
        dO[2] = (rn_half)(z.o2 * rscale);
    }
    half8 dr2f[4], dr1f[4];
    {
        f32x16 b0 = rn_zero16(), b1 = rn_zero16();
        b0 = rn_mfma(rn_frag(sW, 24), dO, b0);
        b1 = rn_mfma(rn_frag(sW, 25), dO, b1);
        rn_acc_to_frags_masked(b0, st.r2[0], st.r2[1], dr2f[0], dr2f[1]);
        rn_acc_to_frags_masked(b1, st.r2[2], st.r2[3], dr2f[2], dr2f[3]);
    }
    {
        f32x16 b0 = rn_zero16(), b1 = rn_zero16();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            b0 = rn_mfma(rn_frag(sW, 26 + q), dr2f[q], b0);
            b1 = rn_mfma(rn_frag(sW, 30 + q), dr2f[q], b1);
        }
        rn_acc_to_frags_masked(b0, st.r1[0], st.r1[1], dr1f[0], dr1f[1]);
        rn_acc_to_frags_masked(b1, st.r1[2], st.r1[3], dr1f[2], dr1f[3]);
    }
    dSH = rn_zero16();
#pragma unroll
    for (int q = 0; q < 4; ++q) dSH = rn_mfma(rn_frag(sWd, q), dr1f[q], dSH);
    half8 dg0, dg1;
    {
        f32x16 b = rn_zero16();
#pragma unroll
        for (int q = 0; q < 4; ++q) b = rn_mfma(rn_frag(sW, 34 + q), dr1f[q], b);
        b *= gscale / rscale;
        if (h == 0) b[8] = z.gsig * gscale;
        rn_acc_to_frags<false>(b, dg0, dg1);
    }
    half8 dh1f[4];
    {
        f32x16 b0 = rn_zero16(), b1 = rn_zero16();
        b0 = rn_mfma(rn_frag(sW, 38), dg0, b0); b0 = rn_mfma(rn_frag(sW, 39), dg1, b0);
        b1 = rn_mfma(rn_frag(sW, 40), dg0, b1); b1 = rn_mfma(rn_frag(sW, 41), dg1, b1);
        rn_acc_to_frags_masked(b0, st.h1[0], st.h1[1], dh1f[0], dh1f[1]);
        rn_acc_to_frags_masked(b1, st.h1[2], st.h1[3], dh1f[2], dh1f[3]);
    }
    dE = rn_zero16();
#pragma unroll
    for (int q = 0; q < 4; ++q) dE = rn_mfma(rn_frag(sW, 42 + q), dh1f[q], dE);
    ginv = 1.0f / gscale;
    rinv = 1.0f / rscale;
}

// dL/du of the lane's sample from its x-half's corners (partial: the other
// half adds its own).  sD: the sample's 32 dL/dencoding values (row order).
__device__ __forceinline__ void encode_grad_lane(const FieldArgs& a, const LvTab& T,
                                                 __amdgpu_buffer_rsrc_t rs, int h, float ux,
                                                 float uy, float uz, bool valid, const float* sD,
                                                 float& gx, float& gy, float& gz) {
    gx = gy = gz = 0.f;
    const float sx = h ? 1.0f : -1.0f;
#pragma unroll
    for (int lb = 0; lb < RN_L; lb += 4) {
        uint32_t raw[16];
        LevelPos P[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const LvConst lc = lv_const(T, a.gm, lb + u);
            P[u] = level_pos(lc.sc, ux, uy, uz);
            const uint32_t ob = valid ? lc.off : (RN_OOB >> 2);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t idx = grid_index(lc, P[u].gx + (uint32_t)h, P[u].gy + (r & 1),
                                                P[u].gz + (r >> 1));
                raw[4 * u + r] = __builtin_amdgcn_raw_buffer_load_b32(rs, (ob + idx) << 2, 0, 0);
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int L = lb + u;
            const float e0 = sD[enc_row(L, 0)], e1 = sD[enc_row(L, 1)];
            const float wx = h ? P[u].fx : 1.0f - P[u].fx;
            float dx = 0.f, dy = 0.f, dz = 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t v = raw[4 * u + r];
                const float v0 = (float)__builtin_bit_cast(rn_half, (uint16_t)(v & 0xffffu));
                const float v1 = (float)__builtin_bit_cast(rn_half, (uint16_t)(v >> 16));
                const float sr = fmaf(e1, v1, e0 * v0);
                const float wy = (r & 1) ? P[u].fy : 1.0f - P[u].fy;
                const float wz = (r >> 1) ? P[u].fz : 1.0f - P[u].fz;
                const float sy = (r & 1) ? 1.0f : -1.0f, sz = (r >> 1) ? 1.0f : -1.0f;
                dx = fmaf(sr, sx * (wy * wz), dx);
                dy = fmaf(sr, wx * sy * wz, dy);
                dz = fmaf(sr, wx * wy * sz, dz);
            }
            const float sc = T.sc[L];
            gx = fmaf(sc, dx, gx); gy = fmaf(sc, dy, gy); gz = fmaf(sc, dz, gz);
        }
    }
}

__device__ __forceinline__ float swap_add(float v) {
    const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                    false);
    return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}

// SH degree 4 (tcnn, sh_lane) Jacobian: the lane's 8 dSH rows -> partial
// dL/d(x, y, z) of the SH input (x = 2 ((d/|d| + 1)/2) - 1)
__device__ __forceinline__ void sh_grad_lane(const f32x16& dSH, float rinv, float x, float y,
                                             float z, float& gx, float& gy, float& gz) {
    const int h = rn_lane() >> 5;
    float g[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) g[i] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
        g[row] = dSH[i] * rinv;
    }
    const float c1 = 0.48860251190291987f, c4 = 1.0925484305920792f, c6 = 0.94617469575755997f,
                c8 = 0.54627421529603959f, c9 = 0.59004358992664352f, c10 = 2.8906114426405538f,
                c11 = 0.45704579946446572f, c12 = 0.3731763325901154f, c14 = 1.4453057213202769f,
                c15 = 0.59004358992664352f;
    const float x2 = x * x, y2 = y * y, z2 = z * z;
    gx = -c1 * g[3] + c4 * y * g[4] - c4 * z * g[7] + 2.0f * c8 * x * g[8]
         - 6.0f * c9 * x * y * g[9] + c10 * y * z * g[10] + c11 * (1.0f - 5.0f * z2) * g[13]
         + 2.0f * c14 * x * z * g[14] + c15 * (3.0f * y2 - 3.0f * x2) * g[15];
    gy = -c1 * g[1] + c4 * x * g[4] - c4 * z * g[5] - 2.0f * c8 * y * g[8]
         + c9 * (3.0f * y2 - 3.0f * x2) * g[9] + c10 * x * z * g[10]
         + c11 * (1.0f - 5.0f * z2) * g[11] - 2.0f * c14 * y * z * g[14] + 6.0f * c15 * x * y * g[15];
    gz = c1 * g[2] - c4 * y * g[5] + 2.0f * c6 * z * g[6] - c4 * x * g[7] + c10 * x * y * g[10]
         - 10.0f * c11 * y * z * g[11] + c12 * (15.0f * z2 - 3.0f) * g[12]
         - 10.0f * c11 * x * z * g[13] + c14 * (x2 - y2) * g[14];
}

template <int MODE, int CACHE>
__global__ void __launch_bounds__(DIN_WAVES * 64)
k_field_dinput(FieldArgs a, const rn_half* __restrict__ dfrags, float* __restrict__ dxyz,
               float* __restrict__ ddir) {
    __shared__ __attribute__((aligned(16))) rn_half sW[FIELD_FRAGS * RN_FRAG_HALFS];
    __shared__ __attribute__((aligned(16))) rn_half sWd[DIN_FRAGS * RN_FRAG_HALFS];
    __shared__ float sD[DIN_WAVES][32][33];
    __shared__ LvTab sT;
    const int k = blockIdx.y;
    rn_block_copy16(sW, a.frags + (size_t)k * FIELD_FRAGS * RN_FRAG_HALFS,
                    FIELD_FRAGS * RN_FRAG_BYTES);
    rn_block_copy16(sWd, dfrags + (size_t)k * DIN_FRAGS * RN_FRAG_HALFS, DIN_FRAGS * RN_FRAG_BYTES);
    lv_stage(sT, a.gm);
    __syncthreads();
    int64_t base, n;
    sample_range(a, MODE, k, base, n);
    const int64_t n_tiles = (n + 31) / 32;
    const int wid = threadIdx.x / RN_WAVE;
    const int lane = rn_lane(), c = lane & 31, h = lane >> 5;
    const __amdgpu_buffer_rsrc_t rs = rn_rsrc(a.grid, a.grid_bytes);
    for (int64_t tile = (int64_t)blockIdx.x * DIN_WAVES + wid; tile < n_tiles;
         tile += (int64_t)gridDim.x * DIN_WAVES) {
        rn_lds_order();
        FwdState st;
        bool valid; int64_t s; float ux, uy, uz;
        tile_forward<MODE, CACHE>(a, sT, sW, base, n, tile, st, valid, s, ux, uy, uz);
        const Seeds z = field_seeds(a, st, valid, s);
        f32x16 dE, dSH;
        float ginv, rinv;
        dx_chain(sW, sWd, st, z, dE, ginv, dSH, rinv);
        // dL/dencoding of the tile's samples -> LDS, row order (feature f)
#pragma unroll
        for (int i = 0; i < 16; ++i) sD[wid][c][(i & 3) + 8 * (i >> 2) + 4 * h] = dE[i] * ginv;
        rn_lds_order();
        float gx, gy, gz;
        encode_grad_lane(a, sT, rs, h, ux, uy, uz, valid, &sD[wid][c][0], gx, gy, gz);
        gx = swap_add(gx); gy = swap_add(gy); gz = swap_add(gz);
        // sample position and direction (again: the loader's registers are gone)
        float x = 0.f, y = 0.f, zz = 0.f, dx = 1.f, dy = 0.f, dz = 0.f;
        if (valid) load_sample<MODE>(a, s, x, y, zz, dx, dy, dz);
        const float nrm = sqrtf(dx * dx + dy * dy + dz * dz);
        const float nx = dx / nrm, ny = dy / nrm, nz = dz / nrm;
        const float shx = fmaf((nx + 1.0f) / 2.0f, 2.0f, -1.0f);
        const float shy = fmaf((ny + 1.0f) / 2.0f, 2.0f, -1.0f);
        const float shz = fmaf((nz + 1.0f) / 2.0f, 2.0f, -1.0f);
        float sgx, sgy, sgz;
        sh_grad_lane(dSH, rinv, shx, shy, shz, sgx, sgy, sgz);
        sgx = swap_add(sgx); sgy = swap_add(sgy); sgz = swap_add(sgz);
        if (valid && h == 0) {
            // networks.py:300-301  clip((x - min) / (max - min), 0, 1)
            const float px = (x - a.xyz_min[0]) / a.extent[0];
            const float py = (y - a.xyz_min[1]) / a.extent[1];
            const float pz = (zz - a.xyz_min[2]) / a.extent[2];
            dxyz[3 * s + 0] = (px >= 0.f && px <= 1.f) ? gx / a.extent[0] : 0.f;
            dxyz[3 * s + 1] = (py >= 0.f && py <= 1.f) ? gy / a.extent[1] : 0.f;
            dxyz[3 * s + 2] = (pz >= 0.f && pz <= 1.f) ? gz / a.extent[2] : 0.f;
            // d (d/|d|): (g - d^ (d^ . g)) / |d|   (the (x+1)/2 -> 2x-1 maps cancel)
            const float dot = nx * sgx + ny * sgy + nz * sgz;
            ddir[3 * s + 0] = (sgx - nx * dot) / nrm;
            ddir[3 * s + 1] = (sgy - ny * dot) / nrm;
            ddir[3 * s + 2] = (sgz - nz * dot) / nrm;
        }
    }
}

// MNGP.density (networks.py:291-309): grid + geo MLP; sigma = TruncExp(h0)
// from the fp32 accumulator (as the full forward), feat = h[1:17] (f16).
__global__ void __launch_bounds__(256)
k_field_density(FieldArgs a, float* __restrict__ feat_out) {
    __shared__ __attribute__((aligned(16))) rn_half sW[8 * RN_FRAG_HALFS];   // geo frags 0..7
    __shared__ LvTab sT;
    rn_block_copy16(sW, a.frags, 8 * RN_FRAG_BYTES);
    lv_stage(sT, a.gm);
    __syncthreads();
    const int64_t n = a.n_fixed;
    const int64_t n_tiles = (n + 31) / 32;
    const int waves = blockDim.x / RN_WAVE;
    const int lane = rn_lane(), c = lane & 31, h = lane >> 5;
    const __amdgpu_buffer_rsrc_t rs = rn_rsrc(a.grid, a.grid_bytes);
    for (int64_t tile = (int64_t)blockIdx.x * waves + threadIdx.x / RN_WAVE; tile < n_tiles;
         tile += (int64_t)gridDim.x * waves) {
        rn_lds_order();
        const int64_t i = tile * 32 + c;
        const bool valid = i < n;
        const int64_t s = valid ? i : 0;
        float x = 0.f, y = 0.f, z = 0.f;
        if (valid) { x = a.xyzs[3 * s]; y = a.xyzs[3 * s + 1]; z = a.xyzs[3 * s + 2]; }
        const float ux = unit_coord(x, a.xyz_min[0], a.extent[0]);
        const float uy = unit_coord(y, a.xyz_min[1], a.extent[1]);
        const float uz = unit_coord(z, a.xyz_min[2], a.extent[2]);
        half8 e0, e1;
        encode_lane(a, sT, rs, h, ux, uy, uz, valid, e0, e1);
        f32x16 a0 = rn_zero16(), a1 = rn_zero16();
        a0 = rn_mfma(rn_frag(sW, 0), e0, a0); a0 = rn_mfma(rn_frag(sW, 1), e1, a0);
        a1 = rn_mfma(rn_frag(sW, 2), e0, a1); a1 = rn_mfma(rn_frag(sW, 3), e1, a1);
        half8 h1[4];
        rn_acc_to_frags<true>(a0, h1[0], h1[1]);
        rn_acc_to_frags<true>(a1, h1[2], h1[3]);
        f32x16 g = rn_zero16();
#pragma unroll
        for (int q = 0; q < 4; ++q) g = rn_mfma(rn_frag(sW, 4 + q), h1[q], g);
        if (!valid) continue;
        if (h == 0) a.sigma[s] = expf(g[8]);
        if (feat_out) {
            // rows 0..15 = geo outputs 1..16: reg i of half h <-> row (i&3) + 8(i>>2) + 4h
#pragma unroll
            for (int i = 0; i < 8; ++i)
                feat_out[16 * s + (i & 3) + 8 * (i >> 2) + 4 * h] = (float)(rn_half)g[i];
        }
    }
}

// ---------------------------------------------------------------------------
// Sampled occupancy-grid update on the device (networks.py:345-409 with
// warmup False, all K sub-NeRFs and C cascades per launch, no host sync).
// The reference draws, per (sub-NeRF k, cascade c), M = G^3/4 uniform cells
// and M cells uniformly among those with density > threshold (with
// replacement), jitters each in its cell, evaluates sigma there and writes it
// with an index_put (density_grid_tmp[c, indices] = sigma, networks.py:394):
// a cell drawn several times keeps ONE of its draws (whichever write lands
// last), and all draws of a cell are i.i.d. jittered points.  So what matters
// per cell is only WHETHER it is drawn, and at which jittered point: here
// cell j of segment (k, c) is drawn with probability 1 - e^-(M / G^3 +
// [occupied] M / n_occupied) (the multinomial counts' Poisson limit: the
// reference's hit rates), decided by a counter-based hash of (seed, k, c, j)
// instead of torch's generator (identical on every rank for the same seed),
// and evaluated once, at the jitter of its first draw.  The drawn cells are
// listed in cell (Morton) order and evaluated in that order, so consecutive
// samples share grid lines as the warm-up's ordered sweep does.
// ---------------------------------------------------------------------------
#define DU_BLK 1024        // cells per counting block (G^3 is a multiple)

__device__ __forceinline__ uint64_t du_mix(uint64_t z) {      // splitmix64 finaliser
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint32_t du_hash(uint64_t seed, uint32_t seg, uint32_t i, uint32_t st) {
    return (uint32_t)(du_mix(seed * 0x9e3779b97f4a7c15ull + (((uint64_t)seg << 32) | i) +
                             (uint64_t)st * 0xd1b54a32d192ed03ull) >> 32);
}
__device__ __forceinline__ float du_unit(uint32_t h) { return (float)(h >> 8) * (1.0f / 16777216.0f); }

// a draw with probability 1 - e^-lam from the uniform word h
__device__ __forceinline__ bool du_hit(float lam, uint32_t h) {
    return lam > 0.f && du_unit(h) >= expf(-lam);
}

struct DensityUpd {
    const float* const* grids;      // [K] -> (C, G3) density grids
    uint8_t* const* bitfields;      // [K] -> C G3 / 8 bytes
    float* tmp;                     // (K, C, G3) sampled sigma, zero on entry
    uint32_t* list;                 // (K C G3) drawn cells, cell-ordered: cell | c << 26
    int32_t* blk;                   // (K C G3 / DU_BLK + 1) occupied counts -> offsets
    int32_t* dblk;                  // (K C G3 / DU_BLK + 1) draw counts -> offsets
    float* part;                    // (K, DU_PART, 2) partial sums / counts of positives
    float* thr_out;                 // [K] packbits threshold min(mean, thr)
    uint64_t seed;
    int K, C, G, M;
    int all;                        // warm-up: every cell drawn
    float thr, decay, scale;
};
#define DU_PART 512

// 1. per-block count of occupied cells (dg > thr) over all (k, c)
__global__ void __launch_bounds__(256)
k_du_count(DensityUpd u) {
    const int64_t G3 = (int64_t)u.G * u.G * u.G, seg_blocks = G3 / DU_BLK;
    const int64_t b = blockIdx.x;
    const int64_t seg = b / seg_blocks, k = seg / u.C, c = seg % u.C;
    const float* g = u.grids[k] + c * G3 + (b % seg_blocks) * DU_BLK;
    int n = 0;
    for (int j = threadIdx.x; j < DU_BLK; j += blockDim.x) n += g[j] > u.thr;
    __shared__ int sN;
    if (threadIdx.x == 0) sN = 0;
    __syncthreads();
    n = (int)rn_wave_sum((float)n);
    if (rn_lane() == 0) atomicAdd(&sN, n);
    __syncthreads();
    if (threadIdx.x == 0) u.blk[b] = sN;
}

// 2. exclusive scan of per-block counts (one block, fixed order); v[nb] = total
__global__ void __launch_bounds__(1024)
k_du_scan(int32_t* __restrict__ v, int nb) {
    __shared__ int sPart[1024];
    const int t = threadIdx.x, per = (nb + 1023) / 1024;
    int acc = 0;
    for (int j = 0; j < per; ++j) { const int q = t * per + j; if (q < nb) acc += v[q]; }
    sPart[t] = acc;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {           // Hillis-Steele, inclusive
        const int x = t >= off ? sPart[t - off] : 0;
        __syncthreads();
        sPart[t] += x;
        __syncthreads();
    }
    int run = t ? sPart[t - 1] : 0;
    for (int j = 0; j < per; ++j) {
        const int q = t * per + j;
        if (q < nb) { const int x = v[q]; v[q] = run; run += x; }
    }
    if (t == 1023) v[nb] = sPart[1023];
}

// is cell j of segment seg drawn (uniform or occupied draws; the occupied
// rate needs the segment's count)?
__device__ __forceinline__ bool du_drawn(const DensityUpd& u, int64_t seg, uint32_t j,
                                         bool occupied, float lam_o) {
    return u.all || du_hit(0.25f, du_hash(u.seed, (uint32_t)seg, j, 0)) ||             // M / G^3
           (occupied && du_hit(lam_o, du_hash(u.seed, (uint32_t)seg, j, 1)));  // M / n_occupied
}

__device__ __forceinline__ float du_lam_occ(const DensityUpd& u, int64_t seg, int64_t seg_blocks) {
    const int32_t no = u.blk[(seg + 1) * seg_blocks] - u.blk[seg * seg_blocks];
    return no > 0 ? (float)u.M / (float)no : 0.f;
}

// 3. per-block count of drawn cells.  MODE 0: counts -> dblk; MODE 1: the
// ordered list (each lane writes its cell at its prefix position)
template <int MODE>
__global__ void __launch_bounds__(256)
k_du_draws(DensityUpd u, int64_t cap) {
    const int64_t G3 = (int64_t)u.G * u.G * u.G, seg_blocks = G3 / DU_BLK;
    const int64_t b = blockIdx.x;
    const int64_t seg = b / seg_blocks, k = seg / u.C, c = seg % u.C;
    const int64_t j0 = (b % seg_blocks) * DU_BLK;
    const float* g = u.grids[k] + c * G3 + j0;
    const float lam_o = du_lam_occ(u, seg, seg_blocks);
    __shared__ int sWave[4];
    int64_t base = MODE ? u.dblk[b] : 0;
    int total = 0;
    for (int j = 0; j < DU_BLK; j += blockDim.x) {
        const uint32_t cell = (uint32_t)(j0 + j + threadIdx.x);
        const int n = du_drawn(u, seg, cell, g[j + threadIdx.x] > u.thr, lam_o) ? 1 : 0;
        if (MODE == 0) { total += n; continue; }
        const int incl = rn_wave_incl_sum_i(n);
        const int w = threadIdx.x / RN_WAVE;
        if (rn_lane() == 63) sWave[w] = incl;
        __syncthreads();
        int before = 0;
        for (int q = 0; q < w; ++q) before += sWave[q];
        const int tot = sWave[0] + sWave[1] + sWave[2] + sWave[3];
        const int64_t p0 = base + before + incl - n;
        if (n && p0 < cap) u.list[p0] = cell | ((uint32_t)c << 26);
        base += tot;
        __syncthreads();
    }
    if (MODE == 0) {
        __shared__ int sN;
        if (threadIdx.x == 0) sN = 0;
        __syncthreads();
        total = (int)rn_wave_sum((float)total);
        if (rn_lane() == 0) atomicAdd(&sN, total);
        __syncthreads();
        if (threadIdx.x == 0) u.dblk[b] = sN;
    }
}

// 4. the drawn cells of sub-NeRF k (blockIdx.y), in cell order: jitter,
// sigma (grid + geo MLP, as k_field_density), tmp[cell] = sigma
__global__ void __launch_bounds__(256)
k_du_sample(FieldArgs a, DensityUpd u, int64_t cap) {
    __shared__ __attribute__((aligned(16))) rn_half sW[8 * RN_FRAG_HALFS];
    __shared__ LvTab sT;
    const int k = blockIdx.y;
    rn_block_copy16(sW, a.frags + (size_t)k * FIELD_FRAGS * RN_FRAG_HALFS, 8 * RN_FRAG_BYTES);
    lv_stage(sT, a.gm);
    __syncthreads();
    const int64_t G3 = (int64_t)u.G * u.G * u.G, seg_blocks = G3 / DU_BLK;
    const int64_t lo = min((int64_t)u.dblk[(int64_t)k * u.C * seg_blocks], cap);
    const int64_t hi = min((int64_t)u.dblk[(int64_t)(k + 1) * u.C * seg_blocks], cap);
    const int64_t n = hi - lo;
    const int64_t n_tiles = (n + 31) / 32;
    const int waves = blockDim.x / RN_WAVE;
    const int lane = rn_lane(), cl = lane & 31, h = lane >> 5;
    const __amdgpu_buffer_rsrc_t rs = rn_rsrc(a.grid, a.grid_bytes);
    for (int64_t tile = (int64_t)blockIdx.x * waves + threadIdx.x / RN_WAVE; tile < n_tiles;
         tile += (int64_t)gridDim.x * waves) {
        rn_lds_order();
        const int64_t q = tile * 32 + cl;
        const bool valid = q < n;
        const uint32_t e = valid ? u.list[lo + q] : 0u;
        const uint32_t cell = e & 0x1fffffu;
        const int c = (int)(e >> 26);
        const int seg = k * u.C + c;
        // networks.py:386-391: cell centre of cascade c, jittered by +-half a cell
        const float sc = fminf(scalbnf(1.0f, c - 1), u.scale);
        const float hgs = sc / u.G;
        const float gm1 = (float)(u.G - 1);
        const float cx = (float)rn_morton3d_invert(cell), cy = (float)rn_morton3d_invert(cell >> 1),
                    cz = (float)rn_morton3d_invert(cell >> 2);
        const uint32_t di = cell << 5;                 // the cell's first draw
        const float jx = du_unit(du_hash(u.seed, seg, di, 2)), jy = du_unit(du_hash(u.seed, seg, di, 3)),
                    jz = du_unit(du_hash(u.seed, seg, di, 4));
        const float x = ((cx / gm1) * 2.0f - 1.0f) * (sc - hgs) + (jx * 2.0f - 1.0f) * hgs;
        const float y = ((cy / gm1) * 2.0f - 1.0f) * (sc - hgs) + (jy * 2.0f - 1.0f) * hgs;
        const float z = ((cz / gm1) * 2.0f - 1.0f) * (sc - hgs) + (jz * 2.0f - 1.0f) * hgs;
        const float ux = unit_coord(x, a.xyz_min[0], a.extent[0]);
        const float uy = unit_coord(y, a.xyz_min[1], a.extent[1]);
        const float uz = unit_coord(z, a.xyz_min[2], a.extent[2]);
        half8 e0, e1;
        encode_lane(a, sT, rs, h, ux, uy, uz, valid, e0, e1);
        f32x16 a0 = rn_zero16(), a1 = rn_zero16();
        a0 = rn_mfma(rn_frag(sW, 0), e0, a0); a0 = rn_mfma(rn_frag(sW, 1), e1, a0);
        a1 = rn_mfma(rn_frag(sW, 2), e0, a1); a1 = rn_mfma(rn_frag(sW, 3), e1, a1);
        half8 h1[4];
        rn_acc_to_frags<true>(a0, h1[0], h1[1]);
        rn_acc_to_frags<true>(a1, h1[2], h1[3]);
        f32x16 gg = rn_zero16();
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) gg = rn_mfma(rn_frag(sW, 4 + qq), h1[qq], gg);
        if (valid && h == 0) u.tmp[(int64_t)seg * G3 + cell] = expf(gg[8]);   // one per cell
    }
}

// 5. grid = dg < 0 ? dg : max(dg * decay, tmp) in place; per-block partial sum
// and count of the positive cells (fixed slots: the mean is deterministic)
__global__ void __launch_bounds__(256)
k_du_decay(DensityUpd u) {
    const int k = blockIdx.y;
    const int64_t n = (int64_t)u.C * u.G * u.G * u.G;
    float* g = const_cast<float*>(u.grids[k]);
    const float* t = u.tmp + (int64_t)k * n;
    float s = 0.f, cnt = 0.f;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
         e += (int64_t)gridDim.x * blockDim.x) {
        const float d = g[e];
        const float v = d < 0.f ? d : fmaxf(d * u.decay, t[e]);
        g[e] = v;
        if (v > 0.f) { s += v; cnt += 1.f; }
    }
    __shared__ float sS[4], sC[4];
    s = rn_wave_sum(s); cnt = rn_wave_sum(cnt);
    const int w = threadIdx.x / RN_WAVE;
    if (rn_lane() == 0) { sS[w] = s; sC[w] = cnt; }
    __syncthreads();
    if (threadIdx.x == 0) {
        u.part[((int64_t)k * DU_PART + blockIdx.x) * 2] = (sS[0] + sS[1]) + (sS[2] + sS[3]);
        u.part[((int64_t)k * DU_PART + blockIdx.x) * 2 + 1] = (sC[0] + sC[1]) + (sC[2] + sC[3]);
    }
}

// 6. mean of the positive densities -> threshold min(mean, thr), per model
__global__ void __launch_bounds__(64)
k_du_mean(DensityUpd u) {
    const int k = blockIdx.x;
    double s = 0.0, c = 0.0;
    if (threadIdx.x == 0) {
        for (int b = 0; b < DU_PART; ++b) {
            s += u.part[((int64_t)k * DU_PART + b) * 2];
            c += u.part[((int64_t)k * DU_PART + b) * 2 + 1];
        }
        const float mean = c > 0.0 ? (float)(s / c) : 0.f;
        u.thr_out[k] = fminf(mean, u.thr);
    }
}

// 7. packbits (raymarching.cu:141-161) at the device threshold
__global__ void __launch_bounds__(256)
k_du_pack(DensityUpd u) {
    const int k = blockIdx.y;
    const int64_t n_bytes = (int64_t)u.C * u.G * u.G * u.G / 8;
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n_bytes) return;
    const float th = u.thr_out[k];
    const float* g = u.grids[k] + 8 * b;
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) bits |= (g[j] > th ? 1u : 0u) << j;
    u.bitfields[k][b] = (uint8_t)bits;
}

inline int nblk(int64_t n, int t) { return (int)((n + t - 1) / t); }

}  // namespace

extern "C" {

int rn_field_dinput(const float* xyzs, const float* dirs, int64_t n_samples, const float* ts,
                    const int32_t* ray_of, const float* rays_o, const float* rays_d,
                    const int32_t* seg_base, const int32_t* seg_count, int32_t n_models,
                    const void* grid_f16, const uint32_t* level_offset,
                    const uint32_t* level_hsize, const uint32_t* level_res,
                    const float* level_scale, const float* xyz_min, const float* extent,
                    const void* frags, const void* dinput_frags, const float* dL_dsigma,
                    const float* dL_drgb, const void* feat_cache, float* dL_dxyz,
                    float* dL_ddir, int32_t blocks_per_model, void* stream) {
    RN_CHECK_ARG(n_models >= 1 && n_samples >= 0 && blocks_per_model >= 1, "bad sizes");
    RN_CHECK_ARG(grid_f16 && level_offset && level_hsize && level_res && level_scale && xyz_min &&
                 extent && frags && dinput_frags && dL_dsigma && dL_drgb && dL_dxyz && dL_ddir,
                 "null pointer");
    FieldArgs a{};
    fill_args(a, xyz_min, extent, level_offset, level_hsize, level_res, level_scale);
    a.grid = (const rn_half*)grid_f16; a.frags = (const rn_half*)frags;
    a.dsigma = dL_dsigma; a.drgb = dL_drgb; a.feat = (rn_half*)feat_cache;
    const rn_half* df = (const rn_half*)dinput_frags;
    dim3 grid(blocks_per_model, n_models);
    hipStream_t st = (hipStream_t)stream;
    if (xyzs) {
        RN_CHECK_ARG(dirs && n_models == 1, "xyz mode needs dirs and a single model");
        if (n_samples == 0) return 0;
        a.xyzs = xyzs; a.dirs = dirs; a.n_fixed = n_samples;
        if (feat_cache) k_field_dinput<0, CACHE_READ><<<grid, DIN_WAVES * 64, 0, st>>>(a, df, dL_dxyz, dL_ddir);
        else k_field_dinput<0, CACHE_NONE><<<grid, DIN_WAVES * 64, 0, st>>>(a, df, dL_dxyz, dL_ddir);
    } else {
        RN_CHECK_ARG(ts && ray_of && rays_o && rays_d && seg_base && seg_count,
                     "compact mode needs ts/ray_of/rays/segments");
        a.ts = ts; a.ray_of = ray_of; a.rays_o = rays_o; a.rays_d = rays_d;
        a.seg_base = seg_base; a.seg_count = seg_count;
        if (feat_cache) k_field_dinput<1, CACHE_READ><<<grid, DIN_WAVES * 64, 0, st>>>(a, df, dL_dxyz, dL_ddir);
        else k_field_dinput<1, CACHE_NONE><<<grid, DIN_WAVES * 64, 0, st>>>(a, df, dL_dxyz, dL_ddir);
    }
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_density_update_sampled(const void* grid_ptrs, const void* bitfield_ptrs, int32_t n_models,
                              int32_t cascades, int32_t grid_size, float scale,
                              float density_threshold, float decay, uint64_t seed,
                              const void* grid_f16, const uint32_t* level_offset,
                              const uint32_t* level_hsize, const uint32_t* level_res,
                              const float* level_scale, const float* xyz_min, const float* extent,
                              const void* frags, float* tmp, int32_t* occ, int32_t* blk,
                              float* part, float* thr_out, int32_t all_cells, void* stream) {
    RN_CHECK_ARG(n_models >= 1 && cascades >= 1 && cascades <= 32 && grid_size == 128,
                 "bad sizes (grid_size 128, cascades <= 32)");
    RN_CHECK_ARG(grid_ptrs && bitfield_ptrs && grid_f16 && level_offset && level_hsize &&
                 level_res && level_scale && xyz_min && extent && frags && tmp && occ && blk &&
                 part && thr_out, "null pointer");
    FieldArgs a{};
    fill_args(a, xyz_min, extent, level_offset, level_hsize, level_res, level_scale);
    a.grid = (const rn_half*)grid_f16; a.frags = (const rn_half*)frags;
    const int64_t G3 = (int64_t)grid_size * grid_size * grid_size;
    const int64_t n_all = (int64_t)n_models * cascades * G3;
    const int nb = (int)(n_all / DU_BLK);
    DensityUpd u{};
    u.grids = (const float* const*)grid_ptrs; u.bitfields = (uint8_t* const*)bitfield_ptrs;
    u.tmp = tmp; u.list = (uint32_t*)occ; u.blk = blk; u.dblk = blk + nb + 1;
    u.part = part; u.thr_out = thr_out;
    u.seed = seed; u.K = n_models; u.C = cascades; u.G = grid_size;
    u.M = (int)(G3 / 4);                                  // networks.py:378: grid_size**3 // 4
    u.thr = density_threshold; u.decay = decay; u.scale = scale;
    u.all = all_cells != 0;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(tmp, 0, sizeof(float) * n_all, st) != hipSuccess) {
        rn_set_error("%s: memset failed", __func__);
        return 2;
    }
    k_du_count<<<nb, 256, 0, st>>>(u);
    k_du_scan<<<1, 1024, 0, st>>>(u.blk, nb);
    k_du_draws<0><<<nb, 256, 0, st>>>(u, n_all);
    k_du_scan<<<1, 1024, 0, st>>>(u.dblk, nb);
    k_du_draws<1><<<nb, 256, 0, st>>>(u, n_all);
    // drawn cells: at most 2 M per (sub-NeRF, cascade) on average (1 - e^-1/4
    // of G^3 plus the occupied ones); the kernel strides over the device count
    const int64_t tiles = ((all_cells ? G3 : 2 * (int64_t)u.M) * cascades + 31) / 32;
    const int sb = (int)(tiles / 4 + 1 < 2048 ? tiles / 4 + 1 : 2048);
    k_du_sample<<<dim3(sb, n_models), 256, 0, st>>>(a, u, n_all);
    k_du_decay<<<dim3(DU_PART, n_models), 256, 0, st>>>(u);
    k_du_mean<<<n_models, 64, 0, st>>>(u);
    k_du_pack<<<dim3(nblk(cascades * G3 / 8, 256), n_models), 256, 0, st>>>(u);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_field_density(const float* xyzs, int64_t n_samples, const void* grid_f16,
                     const uint32_t* level_offset, const uint32_t* level_hsize,
                     const uint32_t* level_res, const float* level_scale, const float* xyz_min,
                     const float* extent, const void* frags, float* sigma, float* geo_feat,
                     void* stream) {
    RN_CHECK_ARG(n_samples >= 0, "bad sizes");
    if (n_samples == 0) return 0;
    RN_CHECK_ARG(xyzs && grid_f16 && level_offset && level_hsize && level_res && level_scale &&
                 xyz_min && extent && frags && sigma, "null pointer");
    FieldArgs a{};
    fill_args(a, xyz_min, extent, level_offset, level_hsize, level_res, level_scale);
    a.grid = (const rn_half*)grid_f16; a.frags = (const rn_half*)frags;
    a.xyzs = xyzs; a.n_fixed = n_samples; a.sigma = sigma;
    const int64_t tiles = (n_samples + 31) / 32;
    const int blocks = (int)(tiles / 4 + 1 < 8192 ? tiles / 4 + 1 : 8192);
    k_field_density<<<blocks, 256, 0, (hipStream_t)stream>>>(a, geo_feat);
    RN_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
