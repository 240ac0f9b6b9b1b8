// Field device code shared by field.hip (forward / backward / merged kernels)
// and field_aux.hip (input gradients, density-only evaluation): level tables,
// the hash-grid encoder, SH, the MFMA MLP forward and the sample loaders.
// Reference: models/networks.py:229-328 (see field.hip header).
#pragma once
#include "rn_mlp.h"
#pragma clang fp contract(off)

#define RN_L 16
#define FIELD_FWD_FRAGS 24
#define FIELD_FRAGS 46
#define FIELD_PARAMS 9472
#define FIELD_DW_TILES 12
#ifndef FWD_MIN_WAVES
#define FWD_MIN_WAVES 2
#endif

struct GridMeta {
    uint32_t offset[RN_L];  // level offset in entries (1 entry = 2 halfs)
    uint32_t hsize[RN_L];   // entries in level (tcnn params_in_level)
    uint32_t res[RN_L];     // grid resolution
    float scale[RN_L];      // tcnn grid_scale (host-computed fp32)
    uint32_t dense_mask;    // bit l set: dense indexing
    uint32_t pow2_mask;     // bit l set: hsize is a power of two
};

struct FieldArgs {
    // sample inputs: MODE 0 = xyzs/dirs arrays, MODE 1 = compact (t, ray)
    const float* xyzs; const float* dirs;
    const float* ts; const int32_t* ray_of; const float* rays_o; const float* rays_d;
    const int32_t* seg_base; const int32_t* seg_count;   // per model, device (MODE 1)
    int64_t n_fixed;                                      // MODE 0 sample count
    const rn_half* grid;      // [entries][2] f16
    float* grid_grad;         // [entries][2] f32
    const rn_half* frags;     // [K][FIELD_FRAGS][512]
    float* dw;                // [K][FIELD_PARAMS]
    float* sigma; float* rgb; // forward outputs
    const float* dsigma; const float* drgb;               // backward seeds
    rn_half* feat;            // optional encoding cache: [sample tiles][64 lanes][16] f16
    const uint32_t* planes;   // level-partitioned encoding: [16 levels][plane_stride] f16x2
    int64_t plane_stride;
    float xyz_min[3]; float extent[3];
    uint32_t grid_bytes;      // byte size of the f16 table (= of the f32 grad / 2)
    int dbg;                  // ablation flags (rn_set_debug_flags), 0 in production
    GridMeta gm;
};

namespace {


__device__ __forceinline__ void sample_range(const FieldArgs& a, int MODE, int k, int64_t& base,
                                             int64_t& n) {
    if (MODE == 0) { base = 0; n = a.n_fixed; }
    else { base = a.seg_base[k]; n = a.seg_count[k]; }
}

// load the sample's position and direction
template <int MODE>
__device__ __forceinline__ void load_sample(const FieldArgs& a, int64_t s, float& x, float& y,
                                            float& z, float& dx, float& dy, float& dz) {
    if (MODE == 0) {
        x = a.xyzs[3 * s]; y = a.xyzs[3 * s + 1]; z = a.xyzs[3 * s + 2];
        dx = a.dirs[3 * s]; dy = a.dirs[3 * s + 1]; dz = a.dirs[3 * s + 2];
    } else {
        // ablation 8192 (timing only): no dependent ray lookup
        const int r = (rn_dbg(a.dbg) & 8192) ? 0 : a.ray_of[s];
        const float t = a.ts[s];
        dx = a.rays_d[3 * r]; dy = a.rays_d[3 * r + 1]; dz = a.rays_d[3 * r + 2];
        // bit-identical to the march's sample position (march.hip march_step)
        x = fmaf(t, dx, a.rays_o[3 * r]);
        y = fmaf(t, dy, a.rays_o[3 * r + 1]);
        z = fmaf(t, dz, a.rays_o[3 * r + 2]);
    }
}

// networks.py:300-301  x = clip((x - xyz_min) / (xyz_max - xyz_min), 0, 1)
__device__ __forceinline__ float unit_coord(float v, float mn, float ext) {
    return fminf(fmaxf((v - mn) / ext, 0.0f), 1.0f);
}

__device__ __forceinline__ int lane_level(int q, int h) { return 2 * h + (q & 1) + 4 * (q >> 1); }

// Level table staged in LDS: lanes index it with a lane-dependent level, which
// from the kernel-argument segment would be a global load per access.
struct LvTab {
    uint32_t off[RN_L];
    uint32_t hs[RN_L];
    uint32_t res[RN_L];
    uint32_t res2[RN_L];
    float sc[RN_L];
};

__device__ __forceinline__ void lv_stage(LvTab& t, const GridMeta& gm) {
    const int i = threadIdx.x;
    if (i < RN_L) {
        t.off[i] = gm.offset[i]; t.hs[i] = gm.hsize[i]; t.res[i] = gm.res[i]; t.sc[i] = gm.scale[i];
        t.res2[i] = gm.res[i] * gm.res[i];
    }
}

// Per-lane constants of one level, hoisted out of sample loops.
struct LvConst {
    uint32_t off, hs, res, res2;
    float sc;
    bool dense;
};

__device__ __forceinline__ LvConst lv_const(const LvTab& T, const GridMeta& gm, int l) {
    LvConst c;
    c.off = T.off[l]; c.hs = T.hs[l]; c.res = T.res[l]; c.res2 = T.res2[l]; c.sc = T.sc[l];
    c.dense = (gm.dense_mask >> l) & 1u;
    return c;
}

// tcnn grid_index (Linear, coherent prime hash), branch-free.  Dense levels:
// index < res^3 + res^2 + res < 2*hsize, so `% hsize` is one conditional
// subtract; hashed levels have hsize = 2^log2_T, so it is a mask.
__device__ __forceinline__ uint32_t grid_index(const LvConst& c, uint32_t x, uint32_t y, uint32_t z) {
    // dense levels: res <= 128 (res^3 <= hsize), so u24 multiplies are exact
    const uint32_t di = x + __umul24(y, c.res) + __umul24(z, c.res2);
    const uint32_t hi = x ^ (y * 2654435761u) ^ (z * 805459861u);
    const uint32_t dm = di >= c.hs ? di - c.hs : di;
    return c.dense ? dm : (hi & (c.hs - 1u));
}

struct LevelPos { uint32_t gx, gy, gz; float fx, fy, fz; };

__device__ __forceinline__ LevelPos level_pos(float sc, float ux, float uy, float uz) {
    LevelPos p;
    float px = fmaf(sc, ux, 0.5f), py = fmaf(sc, uy, 0.5f), pz = fmaf(sc, uz, 0.5f);
    // cell = floor, fraction = p - floor(p): v_cvt_flr_i32_f32 + v_fract_f32
    // per axis (floor, convert and subtract took three).  p >= 0.5 (unit
    // coordinates are clamped to [0, 1]), where p - floor(p) is exact and
    // below 1, which is what v_fract_f32 returns
    // (the compiler keeps floor + convert: v_cvt_flr_i32_f32 written out)
    auto cvt_flr = [](float v) {
        int r;
        asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(v));
        return (uint32_t)r;
    };
    p.gx = cvt_flr(px); p.gy = cvt_flr(py); p.gz = cvt_flr(pz);
    p.fx = __builtin_amdgcn_fractf(px); p.fy = __builtin_amdgcn_fractf(py); p.fz = __builtin_amdgcn_fractf(pz);
    return p;
}

__device__ __forceinline__ float corner_weight(const LevelPos& p, int c) {
    float w = 1.0f;
    w *= (c & 1) ? p.fx : 1.0f - p.fx;
    w *= (c & 2) ? p.fy : 1.0f - p.fy;
    w *= (c & 4) ? p.fz : 1.0f - p.fz;
    return w;
}

__device__ __forceinline__ uint32_t corner_index(const LvConst& c, const LevelPos& p, int corner) {
    return grid_index(c, p.gx + (corner & 1), p.gy + ((corner >> 1) & 1), p.gz + ((corner >> 2) & 1));
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rn_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes,
                                             0x00020000);
}

#define RN_OOB 0x80000000u   // buffer offset past num_records: load returns 0

// hash-grid encoding of the tile's 32 samples -> the two B fragments.
//
// Lane (c, h): sample c.  For every level the lane gathers the corners with
// x bit = h of the 4 (y, z) rows, so ONE gather instruction covers the two
// x-neighbours of a row for 32 samples: both sit in one 128-B line almost
// always, and the cost of a gather instruction on gfx950 is its number of
// distinct lines (measured: the same stream with every lane of an instruction
// in one line runs as fast as with no memory access at all, r01 ablation
// f1024).  28 lines/sample instead of 53 with one corner of two levels per
// instruction (tools/atomic_sim.py's replay of the bench samples).  A lane
// per (sample, level) with all 8 corners does 40 % less VALU work (position
// and row hash once per sample) but is 5 % slower: its instructions touch
// twice the lines (profiles/r01/ablate_fwd_levelsplit.json).
// The two x-halves of each level are summed across the wave halves with
// v_permlane32_swap (x0 half first, so both lanes hold the same value); each
// lane keeps the 8 levels of its B-fragment rows (lane_level).
// Gathers: 32-bit buffer offsets, 4 levels (16 loads) in flight per batch;
// invalid lanes read out of range (zero, no memory access).
__device__ __forceinline__ void encode_lane(const FieldArgs& a, const LvTab& T,
                                            __amdgpu_buffer_rsrc_t rs, int h, float ux, float uy,
                                            float uz, bool valid, half8& e0, half8& e1) {
    float f[16];
    const bool load = valid && !(rn_dbg(a.dbg) & 128);
#pragma unroll
    for (int lb = 0; lb < RN_L; lb += 4) {
        // per level: the cell's x, the weights' fractions, and the x-free part
        // of tcnn grid_index for the 4 (y, z) rows: dense levels
        // y res + z res^2 (+ res / res^2; u24 exact, res <= 128), hashed
        // y P1 ^ z P2 with (y+1) P1 = y P1 + P1.  Both wave halves need them
        // for the same sample, so each half computes one level of a pair and
        // v_permlane32_swap hands it to the other (lanes 0-31: level lb + up,
        // lanes 32-63: lb + up + 1).
        uint32_t GX[4], ROW[4][4];
        float FX[4], FY[4], FZ[4];
#pragma unroll
        for (int up = 0; up < 4; up += 2) {
            const LvConst lm = lv_const(T, a.gm, lb + up + h);
            const LevelPos p = level_pos(lm.sc, ux, uy, uz);
            uint32_t rw[4];
            if (lm.dense) {
                const uint32_t b = __umul24(p.gy, lm.res) + __umul24(p.gz, lm.res2);
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    rw[r] = b + ((r & 1) ? lm.res : 0u) + ((r >> 1) ? lm.res2 : 0u);
            } else {
                const uint32_t y0 = p.gy * 2654435761u, z0 = p.gz * 805459861u;
                const uint32_t y1 = y0 + 2654435761u, z1 = z0 + 805459861u;
#pragma unroll
                for (int r = 0; r < 4; ++r) rw[r] = ((r & 1) ? y1 : y0) ^ ((r >> 1) ? z1 : z0);
            }
            auto xch = [&](uint32_t v, uint32_t& lo, uint32_t& hi) {
                const auto r2 = __builtin_amdgcn_permlane32_swap(v, v, false, false);
                lo = r2[0]; hi = r2[1];
            };
            uint32_t t0, t1;
            xch(p.gx, GX[up], GX[up + 1]);
            xch(__float_as_uint(p.fx), t0, t1); FX[up] = __uint_as_float(t0); FX[up + 1] = __uint_as_float(t1);
            xch(__float_as_uint(p.fy), t0, t1); FY[up] = __uint_as_float(t0); FY[up + 1] = __uint_as_float(t1);
            xch(__float_as_uint(p.fz), t0, t1); FZ[up] = __uint_as_float(t0); FZ[up + 1] = __uint_as_float(t1);
#pragma unroll
            for (int r = 0; r < 4; ++r) xch(rw[r], ROW[up][r], ROW[up + 1][r]);
        }
        uint32_t off[16];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            // the lane's 4 corners of level lb + u: x = gx + h on the 4 rows.
            // The level is wave-uniform here, so only one branch runs.
            const LvConst lc = lv_const(T, a.gm, lb + u);
            const uint32_t x = GX[u] + (uint32_t)h;
            uint32_t idx[4];
            if (lc.dense) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const uint32_t d = x + ROW[u][r];
                    idx[r] = min(d, d - lc.hs);      // d >= hs ? d - hs : d  (d < 2 hs)
                }
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) idx[r] = (x ^ ROW[u][r]) & (lc.hs - 1u);
            }
            // one v_add_lshl per corner; invalid lanes start past num_records
            // (the table is < 2^31 B)
            const uint32_t ob = load ? lc.off : (RN_OOB >> 2);
#pragma unroll
            for (int r = 0; r < 4; ++r) off[4 * u + r] = (ob + idx[r]) << 2;
        }
        uint32_t raw[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) raw[i] = __builtin_amdgcn_raw_buffer_load_b32(rs, off[i], 0, 0);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            float a0 = 0.f, a1 = 0.f;
            // corner weight (wx * wy) * wz, tcnn's dimension order
            const float wx = h ? FX[u] : 1.0f - FX[u];
            const float wy0 = 1.0f - FY[u], wz0 = 1.0f - FZ[u];
            const float wxy0 = wx * wy0, wxy1 = wx * FY[u];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float w = ((r & 1) ? wxy1 : wxy0) * ((r >> 1) ? FZ[u] : wz0);
                const uint32_t v = raw[4 * u + r];
                a0 = fmaf(w, (float)__builtin_bit_cast(rn_half, (uint16_t)(v & 0xffffu)), a0);
                a1 = fmaf(w, (float)__builtin_bit_cast(rn_half, (uint16_t)(v >> 16)), a1);
            }
            // x0 half (lanes 0-31) + x1 half (lanes 32-63), same order in both
            const auto s0 = __builtin_amdgcn_permlane32_swap(__float_as_uint(a0), __float_as_uint(a0), false, false);
            const auto s1 = __builtin_amdgcn_permlane32_swap(__float_as_uint(a1), __float_as_uint(a1), false, false);
            const float v0 = __uint_as_float(s0[0]) + __uint_as_float(s0[1]);
            const float v1 = __uint_as_float(s1[0]) + __uint_as_float(s1[1]);
            // level L = lb + u belongs to the lanes with h == (L >> 1) & 1, at
            // k-slot q = (L & 1) + 2 * (L >> 2)
            const int L = lb + u, q = (L & 1) + 2 * (L >> 2);
            if (((L >> 1) & 1) == h) { f[2 * q] = v0; f[2 * q + 1] = v1; }
        }
        // keep at most one batch of gathers in flight per wave: bounds VGPRs so
        // more waves fit (TLP hides the L2/MALL latency instead of ILP)
#ifndef FWD_NO_SCHED_BARRIER
        __builtin_amdgcn_sched_barrier(0);
#endif
    }
    // element j of k-step s <-> level lane_level(4s + (j>>1), h), feature j&1
#pragma unroll
    for (int j = 0; j < 8; ++j) { e0[j] = (rn_half)f[j]; e1[j] = (rn_half)f[8 + j]; }
}

// A level's constants for a wave-uniform level index, in SGPRs
__device__ __forceinline__ LvConst lv_const_uniform(const LvTab& T, const GridMeta& gm, int l) {
    const LvConst c = lv_const(T, gm, l);
    LvConst u;
    u.off = (uint32_t)__builtin_amdgcn_readfirstlane((int)c.off);
    u.hs = (uint32_t)__builtin_amdgcn_readfirstlane((int)c.hs);
    u.res = (uint32_t)__builtin_amdgcn_readfirstlane((int)c.res);
    u.res2 = (uint32_t)__builtin_amdgcn_readfirstlane((int)c.res2);
    u.sc = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(c.sc)));
    u.dense = c.dense;
    return u;
}

// One level of two tiles (32 samples each), the same arithmetic per (sample,
// level) as encode_lane (bit-identical features): wave half h computes the
// cell position and row hashes of sample c of tile h, v_permlane32_swap hands
// them across, every lane gathers the 4 rows of its x-half for both tiles,
// and the x-halves are summed with a second swap.  The level is wave-uniform
// (lv_const_uniform): dense / hashed are scalar branches.  valid0 / valid1:
// sample c of tile 0 / 1 exists (invalid samples gather nothing).  Returns
// the features of the lane's own sample (tile h) as packed f16x2.
// (Round 3 first paired two levels per tile instead: an XCD then gathered from
// both its levels' tables at once, 4 MB for two hashed levels = its whole L2.)
__device__ __forceinline__ uint32_t encode_tiles(const FieldArgs& a, __amdgpu_buffer_rsrc_t rs,
                                                 int h, const LvConst& L, float ux, float uy,
                                                 float uz, bool valid0, bool valid1) {
    uint32_t GX[2], ROW[2][4];
    float FX[2], FY[2], FZ[2];
    const int dn = __builtin_amdgcn_readfirstlane((int)L.dense);
    {
        const LevelPos p = level_pos(L.sc, ux, uy, uz);
        uint32_t rw[4];
        if (dn) {                                // scalar branch
            const uint32_t b = __umul24(p.gy, L.res) + __umul24(p.gz, L.res2);
#pragma unroll
            for (int r = 0; r < 4; ++r) rw[r] = b + ((r & 1) ? L.res : 0u) + ((r >> 1) ? L.res2 : 0u);
        } else {
            const uint32_t y0 = p.gy * 2654435761u, z0 = p.gz * 805459861u;
            const uint32_t y1 = y0 + 2654435761u, z1 = z0 + 805459861u;
#pragma unroll
            for (int r = 0; r < 4; ++r) rw[r] = ((r & 1) ? y1 : y0) ^ ((r >> 1) ? z1 : z0);
        }
        auto xch = [&](uint32_t v, uint32_t& lo, uint32_t& hi) {
            const auto r2 = __builtin_amdgcn_permlane32_swap(v, v, false, false);
            lo = r2[0]; hi = r2[1];
        };
        uint32_t t0, t1;
        xch(p.gx, GX[0], GX[1]);
        xch(__float_as_uint(p.fx), t0, t1); FX[0] = __uint_as_float(t0); FX[1] = __uint_as_float(t1);
        xch(__float_as_uint(p.fy), t0, t1); FY[0] = __uint_as_float(t0); FY[1] = __uint_as_float(t1);
        xch(__float_as_uint(p.fz), t0, t1); FZ[0] = __uint_as_float(t0); FZ[1] = __uint_as_float(t1);
#pragma unroll
        for (int r = 0; r < 4; ++r) xch(rw[r], ROW[0][r], ROW[1][r]);
    }
    const bool noload = rn_dbg(a.dbg) & 128;
    uint32_t off[8];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const uint32_t x = GX[u] + (uint32_t)h;
        const uint32_t ob = ((u ? valid1 : valid0) && !noload) ? L.off : (RN_OOB >> 2);
        if (dn) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t d = x + ROW[u][r];
                off[4 * u + r] = (ob + min(d, d - L.hs)) << 2;
            }
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) off[4 * u + r] = (ob + ((x ^ ROW[u][r]) & (L.hs - 1u))) << 2;
        }
    }
    uint32_t raw[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) raw[i] = __builtin_amdgcn_raw_buffer_load_b32(rs, off[i], 0, 0);
    uint32_t res = 0u;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        float a0 = 0.f, a1 = 0.f;
        const float wx = h ? FX[u] : 1.0f - FX[u];
        const float wy0 = 1.0f - FY[u], wz0 = 1.0f - FZ[u];
        const float wxy0 = wx * wy0, wxy1 = wx * FY[u];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float w = ((r & 1) ? wxy1 : wxy0) * ((r >> 1) ? FZ[u] : wz0);
            const uint32_t v = raw[4 * u + r];
            a0 = fmaf(w, (float)__builtin_bit_cast(rn_half, (uint16_t)(v & 0xffffu)), a0);
            a1 = fmaf(w, (float)__builtin_bit_cast(rn_half, (uint16_t)(v >> 16)), a1);
        }
        const auto s0 = __builtin_amdgcn_permlane32_swap(__float_as_uint(a0), __float_as_uint(a0), false, false);
        const auto s1 = __builtin_amdgcn_permlane32_swap(__float_as_uint(a1), __float_as_uint(a1), false, false);
        const float v0 = __uint_as_float(s0[0]) + __uint_as_float(s0[1]);
        const float v1 = __uint_as_float(s1[0]) + __uint_as_float(s1[1]);
        const uint32_t pk = (uint32_t)__builtin_bit_cast(uint16_t, (rn_half)v0) |
                            ((uint32_t)__builtin_bit_cast(uint16_t, (rn_half)v1) << 16);
        if (u == h) res = pk;
    }
    return res;
}

// tcnn SphericalHarmonics degree 4 on (d/|d| + 1)/2 (networks.py:324-325)
__device__ __forceinline__ half8 sh_lane(float dx, float dy, float dz, int h) {
    const float n = sqrtf(dx * dx + dy * dy + dz * dz);
    const float x = fmaf((dx / n + 1.0f) / 2.0f, 2.0f, -1.0f);
    const float y = fmaf((dy / n + 1.0f) / 2.0f, 2.0f, -1.0f);
    const float z = fmaf((dz / n + 1.0f) / 2.0f, 2.0f, -1.0f);
    const float xy = x * y, xz = x * z, yz = y * z, x2 = x * x, y2 = y * y, z2 = z * z;
    float o[16];
    o[0] = 0.28209479177387814f;
    o[1] = -0.48860251190291987f * y;
    o[2] = 0.48860251190291987f * z;
    o[3] = -0.48860251190291987f * x;
    o[4] = 1.0925484305920792f * xy;
    o[5] = -1.0925484305920792f * yz;
    o[6] = 0.94617469575755997f * z2 - 0.31539156525251999f;
    o[7] = -1.0925484305920792f * xz;
    o[8] = 0.54627421529603959f * x2 - 0.54627421529603959f * y2;
    o[9] = 0.59004358992664352f * y * (-3.0f * x2 + y2);
    o[10] = 2.8906114426405538f * xy * z;
    o[11] = 0.45704579946446572f * y * (1.0f - 5.0f * z2);
    o[12] = 0.3731763325901154f * z * (5.0f * z2 - 3.0f);
    o[13] = 0.45704579946446572f * x * (1.0f - 5.0f * z2);
    o[14] = 1.4453057213202769f * z * (x2 - y2);
    o[15] = 0.59004358992664352f * x * (-x2 + 3.0f * y2);
    half8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int c0 = 8 * (j >> 2) + (j & 3);  // h = 0 coefficient; h = 1 adds 4
        r[j] = (rn_half)(h ? o[c0 + 4] : o[c0]);
    }
    return r;
}

struct FwdState {
    half8 e0, e1;          // encoding (k-steps 0, 1)
    half8 h1[4];           // geo hidden (ReLU, f16)
    half8 gin;             // geo outputs 1..16 (f16) = rgb-net input k-step 1
    half8 sh;              // SH (f16)             = rgb-net input k-step 0
    half8 r1[4], r2[4];    // rgb hidden
    float g0;              // geo output 0 (fp32 accumulator), lanes h == 0
    f32x16 out;            // rgb pre-activation (rows 0..2 on lanes h == 0)
};

// forward MLP chain on a 32-sample tile; frag base in LDS
__device__ __forceinline__ void mlp_forward(const rn_half* W, FwdState& st) {
    // geo layer 1: 32 -> 64
    f32x16 a0 = rn_zero16(), a1 = rn_zero16();
    a0 = rn_mfma(rn_frag(W, 0), st.e0, a0); a0 = rn_mfma(rn_frag(W, 1), st.e1, a0);
    a1 = rn_mfma(rn_frag(W, 2), st.e0, a1); a1 = rn_mfma(rn_frag(W, 3), st.e1, a1);
    rn_acc_to_frags<true>(a0, st.h1[0], st.h1[1]);
    rn_acc_to_frags<true>(a1, st.h1[2], st.h1[3]);
    // geo layer 2: 64 -> 17 (acc rows 0..15 = outputs 1..16, row 16 = output 0)
    f32x16 g = rn_zero16();
#pragma unroll
    for (int q = 0; q < 4; ++q) g = rn_mfma(rn_frag(W, 4 + q), st.h1[q], g);
    half8 gk1;
    rn_acc_to_frags<false>(g, st.gin, gk1);
    // sigma = TruncExp(h0) from the fp32 accumulator (wider than tcnn's f16
    // output; acc reg 8 of lanes h == 0 is row 16 = geo output 0)
    st.g0 = g[8];
    // rgb layer 1: [SH | geo 1..16] -> 64
    a0 = rn_zero16(); a1 = rn_zero16();
    a0 = rn_mfma(rn_frag(W, 8), st.sh, a0); a0 = rn_mfma(rn_frag(W, 9), st.gin, a0);
    a1 = rn_mfma(rn_frag(W, 10), st.sh, a1); a1 = rn_mfma(rn_frag(W, 11), st.gin, a1);
    rn_acc_to_frags<true>(a0, st.r1[0], st.r1[1]);
    rn_acc_to_frags<true>(a1, st.r1[2], st.r1[3]);
    // rgb layer 2: 64 -> 64
    a0 = rn_zero16(); a1 = rn_zero16();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        a0 = rn_mfma(rn_frag(W, 12 + q), st.r1[q], a0);
        a1 = rn_mfma(rn_frag(W, 16 + q), st.r1[q], a1);
    }
    rn_acc_to_frags<true>(a0, st.r2[0], st.r2[1]);
    rn_acc_to_frags<true>(a1, st.r2[2], st.r2[3]);
    // rgb layer 3: 64 -> 3
    st.out = rn_zero16();
#pragma unroll
    for (int q = 0; q < 4; ++q) st.out = rn_mfma(rn_frag(W, 20 + q), st.r2[q], st.out);
}

__device__ __forceinline__ float sigmoidf(float x) { return 1.0f / (1.0f + expf(-x)); }

enum { CACHE_NONE = 0, CACHE_WRITE = 1, CACHE_READ = 2,
       CACHE_READ_NT = 3,     // READ past L1: written by other waves of this kernel
       CACHE_PLANES = 4 };    // encoding from the level planes; the cache slot (if any) written

// forward of one 32-sample tile for the lanes' samples `s` (valid lanes only
// load); fc: this lane's encoding-cache slot (CACHE_WRITE writes it on every
// lane, CACHE_READ reads it on valid lanes)
template <int CACHE>
__device__ __forceinline__ void tile_forward_pos(const FieldArgs& a, const LvTab& T, const rn_half* W,
                                                 float x, float y, float z, float dx, float dy,
                                                 float dz, bool valid, half8* fc, FwdState& st,
                                                 float& ux, float& uy, float& uz);

template <int MODE, int CACHE>
__device__ __forceinline__ void tile_forward_s(const FieldArgs& a, const LvTab& T, const rn_half* W,
                                               int64_t s, bool valid, half8* fc, FwdState& st,
                                               float& ux, float& uy, float& uz) {
    float x = 0.f, y = 0.f, z = 0.f, dx = 1.f, dy = 0.f, dz = 0.f;
    if (CACHE == CACHE_PLANES) {
        // lane (c, h) holds levels lane_level(q, h), q = 0..7: e0 = q 0-3, e1 = q 4-7
        const int h = rn_lane() >> 5;
        typedef uint32_t u4v __attribute__((ext_vector_type(4)));
        u4v w0 = {0u, 0u, 0u, 0u}, w1 = {0u, 0u, 0u, 0u};
        if (valid) {
            const uint32_t* pl = a.planes + s;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                w0[q] = pl[(size_t)lane_level(q, h) * a.plane_stride];
                w1[q] = pl[(size_t)lane_level(q + 4, h) * a.plane_stride];
            }
        }
        st.e0 = __builtin_bit_cast(half8, w0); st.e1 = __builtin_bit_cast(half8, w1);
    }
    if (valid) load_sample<MODE>(a, s, x, y, z, dx, dy, dz);
    tile_forward_pos<CACHE>(a, T, W, x, y, z, dx, dy, dz, valid, fc, st, ux, uy, uz);
}

// MODE 1 with the chunk's rays [r0, r0 + nr) staged in LDS (6 floats per ray:
// origin, direction): the ray lookup of a sample is an LDS read instead of a
// second dependent global load; rays outside the table (nr = 0: the chunk had
// too many) come from global memory.  Same arithmetic as load_sample<1>.
template <int CACHE>
__device__ __forceinline__ void tile_forward_rays(const FieldArgs& a, const LvTab& T,
                                                  const rn_half* W, int64_t s, bool valid,
                                                  half8* fc, const float* sRays, int r0, int nr,
                                                  FwdState& st, float& ux, float& uy, float& uz) {
    float x = 0.f, y = 0.f, z = 0.f, dx = 1.f, dy = 0.f, dz = 0.f;
    if (valid) {
        const int r = a.ray_of[s];
        const float t = a.ts[s];
        const uint32_t q = (uint32_t)(r - r0);
        float ox, oy, oz;
        if (q < (uint32_t)nr) {
            typedef __attribute__((address_space(3))) const float lds_f;
            lds_f* p = (lds_f*)sRays + 6 * q;
            ox = p[0]; oy = p[1]; oz = p[2]; dx = p[3]; dy = p[4]; dz = p[5];
        } else {
            ox = a.rays_o[3 * r]; oy = a.rays_o[3 * r + 1]; oz = a.rays_o[3 * r + 2];
            dx = a.rays_d[3 * r]; dy = a.rays_d[3 * r + 1]; dz = a.rays_d[3 * r + 2];
        }
        x = fmaf(t, dx, ox);
        y = fmaf(t, dy, oy);
        z = fmaf(t, dz, oz);
    }
    tile_forward_pos<CACHE>(a, T, W, x, y, z, dx, dy, dz, valid, fc, st, ux, uy, uz);
}

// the same for positions / directions already in registers (invalid lanes:
// any finite values; their gathers are skipped)
template <int CACHE>
__device__ __forceinline__ void tile_forward_pos(const FieldArgs& a, const LvTab& T, const rn_half* W,
                                                 float x, float y, float z, float dx, float dy,
                                                 float dz, bool valid, half8* fc, FwdState& st,
                                                 float& ux, float& uy, float& uz) {
    const int h = rn_lane() >> 5;
    ux = unit_coord(x, a.xyz_min[0], a.extent[0]);
    uy = unit_coord(y, a.xyz_min[1], a.extent[1]);
    uz = unit_coord(z, a.xyz_min[2], a.extent[2]);
    if (CACHE == CACHE_PLANES) {
        // st.e0 / st.e1 were loaded from the level planes (tile_forward_s)
        if (valid && fc) { fc[0] = st.e0; fc[1] = st.e1; }
    } else if (CACHE == CACHE_READ || CACHE == CACHE_READ_NT) {
        // lanes past the segment end (the backward walks whole 8-tile
        // iterations) were never written: zero encoding, as the gather path
        st.e0 = rn_zero8(); st.e1 = rn_zero8();
        if (valid && CACHE == CACHE_READ) { st.e0 = fc[0]; st.e1 = fc[1]; }
        if (valid && CACHE == CACHE_READ_NT) {
            st.e0 = __builtin_nontemporal_load(fc);
            st.e1 = __builtin_nontemporal_load(fc + 1);
        }
    } else {
        if (rn_dbg(a.dbg) & 256) { st.e0 = rn_zero8(); st.e1 = rn_zero8(); asm volatile("" :: "v"(ux), "v"(uy), "v"(uz)); }
        else encode_lane(a, T, rn_rsrc(a.grid, a.grid_bytes), h, ux, uy, uz, valid, st.e0, st.e1);
        if (CACHE == CACHE_WRITE && valid) { fc[0] = st.e0; fc[1] = st.e1; }
    }
    st.sh = sh_lane(dx, dy, dz, h);
    if (rn_dbg(a.dbg) & 4096) {                 // ablation: no MLP (outputs are garbage)
        st.out = rn_zero16(); st.g0 = 0.f;
        asm volatile("" :: "v"(st.e0), "v"(st.e1), "v"(st.sh));
    } else {
        mlp_forward(W, st);
    }
}

// encoding-cache slot of global sample s: 32-sample tiles of the sample
// array, lane-linear (lane c + 32h holds sample c's k-steps of half h)
__device__ __forceinline__ half8* cache_slot(const FieldArgs& a, int64_t s) {
    return reinterpret_cast<half8*>(a.feat) + ((s >> 5) * 64 + (s & 31) + 32 * (rn_lane() >> 5)) * 2;
}

template <int MODE, int CACHE>
__device__ __forceinline__ void tile_forward(const FieldArgs& a, const LvTab& T, const rn_half* W,
                                             int64_t base, int64_t n, int64_t tile, FwdState& st,
                                             bool& valid, int64_t& s, float& ux, float& uy,
                                             float& uz) {
    const int lane = rn_lane(), c = lane & 31;
    const int64_t i = tile * 32 + c;
    valid = i < n;
    s = base + (valid ? i : 0);
    // the encoding cache is indexed by 32-sample tile of the global sample
    // array (segment bases are 128-aligned); lane-linear, 32 B per lane
    half8* fc = CACHE == CACHE_NONE ? nullptr
              : reinterpret_cast<half8*>(a.feat) + (((base >> 5) + tile) * 64 + lane) * 2;
    tile_forward_s<MODE, CACHE>(a, T, W, s, valid, fc, st, ux, uy, uz);
}

// host: kernel arguments from the C-ABI level table
int fill_args(FieldArgs& a, const float* xyz_min, const float* extent, const uint32_t* offsets,
              const uint32_t* hsize, const uint32_t* res, const float* scale) {
    for (int d = 0; d < 3; ++d) { a.xyz_min[d] = xyz_min[d]; a.extent[d] = extent[d]; }
    a.gm.dense_mask = 0;
    a.gm.pow2_mask = 0;
    a.grid_bytes = 4u * (offsets[RN_L - 1] + hsize[RN_L - 1]);
    for (int l = 0; l < RN_L; ++l) {
        a.gm.offset[l] = offsets[l]; a.gm.hsize[l] = hsize[l]; a.gm.res[l] = res[l];
        a.gm.scale[l] = scale[l];
        const uint64_t r = res[l];
        if (r * r * r <= (uint64_t)hsize[l]) a.gm.dense_mask |= 1u << l;
        if (hsize[l] && (hsize[l] & (hsize[l] - 1u)) == 0) a.gm.pow2_mask |= 1u << l;
    }
    return 0;
}

}  // namespace
