// Fused test-time render for gfx950.
//
// Reference: models/ml_rendering.py:81-155 (__render_rays_test) and
// models/rendering.py:113-189: a host loop that, per iteration, marches
// `step` samples for every alive ray (raymarching.cu:335-404), evaluates the
// field on the valid ones, composites them (volumerendering.cu:206-286,
// T = 1 - opacity at every call) and drops the finished rays.  Every
// iteration is a round of launches plus host synchronisation; the march of a
// ray is the same fixed t sequence whatever `step` is (hits_t carries t).
//
// Here one wave renders one ray from start to finish in tiles of 32 samples:
// march_ray_wave (the same chain walk as the training march, test-time dt
// quirk, negative t1 allowed as the test march does) fills the wave's LDS
// slots with the next <= 32 occupied samples; the field evaluates them as one
// MFMA tile (tile_forward_pos: the forward kernels' arithmetic, so sigma / rgb
// are bit-identical to rn_field_fwd's); the composite folds them serially in
// the reference's order and arithmetic (T = 1 - opacity at the tile start,
// as at the start of each composite_test_fw call) and stops at T <= thr.
// Rays go round-robin over the grid's waves (hundreds of rays per wave at
// image sizes, so their different lengths even out); gridDim.y = sub-NeRF.  No host loop, no compaction, no synchronisation.
//
// Differences from the reference loop, all below float rounding of the
// outputs: the composite restarts T from the opacity every 32 samples instead
// of every `step` samples; `total_samples` counts the samples marched per
// tile (the reference counts per iteration); a ray is capped at max_samples
// samples (the reference caps the loop's summed step sizes, so a ray that
// never terminates gets 1024..1087).
#include "rn_field.h"
#include "rn_march.h"
#pragma clang fp contract(off)

namespace {

#define RT_WAVES 4
#ifndef RT_MIN_BLOCKS
#define RT_MIN_BLOCKS 1      // 2 waves per SIMD (146 VGPRs); 3 (min 2 blocks, 2x the grid) was
                             // slower: 800x800 image 103 -> 111 ms (K 2), 113 -> 134 ms (K 4, scale 16)
#endif

// the wave's tile slots in LDS (march_ray_wave's emitting lanes write them)
struct TileSink {
    float* ts; float* dts;
    __device__ __forceinline__ void emit(int s, float, float, float, float t, float dt) const {
        ts[s] = t; dts[s] = dt;
    }
};

struct RenderArgs {
    const float* hits;            // [B][2]: t1 (NEAR_DISTANCE-clamped), t2
    const uint8_t* bitfields;     // [K][bitfield_bytes]
    int64_t bitfield_bytes;
    MarchCfg mc;
    float* opacity; float* depth; float* rgb;   // [K][B], [K][B], [K][B][3]
    int32_t* n_samples;           // [K][B] samples marched
    int n_rays; int max_samples; float thr;
};

__device__ __forceinline__ float rd_lane(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

__global__ void __launch_bounds__(RT_WAVES * 64, RT_MIN_BLOCKS)
k_render_test(FieldArgs a, RenderArgs g) {
    __shared__ __attribute__((aligned(16))) rn_half sW[FIELD_FWD_FRAGS * RN_FRAG_HALFS];
    __shared__ LvTab sT;
    __shared__ float sTs[RT_WAVES][32], sDt[RT_WAVES][32];
    const int k = blockIdx.y;
    rn_block_copy16(sW, a.frags + (size_t)k * FIELD_FRAGS * RN_FRAG_HALFS,
                    FIELD_FWD_FRAGS * RN_FRAG_BYTES);
    lv_stage(sT, a.gm);
    __syncthreads();
    const int wid = threadIdx.x / RN_WAVE, lane = rn_lane(), c = lane & 31;
    const uint8_t* bits = g.bitfields + (size_t)k * g.bitfield_bytes;
    const TileSink sink{sTs[wid], sDt[wid]};
    // rays round-robin over the grid's waves (the wave index is scalar, so
    // every loop bound below stays wave-uniform)
    const int wave0 = __builtin_amdgcn_readfirstlane(blockIdx.x * RT_WAVES + wid);
    const int n_waves = gridDim.x * RT_WAVES;
    for (int r = wave0; r < g.n_rays; r += n_waves) {
        const float ox = a.rays_o[3 * r], oy = a.rays_o[3 * r + 1], oz = a.rays_o[3 * r + 2];
        const float dx = a.rays_d[3 * r], dy = a.rays_d[3 * r + 1], dz = a.rays_d[3 * r + 2];
        float t = g.hits[2 * r];
        const float t2 = g.hits[2 * r + 1];
        float co = 0.f, cr = 0.f, cg = 0.f, cb = 0.f, cd = 0.f;
        int n_tot = 0, tiles = 0;
        for (;;) {
            if (++tiles > g.max_samples) { n_tot = -1; break; }    // cannot happen: n >= 1 per tile
            const int cap = min(32, g.max_samples - n_tot);
            const int n = __builtin_amdgcn_readfirstlane(march_ray_wave<true, TileSink, true>(
                ox, oy, oz, dx, dy, dz, t, t2, cap, 0, bits, g.mc, sink));
            n_tot += n;
            if (n == 0) break;
            // the slots were written by other lanes of this wave: LDS
            // operations of one wave complete in order; keep the compiler
            // from moving the reads above the writes
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            const bool valid = c < n;
            const float tc = valid ? sTs[wid][c] : 0.f, dtc = valid ? sDt[wid][c] : 0.f;
            // raymarching.cu:376-377: t += dt after an occupied sample
            t = sTs[wid][n - 1] + sDt[wid][n - 1];
            // bit-identical to the march's positions (fmaf(t, d, o))
            const float x = fmaf(tc, dx, ox), y = fmaf(tc, dy, oy), z = fmaf(tc, dz, oz);
            FwdState st;
            float ux, uy, uz;
            tile_forward_pos<CACHE_NONE>(a, sT, sW, x, y, z, dx, dy, dz, valid, nullptr, st,
                                         ux, uy, uz);
            // lanes 0..31 (h == 0) hold sample c's outputs, as rn_field_fwd writes them
            const float sig = expf(st.g0);
            const float r0 = sigmoidf(st.out[0]), r1 = sigmoidf(st.out[1]), r2 = sigmoidf(st.out[2]);
            // volumerendering.cu:206-286 in its order and arithmetic
            float T = 1.0f - co;
            bool stop = false;
            for (int s = 0; s < n; ++s) {
                const float ts_ = rd_lane(tc, s), dl = rd_lane(dtc, s);
                const float al = 1.0f - rn_exp_det(-rd_lane(sig, s) * dl);
                const float w = al * T;
                cr = fmaf(w, rd_lane(r0, s), cr);
                cg = fmaf(w, rd_lane(r1, s), cg);
                cb = fmaf(w, rd_lane(r2, s), cb);
                cd = fmaf(w, ts_, cd);
                co += w;
                T *= 1.0f - al;
                if (T <= g.thr) { stop = true; break; }
            }
            if (stop || n < cap || n_tot >= g.max_samples) break;
            // every lane is done with the slots before the next march rewrites them
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
        if (lane == 0) {
            const size_t o = (size_t)k * g.n_rays + r;
            g.opacity[o] = co; g.depth[o] = cd;
            g.rgb[3 * o] = cr; g.rgb[3 * o + 1] = cg; g.rgb[3 * o + 2] = cb;
            g.n_samples[o] = n_tot;
        }
    }
}

}  // namespace

extern "C" {

int rn_render_test(const float* rays_o, const float* rays_d, const float* hits_t, int64_t n_rays,
                   int32_t n_models, const uint8_t* density_bitfields, int64_t bitfield_bytes,
                   int32_t cascades, float scale, float exp_step_factor, int32_t grid_size,
                   int32_t max_samples, const void* grid_f16, const uint32_t* level_offset,
                   const uint32_t* level_hsize, const uint32_t* level_res,
                   const float* level_scale, const float* xyz_min, const float* extent,
                   const void* frags, float T_threshold, float* opacity,
                   float* depth, float* rgb, int32_t* n_samples, int32_t blocks, void* stream) {
    RN_CHECK_ARG(n_rays >= 0 && n_rays < (1ll << 31) && n_models >= 1 && cascades >= 1 &&
                 grid_size >= 1 && max_samples >= 1 && blocks >= 1 && bitfield_bytes >= 1,
                 "bad sizes");
    if (n_rays == 0) return 0;
    RN_CHECK_ARG(rays_o && rays_d && hits_t && density_bitfields && grid_f16 && level_offset &&
                 level_hsize && level_res && level_scale && xyz_min && extent && frags &&
                 opacity && depth && rgb && n_samples, "null pointer");
    FieldArgs a{};
    fill_args(a, xyz_min, extent, level_offset, level_hsize, level_res, level_scale);
    a.grid = (const rn_half*)grid_f16; a.frags = (const rn_half*)frags;
    a.rays_o = rays_o; a.rays_d = rays_d;
    RenderArgs g{};
    g.hits = hits_t; g.bitfields = density_bitfields; g.bitfield_bytes = bitfield_bytes;
    // raymarching.cu:370,399: the test march hands `cascades` to calc_dt as its scale
    g.mc.cascades = cascades; g.mc.grid_size = grid_size; g.mc.max_samples = max_samples;
    g.mc.scale = scale; g.mc.dt_scale = (float)cascades; g.mc.esf = exp_step_factor; g.mc.abl = 0;
    g.opacity = opacity; g.depth = depth; g.rgb = rgb; g.n_samples = n_samples;
    g.n_rays = (int)n_rays; g.max_samples = max_samples; g.thr = T_threshold;
    hipStream_t st = (hipStream_t)stream;
    k_render_test<<<dim3(blocks, n_models), RT_WAVES * 64, 0, st>>>(a, g);
    RN_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
