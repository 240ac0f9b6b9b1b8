// Occupancy-grid ray marching for gfx950.
//
// Reference: models/csrc/raymarching.cu:166-332 (raymarching_train_kernel),
//            :335-454 (raymarching_test_kernel), intersection.cu:5-56 (AABB).
//
// Differences by design:
//  * deterministic slot allocation: count pass -> exclusive scan -> write pass
//    (the reference allocates with atomicAdd, so its row order is random; we
//    emit rays_a in ray order, start = exclusive prefix of the counts);
//  * outputs are exactly sized; no B*max_samples zero-fill;
//  * the fused multi-sub-NeRF path marches all K sub-NeRFs in one launch,
//    does the ray/AABB test + NEAR_DISTANCE clamp inline, and stores a compact
//    12 B sample record (t, dt, ray) instead of 32 B (xyz, dir, t, dt):
//    xyz is recomputed bit-identically downstream as fmaf(t, d, o).
#include "rn_march.h"
#include "rn_bin.h"      // rn_debug_flags_internal
#pragma clang fp contract(off)

namespace {

// ----------------------------------------------------------------------------
// drop-in path: one sub-NeRF, hits_t given (vren.raymarching_train)
// ----------------------------------------------------------------------------
__device__ __forceinline__ float perturbed_t1(float t1, float noise, const MarchCfg& c) {
    if (t1 >= 0) {  // raymarching.cu:195-198
        const float dt = rn_calc_dt(t1, c.esf, c.max_samples, c.grid_size, c.dt_scale);
        t1 = fmaf(dt, noise, t1);
    }
    return t1;
}

__global__ void __launch_bounds__(256)
k_march_train_count(int n_rays, const float* __restrict__ rays_o, const float* __restrict__ rays_d,
                    const float* __restrict__ hits_t, const float* __restrict__ noise,
                    const uint8_t* __restrict__ bitfield, MarchCfg c, int32_t* __restrict__ counts) {
    const int r = blockIdx.x * (blockDim.x / RN_WAVE) + threadIdx.x / RN_WAVE;   // one wave per ray
    if (r >= n_rays) return;
    const float t1 = perturbed_t1(hits_t[2 * r], noise[r], c);
    const int n = march_ray_wave<false>(rays_o[3 * r], rays_o[3 * r + 1], rays_o[3 * r + 2],
                                        rays_d[3 * r], rays_d[3 * r + 1], rays_d[3 * r + 2],
                                        t1, hits_t[2 * r + 1], c.max_samples, 0, bitfield, c,
                                        NoSink{});
    if (rn_lane() == 0) counts[r] = n;
}

__global__ void __launch_bounds__(256)
k_march_train_write(int n_rays, const float* __restrict__ rays_o, const float* __restrict__ rays_d,
                    const float* __restrict__ hits_t, const float* __restrict__ noise,
                    const uint8_t* __restrict__ bitfield, MarchCfg c,
                    const int32_t* __restrict__ counts, const int32_t* __restrict__ offsets,
                    int64_t* __restrict__ rays_a, float* __restrict__ xyzs,
                    float* __restrict__ dirs, float* __restrict__ deltas, float* __restrict__ ts) {
    const int r = blockIdx.x * (blockDim.x / RN_WAVE) + threadIdx.x / RN_WAVE;   // one wave per ray
    if (r >= n_rays) return;
    const int n = counts[r], start = offsets[r];
    if (rn_lane() == 0) { rays_a[3 * r + 0] = r; rays_a[3 * r + 1] = start; rays_a[3 * r + 2] = n; }
    if (n == 0) return;
    const float dx = rays_d[3 * r], dy = rays_d[3 * r + 1], dz = rays_d[3 * r + 2];
    const float t1 = perturbed_t1(hits_t[2 * r], noise[r], c);
    RefSink sink{xyzs, dirs, ts, deltas, dx, dy, dz};
    march_ray_wave<true>(rays_o[3 * r], rays_o[3 * r + 1], rays_o[3 * r + 2], dx, dy, dz,
                         t1, hits_t[2 * r + 1], n, start, bitfield, c, sink);
}

// ----------------------------------------------------------------------------
// single-block exclusive scan with per-segment alignment.
//   counts: [n_seg][n_per]  ->  offsets (same shape), seg_base[n_seg],
//   seg_count[n_seg], meta[0] = aligned end, meta[1] = unaligned total.
// segment k starts at seg_base[k] = align_up(seg_base[k-1] + seg_count[k-1]).
// ----------------------------------------------------------------------------
__global__ void __launch_bounds__(1024)
k_scan_segments(int n_seg, int n_per, int align, const int32_t* __restrict__ counts,
                int32_t* __restrict__ offsets, int32_t* __restrict__ seg_base,
                int32_t* __restrict__ seg_count, int32_t* __restrict__ meta) {
    // SCAN_PT consecutive elements per thread per pass: one wave scan and one
    // cross-wave scan per SCAN_PT * blockDim elements (a latency-bound chain)
    constexpr int SCAN_PT = 4;
    __shared__ int wsum[16];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int nthr = blockDim.x, nw = nthr >> 6;
    int base = 0, total = 0;
    for (int k = 0; k < n_seg; ++k) {
        const int32_t* cin = counts + (size_t)k * n_per;
        int32_t* cout = offsets + (size_t)k * n_per;
        int carry = 0;
        for (int c0 = 0; c0 < n_per; c0 += nthr * SCAN_PT) {
            const int i0 = c0 + tid * SCAN_PT;
            int v[SCAN_PT], loc = 0;
#pragma unroll
            for (int j = 0; j < SCAN_PT; ++j) {
                v[j] = i0 + j < n_per ? cin[i0 + j] : 0;
                loc += v[j];
            }
            const int incl = rn_wave_incl_sum_i(loc);
            if (lane == 63) wsum[wid] = incl;
            __syncthreads();
            if (wid == 0) {
                int s = lane < nw ? wsum[lane] : 0;
                s = rn_wave_incl_sum_i(s);
                if (lane < nw) wsum[lane] = s;
            }
            __syncthreads();
            int run = base + carry + (wid > 0 ? wsum[wid - 1] : 0) + incl - loc;
#pragma unroll
            for (int j = 0; j < SCAN_PT; ++j) {
                if (i0 + j < n_per) cout[i0 + j] = run;
                run += v[j];
            }
            const int chunk_total = wsum[nw - 1];
            __syncthreads();
            carry += chunk_total;
        }
        if (tid == 0) { seg_base[k] = base; seg_count[k] = carry; }
        total += carry;
        base = ((base + carry + align - 1) / align) * align;
    }
    if (tid == 0) { meta[0] = base; meta[1] = total; }
}

// The same scan with one block per segment (n_seg <= SCAN_PAR_MAX): block k
// sums the counts of segments 0..k (all loads independent, many in flight),
// derives its base from the aligned totals before it, and scans only its own
// segment.  The single block walked the segments one after another, a chain of
// n_seg x n_per / 4096 passes (C5: 16 passes, 0.04 ms).
#define SCAN_PAR_MAX 16
__global__ void __launch_bounds__(1024)
k_scan_segments_par(int n_seg, int n_per, int align, const int32_t* __restrict__ counts,
                    int32_t* __restrict__ offsets, int32_t* __restrict__ seg_base,
                    int32_t* __restrict__ seg_count, int32_t* __restrict__ meta) {
    constexpr int SCAN_PT = 4;
    __shared__ int wpart[16][SCAN_PAR_MAX];
    __shared__ int totals[SCAN_PAR_MAX];
    __shared__ int wsum[16];
    const int k = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int nthr = blockDim.x, nw = nthr >> 6;
    int part[SCAN_PAR_MAX];
#pragma unroll
    for (int j = 0; j < SCAN_PAR_MAX; ++j) part[j] = 0;
    // segments 0..k (block-uniform guards, static indices: part[] stays in
    // registers)
    for (int i = tid; i < n_per; i += nthr) {
#pragma unroll
        for (int j = 0; j < SCAN_PAR_MAX; ++j)
            if (j <= k) part[j] += counts[(size_t)j * n_per + i];
    }
#pragma unroll
    for (int j = 0; j < SCAN_PAR_MAX; ++j) {
        if (j <= k) {
            const int t = rn_wave_incl_sum_i(part[j]);
            if (lane == 63) wpart[wid][j] = t;
        }
    }
    __syncthreads();
    if (tid <= k) {
        int t = 0;
        for (int w = 0; w < nw; ++w) t += wpart[w][tid];
        totals[tid] = t;
    }
    __syncthreads();
    int base = 0, total = 0;
    for (int j = 0; j < k; ++j) {
        base = ((base + totals[j] + align - 1) / align) * align;
        total += totals[j];
    }
    const int32_t* cin = counts + (size_t)k * n_per;
    int32_t* cout = offsets + (size_t)k * n_per;
    int carry = 0;
    for (int c0 = 0; c0 < n_per; c0 += nthr * SCAN_PT) {
        const int i0 = c0 + tid * SCAN_PT;
        int v[SCAN_PT], loc = 0;
#pragma unroll
        for (int j = 0; j < SCAN_PT; ++j) {
            v[j] = i0 + j < n_per ? cin[i0 + j] : 0;
            loc += v[j];
        }
        const int incl = rn_wave_incl_sum_i(loc);
        if (lane == 63) wsum[wid] = incl;
        __syncthreads();
        if (wid == 0) {
            int s = lane < nw ? wsum[lane] : 0;
            s = rn_wave_incl_sum_i(s);
            if (lane < nw) wsum[lane] = s;
        }
        __syncthreads();
        int run = base + carry + (wid > 0 ? wsum[wid - 1] : 0) + incl - loc;
#pragma unroll
        for (int j = 0; j < SCAN_PT; ++j) {
            if (i0 + j < n_per) cout[i0 + j] = run;
            run += v[j];
        }
        const int chunk_total = wsum[nw - 1];
        __syncthreads();
        carry += chunk_total;
    }
    if (tid == 0) {
        seg_base[k] = base; seg_count[k] = carry;
        if (k == n_seg - 1) {
            meta[0] = ((base + carry + align - 1) / align) * align;
            meta[1] = total + carry;
        }
    }
}

// ----------------------------------------------------------------------------
// fused multi-sub-NeRF march (ml_rendering.py:47-52 + __render_rays_train
// :174-179): AABB + NEAR clamp + jitter + count for K sub-NeRFs in one launch.
// thread -> (k, r); bitfields: [K][bitfield_bytes]; noise: [K][B]
// ----------------------------------------------------------------------------
template <bool STAGE>
__global__ void __launch_bounds__(256)
k_ml_march_count(int n_rays, int K, const float* __restrict__ rays_o,
                 const float* __restrict__ rays_d, const float* __restrict__ center,
                 const float* __restrict__ half_size, float near_distance,
                 const float* __restrict__ noise, const uint8_t* __restrict__ bitfields,
                 int64_t bitfield_bytes, MarchCfg c, int32_t* __restrict__ counts,
                 float* __restrict__ stage_ts, float* __restrict__ stage_dt) {
    const int gid = blockIdx.x * (blockDim.x / RN_WAVE) + threadIdx.x / RN_WAVE;  // wave per (k, ray)
    if (gid >= n_rays * K) return;
    const int k = gid / n_rays, r = gid - k * n_rays;
    const float ox = rays_o[3 * r], oy = rays_o[3 * r + 1], oz = rays_o[3 * r + 2];
    const float dx = rays_d[3 * r], dy = rays_d[3 * r + 1], dz = rays_d[3 * r + 2];
    float t1, t2;
    aabb(ox, oy, oz, dx, dy, dz, center, half_size, t1, t2);
    if (!(t2 > 0)) { t1 = -1.0f; t2 = -1.0f; }              // intersection.cu:48
    else { t1 = fmaxf(t1, 0.0f); if (t1 < near_distance) t1 = near_distance; }
    t1 = perturbed_t1(t1, noise[gid], c);
    int n;
    if (STAGE)
        n = march_ray_wave<true>(ox, oy, oz, dx, dy, dz, t1, t2, c.max_samples,
                                 gid * c.max_samples, bitfields + (size_t)k * bitfield_bytes, c,
                                 StageSink{stage_ts, stage_dt});
    else
        n = march_ray_wave<false>(ox, oy, oz, dx, dy, dz, t1, t2, c.max_samples, 0,
                                  bitfields + (size_t)k * bitfield_bytes, c, NoSink{});
    if (rn_lane() == 0) counts[gid] = n;
}

// staged samples -> compact model-major layout at the scanned offsets
__global__ void __launch_bounds__(256)
k_ml_compact(int n_rays, int K, int max_samples, const int32_t* __restrict__ counts,
             const int32_t* __restrict__ offsets, const float* __restrict__ stage_ts,
             const float* __restrict__ stage_dt, float* __restrict__ ts,
             float* __restrict__ deltas, int32_t* __restrict__ ray_of) {
    const int gid = blockIdx.x * (blockDim.x / RN_WAVE) + threadIdx.x / RN_WAVE;
    if (gid >= n_rays * K) return;
    const int r = gid % n_rays;
    const int n = counts[gid], o = offsets[gid];
    const size_t src = (size_t)gid * max_samples;
    for (int i = rn_lane(); i < n; i += RN_WAVE) {
        ts[o + i] = stage_ts[src + i];
        deltas[o + i] = stage_dt[src + i];
        ray_of[o + i] = r;
    }
}

__global__ void __launch_bounds__(256)
k_ml_march_write(int n_rays, int K, const float* __restrict__ rays_o,
                 const float* __restrict__ rays_d, const float* __restrict__ center,
                 const float* __restrict__ half_size, float near_distance,
                 const float* __restrict__ noise, const uint8_t* __restrict__ bitfields,
                 int64_t bitfield_bytes, MarchCfg c, const int32_t* __restrict__ counts,
                 const int32_t* __restrict__ offsets, float* __restrict__ ts,
                 float* __restrict__ deltas, int32_t* __restrict__ ray_of) {
    const int gid = blockIdx.x * (blockDim.x / RN_WAVE) + threadIdx.x / RN_WAVE;  // wave per (k, ray)
    if (gid >= n_rays * K) return;
    const int n = counts[gid];
    if (n == 0) return;
    const int k = gid / n_rays, r = gid - k * n_rays;
    const float ox = rays_o[3 * r], oy = rays_o[3 * r + 1], oz = rays_o[3 * r + 2];
    const float dx = rays_d[3 * r], dy = rays_d[3 * r + 1], dz = rays_d[3 * r + 2];
    float t1, t2;
    aabb(ox, oy, oz, dx, dy, dz, center, half_size, t1, t2);
    t1 = fmaxf(t1, 0.0f);
    if (t1 < near_distance) t1 = near_distance;
    t1 = perturbed_t1(t1, noise[gid], c);
    CompactSink sink{ts, deltas, ray_of, r};
    march_ray_wave<true>(ox, oy, oz, dx, dy, dz, t1, t2, n, offsets[gid],
                         bitfields + (size_t)k * bitfield_bytes, c, sink);
}

// ----------------------------------------------------------------------------
// test-time march (raymarching.cu:335-404) incl. the calc_dt(cascades) quirk
// ----------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
k_march_test(int n_alive, const float* __restrict__ rays_o, const float* __restrict__ rays_d,
             float* __restrict__ hits_t, const int64_t* __restrict__ alive,
             const uint8_t* __restrict__ bitfield, MarchCfg c, int n_samples,
             float* __restrict__ xyzs, float* __restrict__ dirs, float* __restrict__ deltas,
             float* __restrict__ ts, int32_t* __restrict__ n_eff) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= n_alive) return;
    const int64_t r = alive[n];
    const float ox = rays_o[3 * r], oy = rays_o[3 * r + 1], oz = rays_o[3 * r + 2];
    const float dx = rays_d[3 * r], dy = rays_d[3 * r + 1], dz = rays_d[3 * r + 2];
    const float dxi = 1.0f / dx, dyi = 1.0f / dy, dzi = 1.0f / dz;
    float t = hits_t[2 * r];
    const float t2 = hits_t[2 * r + 1];
    int s = 0;
    const size_t row = (size_t)n * n_samples;
    while (t < t2 && s < n_samples) {
        float x, y, z, dt;
        if (march_step(t, ox, oy, oz, dx, dy, dz, dxi, dyi, dzi, bitfield, c, x, y, z, dt)) {
            const size_t o = row + s;
            xyzs[3 * o] = x; xyzs[3 * o + 1] = y; xyzs[3 * o + 2] = z;
            dirs[3 * o] = dx; dirs[3 * o + 1] = dy; dirs[3 * o + 2] = dz;
            ts[o] = t; deltas[o] = dt;
            t += dt;
            hits_t[2 * r] = t;
            s++;
        }
    }
    n_eff[n] = s;
}

// ----------------------------------------------------------------------------
// ray/AABB intersection (intersection.cu:25-100), deterministic: hits for a
// ray are kept in voxel order (first max_hits), then sorted by t_near with
// the reference's torch::sort semantics (unfilled -1 slots sort first).
// ----------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
k_ray_aabb(int n_rays, int n_vox, int max_hits, const float* __restrict__ rays_o,
           const float* __restrict__ rays_d, const float* __restrict__ centers,
           const float* __restrict__ halfs, int32_t* __restrict__ hit_cnt,
           float* __restrict__ hits_t, int64_t* __restrict__ hit_idx) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rays) return;
    const float ox = rays_o[3 * r], oy = rays_o[3 * r + 1], oz = rays_o[3 * r + 2];
    const float dx = rays_d[3 * r], dy = rays_d[3 * r + 1], dz = rays_d[3 * r + 2];
    float* ht = hits_t + (size_t)r * max_hits * 2;
    int64_t* hi = hit_idx + (size_t)r * max_hits;
    for (int m = 0; m < max_hits; ++m) { ht[2 * m] = -1.0f; ht[2 * m + 1] = -1.0f; hi[m] = -1; }
    int cnt = 0;
    for (int v = 0; v < n_vox; ++v) {
        float t1, t2;
        aabb(ox, oy, oz, dx, dy, dz, centers + 3 * v, halfs + 3 * v, t1, t2);
        if (t2 > 0) {
            if (cnt < max_hits) {
                ht[2 * cnt] = fmaxf(t1, 0.0f); ht[2 * cnt + 1] = t2; hi[cnt] = v;
            }
            cnt++;
        }
    }
    hit_cnt[r] = cnt;
    // stable insertion sort of the max_hits slots by t_near (torch::sort asc)
    for (int a = 1; a < max_hits; ++a) {
        const float k0 = ht[2 * a], k1 = ht[2 * a + 1];
        const int64_t kv = hi[a];
        int b = a - 1;
        while (b >= 0 && ht[2 * b] > k0) {
            ht[2 * (b + 1)] = ht[2 * b]; ht[2 * (b + 1) + 1] = ht[2 * b + 1]; hi[b + 1] = hi[b];
            --b;
        }
        ht[2 * (b + 1)] = k0; ht[2 * (b + 1) + 1] = k1; hi[b + 1] = kv;
    }
}

inline MarchCfg make_cfg(int cascades, int grid_size, int max_samples, float scale,
                         float dt_scale, float esf) {
    MarchCfg c;
    c.cascades = cascades; c.grid_size = grid_size; c.max_samples = max_samples;
    c.scale = scale; c.dt_scale = dt_scale; c.esf = esf; c.abl = 0;
    return c;
}

// intersection.cu:103-150 (ray/sphere) with the t_near sort of :191-195.
__global__ void __launch_bounds__(256)
k_ray_sphere(int n_rays, int n_sph, int max_hits, const float* __restrict__ rays_o,
             const float* __restrict__ rays_d, const float* __restrict__ centers,
             const float* __restrict__ radii, int32_t* __restrict__ hit_cnt,
             float* __restrict__ hits_t, int64_t* __restrict__ hit_idx) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rays) return;
    const float ox = rays_o[3 * r], oy = rays_o[3 * r + 1], oz = rays_o[3 * r + 2];
    const float dx = rays_d[3 * r], dy = rays_d[3 * r + 1], dz = rays_d[3 * r + 2];
    float* ht = hits_t + (size_t)r * max_hits * 2;
    int64_t* hi = hit_idx + (size_t)r * max_hits;
    for (int m = 0; m < max_hits; ++m) { ht[2 * m] = -1.0f; ht[2 * m + 1] = -1.0f; hi[m] = -1; }
    const float a = dx * dx + dy * dy + dz * dz;
    int cnt = 0;
    for (int v = 0; v < n_sph; ++v) {
        const float cx = ox - centers[3 * v], cy = oy - centers[3 * v + 1],
                    cz = oz - centers[3 * v + 2];
        const float hb = dx * cx + dy * cy + dz * cz;
        const float c = (cx * cx + cy * cy + cz * cz) - radii[v] * radii[v];
        const float disc = hb * hb - a * c;
        float t1 = -1.0f, t2 = -1.0f;
        if (!(disc < 0)) {
            const float q = sqrtf(disc);
            t1 = (-hb - q) / a;
            t2 = (-hb + q) / a;
        }
        if (t2 > 0) {
            if (cnt < max_hits) {
                ht[2 * cnt] = fmaxf(t1, 0.0f); ht[2 * cnt + 1] = t2; hi[cnt] = v;
            }
            cnt++;
        }
    }
    hit_cnt[r] = cnt;
    for (int i = 1; i < max_hits; ++i) {
        const float k0 = ht[2 * i], k1 = ht[2 * i + 1];
        const int64_t kv = hi[i];
        int b = i - 1;
        while (b >= 0 && ht[2 * b] > k0) {
            ht[2 * (b + 1)] = ht[2 * b]; ht[2 * (b + 1) + 1] = ht[2 * b + 1]; hi[b + 1] = hi[b];
            --b;
        }
        ht[2 * (b + 1)] = k0; ht[2 * (b + 1) + 1] = k1; hi[b + 1] = kv;
    }
}

// RayMarcher.backward (custom_functions.py:102-112, torch_scatter.segment_csr):
// per rays_a row, dL/drays_o = sum dL/dxyz and dL/drays_d = sum (dL/dxyz * t +
// dL/ddir) over the row's samples.  One wave per row, coalesced strided reads.
__global__ void __launch_bounds__(256)
k_march_train_bw(int n_rows, const float* __restrict__ gx, const float* __restrict__ gd,
                 const float* __restrict__ ts, const int64_t* __restrict__ rays_a,
                 float* __restrict__ go, float* __restrict__ gdir) {
    const int row = blockIdx.x * (blockDim.x / RN_WAVE) + (threadIdx.x / RN_WAVE);
    if (row >= n_rows) return;
    const int lane = rn_lane();
    const int64_t start = rays_a[3 * row + 1];
    const int n = (int)rays_a[3 * row + 2];
    float o0 = 0.f, o1 = 0.f, o2 = 0.f, d0 = 0.f, d1 = 0.f, d2 = 0.f;
    for (int i = lane; i < n; i += RN_WAVE) {
        const int64_t s = start + i;
        const float t = ts[s];
        const float x0 = gx[3 * s], x1 = gx[3 * s + 1], x2 = gx[3 * s + 2];
        o0 += x0; o1 += x1; o2 += x2;
        d0 += x0 * t + gd[3 * s]; d1 += x1 * t + gd[3 * s + 1]; d2 += x2 * t + gd[3 * s + 2];
    }
    o0 = rn_wave_sum(o0); o1 = rn_wave_sum(o1); o2 = rn_wave_sum(o2);
    d0 = rn_wave_sum(d0); d1 = rn_wave_sum(d1); d2 = rn_wave_sum(d2);
    if (lane == 0) {
        go[3 * row] = o0; go[3 * row + 1] = o1; go[3 * row + 2] = o2;
        gdir[3 * row] = d0; gdir[3 * row + 1] = d1; gdir[3 * row + 2] = d2;
    }
}

// RayMarcher.backward (custom_functions.py:102-112) for the fused layout: per
// ray, over the K sub-NeRFs' (t, ray) segments, dL/drays_o = sum dL/dxyz and
// dL/drays_d = sum (dL/dxyz t + dL/ddir); sample positions are fmaf(t, d, o).
// Wave per ray, fixed summation order (deterministic).
__global__ void __launch_bounds__(256)
k_ml_march_bw(int n_rays, int K, const int32_t* __restrict__ counts,
              const int32_t* __restrict__ offsets, const float* __restrict__ ts,
              const float* __restrict__ gx, const float* __restrict__ gd,
              float* __restrict__ go, float* __restrict__ gdir) {
    const int r = blockIdx.x * (blockDim.x / RN_WAVE) + (threadIdx.x / RN_WAVE);
    if (r >= n_rays) return;
    const int lane = rn_lane();
    float o0 = 0.f, o1 = 0.f, o2 = 0.f, d0 = 0.f, d1 = 0.f, d2 = 0.f;
    for (int k = 0; k < K; ++k) {
        const int64_t start = offsets[(int64_t)k * n_rays + r];
        const int n = counts[(int64_t)k * n_rays + r];
        for (int i = lane; i < n; i += RN_WAVE) {
            const int64_t s = start + i;
            const float t = ts[s];
            const float x0 = gx[3 * s], x1 = gx[3 * s + 1], x2 = gx[3 * s + 2];
            o0 += x0; o1 += x1; o2 += x2;
            d0 += fmaf(x0, t, gd[3 * s]); d1 += fmaf(x1, t, gd[3 * s + 1]);
            d2 += fmaf(x2, t, gd[3 * s + 2]);
        }
    }
    o0 = rn_wave_sum(o0); o1 = rn_wave_sum(o1); o2 = rn_wave_sum(o2);
    d0 = rn_wave_sum(d0); d1 = rn_wave_sum(d1); d2 = rn_wave_sum(d2);
    if (lane == 0) {
        go[3 * r] = o0; go[3 * r + 1] = o1; go[3 * r + 2] = o2;
        gdir[3 * r] = d0; gdir[3 * r + 1] = d1; gdir[3 * r + 2] = d2;
    }
}

inline int nblk(int64_t n, int t) { return (int)((n + t - 1) / t); }

}  // namespace

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

int rn_ray_aabb_intersect(const float* rays_o, const float* rays_d, const float* centers,
                          const float* half_sizes, int64_t n_rays, int64_t n_voxels,
                          int32_t max_hits, int32_t* hit_cnt, float* hits_t,
                          int64_t* hits_voxel_idx, void* stream) {
    RN_CHECK_ARG(n_rays >= 0 && n_voxels >= 0 && max_hits >= 1, "bad sizes");
    if (n_rays == 0) return 0;
    RN_CHECK_ARG(rays_o && rays_d && centers && half_sizes && hit_cnt && hits_t && hits_voxel_idx,
                 "null pointer");
    k_ray_aabb<<<nblk(n_rays, 256), 256, 0, (hipStream_t)stream>>>(
        (int)n_rays, (int)n_voxels, max_hits, rays_o, rays_d, centers, half_sizes, hit_cnt,
        hits_t, hits_voxel_idx);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_raymarching_train_count(const float* rays_o, const float* rays_d, const float* hits_t,
                               const uint8_t* density_bitfield, int32_t cascades, float scale,
                               float exp_step_factor, const float* noise, int32_t grid_size,
                               int32_t max_samples, int64_t n_rays, int32_t* counts,
                               void* stream) {
    RN_CHECK_ARG(n_rays >= 0 && cascades >= 1 && grid_size >= 1 && grid_size <= 1024 &&
                 max_samples >= 1, "bad sizes");
    if (n_rays == 0) return 0;
    RN_CHECK_ARG(rays_o && rays_d && hits_t && density_bitfield && noise && counts, "null pointer");
    MarchCfg c = make_cfg(cascades, grid_size, max_samples, scale, scale, exp_step_factor);
    k_march_train_count<<<nblk(n_rays, 4), 256, 0, (hipStream_t)stream>>>(
        (int)n_rays, rays_o, rays_d, hits_t, noise, density_bitfield, c, counts);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_scan_segments(const int32_t* counts, int32_t n_seg, int64_t n_per, int32_t align,
                     int32_t* offsets, int32_t* seg_base, int32_t* seg_count, int32_t* meta,
                     void* stream) {
    RN_CHECK_ARG(n_seg >= 1 && n_per >= 0 && align >= 1, "bad sizes");
    RN_CHECK_ARG(counts && offsets && seg_base && seg_count && meta, "null pointer");
    // (two segments: the single block's four passes measured 0.014 ms against
    // 0.016; K = 8 at C5 0.041 -> 0.029)
    if (n_seg > 2 && n_seg <= SCAN_PAR_MAX)
        k_scan_segments_par<<<n_seg, 1024, 0, (hipStream_t)stream>>>(
            n_seg, (int)n_per, align, counts, offsets, seg_base, seg_count, meta);
    else
        k_scan_segments<<<1, 1024, 0, (hipStream_t)stream>>>(n_seg, (int)n_per, align, counts,
                                                             offsets, seg_base, seg_count, meta);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_raymarching_train_write(const float* rays_o, const float* rays_d, const float* hits_t,
                               const uint8_t* density_bitfield, int32_t cascades, float scale,
                               float exp_step_factor, const float* noise, int32_t grid_size,
                               int32_t max_samples, int64_t n_rays, const int32_t* counts,
                               const int32_t* offsets, int64_t* rays_a, float* xyzs, float* dirs,
                               float* deltas, float* ts, void* stream) {
    RN_CHECK_ARG(n_rays >= 0 && cascades >= 1 && grid_size >= 1 && max_samples >= 1, "bad sizes");
    if (n_rays == 0) return 0;
    RN_CHECK_ARG(rays_o && rays_d && hits_t && density_bitfield && noise && counts && offsets &&
                 rays_a, "null pointer");
    MarchCfg c = make_cfg(cascades, grid_size, max_samples, scale, scale, exp_step_factor);
    k_march_train_write<<<nblk(n_rays, 4), 256, 0, (hipStream_t)stream>>>(
        (int)n_rays, rays_o, rays_d, hits_t, noise, density_bitfield, c, counts, offsets, rays_a,
        xyzs, dirs, deltas, ts);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_raymarching_test(const float* rays_o, const float* rays_d, float* hits_t,
                        const int64_t* alive_indices, int64_t n_alive,
                        const uint8_t* density_bitfield, int32_t cascades, float scale,
                        float exp_step_factor, int32_t grid_size, int32_t max_samples,
                        int32_t n_samples, float* xyzs, float* dirs, float* deltas, float* ts,
                        int32_t* n_eff_samples, void* stream) {
    RN_CHECK_ARG(n_alive >= 0 && cascades >= 1 && grid_size >= 1 && max_samples >= 1 &&
                 n_samples >= 1, "bad sizes");
    if (n_alive == 0) return 0;
    RN_CHECK_ARG(rays_o && rays_d && hits_t && alive_indices && density_bitfield && xyzs && dirs &&
                 deltas && ts && n_eff_samples, "null pointer");
    // raymarching.cu:370,399: calc_dt receives `cascades` as its scale argument
    MarchCfg c = make_cfg(cascades, grid_size, max_samples, scale, (float)cascades,
                          exp_step_factor);
    k_march_test<<<nblk(n_alive, 256), 256, 0, (hipStream_t)stream>>>(
        (int)n_alive, rays_o, rays_d, hits_t, alive_indices, density_bitfield, c, n_samples, xyzs,
        dirs, deltas, ts, n_eff_samples);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_ml_march_count(const float* rays_o, const float* rays_d, const float* center,
                      const float* half_size, float near_distance, const float* noise,
                      const uint8_t* density_bitfields, int64_t bitfield_bytes, int32_t n_models,
                      int32_t cascades, float scale, float exp_step_factor, int32_t grid_size,
                      int32_t max_samples, int64_t n_rays, int32_t* counts, float* stage_ts,
                      float* stage_deltas, void* stream) {
    RN_CHECK_ARG(n_rays >= 0 && n_models >= 1 && cascades >= 1 && grid_size >= 1 &&
                 max_samples >= 1, "bad sizes");
    RN_CHECK_ARG((stage_ts == nullptr) == (stage_deltas == nullptr), "stage_ts/stage_deltas: both or neither");
    RN_CHECK_ARG(n_rays * n_models * (int64_t)max_samples < (int64_t)1 << 31, "staging too large");
    RN_CHECK_ARG(bitfield_bytes >= (int64_t)cascades * grid_size * grid_size * grid_size / 8,
                 "bitfield too small");
    if (n_rays == 0) return 0;
    RN_CHECK_ARG(rays_o && rays_d && center && half_size && noise && density_bitfields && counts,
                 "null pointer");
    MarchCfg c = make_cfg(cascades, grid_size, max_samples, scale, scale, exp_step_factor);
    c.abl = rn_dbg(rn_debug_flags_internal() >> 24) & 1;
    if (stage_ts)
        k_ml_march_count<true><<<nblk(n_rays * n_models, 4), 256, 0, (hipStream_t)stream>>>(
            (int)n_rays, n_models, rays_o, rays_d, center, half_size, near_distance, noise,
            density_bitfields, bitfield_bytes, c, counts, stage_ts, stage_deltas);
    else
        k_ml_march_count<false><<<nblk(n_rays * n_models, 4), 256, 0, (hipStream_t)stream>>>(
            (int)n_rays, n_models, rays_o, rays_d, center, half_size, near_distance, noise,
            density_bitfields, bitfield_bytes, c, counts, nullptr, nullptr);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_ml_march_write(const float* rays_o, const float* rays_d, const float* center,
                      const float* half_size, float near_distance, const float* noise,
                      const uint8_t* density_bitfields, int64_t bitfield_bytes, int32_t n_models,
                      int32_t cascades, float scale, float exp_step_factor, int32_t grid_size,
                      int32_t max_samples, int64_t n_rays, const int32_t* counts,
                      const int32_t* offsets, float* ts, float* deltas, int32_t* ray_of,
                      void* stream) {
    RN_CHECK_ARG(n_rays >= 0 && n_models >= 1 && cascades >= 1 && grid_size >= 1 &&
                 max_samples >= 1, "bad sizes");
    if (n_rays == 0) return 0;
    RN_CHECK_ARG(rays_o && rays_d && center && half_size && noise && density_bitfields && counts &&
                 offsets && ts && deltas && ray_of, "null pointer");
    MarchCfg c = make_cfg(cascades, grid_size, max_samples, scale, scale, exp_step_factor);
    k_ml_march_write<<<nblk(n_rays * n_models, 4), 256, 0, (hipStream_t)stream>>>(
        (int)n_rays, n_models, rays_o, rays_d, center, half_size, near_distance, noise,
        density_bitfields, bitfield_bytes, c, counts, offsets, ts, deltas, ray_of);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_ml_compact(const int32_t* counts, const int32_t* offsets, int64_t n_rays, int32_t n_models,
                  int32_t max_samples, const float* stage_ts, const float* stage_deltas,
                  float* ts, float* deltas, int32_t* ray_of, void* stream) {
    RN_CHECK_ARG(n_rays >= 0 && n_models >= 1 && max_samples >= 1, "bad sizes");
    if (n_rays == 0) return 0;
    RN_CHECK_ARG(counts && offsets && stage_ts && stage_deltas && ts && deltas && ray_of,
                 "null pointer");
    k_ml_compact<<<nblk(n_rays * n_models, 4), 256, 0, (hipStream_t)stream>>>(
        (int)n_rays, n_models, max_samples, counts, offsets, stage_ts, stage_deltas, ts, deltas,
        ray_of);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_ray_sphere_intersect(const float* rays_o, const float* rays_d, const float* centers,
                            const float* radii, int64_t n_rays, int64_t n_spheres,
                            int32_t max_hits, int32_t* hit_cnt, float* hits_t,
                            int64_t* hits_sphere_idx, void* stream) {
    RN_CHECK_ARG(n_rays >= 0 && n_spheres >= 0 && max_hits >= 1, "bad sizes");
    if (n_rays == 0) return 0;
    RN_CHECK_ARG(rays_o && rays_d && hit_cnt && hits_t && hits_sphere_idx, "null pointer");
    RN_CHECK_ARG(n_spheres == 0 || (centers && radii), "null pointer");
    k_ray_sphere<<<nblk(n_rays, 256), 256, 0, (hipStream_t)stream>>>(
        (int)n_rays, (int)n_spheres, max_hits, rays_o, rays_d, centers, radii, hit_cnt, hits_t,
        hits_sphere_idx);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_raymarching_train_bw(const float* dL_dxyzs, const float* dL_ddirs, const float* ts,
                            const int64_t* rays_a, int64_t n_rows, float* dL_drays_o,
                            float* dL_drays_d, void* stream) {
    RN_CHECK_ARG(n_rows >= 0, "bad sizes");
    if (n_rows == 0) return 0;
    RN_CHECK_ARG(dL_dxyzs && dL_ddirs && ts && rays_a && dL_drays_o && dL_drays_d,
                 "null pointer");
    k_march_train_bw<<<nblk(n_rows, 4), 256, 0, (hipStream_t)stream>>>(
        (int)n_rows, dL_dxyzs, dL_ddirs, ts, rays_a, dL_drays_o, dL_drays_d);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_ml_march_bw(const int32_t* counts, const int32_t* offsets, int64_t n_rays,
                   int32_t n_models, const float* ts, const float* dL_dxyzs,
                   const float* dL_ddirs, float* dL_drays_o, float* dL_drays_d, void* stream) {
    RN_CHECK_ARG(n_rays >= 0 && n_models >= 1, "bad sizes");
    if (n_rays == 0) return 0;
    RN_CHECK_ARG(counts && offsets && ts && dL_dxyzs && dL_ddirs && dL_drays_o && dL_drays_d,
                 "null pointer");
    k_ml_march_bw<<<nblk(n_rays, 4), 256, 0, (hipStream_t)stream>>>(
        (int)n_rays, n_models, counts, offsets, ts, dL_dxyzs, dL_ddirs, dL_drays_o, dL_drays_d);
    RN_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
