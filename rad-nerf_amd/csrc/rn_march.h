// Occupancy-grid march device code shared by march.hip (training / test
// marches) and render.hip (fused test-time render): the reference's step
// (raymarching.cu:200-279, :364-395) and the wave-per-ray chain walk.
#pragma once
#include "rn_common.h"
#pragma clang fp contract(off)

namespace {

struct MarchCfg {
    int cascades;
    int grid_size;
    int max_samples;
    float scale;      // used for mip_bound and (train) calc_dt
    float dt_scale;   // `scale` argument handed to calc_dt (== cascades for test)
    float esf;
    int abl;          // timing studies only (debug bit 24): 1 = no t chain (wrong t)
};

struct NoSink {
    __device__ __forceinline__ void emit(int, float, float, float, float, float) const {}
};

// xyz/dir/t/dt sink with the reference layout (raymarching.cu:265-267)
struct RefSink {
    float* __restrict__ xyzs; float* __restrict__ dirs;
    float* __restrict__ ts;   float* __restrict__ deltas;
    float dx, dy, dz;
    __device__ __forceinline__ void emit(int s, float x, float y, float z, float t, float dt) const {
        xyzs[3 * s + 0] = x; xyzs[3 * s + 1] = y; xyzs[3 * s + 2] = z;
        dirs[3 * s + 0] = dx; dirs[3 * s + 1] = dy; dirs[3 * s + 2] = dz;
        ts[s] = t; deltas[s] = dt;
    }
};

// staging sink of the single-pass fused march: per-(model, ray) slots of
// max_samples records (t, dt), compacted after the scan by k_ml_compact
struct StageSink {
    float* __restrict__ ts; float* __restrict__ deltas;
    __device__ __forceinline__ void emit(int s, float, float, float, float t, float dt) const {
        ts[s] = t; deltas[s] = dt;
    }
};

// compact sink for the fused path: t, dt and owning ray
struct CompactSink {
    float* __restrict__ ts; float* __restrict__ deltas; int32_t* __restrict__ ray_of;
    int ray;
    __device__ __forceinline__ void emit(int s, float, float, float, float t, float dt) const {
        ts[s] = t; deltas[s] = dt; ray_of[s] = ray;
    }
};

// 1 / mip_bound with mip_bound = fminf(2^(mip-1), scale) (raymarching.cu:
// 213-214), bit-exact without a per-query division: the reciprocal of a power
// of two is exact, and 1 / scale is loop-invariant
__device__ __forceinline__ float mip_bound_inv(int mip, float scale) {
    return scalbnf(1.0f, mip - 1) < scale ? scalbnf(1.0f, 1 - mip) : 1.0f / scale;
}

// One occupancy query + step of raymarching.cu:205-233.  Returns true if the
// cell at t is occupied; otherwise advances t past the cell exit.
__device__ __forceinline__ bool march_step(float& t, float ox, float oy, float oz,
                                           float dx, float dy, float dz,
                                           float dxi, float dyi, float dzi,
                                           const uint8_t* __restrict__ bitfield,
                                           const MarchCfg& c, float& x, float& y,
                                           float& z, float& dt) {
    const uint32_t g3 = (uint32_t)c.grid_size * c.grid_size * c.grid_size;
    const float gsi = 1.0f / c.grid_size;
    x = fmaf(t, dx, ox); y = fmaf(t, dy, oy); z = fmaf(t, dz, oz);
    dt = rn_calc_dt(t, c.esf, c.max_samples, c.grid_size, c.dt_scale);
    const int mip = max(rn_mip_from_pos(x, y, z, c.cascades),
                        rn_mip_from_dt(dt, c.grid_size, c.cascades));
    const float mb = fminf(scalbnf(1.0f, mip - 1), c.scale);
    const float mbi = mip_bound_inv(mip, c.scale);
    const float gm1 = c.grid_size - 1.0f;
    const int nx = (int)rn_clampf(0.5f * fmaf(x, mbi, 1.0f) * c.grid_size, 0.0f, gm1);
    const int ny = (int)rn_clampf(0.5f * fmaf(y, mbi, 1.0f) * c.grid_size, 0.0f, gm1);
    const int nz = (int)rn_clampf(0.5f * fmaf(z, mbi, 1.0f) * c.grid_size, 0.0f, gm1);
    const uint32_t idx = mip * g3 + rn_morton3d(nx, ny, nz);
    const bool occ = bitfield[idx / 8] & (1 << (idx % 8));
    if (occ) return true;
    const float tx = fmaf(fmaf(fmaf(0.5f, rn_signf(dx), nx + 0.5f) * gsi, 2.0f, -1.0f), mb, -x) * dxi;
    const float ty = fmaf(fmaf(fmaf(0.5f, rn_signf(dy), ny + 0.5f) * gsi, 2.0f, -1.0f), mb, -y) * dyi;
    const float tz = fmaf(fmaf(fmaf(0.5f, rn_signf(dz), nz + 0.5f) * gsi, 2.0f, -1.0f), mb, -z) * dzi;
    const float t_target = t + fmaxf(0.0f, fminf(tx, fminf(ty, tz)));
    do {
        t += rn_calc_dt(t, c.esf, c.max_samples, c.grid_size, c.dt_scale);
    } while (t < t_target);
    return false;
}

// Occupancy query of raymarching.cu:205-224 at t: occupied?  If not, the skip
// target of :225-230 (exit of the cell at its mip level).
__device__ __forceinline__ bool march_query(float t, float ox, float oy, float oz,
                                            float dx, float dy, float dz,
                                            float dxi, float dyi, float dzi,
                                            const uint8_t* __restrict__ bitfield,
                                            const MarchCfg& c, float& x, float& y, float& z,
                                            float& dt, float& t_target) {
    const uint32_t g3 = (uint32_t)c.grid_size * c.grid_size * c.grid_size;
    const float gsi = 1.0f / c.grid_size;
    x = fmaf(t, dx, ox); y = fmaf(t, dy, oy); z = fmaf(t, dz, oz);
    dt = rn_calc_dt(t, c.esf, c.max_samples, c.grid_size, c.dt_scale);
    const int mip = max(rn_mip_from_pos(x, y, z, c.cascades),
                        rn_mip_from_dt(dt, c.grid_size, c.cascades));
    const float mb = fminf(scalbnf(1.0f, mip - 1), c.scale);
    const float mbi = mip_bound_inv(mip, c.scale);
    const float gm1 = c.grid_size - 1.0f;
    const int nx = (int)rn_clampf(0.5f * fmaf(x, mbi, 1.0f) * c.grid_size, 0.0f, gm1);
    const int ny = (int)rn_clampf(0.5f * fmaf(y, mbi, 1.0f) * c.grid_size, 0.0f, gm1);
    const int nz = (int)rn_clampf(0.5f * fmaf(z, mbi, 1.0f) * c.grid_size, 0.0f, gm1);
    const uint32_t idx = mip * g3 + rn_morton3d(nx, ny, nz);
    const bool occ = bitfield[idx / 8] & (1 << (idx % 8));
    const float tx = fmaf(fmaf(fmaf(0.5f, rn_signf(dx), nx + 0.5f) * gsi, 2.0f, -1.0f), mb, -x) * dxi;
    const float ty = fmaf(fmaf(fmaf(0.5f, rn_signf(dy), ny + 0.5f) * gsi, 2.0f, -1.0f), mb, -y) * dyi;
    const float tz = fmaf(fmaf(fmaf(0.5f, rn_signf(dz), nz + 0.5f) * gsi, 2.0f, -1.0f), mb, -z) * dzi;
    t_target = t + fmaxf(0.0f, fminf(tx, fminf(ty, tz)));
    return occ;
}

// One ray marched by a whole wave (raymarching.cu:200-279, bit-exact).
//
// The reference marches a ray serially: at the current t it queries the cell;
// occupied -> emit, t += dt(t); empty -> repeat t += dt(t) until t >= the
// cell's exit.  Either way t only ever advances by t += dt(t), so the values
// t_k visited form ONE fixed sequence; occupancy only decides which k are
// queried (the chain) and emitted.  The wave evaluates 64 consecutive t_k per
// chunk (lane j: t_{base+j}, the same float additions in the same order),
// queries all of them in parallel (one bitfield load per lane instead of one
// dependent load per step), and then walks the chain through the chunk with
// scalar ops: next(k) = k + 1 if occupied, else the first k' > k with
// t_k' >= target(k) (the do-while of :228-230).  The chain is the reference's
// sequence of queries, so counts and samples are identical; the serial
// latency per step drops from a dependent L2 load to a few scalar ops.
// NEG: march from a negative t1 too (the test-time march, raymarching.cu:
// 364-365, starts wherever hits_t says; the training march requires t1 >= 0)
template <bool WRITE, typename Sink, bool NEG = false>
__device__ int march_ray_wave(float ox, float oy, float oz, float dx, float dy, float dz,
                              float t1, float t2, int cap, int start,
                              const uint8_t* __restrict__ bitfield, const MarchCfg& c,
                              const Sink& sink) {
    const int lane = rn_lane();
    if (!((NEG || 0.0f <= t1) && t1 < t2) || cap <= 0) return 0;
    const float dxi = 1.0f / dx, dyi = 1.0f / dy, dzi = 1.0f / dz;
    const uint64_t lt_mask = (1ull << lane) - 1ull;
    float tb = t1;                 // t at the chunk's first step (wave-uniform)
    float need = -INFINITY;        // chain resumes at the first step with t >= need
    int n = 0;
    int chunks = 0;
    while (true) {
        // every chunk advances t by 64 steps; bound the walk anyway (a t so
        // large that t + dt == t would never reach t2)
        if (NEG && ++chunks > (1 << 16)) break;
        float t = tb;
        if (c.esf == 0.0f) {            // constant dt (scale <= 0.5 scenes): same adds, no clamp
            const float d0 = rn_calc_dt(0.0f, c.esf, c.max_samples, c.grid_size, c.dt_scale);
            // Inside one binade [2^e, 2^(e+1)) every t is a multiple of its ulp
            // u and fl(t + d0) = t + r with r = round_u(d0) the same for every
            // t (round-to-nearest is translation invariant on that grid; with
            // a tie, only the first step can differ, which the second-step
            // comparison rejects).  So t_j = tb + j r exactly, one fma per
            // lane, whenever the chunk stays inside tb's binade; otherwise
            // the serial adds below.
            const float s1 = tb + d0, r = s1 - tb, s2 = s1 + d0;
            const float bend = __uint_as_float((__float_as_uint(tb) & 0x7f800000u) + 0x00800000u);
            const float tj = fmaf((float)lane, r, tb);
            if (s2 - s1 == r && tb > 0.0f && __builtin_amdgcn_ballot_w64(!(tj < bend)) == 0) {
                t = tj;
            } else {
#pragma unroll 16
                for (int i = 0; i < RN_WAVE - 1; ++i) { const float nt = t + d0; t = i < lane ? nt : t; }
            }
        } else if (rn_dbg(c.abl) & 1) {  // timing only: the chain's cost
            t = fmaf((float)lane, rn_calc_dt(tb, c.esf, c.max_samples, c.grid_size, c.dt_scale), tb);
        } else {
#pragma unroll 8
            for (int i = 0; i < RN_WAVE - 1; ++i) {
                const float nt = t + rn_calc_dt(t, c.esf, c.max_samples, c.grid_size, c.dt_scale);
                t = i < lane ? nt : t;
            }
        }
        const bool alive = t < t2;                      // a prefix of the lanes
        float x, y, z, dt, target;
        const bool occ = march_query(t, ox, oy, oz, dx, dy, dz, dxi, dyi, dzi, bitfield, c,
                                     x, y, z, dt, target) && alive;
        const uint64_t alive_m = __builtin_amdgcn_ballot_w64(alive);
        const uint64_t occ_m = __builtin_amdgcn_ballot_w64(occ);
        // walk the chain through this chunk (scalar).  A run of occupied steps
        // is on the chain as a whole (next(k) = k + 1), so one iteration per
        // run and one per empty query.
        uint64_t mark = 0;
        const uint64_t cand = __builtin_amdgcn_ballot_w64(alive && t >= need);
        int cur = cand ? __builtin_ctzll(cand) : RN_WAVE;
        int emitted = 0;
        bool full = false;
        const bool capfree = n + RN_WAVE < cap;          // this chunk cannot reach the cap
        while (cur < RN_WAVE) {
            const uint64_t from = ~0ull << cur;
            if ((occ_m >> cur) & 1ull) {
                const uint64_t stop = ~occ_m & from;
                const int end = stop ? __builtin_ctzll(stop) : RN_WAVE;
                need = -INFINITY;
                if (!capfree && n + emitted + (end - cur) >= cap) {
                    const int e2 = cur + (cap - n - emitted);
                    mark |= from & (e2 < RN_WAVE ? ~(~0ull << e2) : ~0ull);
                    emitted += e2 - cur;
                    full = true;
                    break;
                }
                mark |= from & ((stop & (0ull - stop)) - 1ull);   // steps [cur, end)
                emitted += end - cur;
                cur = (end < RN_WAVE && ((alive_m >> end) & 1ull)) ? end : RN_WAVE;
            } else {
                mark |= 1ull << cur;
                need = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(target), cur));
                const uint64_t nxt = __builtin_amdgcn_ballot_w64(alive && t >= need) & (from << 1);
                cur = nxt ? __builtin_ctzll(nxt) : RN_WAVE;
            }
        }
        const uint64_t emit_m = mark & occ_m;
        if (WRITE && ((emit_m >> lane) & 1ull))
            sink.emit(start + n + __builtin_popcountll(emit_m & lt_mask), x, y, z, t, dt);
        n += __builtin_popcountll(emit_m);
        if (full || alive_m != ~0ull) break;            // cap reached, or the ray left [t1, t2)
        const float tl = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t), RN_WAVE - 1));
        tb = tl + rn_calc_dt(tl, c.esf, c.max_samples, c.grid_size, c.dt_scale);
        if (!(tb < t2)) break;
    }
    return n;
}

// intersection.cu:5-22 (_ray_aabb_intersect) for a single box
__device__ __forceinline__ void aabb(float ox, float oy, float oz, float dx, float dy, float dz,
                                     const float* __restrict__ c, const float* __restrict__ h,
                                     float& t1, float& t2) {
    const float ix = 1.0f / dx, iy = 1.0f / dy, iz = 1.0f / dz;
    const float ax = (c[0] - h[0] - ox) * ix, bx = (c[0] + h[0] - ox) * ix;
    const float ay = (c[1] - h[1] - oy) * iy, by = (c[1] + h[1] - oy) * iy;
    const float az = (c[2] - h[2] - oz) * iz, bz = (c[2] + h[2] - oz) * iz;
    const float n = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    const float f = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
    if (n > f) { t1 = -1.0f; t2 = -1.0f; } else { t1 = n; t2 = f; }
}

}  // namespace
