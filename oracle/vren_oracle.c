/*
 * ORACLE — test infrastructure only.  Serial CPU restatement of the reference
 * `vren` kernels of thu-nics/Rad-NeRF (models/csrc/{raymarching,volumerendering,intersection}.cu), used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.
 * Never linked into or called by the product (rad-nerf_amd/).
 *
 * Parity status: UNPINNED against the reference itself — the reference ships
 * no tests, fixtures or golden vectors for this path and
 * its CUDA extension cannot be built or run in this image (it needs
 * cuda_runtime.h / nvcc).  The restatement is pinned by analytic known-answer
 * tests (tests/test_oracle.py) derived from the cited formulas.
 *
 * Contraction policy: compiled with -ffp-contract=off; the
 * multiply-adds that nvcc fuses in the reference are explicit fmaf() calls at
 * exactly the sites the HIP kernels use them.
 * Threads: rays (segments) are independent, so march and composite loops run
 * under OpenMP (OMP_NUM_THREADS); the march counts first, takes ray-order
 * starts serially, then writes.  Results do not depend on the thread count.
 * Ordering: the reference allocates sample slots with atomicAdd
 * (raymarching.cu:237-238), so its row order is nondeterministic; this oracle
 * uses ray order with start = exclusive prefix of the per-ray counts.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define SQRT3 1.73205080757f

/* helper_math.h:280-283 */
static float clampf_(float f, float a, float b) { return fmaxf(a, fminf(f, b)); }
/* raymarching.cu:7 */
static float signf_(float x) { return copysignf(1.0f, x); }

/* exp(x) as one fixed sequence of IEEE-754 single operations: the
 * compositing exponent of volumerendering.cu:31 (`__expf(-sigma*delta)`, CUDA's
 * ex2.approx) restated with a formulation the GPU kernels evaluate with the
 * same operations, so transmittance and the early-termination sample match
 * bit for bit.  Range reduction x = k*ln2 + r (Cody-Waite: 15-bit head + tail),
 * degree-7 Taylor polynomial in Horner form with fmaf, exact ldexpf.
 * Within 1 ulp of exp for x in [-87, 0]. */
float oracle_det_expf(float x);
static float det_expf(float x) {
    if (!(x >= -87.0f)) return x != x ? x : 0.0f;
    if (x > 88.0f) return INFINITY;
    const float k = rintf(x * 1.44269502162933349609375f);
    float r = fmaf(k, -0.693145751953125f, x);
    r = fmaf(k, -1.428606765330187045037746429443359375e-06f, r);
    float p = 1.98412701138295233249664306640625e-04f;
    p = fmaf(p, r, 1.388888922519981861114501953125e-03f);
    p = fmaf(p, r, 8.333333767950534820556640625e-03f);
    p = fmaf(p, r, 4.16666679084300994873046875000e-02f);
    p = fmaf(p, r, 1.66666671633720397949218750000e-01f);
    p = fmaf(p, r, 0.5f);
    p = fmaf(p, r, 1.0f);
    p = fmaf(p, r, 1.0f);
    return ldexpf(p, (int)k);
}
/* raymarching.cu:11-13 */
static float calc_dt(float t, float esf, int max_samples, int grid_size, float scale) {
    return clampf_(t * esf, SQRT3 / max_samples, SQRT3 * 2 * scale / grid_size);
}
/* raymarching.cu:19-23 */
static int mip_from_pos(float x, float y, float z, int cascades) {
    const float mx = fmaxf(fabsf(x), fmaxf(fabsf(y), fabsf(z)));
    int e;
    frexpf(mx, &e);
    int m = e + 1;
    if (m < 0) m = 0;
    return m < cascades - 1 ? m : cascades - 1;
}
/* raymarching.cu:29-32 */
static int mip_from_dt(float dt, int grid_size, int cascades) {
    int e;
    frexpf(dt * grid_size, &e);
    int m = e;
    if (m < 0) m = 0;
    return m < cascades - 1 ? m : cascades - 1;
}
/* raymarching.cu:35-60 */
static uint32_t expand_bits(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}
uint32_t oracle_morton3d_one(uint32_t x, uint32_t y, uint32_t z) {
    return expand_bits(x) | (expand_bits(y) << 1) | (expand_bits(z) << 2);
}
uint32_t oracle_morton3d_invert_one(uint32_t x) {
    x = x & 0x49249249u;
    x = (x | (x >> 2)) & 0xc30c30c3u;
    x = (x | (x >> 4)) & 0x0f00f00fu;
    x = (x | (x >> 8)) & 0xff0000ffu;
    x = (x | (x >> 16)) & 0x0000ffffu;
    return x;
}

void oracle_morton3d(const int32_t* coords, int64_t n, int32_t* out) {
    for (int64_t i = 0; i < n; ++i)
        out[i] = (int32_t)oracle_morton3d_one(coords[3 * i], coords[3 * i + 1], coords[3 * i + 2]);
}
void oracle_morton3d_invert(const int32_t* idx, int64_t n, int32_t* coords) {
    for (int64_t i = 0; i < n; ++i) {
        const uint32_t v = (uint32_t)idx[i];
        coords[3 * i] = oracle_morton3d_invert_one(v);
        coords[3 * i + 1] = oracle_morton3d_invert_one(v >> 1);
        coords[3 * i + 2] = oracle_morton3d_invert_one(v >> 2);
    }
}
/* raymarching.cu:122-141 */
void oracle_packbits(const float* grid, int64_t n_bytes, float thr, uint8_t* bits) {
    for (int64_t n = 0; n < n_bytes; ++n) {
        uint8_t b = 0;
        for (int i = 0; i < 8; ++i) b |= (grid[8 * n + i] > thr) ? (uint8_t)(1u << i) : 0;
        bits[n] = b;
    }
}

/* intersection.cu:5-22 + :48-55 for one box */
static void aabb_one(const float* o, const float* d, const float* c, const float* h, float* t1,
                     float* t2) {
    const float ix = 1.0f / d[0], iy = 1.0f / d[1], iz = 1.0f / d[2];
    const float ax = (c[0] - h[0] - o[0]) * ix, bx = (c[0] + h[0] - o[0]) * ix;
    const float ay = (c[1] - h[1] - o[1]) * iy, by = (c[1] + h[1] - o[1]) * iy;
    const float az = (c[2] - h[2] - o[2]) * iz, bz = (c[2] + h[2] - o[2]) * iz;
    const float n = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    const float f = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
    if (n > f) { *t1 = -1.0f; *t2 = -1.0f; } else { *t1 = n; *t2 = f; }
}

/* intersection.cu:25-100 (deterministic voxel order, then sort by t_near) */
void oracle_ray_aabb_intersect(const float* rays_o, const float* rays_d, const float* centers,
                               const float* halfs, int64_t n_rays, int64_t n_vox, int max_hits,
                               int32_t* hit_cnt, float* hits_t, int64_t* hit_idx) {
    for (int64_t r = 0; r < n_rays; ++r) {
        float* ht = hits_t + r * max_hits * 2;
        int64_t* hi = hit_idx + r * max_hits;
        for (int m = 0; m < max_hits; ++m) { ht[2 * m] = -1.f; ht[2 * m + 1] = -1.f; hi[m] = -1; }
        int cnt = 0;
        for (int64_t v = 0; v < n_vox; ++v) {
            float t1, t2;
            aabb_one(rays_o + 3 * r, rays_d + 3 * r, centers + 3 * v, halfs + 3 * v, &t1, &t2);
            if (t2 > 0) {
                if (cnt < max_hits) { ht[2 * cnt] = fmaxf(t1, 0.0f); ht[2 * cnt + 1] = t2; hi[cnt] = v; }
                cnt++;
            }
        }
        hit_cnt[r] = cnt;
        for (int a = 1; a < max_hits; ++a) {  /* stable sort by t_near */
            float k0 = ht[2 * a], k1 = ht[2 * a + 1];
            int64_t kv = hi[a];
            int b = a - 1;
            while (b >= 0 && ht[2 * b] > k0) {
                ht[2 * (b + 1)] = ht[2 * b]; ht[2 * (b + 1) + 1] = ht[2 * b + 1]; hi[b + 1] = hi[b];
                --b;
            }
            ht[2 * (b + 1)] = k0; ht[2 * (b + 1) + 1] = k1; hi[b + 1] = kv;
        }
    }
}

typedef struct { int cascades, grid_size, max_samples; float scale, dt_scale, esf; } cfg_t;

/* raymarching.cu:204-233 (count) / :243-279 (write).  out_* may be NULL. */
static int march(const float* o, const float* d, float t1, float t2, const uint8_t* bits,
                 const cfg_t* c, int count_pass, int n_write, float* xyz, float* dir, float* ts,
                 float* dts) {
    const uint32_t g3 = (uint32_t)c->grid_size * c->grid_size * c->grid_size;
    const float gsi = 1.0f / c->grid_size;
    const float ox = o[0], oy = o[1], oz = o[2], dx = d[0], dy = d[1], dz = d[2];
    const float dxi = 1.0f / dx, dyi = 1.0f / dy, dzi = 1.0f / dz;
    float t = t1;
    int n = 0;
    for (;;) {
        if (count_pass) { if (!(0 <= t && t < t2 && n < c->max_samples)) break; }
        else { if (!(t < t2 && n < n_write)) break; }
        const float x = fmaf(t, dx, ox), y = fmaf(t, dy, oy), z = fmaf(t, dz, oz);
        const float dt = calc_dt(t, c->esf, c->max_samples, c->grid_size, c->dt_scale);
        const int mp = mip_from_pos(x, y, z, c->cascades), md = mip_from_dt(dt, c->grid_size, c->cascades);
        const int mip = mp > md ? mp : md;
        const float mb = fminf(scalbnf(1.0f, mip - 1), c->scale);
        const float mbi = 1 / mb;
        const float gm1 = c->grid_size - 1.0f;
        const int nx = (int)clampf_(0.5f * fmaf(x, mbi, 1.0f) * c->grid_size, 0.0f, gm1);
        const int ny = (int)clampf_(0.5f * fmaf(y, mbi, 1.0f) * c->grid_size, 0.0f, gm1);
        const int nz = (int)clampf_(0.5f * fmaf(z, mbi, 1.0f) * c->grid_size, 0.0f, gm1);
        const uint32_t idx = mip * g3 + oracle_morton3d_one(nx, ny, nz);
        const int occ = bits[idx / 8] & (1 << (idx % 8));
        if (occ) {
            if (!count_pass) {
                xyz[3 * n] = x; xyz[3 * n + 1] = y; xyz[3 * n + 2] = z;
                if (dir) { dir[3 * n] = dx; dir[3 * n + 1] = dy; dir[3 * n + 2] = dz; }
                ts[n] = t; dts[n] = dt;
            }
            t += dt; n++;
        } else {
            const float tx = fmaf(fmaf(fmaf(0.5f, signf_(dx), nx + 0.5f) * gsi, 2.0f, -1.0f), mb, -x) * dxi;
            const float ty = fmaf(fmaf(fmaf(0.5f, signf_(dy), ny + 0.5f) * gsi, 2.0f, -1.0f), mb, -y) * dyi;
            const float tz = fmaf(fmaf(fmaf(0.5f, signf_(dz), nz + 0.5f) * gsi, 2.0f, -1.0f), mb, -z) * dzi;
            const float tt = t + fmaxf(0.0f, fminf(tx, fminf(ty, tz)));
            do { t += calc_dt(t, c->esf, c->max_samples, c->grid_size, c->dt_scale); } while (t < tt);
        }
    }
    return n;
}

/* raymarching.cu:166-332.  Outputs sized for n_rays*max_samples rows (or the
 * caller's capacity `cap`); returns the total sample count (counter[0]). */
int64_t oracle_raymarching_train(const float* rays_o, const float* rays_d, const float* hits_t,
                                 const uint8_t* bits, int cascades, float scale, float esf,
                                 const float* noise, int grid_size, int max_samples,
                                 int64_t n_rays, int64_t cap, int64_t* rays_a, float* xyzs,
                                 float* dirs, float* deltas, float* ts) {
    cfg_t c = {cascades, grid_size, max_samples, scale, scale, esf};
    /* pass 1 (rays independent: OpenMP over rays), count */
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t r = 0; r < n_rays; ++r) {
        float t1 = hits_t[2 * r], t2 = hits_t[2 * r + 1];
        if (t1 >= 0) {  /* raymarching.cu:195-198 */
            const float dt = calc_dt(t1, esf, max_samples, grid_size, scale);
            t1 = fmaf(dt, noise[r], t1);
        }
        rays_a[3 * r] = r;
        rays_a[3 * r + 2] = march(rays_o + 3 * r, rays_d + 3 * r, t1, t2, bits, &c, 1, 0, 0, 0, 0, 0);
    }
    /* ray-order starts (the reference's atomicAdd order is nondeterministic) */
    int64_t start = 0;
    for (int64_t r = 0; r < n_rays; ++r) { rays_a[3 * r + 1] = start; start += rays_a[3 * r + 2]; }
    /* pass 2, write */
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t r = 0; r < n_rays; ++r) {
        const int64_t s0 = rays_a[3 * r + 1];
        const int n = (int)rays_a[3 * r + 2];
        if (n == 0 || s0 + n > cap) continue;
        float t1 = hits_t[2 * r], t2 = hits_t[2 * r + 1];
        if (t1 >= 0) {
            const float dt = calc_dt(t1, esf, max_samples, grid_size, scale);
            t1 = fmaf(dt, noise[r], t1);
        }
        march(rays_o + 3 * r, rays_d + 3 * r, t1, t2, bits, &c, 0, n, xyzs + 3 * s0,
              dirs + 3 * s0, ts + s0, deltas + s0);
    }
    return start;
}

/* raymarching.cu:335-404 (incl. the calc_dt(..., cascades) quirk :370,399) */
void oracle_raymarching_test(const float* rays_o, const float* rays_d, float* hits_t,
                             const int64_t* alive, int64_t n_alive, const uint8_t* bits,
                             int cascades, float scale, float esf, int grid_size,
                             int max_samples, int n_samples, float* xyzs, float* dirs,
                             float* deltas, float* ts, int32_t* n_eff) {
    cfg_t c = {cascades, grid_size, max_samples, scale, (float)cascades, esf};
    const uint32_t g3 = (uint32_t)grid_size * grid_size * grid_size;
    const float gsi = 1.0f / grid_size;
    for (int64_t n = 0; n < n_alive; ++n) {
        const int64_t r = alive[n];
        const float ox = rays_o[3 * r], oy = rays_o[3 * r + 1], oz = rays_o[3 * r + 2];
        const float dx = rays_d[3 * r], dy = rays_d[3 * r + 1], dz = rays_d[3 * r + 2];
        const float dxi = 1.0f / dx, dyi = 1.0f / dy, dzi = 1.0f / dz;
        float t = hits_t[2 * r];
        const float t2 = hits_t[2 * r + 1];
        int s = 0;
        while (t < t2 && s < n_samples) {
            const float x = fmaf(t, dx, ox), y = fmaf(t, dy, oy), z = fmaf(t, dz, oz);
            const float dt = calc_dt(t, esf, max_samples, grid_size, c.dt_scale);
            const int mp = mip_from_pos(x, y, z, cascades), md = mip_from_dt(dt, grid_size, cascades);
            const int mip = mp > md ? mp : md;
            const float mb = fminf(scalbnf(1.0f, mip - 1), scale);
            const float mbi = 1 / mb;
            const float gm1 = grid_size - 1.0f;
            const int nx = (int)clampf_(0.5f * fmaf(x, mbi, 1.0f) * grid_size, 0.0f, gm1);
            const int ny = (int)clampf_(0.5f * fmaf(y, mbi, 1.0f) * grid_size, 0.0f, gm1);
            const int nz = (int)clampf_(0.5f * fmaf(z, mbi, 1.0f) * grid_size, 0.0f, gm1);
            const uint32_t idx = mip * g3 + oracle_morton3d_one(nx, ny, nz);
            if (bits[idx / 8] & (1 << (idx % 8))) {
                const int64_t o = n * n_samples + s;
                xyzs[3 * o] = x; xyzs[3 * o + 1] = y; xyzs[3 * o + 2] = z;
                dirs[3 * o] = dx; dirs[3 * o + 1] = dy; dirs[3 * o + 2] = dz;
                ts[o] = t; deltas[o] = dt;
                t += dt;
                hits_t[2 * r] = t;
                s++;
            } else {
                const float tx = fmaf(fmaf(fmaf(0.5f, signf_(dx), nx + 0.5f) * gsi, 2.0f, -1.0f), mb, -x) * dxi;
                const float ty = fmaf(fmaf(fmaf(0.5f, signf_(dy), ny + 0.5f) * gsi, 2.0f, -1.0f), mb, -y) * dyi;
                const float tz = fmaf(fmaf(fmaf(0.5f, signf_(dz), nz + 0.5f) * gsi, 2.0f, -1.0f), mb, -z) * dzi;
                const float tt = t + fmaxf(0.0f, fminf(tx, fminf(ty, tz)));
                do { t += calc_dt(t, esf, max_samples, grid_size, c.dt_scale); } while (t < tt);
            }
        }
        n_eff[n] = s;
    }
}

/* volumerendering.cu:6-45 */
void oracle_composite_train_fw(const float* sig, const float* rgbs, const float* dl,
                               const float* ts, const int64_t* rays_a, int64_t n_rows, float thr,
                               int64_t* total, float* opacity, float* depth, float* rgb,
                               float* ws) {
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t n = 0; n < n_rows; ++n) {
        const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1];
        const int N = (int)rays_a[3 * n + 2];
        int samples = 0;
        float T = 1.0f;
        while (samples < N) {
            const int64_t s = start + samples;
            const float a = 1.0f - det_expf(-sig[s] * dl[s]);
            const float w = a * T;
            rgb[3 * ray] = fmaf(w, rgbs[3 * s], rgb[3 * ray]);
            rgb[3 * ray + 1] = fmaf(w, rgbs[3 * s + 1], rgb[3 * ray + 1]);
            rgb[3 * ray + 2] = fmaf(w, rgbs[3 * s + 2], rgb[3 * ray + 2]);
            depth[ray] = fmaf(w, ts[s], depth[ray]);
            opacity[ray] += w;
            ws[s] = w;
            T *= 1.0f - a;
            if (T <= thr) break;
            samples++;
        }
        total[ray] = samples;
    }
}

/* volumerendering.cu:87-152 (thrust inclusive_scan restated serially) */
void oracle_composite_train_bw(const float* gO, const float* gD, const float* gRGB,
                               const float* dL_dws, const float* sig, const float* rgbs,
                               const float* ws, const float* dl, const float* ts,
                               const int64_t* rays_a, int64_t n_rows, const float* opacity,
                               const float* depth, const float* rgb, float thr, float* dsig,
                               float* drgb) {
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t n = 0; n < n_rows; ++n) {
        const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1];
        const int N = (int)rays_a[3 * n + 2];
        if (N == 0) continue;
        float* pre = (float*)malloc(sizeof(float) * N);
        float acc = 0.f;
        for (int i = 0; i < N; ++i) { acc += dL_dws[start + i] * ws[start + i]; pre[i] = acc; }
        const float wsum = pre[N - 1];
        const float R = rgb[3 * ray], G = rgb[3 * ray + 1], B = rgb[3 * ray + 2];
        const float O = opacity[ray], D = depth[ray];
        float T = 1.0f, r = 0.f, g = 0.f, b = 0.f, d = 0.f;
        int samples = 0;
        while (samples < N) {
            const int64_t s = start + samples;
            const float a = 1.0f - det_expf(-sig[s] * dl[s]);
            const float w = a * T;
            r = fmaf(w, rgbs[3 * s], r); g = fmaf(w, rgbs[3 * s + 1], g);
            b = fmaf(w, rgbs[3 * s + 2], b); d = fmaf(w, ts[s], d);
            T *= 1.0f - a;
            drgb[3 * s] = gRGB[3 * ray] * w;
            drgb[3 * s + 1] = gRGB[3 * ray + 1] * w;
            drgb[3 * s + 2] = gRGB[3 * ray + 2] * w;
            float v = gRGB[3 * ray] * fmaf(rgbs[3 * s], T, -(R - r));
            v = fmaf(gRGB[3 * ray + 1], fmaf(rgbs[3 * s + 1], T, -(G - g)), v);
            v = fmaf(gRGB[3 * ray + 2], fmaf(rgbs[3 * s + 2], T, -(B - b)), v);
            v = v + gO[ray] * (1 - O);
            v = fmaf(gD[ray], fmaf(ts[s], T, -(D - d)), v);
            v = fmaf(T, dL_dws[s], v) - (wsum - pre[samples]);
            dsig[s] = dl[s] * v;
            if (T <= thr) break;
            samples++;
        }
        free(pre);
    }
}

/* volumerendering.cu:206-250 */
void oracle_composite_test_fw(const float* sig, const float* rgbs, const float* dl,
                              const float* ts, int64_t n_alive, int n_samples, int64_t* alive,
                              float thr, const int32_t* n_eff, float* opacity, float* depth,
                              float* rgb) {
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t n = 0; n < n_alive; ++n) {
        if (n_eff[n] == 0) { alive[n] = -1; continue; }
        const int64_t r = alive[n];
        float T = 1 - opacity[r];
        for (int s = 0; s < n_eff[n]; ++s) {
            const int64_t o = n * n_samples + s;
            const float a = 1.0f - det_expf(-sig[o] * dl[o]);
            const float w = a * T;
            rgb[3 * r] = fmaf(w, rgbs[3 * o], rgb[3 * r]);
            rgb[3 * r + 1] = fmaf(w, rgbs[3 * o + 1], rgb[3 * r + 1]);
            rgb[3 * r + 2] = fmaf(w, rgbs[3 * o + 2], rgb[3 * r + 2]);
            depth[r] = fmaf(w, ts[o], depth[r]);
            opacity[r] += w;
            T *= 1.0f - a;
            if (T <= thr) { alive[n] = -1; break; }
        }
    }
}

/* ml_rendering.py:47-52 + __render_rays_train:174-179 for K models: AABB,
 * NEAR clamp (ml_rendering.py:50), jitter, march.  Counts [K][B]; samples
 * written model-major, ray order, with start offsets in `starts` [K][B]. */
int64_t oracle_ml_march(const float* rays_o, const float* rays_d, const float* center,
                        const float* half_size, float near_distance, const float* noise,
                        const uint8_t* bitfields, int64_t bitfield_bytes, int K, int cascades,
                        float scale, float esf, int grid_size, int max_samples, int64_t n_rays,
                        int64_t cap, int32_t* counts, int64_t* starts, float* xyzs, float* ts,
                        float* deltas) {
    cfg_t c = {cascades, grid_size, max_samples, scale, scale, esf};
    const int64_t n_seg = (int64_t)K * n_rays;
    if (n_seg == 0) return 0;
    /* pass 1 (segments independent: OpenMP), count; pass 2, write */
    for (int pass = 0; pass < 2; ++pass) {
#pragma omp parallel for schedule(dynamic, 16)
        for (int64_t g = 0; g < n_seg; ++g) {
            const int k = (int)(g / n_rays);
            const int64_t r = g - (int64_t)k * n_rays;
            if (pass == 1 && (counts[g] == 0 || starts[g] + counts[g] > cap)) continue;
            float t1, t2;
            aabb_one(rays_o + 3 * r, rays_d + 3 * r, center, half_size, &t1, &t2);
            if (!(t2 > 0)) { t1 = -1.f; t2 = -1.f; }
            else { t1 = fmaxf(t1, 0.0f); if (t1 < near_distance) t1 = near_distance; }
            if (t1 >= 0) {
                const float dt = calc_dt(t1, esf, max_samples, grid_size, scale);
                t1 = fmaf(dt, noise[g], t1);
            }
            const uint8_t* bits = bitfields + k * bitfield_bytes;
            if (pass == 0) {
                counts[g] = march(rays_o + 3 * r, rays_d + 3 * r, t1, t2, bits, &c, 1, 0, 0, 0, 0, 0);
            } else {
                const int64_t s0 = starts[g];
                march(rays_o + 3 * r, rays_d + 3 * r, t1, t2, bits, &c, 0, counts[g], xyzs + 3 * s0,
                      0, ts + s0, deltas + s0);
            }
        }
        if (pass == 0) {
            int64_t start = 0;
            for (int64_t g = 0; g < n_seg; ++g) { starts[g] = start; start += counts[g]; }
            if (cap == 0) return start;
        }
    }
    return starts[n_seg - 1] + counts[n_seg - 1];
}

/* intersection.cu:103-120 (_ray_sphere_intersect) + :123-150 (kernel) + :191-195
 * (sort by t_near).  Deterministic sphere order, then a stable sort. */
void oracle_ray_sphere_intersect(const float* rays_o, const float* rays_d, const float* centers,
                                 const float* radii, int64_t n_rays, int64_t n_sph, int max_hits,
                                 int32_t* hit_cnt, float* hits_t, int64_t* hit_idx) {
    for (int64_t r = 0; r < n_rays; ++r) {
        const float* o = rays_o + 3 * r;
        const float* d = rays_d + 3 * r;
        float* ht = hits_t + r * max_hits * 2;
        int64_t* hi = hit_idx + r * max_hits;
        for (int m = 0; m < max_hits; ++m) { ht[2 * m] = -1.f; ht[2 * m + 1] = -1.f; hi[m] = -1; }
        int cnt = 0;
        for (int64_t s = 0; s < n_sph; ++s) {
            const float cx = o[0] - centers[3 * s], cy = o[1] - centers[3 * s + 1],
                        cz = o[2] - centers[3 * s + 2];
            const float a = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
            const float hb = d[0] * cx + d[1] * cy + d[2] * cz;
            const float c = (cx * cx + cy * cy + cz * cz) - radii[s] * radii[s];
            const float disc = hb * hb - a * c;
            float t1 = -1.f, t2 = -1.f;
            if (!(disc < 0)) {
                const float q = sqrtf(disc);
                t1 = (-hb - q) / a;
                t2 = (-hb + q) / a;
            }
            if (t2 > 0) {
                if (cnt < max_hits) { ht[2 * cnt] = fmaxf(t1, 0.0f); ht[2 * cnt + 1] = t2; hi[cnt] = s; }
                cnt++;
            }
        }
        hit_cnt[r] = cnt;
        for (int a = 1; a < max_hits; ++a) {
            float k0 = ht[2 * a], k1 = ht[2 * a + 1];
            int64_t kv = hi[a];
            int b = a - 1;
            while (b >= 0 && ht[2 * b] > k0) {
                ht[2 * (b + 1)] = ht[2 * b]; ht[2 * (b + 1) + 1] = ht[2 * b + 1]; hi[b + 1] = hi[b];
                --b;
            }
            ht[2 * (b + 1)] = k0; ht[2 * (b + 1) + 1] = k1; hi[b + 1] = kv;
        }
    }
}

/* losses.cu:9-44 (prefix sums), :47-110 (distortion_loss_fw): per rays_a row,
 * serial scans of ws and ws*ts, per-sample term
 *   2*(wts_incl*ws_excl - ws_incl*wts_excl) + 1/3*ws*ws*deltas
 * summed into loss[ray_idx].  loss (n_out) must be zeroed by the caller. */
void oracle_distortion_loss_fw(const float* ws, const float* deltas, const float* ts,
                               const int64_t* rays_a, int64_t n_rows, float* loss,
                               float* ws_incl, float* wts_incl) {
    for (int64_t n = 0; n < n_rows; ++n) {
        const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1], N = rays_a[3 * n + 2];
        float sw = 0.f, swt = 0.f, acc = 0.f;
        for (int64_t i = 0; i < N; ++i) {
            const int64_t s = start + i;
            const float wt = ws[s] * ts[s];
            const float ex_w = sw, ex_wt = swt;
            sw += ws[s];
            swt += wt;
            ws_incl[s] = sw;
            wts_incl[s] = swt;
            const float term = 2.0f * (swt * ex_w - sw * ex_wt) +
                               (1.0f / 3) * ws[s] * ws[s] * deltas[s];
            acc += term;
        }
        loss[ray] = acc;
    }
}

/* losses.cu:113-150 (distortion_loss_bw_kernel) */
void oracle_distortion_loss_bw(const float* dL_dloss, const float* ws_incl, const float* wts_incl,
                               const float* ws, const float* deltas, const float* ts,
                               const int64_t* rays_a, int64_t n_rows, float* dL_dws) {
    for (int64_t n = 0; n < n_rows; ++n) {
        const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1], N = rays_a[3 * n + 2];
        if (N <= 0) continue;
        const int64_t end = start + N - 1;
        const float ws_sum = ws_incl[end], wts_sum = wts_incl[end];
        const float g = dL_dloss[ray];
        for (int64_t s = start; s <= end; ++s) {
            const float front = s == start ? 0.f : ts[s] * ws_incl[s - 1] - wts_incl[s - 1];
            const float back = wts_sum - wts_incl[s] - ts[s] * (ws_sum - ws_incl[s]);
            dL_dws[s] = g * 2 * (front + back);
            dL_dws[s] += g * (2.0f / 3) * ws[s] * deltas[s];
        }
    }
}

/* custom_functions.py:102-112 (RayMarcher.backward, torch_scatter.segment_csr
 * sums over the rays_a segments, in ray-row order) */
void oracle_raymarching_train_bw(const float* dL_dxyzs, const float* dL_ddirs, const float* ts,
                                 const int64_t* rays_a, int64_t n_rows, float* dL_drays_o,
                                 float* dL_drays_d) {
    for (int64_t n = 0; n < n_rows; ++n) {
        const int64_t start = rays_a[3 * n + 1], N = rays_a[3 * n + 2];
        float o[3] = {0, 0, 0}, d[3] = {0, 0, 0};
        for (int64_t s = start; s < start + N; ++s)
            for (int c = 0; c < 3; ++c) {
                o[c] += dL_dxyzs[3 * s + c];
                d[c] += dL_dxyzs[3 * s + c] * ts[s] + dL_ddirs[3 * s + c];
            }
        for (int c = 0; c < 3; ++c) { dL_drays_o[3 * n + c] = o[c]; dL_drays_d[3 * n + c] = d[c]; }
    }
}

/* the compositing exponent, exported for tests/test_oracle.py's accuracy check */
float oracle_det_expf(float x) { return det_expf(x); }

/* thread count of the OpenMP loops (bench.py's CPU-baseline sweep) */
#include <omp.h>
void oracle_set_threads(int n) { if (n > 0) omp_set_num_threads(n); }
