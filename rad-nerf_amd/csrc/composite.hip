// Front-to-back alpha compositing for gfx950: one wavefront per ray segment.
//
// Reference: models/csrc/volumerendering.cu:6-45 (composite_train_fw_kernel),
// :87-152 (composite_train_bw_kernel), :206-250 (composite_test_fw_kernel) and
// the gated combine of models/ml_rendering.py:41-78,192-200.
//
// The reference walks each ray with one thread (serial, uncoalesced, thrust
// inclusive_scan inside the thread).  Here a 64-lane wave walks a segment in
// chunks of 64 consecutive samples (coalesced loads), builds the transmittance
// with a wave prefix-product, finds the early-termination sample with a
// ballot, and replaces the in-thread thrust scan with wave prefix sums.
#include "rn_common.h"
#pragma clang fp contract(off)

namespace {

struct SegOut { float O, D, R, G, B; int used; };

// the chunk's early-termination lane (or -1), bit-exact against the serial
// fold: rn_chunk_break, with the whole-segment serial fold when ambiguous
__device__ __forceinline__ int seg_break(const float* __restrict__ sig,
                                         const float* __restrict__ dl, int64_t start, int n,
                                         int base, float pin, bool valid, float thr) {
    int brk = rn_chunk_break(pin, valid, base + rn_lane(), thr);
    if (brk == -2) {
        const int b = rn_serial_break(sig, dl, start, n, thr);
        brk = (b >= base && b < base + RN_WAVE) ? b - base : -1;
    }
    return brk;
}

// Forward over one segment.  All lanes of the wave call this with the same
// (start, n).  Writes ws for the samples that contribute (<= break sample).
__device__ SegOut seg_forward(const float* __restrict__ sig, const float* __restrict__ rgbs,
                              const float* __restrict__ dl, const float* __restrict__ ts,
                              int64_t start, int n, float thr, float* __restrict__ ws) {
    const int lane = rn_lane();
    float T = 1.0f;
    float aO = 0.f, aD = 0.f, aR = 0.f, aG = 0.f, aB = 0.f;
    int used = n;
    bool done = false;
    for (int base = 0; base < n; base += RN_WAVE) {
        const int i = base + lane;
        const bool valid = i < n;
        if (done) {  // samples past the termination keep ws = 0
            if (valid) ws[start + i] = 0.f;
            continue;
        }
        float a = 0.f, c0 = 0.f, c1 = 0.f, c2 = 0.f, t = 0.f;
        if (valid) {
            const int64_t s = start + i;
            a = 1.0f - rn_exp_det(-sig[s] * dl[s]);
            c0 = rgbs[3 * s]; c1 = rgbs[3 * s + 1]; c2 = rgbs[3 * s + 2]; t = ts[s];
        }
        const float om = 1.0f - a;
        // transmittance after this sample = T * prod_{j<=i} (1-a_j)
        const float pin = rn_wave_incl_prod(lane == 0 ? T * om : om);
        const float pex = rn_wave_shr1(pin, T);
        const float w = a * pex;
        int last = RN_WAVE - 1;
        const int brk = seg_break(sig, dl, start, n, base, pin, valid, thr);
        if (brk >= 0) {
            last = brk;
            used = base + last;
            done = true;
        }
        const bool live = valid && lane <= last;
        if (valid) ws[start + i] = live ? w : 0.f;
        if (live) {
            aR = fmaf(w, c0, aR); aG = fmaf(w, c1, aG); aB = fmaf(w, c2, aB);
            aD = fmaf(w, t, aD); aO += w;
        }
        T = rn_wave_last(pin);
    }
    SegOut o;
    o.O = rn_wave_sum(aO); o.D = rn_wave_sum(aD);
    o.R = rn_wave_sum(aR); o.G = rn_wave_sum(aG); o.B = rn_wave_sum(aB);
    o.used = used;
    return o;
}

// Backward over one segment (volumerendering.cu:109-151).  Seeds are per ray.
__device__ void seg_backward(const float* __restrict__ sig, const float* __restrict__ rgbs,
                             const float* __restrict__ dl, const float* __restrict__ ts,
                             const float* __restrict__ ws, const float* __restrict__ dL_dws,
                             int64_t start, int n, float thr, float R, float G, float B, float O,
                             float D, float gR, float gG, float gB, float gO, float gD,
                             float* __restrict__ dsig, float* __restrict__ drgb) {
    const int lane = rn_lane();
    // total of dL_dws*ws over the whole segment (thrust scan's last element)
    float wsum_part = 0.f;
    if (dL_dws) {
        for (int base = 0; base < n; base += RN_WAVE) {
            const int i = base + lane;
            if (i < n) wsum_part += dL_dws[start + i] * ws[start + i];
        }
    }
    const float wtot = dL_dws ? rn_wave_sum(wsum_part) : 0.f;
    const float gterm_O = gO * (1 - O);
    float T = 1.0f, pr = 0.f, pg = 0.f, pb = 0.f, pd = 0.f, pw = 0.f;
    bool done = false;
    for (int base = 0; base < n; base += RN_WAVE) {
        const int i = base + lane;
        const bool valid = i < n;
        const int64_t s = start + i;
        if (done) {  // past the termination sample: zero gradients
            if (valid) { dsig[s] = 0.f; drgb[3 * s] = 0.f; drgb[3 * s + 1] = 0.f; drgb[3 * s + 2] = 0.f; }
            continue;
        }
        float a = 0.f, c0 = 0.f, c1 = 0.f, c2 = 0.f, t = 0.f, d = 0.f, gw = 0.f, wsv = 0.f;
        if (valid) {
            d = dl[s];
            a = 1.0f - rn_exp_det(-sig[s] * d);
            c0 = rgbs[3 * s]; c1 = rgbs[3 * s + 1]; c2 = rgbs[3 * s + 2]; t = ts[s];
            if (dL_dws) { gw = dL_dws[s]; wsv = ws[s]; }
        }
        const float om = 1.0f - a;
        const float pin = rn_wave_incl_prod(lane == 0 ? T * om : om);
        const float pex = rn_wave_shr1(pin, T);
        const float w = a * pex;
        const int brk = seg_break(sig, dl, start, n, base, pin, valid, thr);
        const bool stop = brk >= 0;
        const int last = stop ? brk : RN_WAVE - 1;
        const bool live = valid && lane <= last;
        // inclusive prefix sums (r, g, b, d accumulate before the gradient)
        const float sr = pr + rn_wave_incl_sum(live ? w * c0 : 0.f);
        const float sg = pg + rn_wave_incl_sum(live ? w * c1 : 0.f);
        const float sb = pb + rn_wave_incl_sum(live ? w * c2 : 0.f);
        const float sd = pd + rn_wave_incl_sum(live ? w * t : 0.f);
        const float sw = pw + rn_wave_incl_sum(valid ? gw * wsv : 0.f);
        if (live) {
            const float Ta = pin;  // T updated before the gradient terms
            drgb[3 * s] = gR * w; drgb[3 * s + 1] = gG * w; drgb[3 * s + 2] = gB * w;
            float acc = gR * fmaf(c0, Ta, -(R - sr));
            acc = fmaf(gG, fmaf(c1, Ta, -(G - sg)), acc);
            acc = fmaf(gB, fmaf(c2, Ta, -(B - sb)), acc);
            acc = acc + gterm_O;
            acc = fmaf(gD, fmaf(t, Ta, -(D - sd)), acc);
            acc = fmaf(Ta, gw, acc) - (wtot - sw);
            dsig[s] = d * acc;
        } else if (valid) {
            dsig[s] = 0.f; drgb[3 * s] = 0.f; drgb[3 * s + 1] = 0.f; drgb[3 * s + 2] = 0.f;
        }
        if (stop) done = true;
        T = rn_wave_last(pin);
        pr = rn_wave_last(sr); pg = rn_wave_last(sg);
        pb = rn_wave_last(sb); pd = rn_wave_last(sd);
        pw = rn_wave_last(sw);
    }
}

// ---------------------------------------------------------------------------
// drop-in kernels (rays_a rows)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
k_composite_fw(int n_rows, const float* __restrict__ sig, const float* __restrict__ rgbs,
               const float* __restrict__ dl, const float* __restrict__ ts,
               const int64_t* __restrict__ rays_a, float thr, int64_t* __restrict__ total,
               float* __restrict__ opacity, float* __restrict__ depth, float* __restrict__ rgb,
               float* __restrict__ ws) {
    const int row = blockIdx.x * (blockDim.x / RN_WAVE) + (threadIdx.x / RN_WAVE);
    if (row >= n_rows) return;
    const int64_t ray = rays_a[3 * row], start = rays_a[3 * row + 1];
    const int n = (int)rays_a[3 * row + 2];
    SegOut o = seg_forward(sig, rgbs, dl, ts, start, n, thr, ws);
    if (rn_lane() == 0) {
        total[ray] = o.used;
        opacity[ray] = o.O; depth[ray] = o.D;
        rgb[3 * ray] = o.R; rgb[3 * ray + 1] = o.G; rgb[3 * ray + 2] = o.B;
    }
}

__global__ void __launch_bounds__(256)
k_composite_bw(int n_rows, const float* __restrict__ gO, const float* __restrict__ gD,
               const float* __restrict__ gRGB, const float* __restrict__ dL_dws,
               const float* __restrict__ sig, const float* __restrict__ rgbs,
               const float* __restrict__ ws, const float* __restrict__ dl,
               const float* __restrict__ ts, const int64_t* __restrict__ rays_a,
               const float* __restrict__ opacity, const float* __restrict__ depth,
               const float* __restrict__ rgb, float thr, float* __restrict__ dsig,
               float* __restrict__ drgb) {
    const int row = blockIdx.x * (blockDim.x / RN_WAVE) + (threadIdx.x / RN_WAVE);
    if (row >= n_rows) return;
    const int64_t ray = rays_a[3 * row], start = rays_a[3 * row + 1];
    const int n = (int)rays_a[3 * row + 2];
    seg_backward(sig, rgbs, dl, ts, ws, dL_dws, start, n, thr, rgb[3 * ray], rgb[3 * ray + 1],
                 rgb[3 * ray + 2], opacity[ray], depth[ray], gRGB[3 * ray], gRGB[3 * ray + 1],
                 gRGB[3 * ray + 2], gO[ray], gD[ray], dsig, drgb);
}

// volumerendering.cu:206-250; thread per alive ray (<= 64 samples per call)
__global__ void __launch_bounds__(256)
k_composite_test(int n_alive, int n_samples, const float* __restrict__ sig,
                 const float* __restrict__ rgbs, const float* __restrict__ dl,
                 const float* __restrict__ ts, int64_t* __restrict__ alive, float thr,
                 const int32_t* __restrict__ n_eff, float* __restrict__ opacity,
                 float* __restrict__ depth, float* __restrict__ rgb) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= n_alive) return;
    if (n_eff[n] == 0) { alive[n] = -1; return; }
    const int64_t r = alive[n];
    float T = 1 - opacity[r];
    float cr = rgb[3 * r], cg = rgb[3 * r + 1], cb = rgb[3 * r + 2], cd = depth[r],
          co = opacity[r];
    const size_t row = (size_t)n * n_samples;
    for (int s = 0; s < n_eff[n]; ++s) {
        const size_t o = row + s;
        const float a = 1.0f - rn_exp_det(-sig[o] * dl[o]);
        const float w = a * T;
        cr = fmaf(w, rgbs[3 * o], cr); cg = fmaf(w, rgbs[3 * o + 1], cg);
        cb = fmaf(w, rgbs[3 * o + 2], cb);
        cd = fmaf(w, ts[o], cd); co += w;
        T *= 1.0f - a;
        if (T <= thr) { alive[n] = -1; break; }
    }
    rgb[3 * r] = cr; rgb[3 * r + 1] = cg; rgb[3 * r + 2] = cb; depth[r] = cd; opacity[r] = co;
}

// ---------------------------------------------------------------------------
// fused ml path: segments addressed by (k, r) -> offsets/counts
// per-model outputs O/D/RGB are [K][B] / [K][B][3] (raw composite, no bg)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
k_ml_composite_fw(int n_rays, int K, const float* __restrict__ sig,
                  const float* __restrict__ rgbs, const float* __restrict__ dl,
                  const float* __restrict__ ts, const int32_t* __restrict__ counts,
                  const int32_t* __restrict__ offsets, float thr, int32_t* __restrict__ used,
                  float* __restrict__ Ok, float* __restrict__ Dk, float* __restrict__ RGBk,
                  float* __restrict__ ws) {
    const int seg = blockIdx.x * (blockDim.x / RN_WAVE) + (threadIdx.x / RN_WAVE);
    if (seg >= n_rays * K) return;
    SegOut o = seg_forward(sig, rgbs, dl, ts, offsets[seg], counts[seg], thr, ws);
    if (rn_lane() == 0) {
        used[seg] = o.used;
        Ok[seg] = o.O; Dk[seg] = o.D;
        RGBk[3 * seg] = o.R; RGBk[3 * seg + 1] = o.G; RGBk[3 * seg + 2] = o.B;
    }
}

// ml_rendering.py:66-68 (+ bg at :192-200), thread per ray, same op order as
// the reference's torch ops:  rgb_i = rgb_i + bg*(1-O_i);  acc = acc + rgb_i*g_i
__global__ void __launch_bounds__(256)
k_ml_combine_fw(int n_rays, int K, const float* __restrict__ gate, const float* __restrict__ Ok,
                const float* __restrict__ Dk, const float* __restrict__ RGBk,
                const float* __restrict__ bg, float* __restrict__ rgb,
                float* __restrict__ opacity, float* __restrict__ depth) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rays) return;
    float ar = 0.f, ag = 0.f, ab = 0.f, ao = 0.f;
    for (int k = 0; k < K; ++k) {
        const int seg = k * n_rays + r;
        const float g = gate[r * K + k];
        const float O = Ok[seg];
        const float om = 1 - O;
        const float cr = RGBk[3 * seg] + bg[0] * om;
        const float cg = RGBk[3 * seg + 1] + bg[1] * om;
        const float cb = RGBk[3 * seg + 2] + bg[2] * om;
        ar = ar + cr * g; ag = ag + cg * g; ab = ab + cb * g;
        ao = ao + O * g;
        depth[r * K + k] = Dk[seg];
    }
    rgb[3 * r] = ar; rgb[3 * r + 1] = ag; rgb[3 * r + 2] = ab; opacity[r] = ao;
}

// backward of the gated combine: d gate (B,K)
__global__ void __launch_bounds__(256)
k_ml_combine_bw(int n_rays, int K, const float* __restrict__ gRGB, const float* __restrict__ gO,
                const float* __restrict__ Ok, const float* __restrict__ RGBk,
                const float* __restrict__ bg, float* __restrict__ dgate) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rays) return;
    const float gr = gRGB[3 * r], gg = gRGB[3 * r + 1], gb = gRGB[3 * r + 2], go = gO[r];
    for (int k = 0; k < K; ++k) {
        const int seg = k * n_rays + r;
        const float O = Ok[seg], om = 1 - O;
        const float cr = RGBk[3 * seg] + bg[0] * om;
        const float cg = RGBk[3 * seg + 1] + bg[1] * om;
        const float cb = RGBk[3 * seg + 2] + bg[2] * om;
        dgate[r * K + k] = gr * cr + gg * cg + gb * cb + go * O;
    }
}

// composite backward with the seeds of the gated combine folded in:
//   dRGB_k = g_k dL/drgb ; dO_k = g_k (dL/dO - bg . dL/drgb) ; dD_k = dL/ddepth[:,k]
__global__ void __launch_bounds__(256)
k_ml_composite_bw(int n_rays, int K, const float* __restrict__ gRGB,
                  const float* __restrict__ gO, const float* __restrict__ gDepth,
                  const float* __restrict__ gate, const float* __restrict__ bg,
                  const float* __restrict__ sig, const float* __restrict__ rgbs,
                  const float* __restrict__ dl, const float* __restrict__ ts,
                  const int32_t* __restrict__ counts, const int32_t* __restrict__ offsets,
                  const float* __restrict__ Ok, const float* __restrict__ Dk,
                  const float* __restrict__ RGBk, float thr, float* __restrict__ dsig,
                  float* __restrict__ drgb) {
    const int seg = blockIdx.x * (blockDim.x / RN_WAVE) + (threadIdx.x / RN_WAVE);
    if (seg >= n_rays * K) return;
    const int k = seg / n_rays, r = seg - k * n_rays;
    const float g = gate[r * K + k];
    const float gr = g * gRGB[3 * r], gg = g * gRGB[3 * r + 1], gb = g * gRGB[3 * r + 2];
    const float bgdot = bg[0] * gRGB[3 * r] + bg[1] * gRGB[3 * r + 1] + bg[2] * gRGB[3 * r + 2];
    const float go = g * (gO[r] - bgdot);
    const float gd = gDepth ? gDepth[r * K + k] : 0.f;
    seg_backward(sig, rgbs, dl, ts, nullptr, nullptr, offsets[seg], counts[seg], thr,
                 RGBk[3 * seg], RGBk[3 * seg + 1], RGBk[3 * seg + 2], Ok[seg], Dk[seg], gr, gg,
                 gb, go, gd, dsig, drgb);
}

// ---------------------------------------------------------------------------
// distortion loss (Mip-NeRF 360 / DVGO-v2), losses.cu:9-150.  The reference
// runs four thrust scans per ray inside one thread plus torch elementwise ops
// and a per-thread thrust::reduce; here one wave per rays_a row does the
// scans as wave prefix sums and reduces the per-sample terms in registers.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
k_distortion_fw(int n_rows, const float* __restrict__ ws, const float* __restrict__ dl,
                const float* __restrict__ ts, const int64_t* __restrict__ rays_a,
                float* __restrict__ loss, float* __restrict__ ws_incl,
                float* __restrict__ wts_incl) {
    const int row = blockIdx.x * (blockDim.x / RN_WAVE) + (threadIdx.x / RN_WAVE);
    if (row >= n_rows) return;
    const int lane = rn_lane();
    const int64_t ray = rays_a[3 * row], start = rays_a[3 * row + 1];
    const int n = (int)rays_a[3 * row + 2];
    float pw = 0.f, pwt = 0.f, acc = 0.f;
    for (int base = 0; base < n; base += RN_WAVE) {
        const int i = base + lane;
        const bool valid = i < n;
        float w = 0.f, t = 0.f, d = 0.f;
        if (valid) { w = ws[start + i]; t = ts[start + i]; d = dl[start + i]; }
        const float wt = w * t;
        const float sw = pw + rn_wave_incl_sum(w);
        const float swt = pwt + rn_wave_incl_sum(wt);
        const float ex_w = rn_wave_shr1(sw, pw), ex_wt = rn_wave_shr1(swt, pwt);   // exclusive scans
        if (valid) {
            ws_incl[start + i] = sw;
            wts_incl[start + i] = swt;
            acc += 2.0f * (swt * ex_w - sw * ex_wt) + (1.0f / 3) * w * w * d;
        }
        pw = rn_wave_last(sw);
        pwt = rn_wave_last(swt);
    }
    acc = rn_wave_sum(acc);
    if (lane == 0) loss[ray] = acc;
}

__global__ void __launch_bounds__(256)
k_distortion_bw(int n_rows, const float* __restrict__ dL_dloss,
                const float* __restrict__ ws_incl, const float* __restrict__ wts_incl,
                const float* __restrict__ ws, const float* __restrict__ dl,
                const float* __restrict__ ts, const int64_t* __restrict__ rays_a,
                float* __restrict__ dL_dws) {
    const int row = blockIdx.x * (blockDim.x / RN_WAVE) + (threadIdx.x / RN_WAVE);
    if (row >= n_rows) return;
    const int lane = rn_lane();
    const int64_t ray = rays_a[3 * row], start = rays_a[3 * row + 1];
    const int n = (int)rays_a[3 * row + 2];
    if (n <= 0) return;
    const int64_t end = start + n - 1;
    const float ws_sum = ws_incl[end], wts_sum = wts_incl[end];
    const float g = dL_dloss[ray];
    for (int base = 0; base < n; base += RN_WAVE) {
        const int i = base + lane;
        if (i >= n) break;
        const int64_t s = start + i;
        const float t = ts[s];
        const float front = i == 0 ? 0.f : t * ws_incl[s - 1] - wts_incl[s - 1];
        const float back = wts_sum - wts_incl[s] - t * (ws_sum - ws_incl[s]);
        float v = g * 2 * (front + back);
        v += g * (2.0f / 3) * ws[s] * dl[s];
        dL_dws[s] = v;
    }
}

inline int nblk(int64_t n, int t) { return (int)((n + t - 1) / t); }

}  // namespace

extern "C" {

int rn_composite_train_fw(const float* sigmas, const float* rgbs, const float* deltas,
                          const float* ts, const int64_t* rays_a, int64_t n_rows,
                          float T_threshold, int64_t* total_samples, float* opacity,
                          float* depth, float* rgb, float* ws, void* stream) {
    RN_CHECK_ARG(n_rows >= 0, "bad sizes");
    if (n_rows == 0) return 0;
    RN_CHECK_ARG(rays_a && total_samples && opacity && depth && rgb, "null pointer");
    k_composite_fw<<<nblk(n_rows, 4), 256, 0, (hipStream_t)stream>>>(
        (int)n_rows, sigmas, rgbs, deltas, ts, rays_a, T_threshold, total_samples, opacity, depth,
        rgb, ws);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_composite_train_bw(const float* dL_dopacity, const float* dL_ddepth, const float* dL_drgb,
                          const float* dL_dws, const float* sigmas, const float* rgbs,
                          const float* ws, const float* deltas, const float* ts,
                          const int64_t* rays_a, int64_t n_rows, const float* opacity,
                          const float* depth, const float* rgb, float T_threshold,
                          float* dL_dsigmas, float* dL_drgbs, void* stream) {
    RN_CHECK_ARG(n_rows >= 0, "bad sizes");
    if (n_rows == 0) return 0;
    RN_CHECK_ARG(dL_dopacity && dL_ddepth && dL_drgb && rays_a && opacity && depth && rgb,
                 "null pointer");
    k_composite_bw<<<nblk(n_rows, 4), 256, 0, (hipStream_t)stream>>>(
        (int)n_rows, dL_dopacity, dL_ddepth, dL_drgb, dL_dws, sigmas, rgbs, ws, deltas, ts, rays_a,
        opacity, depth, rgb, T_threshold, dL_dsigmas, dL_drgbs);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_composite_test_fw(const float* sigmas, const float* rgbs, const float* deltas,
                         const float* ts, int64_t n_alive, int32_t n_samples,
                         int64_t* alive_indices, float T_threshold, const int32_t* n_eff_samples,
                         float* opacity, float* depth, float* rgb, void* stream) {
    RN_CHECK_ARG(n_alive >= 0 && n_samples >= 1, "bad sizes");
    if (n_alive == 0) return 0;
    RN_CHECK_ARG(sigmas && rgbs && deltas && ts && alive_indices && n_eff_samples && opacity &&
                 depth && rgb, "null pointer");
    k_composite_test<<<nblk(n_alive, 256), 256, 0, (hipStream_t)stream>>>(
        (int)n_alive, n_samples, sigmas, rgbs, deltas, ts, alive_indices, T_threshold,
        n_eff_samples, opacity, depth, rgb);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_ml_composite_fw(const float* sigmas, const float* rgbs, const float* deltas,
                       const float* ts, const int32_t* counts, const int32_t* offsets,
                       int64_t n_rays, int32_t n_models, float T_threshold, int32_t* used,
                       float* opacity_k, float* depth_k, float* rgb_k, float* ws, void* stream) {
    RN_CHECK_ARG(n_rays >= 0 && n_models >= 1, "bad sizes");
    if (n_rays == 0) return 0;
    RN_CHECK_ARG(counts && offsets && used && opacity_k && depth_k && rgb_k, "null pointer");
    k_ml_composite_fw<<<nblk(n_rays * n_models, 4), 256, 0, (hipStream_t)stream>>>(
        (int)n_rays, n_models, sigmas, rgbs, deltas, ts, counts, offsets, T_threshold, used,
        opacity_k, depth_k, rgb_k, ws);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_ml_combine_fw(const float* gate, const float* opacity_k, const float* depth_k,
                     const float* rgb_k, const float* bg, int64_t n_rays, int32_t n_models,
                     float* rgb, float* opacity, float* depth, void* stream) {
    RN_CHECK_ARG(n_rays >= 0 && n_models >= 1, "bad sizes");
    if (n_rays == 0) return 0;
    RN_CHECK_ARG(gate && opacity_k && depth_k && rgb_k && bg && rgb && opacity && depth,
                 "null pointer");
    k_ml_combine_fw<<<nblk(n_rays, 256), 256, 0, (hipStream_t)stream>>>(
        (int)n_rays, n_models, gate, opacity_k, depth_k, rgb_k, bg, rgb, opacity, depth);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_ml_combine_bw(const float* dL_drgb, const float* dL_dopacity, const float* opacity_k,
                     const float* rgb_k, const float* bg, int64_t n_rays, int32_t n_models,
                     float* dL_dgate, void* stream) {
    RN_CHECK_ARG(n_rays >= 0 && n_models >= 1, "bad sizes");
    if (n_rays == 0) return 0;
    RN_CHECK_ARG(dL_drgb && dL_dopacity && opacity_k && rgb_k && bg && dL_dgate, "null pointer");
    k_ml_combine_bw<<<nblk(n_rays, 256), 256, 0, (hipStream_t)stream>>>(
        (int)n_rays, n_models, dL_drgb, dL_dopacity, opacity_k, rgb_k, bg, dL_dgate);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_ml_composite_bw(const float* dL_drgb, const float* dL_dopacity, const float* dL_ddepth,
                       const float* gate, const float* bg, const float* sigmas,
                       const float* rgbs, const float* deltas, const float* ts,
                       const int32_t* counts, const int32_t* offsets, const float* opacity_k,
                       const float* depth_k, const float* rgb_k, int64_t n_rays,
                       int32_t n_models, float T_threshold, float* dL_dsigmas, float* dL_drgbs,
                       void* stream) {
    RN_CHECK_ARG(n_rays >= 0 && n_models >= 1, "bad sizes");
    if (n_rays == 0) return 0;
    RN_CHECK_ARG(dL_drgb && dL_dopacity && gate && bg && counts && offsets && opacity_k &&
                 depth_k && rgb_k, "null pointer");
    k_ml_composite_bw<<<nblk(n_rays * n_models, 4), 256, 0, (hipStream_t)stream>>>(
        (int)n_rays, n_models, dL_drgb, dL_dopacity, dL_ddepth, gate, bg, sigmas, rgbs, deltas,
        ts, counts, offsets, opacity_k, depth_k, rgb_k, T_threshold, dL_dsigmas, dL_drgbs);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_distortion_loss_fw(const float* ws, const float* deltas, const float* ts,
                          const int64_t* rays_a, int64_t n_rows, float* loss, float* ws_incl,
                          float* wts_incl, void* stream) {
    RN_CHECK_ARG(n_rows >= 0, "bad sizes");
    if (n_rows == 0) return 0;
    RN_CHECK_ARG(ws && deltas && ts && rays_a && loss && ws_incl && wts_incl, "null pointer");
    k_distortion_fw<<<nblk(n_rows, 4), 256, 0, (hipStream_t)stream>>>(
        (int)n_rows, ws, deltas, ts, rays_a, loss, ws_incl, wts_incl);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_distortion_loss_bw(const float* dL_dloss, const float* ws_incl, const float* wts_incl,
                          const float* ws, const float* deltas, const float* ts,
                          const int64_t* rays_a, int64_t n_rows, float* dL_dws, void* stream) {
    RN_CHECK_ARG(n_rows >= 0, "bad sizes");
    if (n_rows == 0) return 0;
    RN_CHECK_ARG(dL_dloss && ws_incl && wts_incl && ws && deltas && ts && rays_a && dL_dws,
                 "null pointer");
    k_distortion_bw<<<nblk(n_rows, 4), 256, 0, (hipStream_t)stream>>>(
        (int)n_rows, dL_dloss, ws_incl, wts_incl, ws, deltas, ts, rays_a, dL_dws);
    RN_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
