// Training-step epilogue kernels on either side of the hot path (SURVEY.md
// §8(f) rows 2-3):
//
//  * k_nerf_loss: NeRFLoss.forward (losses.py:44-76) as used by
//    train_ml.py:185-192 -- rgb MSE, opacity entropy, CV^2 of the gate
//    importance, depth-mutual -- fused with its own backward: one pass over
//    the rays writes the loss terms AND the seeds dL/drgb, dL/dopacity,
//    dL/ddepth, dL/dgate that FusedMLRenderer.backward consumes (the
//    reference runs ~15 elementwise torch kernels plus their autograd graph).
//  * k_adam: torch.optim.Adam / apex.FusedAdam(eps=1e-15) (train_ml.py:138-153)
//    over the flat fp32 parameter buffer, one pass that also refreshes the f16
//    copy of the hash table the field kernels gather from.
#include "rn_common.h"
#pragma clang fp contract(off)

namespace {

// loss_out: [0] sum over (B,3) of (rgb - t)^2, [1] sum over B of -o log o
// (lambda applied), [2] cv^2 term (lambda applied), [3] sum over (B,K) of the
// depth-mutual term (lambda applied).  The host divides by the element counts.
__global__ void __launch_bounds__(256)
k_nerf_loss(int64_t B, int K, const float* __restrict__ rgb, const float* __restrict__ target,
            const float* __restrict__ opacity, const float* __restrict__ depth,
            const float* __restrict__ gate, const float* __restrict__ importance,
            float lambda_opacity, float lambda_cv, float lambda_dm, float* __restrict__ loss_out,
            float* __restrict__ d_rgb, float* __restrict__ d_opacity, float* __restrict__ d_depth,
            float* __restrict__ d_gate) {
    __shared__ float red[4][RN_WAVE];
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = r < B;
    const bool multi = K > 1;
    // CV^2 of the importance (torch.var: unbiased), losses.py:68-70
    float mu = 0.f, var = 0.f, den = 1.f;
    const bool use_cv = multi && lambda_cv > 0.f;
    if (use_cv) {
        for (int k = 0; k < K; ++k) mu += importance[k];
        mu /= K;
        for (int k = 0; k < K; ++k) { const float e = importance[k] - mu; var += e * e; }
        var /= (K - 1);
        den = mu * mu + 1e-10f;
    }
    float l_rgb = 0.f, l_op = 0.f, l_dm = 0.f;
    if (valid) {
        // rgb MSE, mean over B x 3 (losses.py:51)
        const float inv3b = 1.0f / (3.0f * (float)B);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float e = rgb[3 * r + c] - target[3 * r + c];
            l_rgb += e * e;
            d_rgb[3 * r + c] = 2.0f * e * inv3b;
        }
        // opacity entropy, o = opacity + 1e-10 (losses.py:53-55)
        const float o = opacity[r] + 1e-10f;
        const float lg = logf(o);
        l_op = lambda_opacity * (-o * lg);
        d_opacity[r] = lambda_opacity * (-(lg + 1.0f)) / (float)B;
        // depth-mutual against the detached gate-weighted depth (losses.py:72-73)
        if (multi && lambda_dm > 0.f) {
            float mean_d = 0.f;
            for (int k = 0; k < K; ++k) mean_d += depth[r * K + k] * gate[r * K + k];
            const float s = 2.0f * lambda_dm / ((float)B * K);
            for (int k = 0; k < K; ++k) {
                const float e = depth[r * K + k] - mean_d;
                l_dm += lambda_dm * e * e;
                d_depth[r * K + k] = s * e;
            }
        } else {
            for (int k = 0; k < K; ++k) d_depth[r * K + k] = 0.f;
        }
        // dL/dgate from the CV^2 term: every ray adds to importance_k
        for (int k = 0; k < K; ++k) {
            float g = 0.f;
            if (use_cv) {
                const float e = importance[k] - mu;
                g = lambda_cv * ((2.0f * e / (K - 1)) / den - var * (2.0f * mu / K) / (den * den));
            }
            d_gate[r * K + k] = g;
        }
    }
    // block reduction of the three per-ray sums, one atomic each per block
    const int lane = rn_lane(), wid = threadIdx.x / RN_WAVE;
    float v[3] = {l_rgb, l_op, l_dm};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        float x = v[q];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
        if (lane == 0) red[q][wid] = x;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        float x = 0.f;
        for (int w = 0; w < (int)(blockDim.x / RN_WAVE); ++w) x += red[threadIdx.x][w];
        atomicAdd(&loss_out[threadIdx.x == 2 ? 3 : threadIdx.x], x);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && use_cv) loss_out[2] = lambda_cv * var / den;
}

// Adam with bias correction, in torch.optim.Adam's operation order (no weight
// decay; apex FusedAdam with weight_decay 0 is the same update):
//   m = lerp(m, g, 1-b1) ;  v = v*b2 + (1-b2)*g*g
//   p -= (lr / (1-b1^t)) * m / (sqrt(v) / sqrt(1-b2^t) + eps)
// half_out (optional): f16 copy of p[0, n_half) written in the same pass.
__global__ void __launch_bounds__(256)
k_adam(int64_t n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
       float* __restrict__ v, float step_size, float omb1, float b2, float omb2, float eps,
       float bc2_sqrt, float grad_scale, _Float16* __restrict__ half_out, int64_t n_half) {
    // torch.optim.Adam (single-tensor form): exp_avg.lerp_(g, 1-b1);
    // exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2);
    // p.addcdiv_(exp_avg, exp_avg_sq.sqrt() / sqrt(bc2) + eps, -lr/bc1)
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float gi = g[i] * grad_scale;
        const float m0 = m[i];
        const float mi = m0 + omb1 * (gi - m0);
        const float vi = v[i] * b2 + omb2 * (gi * gi);
        m[i] = mi;
        v[i] = vi;
        const float denom = sqrtf(vi) / bc2_sqrt + eps;
        const float pi = p[i] - step_size * (mi / denom);
        p[i] = pi;
        if (i < n_half) half_out[i] = (_Float16)pi;
    }
}

// train_ml.py:84-96 + datasets/ray_utils.py:45-70 (get_rays) for a batch of
// (image, pixel) picks: rays_d = R dir, rays_o = T, imgs_d = R mean_dir.
// The 3x3 rotation is applied as three dot products in (x, y, z) order.
__global__ void __launch_bounds__(256)
k_get_rays(int64_t n, const float* __restrict__ dirs, const float* __restrict__ poses,
           const int64_t* __restrict__ img_idx, const int64_t* __restrict__ pix_idx,
           const float* __restrict__ mean_dir, float* __restrict__ rays_o,
           float* __restrict__ rays_d, float* __restrict__ imgs_d) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const float* P = poses + 12 * (img_idx ? img_idx[r] : 0);     // (3, 4) row-major
    const float* d = dirs + 3 * (pix_idx ? pix_idx[r] : r);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        rays_d[3 * r + i] = d[0] * P[4 * i] + d[1] * P[4 * i + 1] + d[2] * P[4 * i + 2];
        rays_o[3 * r + i] = P[4 * i + 3];
        if (imgs_d)
            imgs_d[3 * r + i] = mean_dir[0] * P[4 * i] + mean_dir[1] * P[4 * i + 1] +
                                mean_dir[2] * P[4 * i + 2];
    }
}

inline int nblk(int64_t n, int t) { return (int)((n + t - 1) / t); }

}  // namespace

extern "C" {

int rn_nerf_loss(const float* rgb, const float* target_rgb, const float* opacity,
                 const float* depth, const float* gate, const float* importance, int64_t n_rays,
                 int32_t n_models, float lambda_opacity, float lambda_cv, float lambda_dm,
                 float* loss_out, float* dL_drgb, float* dL_dopacity, float* dL_ddepth,
                 float* dL_dgate, void* stream) {
    RN_CHECK_ARG(n_rays >= 1 && n_models >= 1, "bad sizes");
    RN_CHECK_ARG(rgb && target_rgb && opacity && depth && gate && importance && loss_out &&
                 dL_drgb && dL_dopacity && dL_ddepth && dL_dgate, "null pointer");
    if (hipMemsetAsync(loss_out, 0, 4 * sizeof(float), (hipStream_t)stream) != hipSuccess) {
        rn_set_error("rn_nerf_loss: hipMemsetAsync failed");
        return 2;
    }
    k_nerf_loss<<<nblk(n_rays, 256), 256, 0, (hipStream_t)stream>>>(
        n_rays, n_models, rgb, target_rgb, opacity, depth, gate, importance, lambda_opacity,
        lambda_cv, lambda_dm, loss_out, dL_drgb, dL_dopacity, dL_ddepth, dL_dgate);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_adam(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
            double lr, double beta1, double beta2, double eps, int32_t step, float grad_scale,
            void* params_f16, int64_t n_f16, void* stream) {
    RN_CHECK_ARG(n >= 0 && step >= 1 && n_f16 >= 0 && n_f16 <= n, "bad sizes");
    if (n == 0) return 0;
    RN_CHECK_ARG(params && grads && exp_avg && exp_avg_sq && (n_f16 == 0 || params_f16),
                 "null pointer");
    // step constants in double, as torch / apex compute them on the host,
    // rounded once to the kernel's fp32
    const double bc1 = 1.0 - pow(beta1, (double)step);
    const double bc2 = 1.0 - pow(beta2, (double)step);
    const int64_t nb = nblk(n, 256);
    const int blocks = (int)(nb < 256 * 16 ? nb : 256 * 16);
    k_adam<<<blocks, 256, 0, (hipStream_t)stream>>>(
        n, params, grads, exp_avg, exp_avg_sq, (float)(lr / bc1), (float)(1.0 - beta1),
        (float)beta2, (float)(1.0 - beta2), (float)eps, (float)sqrt(bc2), grad_scale,
        (_Float16*)params_f16, n_f16);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_get_rays(const float* directions, const float* poses, const int64_t* img_idxs,
                const int64_t* pix_idxs, int64_t n_rays, const float* mean_dir, float* rays_o,
                float* rays_d, float* imgs_d, void* stream) {
    RN_CHECK_ARG(n_rays >= 0, "bad sizes");
    if (n_rays == 0) return 0;
    RN_CHECK_ARG(directions && poses && rays_o && rays_d && (!imgs_d || mean_dir), "null pointer");
    k_get_rays<<<nblk(n_rays, 256), 256, 0, (hipStream_t)stream>>>(
        n_rays, directions, poses, img_idxs, pix_idxs, mean_dir, rays_o, rays_d, imgs_d);
    RN_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
