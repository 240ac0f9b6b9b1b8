// Occupancy-grid maintenance kernels + library-wide error/version plumbing.
//
// Reference: models/csrc/raymarching.cu:62-161 (morton3D, morton3D_invert,
// packbits), used by MNGP.update_density_grid (models/networks.py:330-409).
#include "rn_common.h"
#include "rn_sig.h"
#include <stdarg.h>
#include <stdio.h>
#pragma clang fp contract(off)

static thread_local char g_err[512] = {0};

extern "C" void rn_set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

namespace {

__global__ void __launch_bounds__(256)
k_morton3d(int64_t n, const int32_t* __restrict__ coords, int32_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = (int32_t)rn_morton3d(coords[3 * i], coords[3 * i + 1], coords[3 * i + 2]);
}

__global__ void __launch_bounds__(256)
k_morton3d_invert(int64_t n, const int32_t* __restrict__ idx, int32_t* __restrict__ coords) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t v = (uint32_t)idx[i];
    coords[3 * i + 0] = rn_morton3d_invert(v >> 0);
    coords[3 * i + 1] = rn_morton3d_invert(v >> 1);
    coords[3 * i + 2] = rn_morton3d_invert(v >> 2);
}

// 16 bytes of bitfield per thread: 128 density cells read as 32 x float4
__global__ void __launch_bounds__(256)
k_packbits(int64_t n_bytes, const float* __restrict__ grid, float thr, uint8_t* __restrict__ bits) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n_bytes) return;
    const float4* g = reinterpret_cast<const float4*>(grid + 8 * b);
    const float4 lo = g[0], hi = g[1];
    uint8_t v = 0;
    v |= (lo.x > thr) << 0; v |= (lo.y > thr) << 1; v |= (lo.z > thr) << 2; v |= (lo.w > thr) << 3;
    v |= (hi.x > thr) << 4; v |= (hi.y > thr) << 5; v |= (hi.z > thr) << 6; v |= (hi.w > thr) << 7;
    bits[b] = v;
}

// tmp[c, indices] = sigma (networks.py:393-394) with duplicate cells resolved
// by their max, deterministically: sigma >= 0, so the int order of the bits is
// the float order and one integer atomicMax per value suffices
__global__ void __launch_bounds__(256)
k_scatter_max(int64_t n, const int64_t* __restrict__ idx, const float* __restrict__ v,
              float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    atomicMax(reinterpret_cast<int*>(out) + idx[i], __float_as_int(fmaxf(v[i], 0.0f)));
}

inline int nblk(int64_t n, int t) { return (int)((n + t - 1) / t); }

}  // namespace

extern "C" {

// ABI history: 2 (round 4) rn_field_bwd_merged takes the page pool of
// fx_mode 4 (binned scatter), its statistics block is named fx_stats;
// rn_grid_bin / rn_grid_sum / rn_grid_binned_fold added.  3 (round 4) the
// fx_stats block grew to 640 B (position-weighted sums wq / we).  4 (round 5)
// binned records are e5m17 (rn_grid_record_encode / _decode), the GbCtl block
// carries a fault word, rn_grid_bin_layout fills 8 values.  5 (round 5) the
// wrap checksums wq / we weight element i by ((i mod 2^24) * 0x9E3779) mod
// 2^32 (a 24-bit multiply), fx_mode 2 refuses grids over 2^24 elements.  6
// (round 5) rn_bwd_plan takes balance_blocks (big chunks a multiple of the
// persistent blocks in number).  7 (round 5) wq / we weight element i by its
// byte offset 4 i; fx_mode 2 takes grids up to 2^28 elements.  8 (round 5)
// rn_bwd_plan can write the level forward's per-position input (prep),
// rn_field_fwd_levels takes prep_ready.  9 (round 6) rn_abi_signatures: the
// per-entry signature table, checked by the binding at load.
int rn_version(void) { return RN_ABI_VERSION; }

const char* rn_abi_signatures(void) { return RN_SIGNATURE_TABLE; }

const char* rn_last_error(void) { return g_err; }

int rn_morton3d(const int32_t* coords, int64_t n, int32_t* indices, void* stream) {
    RN_CHECK_ARG(n >= 0, "bad size");
    if (n == 0) return 0;
    RN_CHECK_ARG(coords && indices, "null pointer");
    k_morton3d<<<nblk(n, 256), 256, 0, (hipStream_t)stream>>>(n, coords, indices);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_morton3d_invert(const int32_t* indices, int64_t n, int32_t* coords, void* stream) {
    RN_CHECK_ARG(n >= 0, "bad size");
    if (n == 0) return 0;
    RN_CHECK_ARG(coords && indices, "null pointer");
    k_morton3d_invert<<<nblk(n, 256), 256, 0, (hipStream_t)stream>>>(n, indices, coords);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_packbits(const float* density_grid, int64_t n_bytes, float density_threshold,
                uint8_t* density_bitfield, void* stream) {
    RN_CHECK_ARG(n_bytes >= 0, "bad size");
    if (n_bytes == 0) return 0;
    RN_CHECK_ARG(density_grid && density_bitfield, "null pointer");
    RN_CHECK_ARG(((uintptr_t)density_grid & 15) == 0, "density_grid must be 16-byte aligned");
    k_packbits<<<nblk(n_bytes, 256), 256, 0, (hipStream_t)stream>>>(n_bytes, density_grid,
                                                                     density_threshold,
                                                                     density_bitfield);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_scatter_max(const int64_t* indices, const float* values, int64_t n, float* out,
                   void* stream) {
    RN_CHECK_ARG(n >= 0, "bad size");
    if (n == 0) return 0;
    RN_CHECK_ARG(indices && values && out, "null pointer");
    k_scatter_max<<<nblk(n, 256), 256, 0, (hipStream_t)stream>>>(n, indices, values, out);
    RN_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
