// A C++ consumer of the C-ABI (include/radnerf.h) with no Python and no torch:
// what a maintainer's own host code (or a cgo / JNI / N-API shim) sees.  It
// runs one ray batch through  rn_ray_aabb_intersect -> near clamp ->
// rn_raymarching_train_count -> rn_scan_segments -> rn_raymarching_train_write
// -> rn_composite_train_fw -> rn_composite_train_bw  (the vren ops of
// models/custom_functions.py:8-159) on device buffers it owns, and writes the
// results for tests/test_gpu_capi.py to check against the CPU oracle.
//
//   capi_smoke <in.bin> <out.bin>
// in : int64 B, int64 bitfield_bytes, float scale, float esf, int32 cascades,
//      rays_o[B*3], rays_d[B*3], noise[B], bitfield[bytes]   (little endian)
// out: int64 total, rays_a[B*3] i64, ts[total], deltas[total], sigma[total],
//      rgbs[total*3], total_samples[B] i64, opacity[B], depth[B], rgb[B*3],
//      dsigma[total], drgb[total*3]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include "radnerf.h"

#define CK(x) do { int _s = (x); if (_s) { fprintf(stderr, "%s -> %d: %s\n", #x, _s, rn_last_error()); return 1; } } while (0)
#define HK(x) do { hipError_t _e = (x); if (_e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(_e)); return 1; } } while (0)

template <typename T> T* dev(size_t n) { void* p = nullptr; if (hipMalloc(&p, n * sizeof(T) + 16) != hipSuccess) { fprintf(stderr, "hipMalloc\n"); exit(1); } return (T*)p; }
template <typename T> void h2d(T* d, const std::vector<T>& h) { (void)hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice); }
template <typename T> std::vector<T> d2h(const T* d, size_t n) { std::vector<T> h(n); (void)hipMemcpy(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost); return h; }
template <typename T> void put(FILE* f, const std::vector<T>& v) { fwrite(v.data(), sizeof(T), v.size(), f); }

int main(int argc, char** argv) {
    if (argc != 3) { fprintf(stderr, "usage: capi_smoke in.bin out.bin\n"); return 2; }
    FILE* fi = fopen(argv[1], "rb");
    if (!fi) return 2;
    int64_t B, nbytes; float scale, esf; int32_t cascades;
    if (fread(&B, 8, 1, fi) != 1 || fread(&nbytes, 8, 1, fi) != 1 || fread(&scale, 4, 1, fi) != 1 ||
        fread(&esf, 4, 1, fi) != 1 || fread(&cascades, 4, 1, fi) != 1) return 2;
    std::vector<float> o(B * 3), d(B * 3), nz(B);
    std::vector<uint8_t> bits(nbytes);
    if (fread(o.data(), 4, B * 3, fi) != (size_t)B * 3 || fread(d.data(), 4, B * 3, fi) != (size_t)B * 3 ||
        fread(nz.data(), 4, B, fi) != (size_t)B || fread(bits.data(), 1, nbytes, fi) != (size_t)nbytes) return 2;
    fclose(fi);
    const int grid = 128, max_samples = 1024;
    hipStream_t st;
    HK(hipStreamCreate(&st));
    float *d_o = dev<float>(B * 3), *d_d = dev<float>(B * 3), *d_nz = dev<float>(B);
    uint8_t* d_bits = dev<uint8_t>(nbytes);
    h2d(d_o, o); h2d(d_d, d); h2d(d_nz, nz); h2d(d_bits, bits);
    // a1: ray-AABB against the scene box, then the NEAR_DISTANCE clamp of
    // ml_rendering.py:48-50 on the host copy
    std::vector<float> center = {0.f, 0.f, 0.f}, half = {scale, scale, scale};
    float *d_c = dev<float>(3), *d_h = dev<float>(3), *d_hits = dev<float>(B * 2);
    int32_t* d_cnt = dev<int32_t>(B);
    int64_t* d_vox = dev<int64_t>(B);
    h2d(d_c, center); h2d(d_h, half);
    CK(rn_ray_aabb_intersect(d_o, d_d, d_c, d_h, B, 1, 1, d_cnt, d_hits, d_vox, st));
    HK(hipStreamSynchronize(st));
    std::vector<float> hits = d2h(d_hits, B * 2);
    for (int64_t r = 0; r < B; ++r)
        if (hits[2 * r] >= 0.f && hits[2 * r] < 0.01f) hits[2 * r] = 0.01f;
    h2d(d_hits, hits);
    // a2: count -> scan -> write
    int32_t *d_counts = dev<int32_t>(B), *d_off = dev<int32_t>(B), *d_base = dev<int32_t>(1),
            *d_segc = dev<int32_t>(1), *d_meta = dev<int32_t>(2);
    CK(rn_raymarching_train_count(d_o, d_d, d_hits, d_bits, cascades, scale, esf, d_nz, grid,
                                  max_samples, B, d_counts, st));
    CK(rn_scan_segments(d_counts, 1, B, 1, d_off, d_base, d_segc, d_meta, st));
    HK(hipStreamSynchronize(st));
    const int64_t total = d2h(d_meta, 2)[1];
    int64_t* d_ra = dev<int64_t>(B * 3);
    float *d_x = dev<float>(total * 3 + 3), *d_dir = dev<float>(total * 3 + 3),
          *d_dt = dev<float>(total + 1), *d_t = dev<float>(total + 1);
    CK(rn_raymarching_train_write(d_o, d_d, d_hits, d_bits, cascades, scale, esf, d_nz, grid,
                                  max_samples, B, d_counts, d_off, d_ra, d_x, d_dir, d_dt, d_t, st));
    HK(hipStreamSynchronize(st));
    std::vector<float> ts = d2h(d_t, total), dts = d2h(d_dt, total);
    // a7/a8: composite a medium defined on the samples (sigma and colour as
    // functions of t), forward then backward with fixed seeds
    std::vector<float> sig(total), rgbs(total * 3);
    for (int64_t s = 0; s < total; ++s) {
        sig[s] = 40.f * (1.f + sinf(7.f * ts[s]));
        for (int c = 0; c < 3; ++c) rgbs[3 * s + c] = 0.5f + 0.5f * cosf(3.f * ts[s] + c);
    }
    float *d_sig = dev<float>(total + 1), *d_rgbs = dev<float>(total * 3 + 3),
          *d_ws = dev<float>(total + 1), *d_op = dev<float>(B), *d_de = dev<float>(B),
          *d_rgb = dev<float>(B * 3);
    int64_t* d_tot = dev<int64_t>(B);
    h2d(d_sig, sig); h2d(d_rgbs, rgbs);
    CK(rn_composite_train_fw(d_sig, d_rgbs, d_dt, d_t, d_ra, B, 1e-4f, d_tot, d_op, d_de, d_rgb,
                             d_ws, st));
    std::vector<float> gO(B), gD(B), gR(B * 3), gW(total + 1, 0.f);
    for (int64_t r = 0; r < B; ++r) {
        gO[r] = 0.1f * sinf(r); gD[r] = 0.05f * cosf(r);
        for (int c = 0; c < 3; ++c) gR[3 * r + c] = 0.2f * sinf(3.f * r + c);
    }
    float *d_gO = dev<float>(B), *d_gD = dev<float>(B), *d_gR = dev<float>(B * 3),
          *d_gW = dev<float>(total + 1), *d_dsig = dev<float>(total + 1),
          *d_drgb = dev<float>(total * 3 + 3);
    h2d(d_gO, gO); h2d(d_gD, gD); h2d(d_gR, gR); h2d(d_gW, gW);
    CK(rn_composite_train_bw(d_gO, d_gD, d_gR, d_gW, d_sig, d_rgbs, d_ws, d_dt, d_t, d_ra, B,
                             d_op, d_de, d_rgb, 1e-4f, d_dsig, d_drgb, st));
    HK(hipStreamSynchronize(st));
    FILE* fo = fopen(argv[2], "wb");
    if (!fo) return 2;
    fwrite(&total, 8, 1, fo);
    put(fo, d2h(d_ra, B * 3)); put(fo, ts); put(fo, dts); put(fo, sig); put(fo, rgbs);
    put(fo, d2h(d_tot, B)); put(fo, d2h(d_op, B)); put(fo, d2h(d_de, B)); put(fo, d2h(d_rgb, B * 3));
    put(fo, d2h(d_dsig, total)); put(fo, d2h(d_drgb, total * 3));
    fclose(fo);
    printf("capi_smoke ok: %lld rays, %lld samples\n", (long long)B, (long long)total);
    return 0;
}
