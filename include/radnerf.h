/*
 * radnerf.h — C ABI of librn.so, the MI355X (gfx950) Rad-NeRF hot path.
 *
 * Every entry point takes plain device pointers + sizes + a hipStream_t passed
 * as `void*`, launches asynchronously on that stream and returns
 *   0 = ok, 1 = invalid argument, 2 = launch failure
 * (rn_last_error() returns a thread-local message).  No torch types appear in
 * any signature.  Each function cites the reference interface it replaces
 * (paths relative to thu-nics/Rad-NeRF).  The Python binding that mirrors the
 * reference's `vren` module lives in rad-nerf_amd/radnerf_amd/vren.py; see
 * INTEGRATION.md for the ctypes/pybind stubs a maintainer would add.
 */
#ifndef RADNERF_H
#define RADNERF_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RN_ABI_VERSION 9   /* rn_version(): bumped on every incompatible ABI change */
#define RN_FX_STATS_BYTES 640   /* the fx_stats block of rn_field_bwd_merged / rn_grid_fx_fold */
int rn_version(void);
const char* rn_last_error(void);
/* the signature of every rn_* entry of this header, as the library was built:
 * "name:codes;..." with one code per parameter (p pointer, i int32, l int64,
 * u uint64, f float, d double), generated from this file at build time
 * (csrc/gen_sig.py).  A binding compares it with its own argument lists and
 * refuses a library built from another revision of the header. */
const char* rn_abi_signatures(void);
/* ablation switches for kernel studies (tools/ablate.py); 0 = production */
void rn_set_debug_flags(int flags);
/* ablation builds (debug flag 4096): per-phase wave cycles of the merged
 * backward, summed over waves, read and cleared (synchronous) */
int rn_debug_cycles(unsigned long long* out);
/* rn_field_fwd_levels' level groups for studies: byte g = levels (lo nibble,
 * hi nibble) of group g, every level exactly once; 0 = default (g, 15 - g) */
int rn_set_level_pairing(uint64_t pairing);

/* ---- ray / AABB -----------------------------------------------------------
 * replaces vren.ray_aabb_intersect  (models/csrc/binding.cpp:4-16,
 * intersection.cu:25-100).  hits_t (n_rays, max_hits, 2), hits_voxel_idx
 * (n_rays, max_hits) are fully written (-1 = no hit).                       */
int rn_ray_aabb_intersect(const float* rays_o, const float* rays_d, const float* centers,
                          const float* half_sizes, int64_t n_rays, int64_t n_voxels,
                          int32_t max_hits, int32_t* hit_cnt, float* hits_t,
                          int64_t* hits_voxel_idx, void* stream);

/* ---- ray / sphere ------------------------------------------------------------
 * replaces vren.ray_sphere_intersect (binding.cpp:19-31, intersection.cu:103-197):
 * t_near clamped at 0, hits sorted by t_near like torch::sort (-1 slots first). */
int rn_ray_sphere_intersect(const float* rays_o, const float* rays_d, const float* centers,
                            const float* radii, int64_t n_rays, int64_t n_spheres,
                            int32_t max_hits, int32_t* hit_cnt, float* hits_t,
                            int64_t* hits_sphere_idx, void* stream);

/* ---- training ray march ----------------------------------------------------
 * replaces vren.raymarching_train (binding.cpp:60-81, raymarching.cu:166-332)
 * as three deterministic steps: count -> rn_scan_segments -> write.
 * hits_t is the (n_rays, 2) near/far slice, noise (n_rays) in [0,1).       */
int rn_raymarching_train_count(const float* rays_o, const float* rays_d, const float* hits_t,
                               const uint8_t* density_bitfield, int32_t cascades, float scale,
                               float exp_step_factor, const float* noise, int32_t grid_size,
                               int32_t max_samples, int64_t n_rays, int32_t* counts,
                               void* stream);
int rn_raymarching_train_write(const float* rays_o, const float* rays_d, const float* hits_t,
                               const uint8_t* density_bitfield, int32_t cascades, float scale,
                               float exp_step_factor, const float* noise, int32_t grid_size,
                               int32_t max_samples, int64_t n_rays, const int32_t* counts,
                               const int32_t* offsets, int64_t* rays_a, float* xyzs, float* dirs,
                               float* deltas, float* ts, void* stream);

/* RayMarcher.backward (custom_functions.py:102-112, torch_scatter.segment_csr):
 * per rays_a row, dL_drays_o = sum dL_dxyzs, dL_drays_d = sum(dL_dxyzs*ts + dL_ddirs). */
int rn_raymarching_train_bw(const float* dL_dxyzs, const float* dL_ddirs, const float* ts,
                            const int64_t* rays_a, int64_t n_rows, float* dL_drays_o,
                            float* dL_drays_d, void* stream);
/* the same for the fused (model-major, per (model, ray) segment) layout of
 * rn_ml_compact: counts / offsets [K][B]; dL_drays_o / dL_drays_d (B, 3)
 * written (sums over the K sub-NeRFs' samples of each ray).                 */
int rn_ml_march_bw(const int32_t* counts, const int32_t* offsets, int64_t n_rays,
                   int32_t n_models, const float* ts, const float* dL_dxyzs,
                   const float* dL_ddirs, float* dL_drays_o, float* dL_drays_d, void* stream);

/* exclusive scan of counts[n_seg][n_per]; segment k starts at an `align`
 * multiple: seg_base[k], seg_count[k]; meta[0] = aligned end, meta[1] = total.
 * (replaces the atomicAdd slot allocation of raymarching.cu:237-238)         */
int rn_scan_segments(const int32_t* counts, int32_t n_seg, int64_t n_per, int32_t align,
                     int32_t* offsets, int32_t* seg_base, int32_t* seg_count, int32_t* meta,
                     void* stream);

/* ---- test-time march -------------------------------------------------------
 * replaces vren.raymarching_test (binding.cpp:84-106, raymarching.cu:335-454);
 * hits_t (n_rays_total, 2) is advanced in place.                            */
int rn_raymarching_test(const float* rays_o, const float* rays_d, float* hits_t,
                        const int64_t* alive_indices, int64_t n_alive,
                        const uint8_t* density_bitfield, int32_t cascades, float scale,
                        float exp_step_factor, int32_t grid_size, int32_t max_samples,
                        int32_t n_samples, float* xyzs, float* dirs, float* deltas, float* ts,
                        int32_t* n_eff_samples, void* stream);

/* ---- fused multi-sub-NeRF march (ml_rendering.py:47-52 + :174-179) -------
 * AABB + NEAR clamp + jitter + march for K models in one launch; counts and
 * noise are [K][n_rays]; writes compact samples (t, dt, ray).
 * Two-pass form: rn_ml_march_count -> rn_scan_segments -> rn_ml_march_write.
 * Single-pass form: rn_ml_march_count with stage_ts/stage_deltas (K*n_rays*
 * max_samples floats each; slot of (k, r) at (k*n_rays + r)*max_samples) ->
 * rn_scan_segments -> rn_ml_compact.                                       */
int rn_ml_march_count(const float* rays_o, const float* rays_d, const float* center,
                      const float* half_size, float near_distance, const float* noise,
                      const uint8_t* density_bitfields, int64_t bitfield_bytes, int32_t n_models,
                      int32_t cascades, float scale, float exp_step_factor, int32_t grid_size,
                      int32_t max_samples, int64_t n_rays, int32_t* counts, float* stage_ts,
                      float* stage_deltas, void* stream);
int rn_ml_compact(const int32_t* counts, const int32_t* offsets, int64_t n_rays, int32_t n_models,
                  int32_t max_samples, const float* stage_ts, const float* stage_deltas,
                  float* ts, float* deltas, int32_t* ray_of, void* stream);
int rn_ml_march_write(const float* rays_o, const float* rays_d, const float* center,
                      const float* half_size, float near_distance, const float* noise,
                      const uint8_t* density_bitfields, int64_t bitfield_bytes, int32_t n_models,
                      int32_t cascades, float scale, float exp_step_factor, int32_t grid_size,
                      int32_t max_samples, int64_t n_rays, const int32_t* counts,
                      const int32_t* offsets, float* ts, float* deltas, int32_t* ray_of,
                      void* stream);

/* ---- compositing -----------------------------------------------------------
 * replaces vren.composite_train_fw / _bw / composite_test_fw
 * (binding.cpp:109-194, volumerendering.cu:6-286).                          */
int rn_composite_train_fw(const float* sigmas, const float* rgbs, const float* deltas,
                          const float* ts, const int64_t* rays_a, int64_t n_rows,
                          float T_threshold, int64_t* total_samples, float* opacity,
                          float* depth, float* rgb, float* ws, void* stream);
int rn_composite_train_bw(const float* dL_dopacity, const float* dL_ddepth, const float* dL_drgb,
                          const float* dL_dws, const float* sigmas, const float* rgbs,
                          const float* ws, const float* deltas, const float* ts,
                          const int64_t* rays_a, int64_t n_rows, const float* opacity,
                          const float* depth, const float* rgb, float T_threshold,
                          float* dL_dsigmas, float* dL_drgbs, void* stream);
int rn_composite_test_fw(const float* sigmas, const float* rgbs, const float* deltas,
                         const float* ts, int64_t n_alive, int32_t n_samples,
                         int64_t* alive_indices, float T_threshold, const int32_t* n_eff_samples,
                         float* opacity, float* depth, float* rgb, void* stream);

/* ---- distortion loss (Mip-NeRF 360 / DVGO-v2) ------------------------------
 * replaces vren.distortion_loss_fw / _bw (binding.cpp:197-231, losses.cu:9-150).
 * fw writes loss[rays_a[n][0]] and the per-sample inclusive scans of ws and
 * ws*ts; bw consumes those scans (losses.py:6-36 DistortionLoss).            */
int rn_distortion_loss_fw(const float* ws, const float* deltas, const float* ts,
                          const int64_t* rays_a, int64_t n_rows, float* loss, float* ws_incl,
                          float* wts_incl, void* stream);
int rn_distortion_loss_bw(const float* dL_dloss, const float* ws_incl, const float* wts_incl,
                          const float* ws, const float* deltas, const float* ts,
                          const int64_t* rays_a, int64_t n_rows, float* dL_dws, void* stream);

/* fused ml path: per-(model, ray) composite + gated combine
 * (ml_rendering.py:41-78 and the bg term of :192-200)                       */
int rn_ml_composite_fw(const float* sigmas, const float* rgbs, const float* deltas,
                       const float* ts, const int32_t* counts, const int32_t* offsets,
                       int64_t n_rays, int32_t n_models, float T_threshold, int32_t* used,
                       float* opacity_k, float* depth_k, float* rgb_k, float* ws, void* stream);
int rn_ml_combine_fw(const float* gate, const float* opacity_k, const float* depth_k,
                     const float* rgb_k, const float* bg, int64_t n_rays, int32_t n_models,
                     float* rgb, float* opacity, float* depth, void* stream);
int rn_ml_combine_bw(const float* dL_drgb, const float* dL_dopacity, const float* opacity_k,
                     const float* rgb_k, const float* bg, int64_t n_rays, int32_t n_models,
                     float* dL_dgate, void* stream);
int rn_ml_composite_bw(const float* dL_drgb, const float* dL_dopacity, const float* dL_ddepth,
                       const float* gate, const float* bg, const float* sigmas,
                       const float* rgbs, const float* deltas, const float* ts,
                       const int32_t* counts, const int32_t* offsets, const float* opacity_k,
                       const float* depth_k, const float* rgb_k, int64_t n_rays,
                       int32_t n_models, float T_threshold, float* dL_dsigmas, float* dL_drgbs,
                       void* stream);

/* ---- field: shared hash grid + per-model geo/rgb MLP -----------------------
 * replaces MNGP.forward / tcnn Encoding+Network fwd/bwd
 * (models/networks.py:229-328, custom_functions.py:162-173).
 * Sample input: xyzs/dirs (n_samples, 3) [single model], or, when xyzs is
 * NULL, compact (ts, ray_of) + rays with per-model seg_base/seg_count.
 * level_* (16 entries) and xyz_min/extent (3) are HOST arrays read at launch;
 * frags = packed f16 weights (device).
 * rn_field_bwd ADDS into grid_grad (fp32, tcnn layout) and dw (fp32, K x
 * FIELD_PARAMS); the caller zeroes them when a fresh gradient is wanted.
 * feat_cache (optional, device, 64 B per sample slot = 32 f16 encodings,
 * indexed like the samples): rn_field_fwd writes the hash-grid encoding there
 * and rn_field_bwd reads it instead of re-gathering the grid.  Pass the same
 * buffer and sample layout to both, or NULL to both.                       */
int rn_field_fwd(const float* xyzs, const float* dirs, int64_t n_samples, const float* ts,
                 const int32_t* ray_of, const float* rays_o, const float* rays_d,
                 const int32_t* seg_base, const int32_t* seg_count, int32_t n_models,
                 const void* grid_f16, const uint32_t* level_offset, const uint32_t* level_hsize,
                 const uint32_t* level_res, const float* level_scale, const float* xyz_min,
                 const float* extent, const void* frags, float* sigma, float* rgb,
                 void* feat_cache, int32_t blocks_per_model, void* stream);
int rn_field_bwd(const float* xyzs, const float* dirs, int64_t n_samples, const float* ts,
                 const int32_t* ray_of, const float* rays_o, const float* rays_d,
                 const int32_t* seg_base, const int32_t* seg_count, int32_t n_models,
                 const void* grid_f16, const uint32_t* level_offset, const uint32_t* level_hsize,
                 const uint32_t* level_res, const float* level_scale, const float* xyz_min,
                 const float* extent, const void* frags, const float* dL_dsigma,
                 const float* dL_drgb, float* grid_grad, float* dw, const void* feat_cache,
                 int32_t blocks_per_model, void* stream);

/* ---- merged field backward (fused training path) ------------------------
 * Same gradients as rn_field_bwd over the compact layout of rn_ml_compact,
 * but the hash-grid gradient of the K sub-NeRFs (which share the grid) is
 * scattered in merged per-ray (ray, t) order, so samples of different models
 * on one ray share atomic requests.
 * rn_bwd_plan builds the merged order (mstart [n_rays + 1] i32, perm [total]
 * i32) and the chunk schedule (chunk_first [cap_chunks + 1] i32: head_chunks
 * chunks ramping from ~0 to head_size merged samples, chunk c of
 * [head_size c (c + 1) / (2 head_chunks), head_size (c + 1) (c + 2) / (2
 * head_chunks)) (one per block, so the blocks' walks start staggered; none
 * when the ramp passes 15/16 of the work), then big chunks up to 15/16 of the work, then
 * min_chunk;
 * the big chunks are max_chunk merged samples, or with balance_blocks > 0 a
 * multiple of balance_blocks in number, each of at most max_chunk (every
 * persistent block takes the same number of them);
 * queue [3] i32 = bwd ticket, chunk count, fwd ticket; chunk_desc
 * [cap_chunks][20] i32 = first ray, end ray, 2 pad, first sample [8], count [8]
 * per model, read by the merged kernels with one 80-B load per ticket).  cap_chunks must bound the chunk
 * count: >= head_chunks + total/max_chunk + total/(8*min_chunk) + max_chunk/min_chunk + 3
 * (+ balance_blocks when balancing): the last big chunk can leave up to
 * max_chunk more samples to the min_chunk tail.  A smaller cap
 * truncates the schedule: the samples past it are not scattered.  With prep (optional, [total] x 4 f32)
 * it also writes each merged position's (unit x, y, z, sample id as i32 bits)
 * for rn_field_fwd_levels (then called with prep_ready = 1): rays_o, rays_d
 * (device) and xyz_min, extent (host, 3 f32 each) are needed only then.
 * rn_field_bwd_merged runs `blocks` persistent blocks pulling chunks; each
 * stages 80-B rows in its scratch slice (scratch: blocks x scratch_rows x 20
 * f32, scratch_rows >= max_chunk + n_models * max_samples) and parks per-model
 * dW accumulators in park (blocks x n_models x 16384 f32).
 * Replaces, with rn_field_bwd, the backward of the tcnn modules called at
 * models/networks.py:300-328 (autograd sums the K sub-NeRFs' gradients into
 * the shared xyz_encoder's).                                               */
int rn_bwd_plan(const int32_t* counts, const int32_t* offsets, const int32_t* seg_base,
                const int32_t* seg_count, const float* ts, int64_t n_rays, int32_t n_models,
                int32_t head_chunks, int32_t head_size, int32_t max_chunk, int32_t min_chunk,
                int32_t balance_blocks, int32_t cap_chunks, int32_t* mstart, int32_t* perm,
                int32_t* chunk_first, int32_t* chunk_desc, int32_t* queue, const float* rays_o,
                const float* rays_d, const float* xyz_min, const float* extent, float* prep,
                void* stream);
int rn_field_bwd_merged(const float* ts, const int32_t* ray_of, const float* rays_o,
                        const float* rays_d, const int32_t* seg_base, const int32_t* seg_count,
                        const int32_t* mstart, const int32_t* perm,
                        const int32_t* chunk_desc, int32_t* queue, int64_t n_rays,
                        int32_t n_models, int32_t max_samples,
                        const void* grid_f16, const uint32_t* level_offset,
                        const uint32_t* level_hsize, const uint32_t* level_res,
                        const float* level_scale, const float* xyz_min, const float* extent,
                        const void* frags, const float* dL_dsigma, const float* dL_drgb,
                        float* grid_grad, float* dw, const void* feat_cache, float* scratch,
                        int64_t scratch_rows, float* park, int32_t max_chunk, int32_t blocks,
                        int32_t* igrad_lo, int32_t* igrad_carry, const float* igrad_scale,
                        int32_t* fx_acc, const float* fx_scale, uint32_t* fx_stats,
                        const int32_t* fx_redo, int32_t fx_mode, void* gb_ctl,
                        uint32_t* gb_page_meta, uint64_t* gb_pages, int32_t gb_pool_pages,
                        void* stream);

/* Fixed-point accumulation of the grid gradient (fx_mode 2, the fused
 * renderer's default; needs the encoding cache).  fx_acc: int32, one
 * per grid_grad element, zero on entry; fx_scale [16] f32 per level: 2^e_l, or
 * 0 for fp32 atomics into grid_grad (the first step); fx_stats: the
 * RN_FX_STATS_BYTES (640-B) per-level statistics block, zero before the first
 * step: u32 vmax[16] (the kernel atomic-maxes the bits of each level's largest
 * |record|), u32 emax[16] (rn_grid_fx_fold: the level's largest |int32 entry|),
 * i64 qsum[16] (the exact sum of each level's integer records), i64 esum[16]
 * (rn_grid_fx_fold: the exact sum of the level's int32 entries), u64 wq[16]
 * and we[16] (the same sums with each element i weighted by its byte offset
 * 4 i, mod 2^64; fixed point needs a grid of at most 2^28 gradient elements,
 * so the weight is injective below 2^30).
 * Each record goes in as rint(v * 2^e_l) with non-returning u32 atomics (the
 * memory side serves them ~27 % faster than f32 adds), so those levels'
 * gradients are order-independent and bitwise reproducible.
 * rn_grid_fx_fold then (1) sets *fx_redo when a level's largest record reached
 * 2^30 units or was not finite, or when the level's entry sum differs from its
 * record sum, plain or weighted (an int32 entry wrapped: many same-sign
 * records; two opposite wraps cancel only in the plain sum), writes the
 * next step's scales
 * (2^(27 - e), |record| < 2^e, capped so the largest entry stays < 2^29 units;
 * a dense level's first fixed-point step 2^(14 - e)) to fx_scale_next and clears
 * the statistics, (2) adds fx_acc * 2^-e_l into grid_grad (skipped when *fx_redo)
 * and re-zeroes fx_acc.  The caller then launches rn_field_bwd_merged with
 * fx_mode 3 and the same fx_scale (fp32 redo of the fixed-point levels' grid
 * scatter, no dW): it returns at once unless *fx_redo is set; and swaps
 * fx_scale_cur / fx_scale_next for the next step.
 * fx_mode 0: fp32 atomics (and the optional igrad_* integer mode).
 * fx_mode 4: binned (rn_grid_bin below): the fixed-point records (e5m17, the
 * largest < 2^38 units) are appended to the gb_* page pool (gb_ctl is reset
 * by the call) instead of atomically added; rn_grid_binned_fold then bins
 * and sums them into grid_grad (fx_acc unused).  A level whose fx_scale is 0
 * goes in by fp32 atomics into grid_grad instead (the renderer zeroes the
 * coarse levels', FusedMLRenderer.bin_f32_levels).
 * fx_mode 5: fx_mode 4 with levels 0-7 by fp32 atomics whatever their scale
 * (the walk's even streams compiled without page code; round 6).            */
int rn_grid_fx_fold(const uint32_t* level_offset, const uint32_t* level_hsize,
                    const uint32_t* level_res, int32_t* fx_acc, const float* fx_scale_cur,
                    float* fx_scale_next, uint32_t* fx_vmax, int32_t* fx_redo, float* grid_grad,
                    void* stream);

/* Binned ("store and sum") grid-gradient scatter, passes 2 and 3
 * (scatter.hip, formats in csrc/rn_bin.h).  Pass 1 is rn_field_bwd_merged
 * with fx_mode 4: it appends each level's fixed-point records (u64: entry
 * index 20 bits, two 22-bit e5m17 features, rn_grid_record_encode) to 64-KB
 * pages of a pool instead of issuing memory-side atomics.  ctl: the 128-B
 * GbCtl block (u32 pages taken, u32 pages per level [16], u32 fault bits:
 * 1 a page meta with a level >= 16 or more than 8192 records, 2 a record
 * index outside its level, 4 a level list past the pool, 8 a page id or run
 * outside the pool / page -- refused, never followed; then u32 sum_fault:
 * the sum passes' bit 8, sticky -- rn_field_bwd_merged zeroes only the first
 * 72 B each step, so a caller reads it back to learn that a sum pass, which
 * runs after the step's redo decision, skipped a run), zero before pass 1;
 * page_meta [pool_pages] u32 (level | count << 8); pages_in / pages_out
 * [pool_pages][8192] u64; desc
 * [pool_pages][256] u32; level_pages [16][pool_pages] u32.
 * rn_grid_bin sorts each page by slice of its level (level_hsize [16]: a
 * slice is the smallest power of two >= 64 entries that cuts the level into
 * <= 128 slices, 4096 at most) in LDS into pages_out and writes each slice's
 * run (start | count << 16) to desc and the page to its level's list.
 * rn_grid_sum (one workgroup per slice, 64 KB of LDS; the same level_hsize)
 * adds the slice's runs of every page of its level into int64
 * accumulators (exact, order-free) and then grid_grad += acc * 2^-e_l
 * (fx_scale) for every touched entry; it returns at once when *redo != 0.
 * Replaces the hash-grid parameter gradient of the tcnn GridEncoding
 * backward behind models/networks.py:300-328.                              */
/* timing studies (debug bit 21): k_grid_sum per-phase wave cycles, read and
 * reset (synchronous): [0..3] phases, [4] waves, [5] run groups, [6] / [7]
 * earliest start / latest end (s_memrealtime ticks, 100 MHz) */
int rn_debug_gb_cycles(unsigned long long* out);
int rn_grid_bin_layout(int32_t* out);   /* host: page records, bins per page, slice
                                          entries, ctl bytes, index bits, value bits,
                                          mantissa bits, target bits (out [8]) */
int rn_grid_slice_bits(const uint32_t* level_hsize, int32_t* out);   /* host: log2 of each
                                          level's slice size (out [16]) */
/* host: a record value x (gradient * 2^e_l) as the walk stores it, e5m17:
 * bits [0, 17) a two's-complement mantissa m, [17, 22) an exponent e, value
 * m * 2^e (e = 0 and m = rint(x) below 2^15; else |m| in [2^14, 2^15]), and
 * back (decode: the exact int64 value the sum pass adds) */
int rn_grid_record_encode(const float* x, int64_t n, uint32_t* out);
int rn_grid_record_decode(const uint32_t* f, int64_t n, int64_t* out);
int rn_grid_bin(const uint32_t* level_hsize, void* ctl, const uint32_t* page_meta,
                const uint64_t* pages_in, uint64_t* pages_out, uint32_t* desc,
                uint32_t* level_pages, int32_t pool_pages, int32_t blocks, void* stream);
/* rn_grid_bin + the binned redo / scale check (a record at 2^46 units, a
 * non-finite one, a pool overflow or a bin-pass fault sets *fx_redo; next
 * scales 2^(38 - e))
 * + rn_grid_sum, for a fx_mode 4 backward; the caller then launches the
 * fx_mode 3 redo exactly as after rn_grid_fx_fold.                         */
/* the first two steps of rn_grid_binned_fold (bin + check); a caller that
 * overlaps the grid gradient's all-reduce with the sum pass then runs
 * rn_grid_sum over the fine levels, starts their collective, and runs it
 * over the coarse ones (the fx_mode 3 redo may go before the sums: they exit
 * at once when *fx_redo is set) */
int rn_grid_bin_check(const uint32_t* level_hsize, void* ctl, const uint32_t* page_meta,
                      const uint64_t* pages_in, uint64_t* pages_out, uint32_t* desc,
                      uint32_t* level_pages, int32_t pool_pages, const float* fx_scale_cur,
                      float* fx_scale_next, uint32_t* fx_stats, int32_t* fx_redo, void* stream);
int rn_grid_binned_fold(const uint32_t* level_offset, const uint32_t* level_hsize, void* ctl,
                        const uint32_t* page_meta, const uint64_t* pages_in, uint64_t* pages_out,
                        uint32_t* desc, uint32_t* level_pages, int32_t pool_pages,
                        const float* fx_scale_cur, float* fx_scale_next, uint32_t* fx_stats,
                        int32_t* fx_redo, float* grid_grad, void* stream);
/* levels [level_lo, level_hi) only (0, 16: all) */
int rn_grid_sum(const uint32_t* level_offset, const uint32_t* level_hsize, const void* ctl,
                const uint32_t* desc, const uint32_t* level_pages, const uint64_t* pages_out,
                int32_t pool_pages, const float* fx_scale, const int32_t* redo, float* grid_grad,
                int32_t level_lo, int32_t level_hi, void* stream);

/* Fused test-time render (ml_rendering.py:81-155 / rendering.py:113-189,
 * raymarching.cu:335-404, volumerendering.cu:206-286): one wave per ray marches
 * its occupied samples 32 at a time (test-time calc_dt with `cascades`),
 * evaluates them as one MFMA field tile and composites them in the
 * reference's order until T <= T_threshold, the box exit or max_samples.
 * All n_models sub-NeRFs in one launch (gridDim.y); hits_t [n_rays][2] is the
 * near-clamped AABB interval (shared by the sub-NeRFs, as ml_rendering.py:
 * 91-94 computes the same one per sub-NeRF); density_bitfields
 * [n_models][bitfield_bytes]; frags [n_models][46 * 512] f16.  Outputs per
 * (sub-NeRF, ray), without background: opacity / depth [n_models][n_rays],
 * rgb [n_models][n_rays][3], n_samples (marched) [n_models][n_rays].
 * Replaces the host loop's
 * vren.raymarching_test + field + vren.composite_test_fw rounds.          */
int rn_render_test(const float* rays_o, const float* rays_d, const float* hits_t, int64_t n_rays,
                   int32_t n_models, const uint8_t* density_bitfields, int64_t bitfield_bytes,
                   int32_t cascades, float scale, float exp_step_factor, int32_t grid_size,
                   int32_t max_samples, const void* grid_f16, const uint32_t* level_offset,
                   const uint32_t* level_hsize, const uint32_t* level_res,
                   const float* level_scale, const float* xyz_min, const float* extent,
                   const void* frags, float T_threshold, float* opacity, float* depth,
                   float* rgb, int32_t* n_samples, int32_t blocks, void* stream);

/* Exact integer accumulation of the merged backward's grid gradient
 * (optional; igrad_lo == NULL keeps fp32 atomics into grid_grad).  With
 * igrad_lo / igrad_carry (int32, one per grid_grad element, zero on entry) and
 * igrad_scale (device f32, from rn_seed_scale), rn_field_bwd_merged adds each
 * contribution as rint(v * scale) with returning u32 atomics plus exact
 * carries; rn_igrad_to_f32 then adds (carry * 2^32 + lo) / scale into
 * grid_grad and re-zeroes the integer arrays.  Order-independent, so the grid
 * gradient is bitwise reproducible.  rn_seed_scale: scale = 2^(26 - e) for the
 * step's largest seed M in [2^(e-1), 2^e) (work: 1 u32 scratch word).      */
int rn_seed_scale(const int32_t* seg_base, const int32_t* seg_count, int32_t n_models,
                  const float* sigma, const float* dL_dsigma, const float* dL_drgb,
                  uint32_t* work, float* scale, void* stream);
int rn_igrad_to_f32(int64_t n, int32_t* igrad_lo, int32_t* igrad_carry, const float* scale,
                    float* grid_grad, void* stream);

/* Merged forward (fused training path, n_models <= 8): same outputs as
 * rn_field_fwd in compact mode, but blocks take rn_bwd_plan's chunks (queue
 * [2] is the forward's ticket) and evaluate the models' tiles of a chunk
 * interleaved, so the K sub-NeRFs' samples of one ray share cached grid
 * lines.  Replaces the per-sub-NeRF MNGP forward (models/networks.py:300-328
 * via ml_rendering.py:174-179).  With mstart and perm (rn_bwd_plan's merged
 * order) and feat_cache, each chunk is first encoded in merged (ray, t, model)
 * order into feat_cache, then the per-model MLP tiles read it back (NULL,
 * NULL: every tile encodes its own samples).  Outputs are identical.       */
int rn_field_fwd_merged(const float* ts, const int32_t* ray_of, const float* rays_o,
                        const float* rays_d, const int32_t* seg_base, const int32_t* seg_count,
                        const int32_t* chunk_desc, int32_t* queue,
                        int64_t n_rays, int32_t n_models, const void* grid_f16,
                        const uint32_t* level_offset, const uint32_t* level_hsize,
                        const uint32_t* level_res, const float* level_scale,
                        const float* xyz_min, const float* extent, const void* frags,
                        float* sigma, float* rgb, void* feat_cache, const int32_t* mstart,
                        const int32_t* perm, int32_t blocks, int32_t threads, void* stream);

/* Level-partitioned merged forward: the same sigma, rgb and feat_cache as
 * rn_field_fwd_merged with the merged-order encoding (bit-exact), in three
 * launches: the merged order's unit coordinates (prep: 16 B per merged
 * sample; skipped with prep_ready != 0, when rn_bwd_plan wrote them), then
 * the encoding split by level (block b encodes levels g and
 * 15 - g, g = b % 8, of every sample into planes[L * plane_stride + s], one
 * f16x2 per level; blocks go to the XCDs round-robin, so each XCD's L2 holds
 * two levels' tables), then the per-model MLP tiles read the planes.
 * plane_stride > every sample index; enc_blocks a multiple of 8; mlp_blocks of
 * 1024 threads.  xq (optional, 96 int32): [8 g + x] = blocks of group g that
 * ran on XCD x (a probe of the mapping), then u64 [32 + g] / [40 + g] the
 * first start / last end of group g's blocks (s_memrealtime, 100 MHz).  Replaces the same reference path as
 * rn_field_fwd_merged (models/networks.py:300-328 via ml_rendering.py:174-179). */
int rn_field_fwd_levels(const float* ts, const int32_t* ray_of, const float* rays_o,
                        const float* rays_d, const int32_t* seg_base, const int32_t* seg_count,
                        int64_t n_rays, int32_t n_models, const void* grid_f16,
                        const uint32_t* level_offset, const uint32_t* level_hsize,
                        const uint32_t* level_res, const float* level_scale,
                        const float* xyz_min, const float* extent, const void* frags,
                        float* sigma, float* rgb, void* feat_cache, const int32_t* mstart,
                        const int32_t* perm, uint32_t* planes, int64_t plane_stride, void* prep,
                        int32_t prep_ready, int32_t enc_blocks, int32_t mlp_blocks, int32_t* xq,
                        void* stream);

/* ---- ray gate (networks.py:1070-1093) --------------------------------------
 * input row r = (in0[r*stride + 0..2], in1[r*stride + 0..2]): pass x (B,6)
 * as (x, x+3, 6) or rays_o/rays_d as (rays_o, rays_d, 3).  importance (K) is
 * accumulated (zero it first) = gate.sum(0).                                */
int rn_gate_fwd(const float* in0, const float* in1, int32_t stride, int64_t n_rays,
                int32_t n_models, const void* frags, float* gate, float* importance,
                int32_t n_blocks, void* stream);
/* rn_gate_bwd: dL_dinput (optional, (B, 6) fp32, written): the gradient into
 * the gate input cat(in0, in1), as tcnn's Network backward provides when the
 * input requires grad (rays_o / rays_d under --optimize_ext,
 * train_ml.py:90-93); needs dinput_frags (4 transposed W0 fragments,
 * radnerf_amd/layout.py gate_dinput_frag_index).                            */
int rn_gate_bwd(const float* in0, const float* in1, int32_t stride, int64_t n_rays,
                int32_t n_models, const void* frags, const float* dL_dgate, float* dw,
                int32_t n_params, const void* dinput_frags, float* dL_dinput,
                int32_t n_blocks, void* stream);

/* ---- field input gradients and density-only evaluation (field_aux.hip) -----
 * rn_field_dinput: dL/dxyz and dL/ddir (fp32, (N, 3) each, written, indexed
 * like the samples) of MNGP.forward (models/networks.py:300-328: clip, hash
 * grid, d/|d|, SH, MLPs) for the seeds dL_dsigma / dL_drgb -- what tcnn's
 * Encoding / Network backward returns for inputs that require grad
 * (--optimize_ext, train_ml.py:90-93; custom_functions.py:102-112 consumes
 * it).  Same sample modes and arguments as rn_field_fwd/_bwd, plus
 * dinput_frags ([K][4][512] f16: the rgb net's SH columns transposed,
 * radnerf_amd/layout.py field_dinput_frag_index) and the optional encoding
 * cache of the forward.
 * rn_field_density: MNGP.density(x, ind, return_feat) (networks.py:291-309):
 * hash grid + geo MLP of one sub-NeRF (frags of that model); sigma (N) and,
 * if geo_feat is not NULL, h[:, 1:17] (N, 16) fp32 of the f16 values.       */
int rn_field_dinput(const float* xyzs, const float* dirs, int64_t n_samples, const float* ts,
                    const int32_t* ray_of, const float* rays_o, const float* rays_d,
                    const int32_t* seg_base, const int32_t* seg_count, int32_t n_models,
                    const void* grid_f16, const uint32_t* level_offset,
                    const uint32_t* level_hsize, const uint32_t* level_res,
                    const float* level_scale, const float* xyz_min, const float* extent,
                    const void* frags, const void* dinput_frags, const float* dL_dsigma,
                    const float* dL_drgb, const void* feat_cache, float* dL_dxyz,
                    float* dL_ddir, int32_t blocks_per_model, void* stream);
/* Occupancy-grid update on the device (MNGP.update_density_grid,
 * networks.py:375-409, train_ml.py:174-177), all n_models sub-NeRFs and
 * cascades in one call, no host synchronisation.  grid_ptrs / bitfield_ptrs:
 * device arrays of n_models pointers to the (cascades, 128^3) f32 density
 * grids (updated in place) and their bitfields.  all_cells != 0: every cell
 * (the warm-up, networks.py:330-343); else per (sub-NeRF, cascade) the cells
 * hit by 128^3/4 uniform draws and 128^3/4 draws among the cells with
 * density > threshold (networks.py:345-372): cell j is drawn with
 * probability 1 - e^-(1/4 + [occupied] (128^3/4) / n_occupied) (the
 * multinomial counts' Poisson limit), decided by a counter-based hash of
 * `seed` (same seed -> same cells on every rank).  Each drawn cell is
 * evaluated ONCE, at a jittered point of its cell (the reference's index_put
 * keeps one of a cell's draws, networks.py:394), in cell (Morton) order:
 * sigma from the grid + geo MLP (frags: [n_models][46 * 512] f16); then
 * grid = grid < 0 ? grid : max(grid * decay, sampled), packbits at
 * min(mean of the positive cells, threshold) (thr_out [n_models]).
 * Scratch: tmp (the sampled sigma, 0 = not drawn), occ (the drawn-cell list)
 * (n_models * cascades * 128^3 f32 / i32), blk (2 * (n_models * cascades *
 * 128^3 / 1024 + 1) i32), part (n_models * 1024 f32).  cascades <= 32.      */
int rn_density_update_sampled(const void* grid_ptrs, const void* bitfield_ptrs, int32_t n_models,
                              int32_t cascades, int32_t grid_size, float scale,
                              float density_threshold, float decay, uint64_t seed,
                              const void* grid_f16, const uint32_t* level_offset,
                              const uint32_t* level_hsize, const uint32_t* level_res,
                              const float* level_scale, const float* xyz_min, const float* extent,
                              const void* frags, float* tmp, int32_t* occ, int32_t* blk,
                              float* part, float* thr_out, int32_t all_cells,
                              void* stream);
int rn_field_density(const float* xyzs, int64_t n_samples, const void* grid_f16,
                     const uint32_t* level_offset, const uint32_t* level_hsize,
                     const uint32_t* level_res, const float* level_scale, const float* xyz_min,
                     const float* extent, const void* frags, float* sigma, float* geo_feat,
                     void* stream);

/* ---- training-step epilogue ---------------------
 * rn_nerf_loss: losses.py:44-76 (NeRFLoss: rgb MSE, opacity entropy, CV^2 of
 * the gate importance, depth-mutual) fused with its backward.  Inputs are the
 * ml_render outputs rgb (B,3), opacity (B), depth (B,K), gating_code (B,K),
 * gating_importance (K).  loss_out[4] = sums of the four terms (lambdas
 * applied; [0] over B*3, [1] over B, [2] the CV^2 scalar, [3] over B*K):
 * divide by the element counts for the reference's per-term means.  Seeds:
 * the gradients of sum(term.mean()) w.r.t. rgb, opacity, depth and gate.
 * rn_adam: torch.optim.Adam step (train_ml.py:138-153, apex FusedAdam with
 * eps 1e-15) over n fp32 params; optional f16 mirror of params[0, n_f16).
 * The hyper-parameters are doubles: the step constants (1-beta, lr/bc1,
 * sqrt(bc2)) are formed in double on the host, as torch does, then rounded
 * once to fp32.                                                              */
int rn_nerf_loss(const float* rgb, const float* target_rgb, const float* opacity,
                 const float* depth, const float* gate, const float* importance, int64_t n_rays,
                 int32_t n_models, float lambda_opacity, float lambda_cv, float lambda_dm,
                 float* loss_out, float* dL_drgb, float* dL_dopacity, float* dL_ddepth,
                 float* dL_dgate, void* stream);
int rn_adam(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
            double lr, double beta1, double beta2, double eps, int32_t step, float grad_scale,
            void* params_f16, int64_t n_f16, void* stream);

/* rn_get_rays: train_ml.py:84-96 + ray_utils.py:45-70 for a batch of picks.
 * directions (P,3) camera-space; poses (I,3,4) c2w; img_idxs (n) or NULL
 * (one pose); pix_idxs (n) or NULL (directions are per ray).  imgs_d (n,3)
 * (the gate's 'image' input: the pose applied to mean_dir) may be NULL.      */
int rn_get_rays(const float* directions, const float* poses, const int64_t* img_idxs,
                const int64_t* pix_idxs, int64_t n_rays, const float* mean_dir, float* rays_o,
                float* rays_d, float* imgs_d, void* stream);

/* ---- parameter packing (f32 master -> f16 MFMA fragments / f16 grid) ------*/
int rn_pack_f16(const float* src, int64_t src_stride, const int32_t* index, int64_t n,
                int32_t n_models, int64_t dst_stride, void* dst, void* stream);
int rn_to_f16(const float* src, int64_t n, void* dst, void* stream);

/* ---- occupancy grid maintenance (raymarching.cu:62-161, "next" row) -------*/
int rn_morton3d(const int32_t* coords, int64_t n, int32_t* indices, void* stream);
int rn_morton3d_invert(const int32_t* indices, int64_t n, int32_t* coords, void* stream);
int rn_packbits(const float* density_grid, int64_t n_bytes, float density_threshold,
                uint8_t* density_bitfield, void* stream);
/* out[indices[i]] = max(out[indices[i]], values[i]) for non-negative values:
 * the density update's `tmp[c, indices] = density(...)` (networks.py:393-394)
 * with duplicate cells resolved deterministically (the reference's
 * index_put keeps an arbitrary one of them).                                */
int rn_scatter_max(const int64_t* indices, const float* values, int64_t n, float* out,
                   void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RADNERF_H */
