// Binned ("store and sum") grid-gradient scatter: the record format and page
// pool shared by the merged backward's walk (field.hip, GM 4) and the bin /
// sum passes (scatter.hip).
//
// Why: at scale 16 the merged backward spent 45 % of its time on memory-side
// u32 atomic requests (C5 8.40 ms with them, 4.66 ms without;
// profiles/r03/ablate_phases_c5_r03b.json): 63.5 walk records per sample
// (tools/records_sim.py), 1.84 records per 64-B request, at 26.6 G requests/s.
// Plain coalesced stores run at ~6 TB/s, so the walk appends its records to
// pages (256 contiguous bytes per 32-record issue), a bin pass sorts every
// page by slice in LDS, and a sum pass adds each slice's records into an
// LDS-resident int64 copy of that slice of the table (exact, order-free, so
// the gradient stays bitwise reproducible) and adds it to grid_grad once.
// Reference: the tcnn hash-grid backward this replaces
// (/root/reference/models/networks.py:300-328 -> tinycudann GridEncoding).
#pragma once
#include <stdint.h>

#define GB_PAGE 8192              // records per page (64 KB)
#define GB_SLICE_BITS 12          // largest slice: 4096 entries (64 KB of int64 pairs in LDS)
#define GB_SLICE (1u << GB_SLICE_BITS)
#define GB_MIN_SLICE_BITS 6       // smallest slice: 64 entries
#define GB_MAX_BINS 256           // slices per level (level sizes <= 2^20 entries)

// A level's slice size: the smallest power of two >= 64 that cuts the level
// into at most 128 slices (4096 at the 2^19-entry hashed levels).  The dense
// coarse levels get small slices, so their records spread over ~64-128
// workgroups of the sum pass instead of 1-23 (level 0 at scale 16 is one 4096
// slice: one workgroup took all its 1M records and set the pass's end).
__host__ __device__ __forceinline__ uint32_t gb_slice_bits(uint32_t hsize) {
    uint32_t b = GB_MIN_SLICE_BITS;
    while (b < GB_SLICE_BITS && (hsize + (1u << b) - 1u) >> b > 128u) ++b;
    return b;
}
#define GB_IDX_BITS 20            // entry index within its level
#define GB_V_BITS 22              // each feature's fixed-point value, two's complement
#define GB_V_MAX ((1 << (GB_V_BITS - 1)) - 1)
#define GB_TARGET_BITS 18         // a level's largest record maps to < 2^18 units (8x headroom)

// Record = u64: [0, 20) entry index within the level, [20, 42) feature 0,
// [42, 64) feature 1 (int22 fixed point in the level's units 2^e_l).  The
// level is the page's (a walk page holds one level's records).
__host__ __device__ __forceinline__ uint64_t gb_pack(uint32_t idx, int32_t q0, int32_t q1) {
    return (uint64_t)(idx & ((1u << GB_IDX_BITS) - 1u)) |
           ((uint64_t)((uint32_t)q0 & ((1u << GB_V_BITS) - 1u)) << GB_IDX_BITS) |
           ((uint64_t)(uint32_t)q1 << (GB_IDX_BITS + GB_V_BITS));
}
__host__ __device__ __forceinline__ uint32_t gb_idx(uint64_t r) {
    return (uint32_t)r & ((1u << GB_IDX_BITS) - 1u);
}
__host__ __device__ __forceinline__ int64_t gb_v0(uint64_t r) {
    return (int64_t)(r << (64 - GB_IDX_BITS - GB_V_BITS)) >> (64 - GB_V_BITS);
}
__host__ __device__ __forceinline__ int64_t gb_v1(uint64_t r) {
    return (int64_t)r >> (GB_IDX_BITS + GB_V_BITS);
}

int rn_debug_flags_internal();    // rn_set_debug_flags (field.hip), host side
// k_fx_check in binned mode (field.hip): redo flag (record growth, pool
// overflow) and the next step's scales
int rn_fx_check_binned(const float* fx_scale_cur, float* fx_scale_next, uint32_t* fx_stats,
                       int32_t* fx_redo, const void* ctl, uint32_t pool_pages, void* stream);

// Device control block (reset to 0 before every backward).
struct GbCtl {
    uint32_t pool_next;           // pages taken by the walk (may exceed the pool: overflow)
    uint32_t level_npages[16];    // pages of each level (the bin pass fills level_pages)
    uint32_t pad[15];
};

// Pool: page_meta[p] = level | count << 8 (written when the page closes);
// pages_in [pool][GB_PAGE] u64 (walk order), pages_out (slice order),
// desc [pool][GB_MAX_BINS] u32 = start | count << 16 of each slice's run in
// pages_out[p], level_pages [16][pool] u32.
struct GbPool {
    GbCtl* ctl;
    uint32_t* page_meta;
    uint64_t* pages_in;
    uint64_t* pages_out;
    uint32_t* desc;
    uint32_t* level_pages;
    uint32_t pool_pages;
    uint8_t slice_bits[16];       // gb_slice_bits of each level's size
};
