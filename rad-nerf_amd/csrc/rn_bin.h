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
#include <stddef.h>
#include <stdint.h>

#ifndef GB_PAGE                   // (-D override: page-size studies)
#define GB_PAGE 8192              // records per page (64 KB)
#endif
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
#define GB_V_BITS 22              // each feature's record value (e5m17, below)
#define GB_M_BITS 17              // two's-complement mantissa
#define GB_E_MAX 31               // 5-bit exponent
#define GB_TARGET_BITS 38         // a level's largest record maps to < 2^38 units (256x headroom)
#define GB_GROWTH_UNITS 70368744177664.f   // 2^46: a record at or past it is not representable

// A record value x (the gradient times the level's 2^e_l, a float; exact,
// since 2^e_l is a power of two) is stored as e5m17: m * 2^e with
//   e = 0,          m = rint(x)            for |x| < 2^15 (exact to one unit),
//   e = E - 14 > 0, m = rint(x * 2^-e)     for 2^E <= |x| < 2^(E+1), E >= 15,
// i.e. |m| <= 2^15 with 14 significant bits past the leading one (relative
// error <= 2^-15 at and above 2^15 units), e <= 31: every |x| < 2^46 is
// representable.  The unit is 2^-38 of the level's largest record of the
// previous step, so only gradients below ~2^-39 of it round to zero.
// Why so fine: with eps = 1e-15, FusedAdam turns any non-zero gradient into an
// lr-sized step, so an entry flushed to zero changes the update as much as a
// wrong sign.  Round 4 stored x as a plain int22 (unit 2^-18 of the largest
// record): at C5's shape 1.3 % of the non-zero entries flushed and 3 Adam
// steps differed from fp32's by 24 % per level; an e4m18 form (unit 2^-27)
// still flushed 0.05 % (4.8 %), all of them entries below half a unit
// (tools/fx_entry_diag.py).  The sum pass adds m << e
// exactly in int64, so the sums stay order-free and bitwise reproducible.
// Overflow margin: a record can reach just under 2^46 units
// before the step is flagged for the redo, so an entry would need ~2^17 such
// records to leave int64 (2^25 at the 2^38 target that scales aim for); a
// scale-16 step puts tens of records on an entry, a coarse dense entry a few
// thousand.
__host__ __device__ __forceinline__ uint32_t gb_encode(float x) {
    const uint32_t E = (__builtin_bit_cast(uint32_t, x) >> 23) & 0xffu;   // biased exponent
    int e = (int)E - (127 + 14);
    e = e < 0 ? 0 : (e > GB_E_MAX ? GB_E_MAX : e);
    // clamped before the conversion (|x| >= 2^46 and NaN: the step is redone)
    const float y = fminf(fmaxf(rintf(ldexpf(x, -e)), -32768.f), 32768.f);
    return ((uint32_t)(int)y & ((1u << GB_M_BITS) - 1u)) | ((uint32_t)e << GB_M_BITS);
}
// The walk's form (field.hip GM 4): the same word for every |x| < 2^46 units
// (there |m| <= 2^15 needs no clamp); a record at or past 2^46, or NaN, sets
// the redo flag through the level's vmax (k_fx_check), and the step's pages
// are discarded, so its word need not saturate
__device__ __forceinline__ uint32_t gb_encode_walk(float x) {
    const uint32_t E = (__builtin_bit_cast(uint32_t, x) >> 23) & 0xffu;
    int e = (int)E - (127 + 14);
    e = e < 0 ? 0 : (e > GB_E_MAX ? GB_E_MAX : e);
    const int m = (int)rintf(ldexpf(x, -e));
    return ((uint32_t)m & ((1u << GB_M_BITS) - 1u)) | ((uint32_t)e << GB_M_BITS);
}
__host__ __device__ __forceinline__ int64_t gb_decode(uint32_t f) {
    const int64_t m = (int64_t)((int32_t)(f << (32 - GB_M_BITS)) >> (32 - GB_M_BITS));
    return m * ((int64_t)1 << ((f >> GB_M_BITS) & (uint32_t)GB_E_MAX));
}

// Record = u64: [0, 20) entry index within the level, [20, 42) feature 0,
// [42, 64) feature 1 (e5m17 fields in the level's units 2^e_l).  The level is
// the page's (a walk page holds one level's records).
__host__ __device__ __forceinline__ uint64_t gb_pack(uint32_t idx, uint32_t f0, uint32_t f1) {
    return (uint64_t)(idx & ((1u << GB_IDX_BITS) - 1u)) |
           ((uint64_t)(f0 & ((1u << GB_V_BITS) - 1u)) << GB_IDX_BITS) |
           ((uint64_t)(f1 & ((1u << GB_V_BITS) - 1u)) << (GB_IDX_BITS + GB_V_BITS));
}
__host__ __device__ __forceinline__ uint32_t gb_idx(uint64_t r) {
    return (uint32_t)r & ((1u << GB_IDX_BITS) - 1u);
}
__host__ __device__ __forceinline__ int64_t gb_v0(uint64_t r) {
    return gb_decode((uint32_t)(r >> GB_IDX_BITS) & ((1u << GB_V_BITS) - 1u));
}
__host__ __device__ __forceinline__ int64_t gb_v1(uint64_t r) {
    return gb_decode((uint32_t)(r >> (GB_IDX_BITS + GB_V_BITS)));
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
    uint32_t fault;               // GB_FAULT_* bits: inputs the passes refused (-> redo)
    // sticky: GB_FAULT_RUN bits of every sum pass since the block was created
    // (the per-step reset stops before it, GB_CTL_RESET_BYTES).  The sum pass
    // runs after the step's check and redo launch, so a run it refuses cannot
    // redo that step any more; the renderer reads this word back with the page
    // count and raises, instead of applying a partial gradient
    // unnoticed.
    uint32_t sum_fault;
    uint32_t pad[13];
};
#define GB_CTL_RESET_BYTES (18 * 4)      // pool_next, level_npages[16], fault
static_assert(offsetof(GbCtl, sum_fault) == GB_CTL_RESET_BYTES, "GbCtl reset span");
static_assert(sizeof(GbCtl) == 128, "GbCtl is 128 B (rn_grid_bin_layout ctl_bytes)");
// fault bits: a page's meta names a level >= 16 or more than GB_PAGE records
// (bin pass); a record's entry index lies outside its level (bin pass); a
// level's page list overflowed the pool (bin pass); a page id or run outside
// the pool / page (sum pass).  The bin pass's faults set the redo flag
// (k_fx_check runs between the bin and sum passes); the sum pass only skips.
#define GB_FAULT_META 1u
#define GB_FAULT_INDEX 2u
#define GB_FAULT_LIST 4u
#define GB_FAULT_RUN 8u

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
    uint32_t hsize[16];           // entries of each level (the bin pass checks indices)
};
