// Fused Rad-NeRF field for gfx950: shared multiresolution hash grid + per
// sub-NeRF geo/rgb MLPs, forward and backward.
//
// Reference (behaviour): models/networks.py:291-328 (MNGP.density/forward),
// :229-289 (tcnn Grid/Hash encoding L=16 F=2 T=2^19 N_min=16, SH degree 4,
// FullyFusedMLP geo 32->64->17, rgb 32->64->64->3 Sigmoid), custom_functions.py
// :162-173 (TruncExp).  tcnn itself is an absent third-party dependency; the
// encoding/SH/MLP semantics restated here are listed in DESIGN.md §2.
//
// Work decomposition: one wave = 32 samples.  Lane (c = lane&31, h = lane>>5)
// owns sample c and 8 of the 16 hash levels, {2h,2h+1,4+2h,5+2h,8+2h,...}: the
// same levels the wave needs in the B operand of the first MFMA layer AND in
// the accumulator of the last backward layer, so the encoding enters and
// leaves the MFMA chain without any data movement.
//
// Kernels:
//  * k_field_fwd / k_field_bwd: one sub-NeRF per blockIdx.y (the drop-in
//    path, one model at a time like the reference).
//  * k_bwd_plan + k_bwd_chunks: merged (ray, t) order of the K models'
//    samples and a chunk schedule of whole rays.
//  * k_field_fwd_merged: the K models' tiles of a chunk interleaved on one
//    CU (their corners share L1 lines).
//  * k_field_bwd_merged: per chunk, the MLP backward model by model, then the
//    hash-grid gradient of all K models scattered in merged per-ray order
//    (row-lane walk + per-stream rings of fp32 atomics; optionally exact
//    integer accumulation).
// Backward MLP: recompute the forward from the encoding cache, run the dX
// chain on MFMA, and form dW = dY . X^T block-cooperatively from sample-major
// LDS images (MFMA again), held in registers across windows.
#include "rn_field.h"
#include "rn_bin.h"
#pragma clang fp contract(off)

static int g_field_dbg = 0;
static uint64_t g_level_pairing = 0;     // rn_field_fwd_levels' level groups (0 = default)
// ablation builds only (flag 4096): per-phase wave cycles of the merged
// backward, summed over waves (s_memtime): [0] MLP phase, [1] walk staging
// (row loads + LDS fill, up to the barrier), [2] walks, [3] chunk tails
// (walk2_end: flush + drain)
__device__ unsigned long long g_rn_cyc[8];

namespace {

template <int MODE, int CACHE>
__global__ void __launch_bounds__(256, FWD_MIN_WAVES)
k_field_fwd(FieldArgs a) {
    __shared__ __attribute__((aligned(16))) rn_half sW[FIELD_FWD_FRAGS * RN_FRAG_HALFS];
    __shared__ LvTab sT;
    const int k = blockIdx.y;
    rn_block_copy16(sW, a.frags + (size_t)k * FIELD_FRAGS * RN_FRAG_HALFS,
                    FIELD_FWD_FRAGS * RN_FRAG_BYTES);
    lv_stage(sT, a.gm);
    __syncthreads();
    int64_t base, n;
    sample_range(a, MODE, k, base, n);
    const int64_t n_tiles = (n + 31) / 32;
    const int waves = blockDim.x / RN_WAVE;
    const int lane = rn_lane(), h = lane >> 5;
    for (int64_t tile = (int64_t)blockIdx.x * waves + threadIdx.x / RN_WAVE; tile < n_tiles;
         tile += (int64_t)gridDim.x * waves) {
        rn_lds_order();   // weights stay in LDS: no hoisting of fragment reads
        FwdState st;
        bool valid; int64_t s; float ux, uy, uz;
        tile_forward<MODE, CACHE>(a, sT, sW, base, n, tile, st, valid, s, ux, uy, uz);
        if (valid && h == 0) {
            // TruncExp.forward on geo output 0 (custom_functions.py:165-167)
            a.sigma[s] = expf(st.g0);
            // Sigmoid output activation in fp32 (tcnn rounds it to f16; the
            // wider output keeps one f16 ulp of rgb off the ray colour)
            a.rgb[3 * s + 0] = sigmoidf(st.out[0]);
            a.rgb[3 * s + 1] = sigmoidf(st.out[1]);
            a.rgb[3 * s + 2] = sigmoidf(st.out[2]);
        }
    }
}

// ---------------------------------------------------------------------------
// Backward.  A block = 8 waves = 256 samples per iteration (one 32-sample tile
// per wave), one model per blockIdx.y, persistent over iterations.
// Weight gradients need a contraction over samples; instead of per-wave LDS
// float atomics (measured ~5.8 ms per step: ds_add_f32 throughput), every
// wave publishes its (dY, X) layer images in LDS and the 12 dW tiles are
// OWNED by waves (1-2 each), which contract over all 256 samples of the block
// (16 MFMAs per tile) into register accumulators that persist across
// iterations and are flushed once with global atomics at the end.
// Gradient scale: one power of two per block iteration (max over the 8 waves'
// seeds); accumulators are rescaled exactly when it changes.
// ---------------------------------------------------------------------------
#define BWD_WAVES 8

// ---------------------------------------------------------------------------
// Hash-grid gradient scatter of one block iteration (256 ray-ordered samples).
//
// Global float atomics on gfx950 execute at the memory side; their cost is one
// 64-B request per distinct 64-B segment a wave instruction touches
// (MI355X_MICROARCH.md "Global float atomics"; measured here: halving the
// active lanes or making every target L2-resident leaves the kernel time
// unchanged, dropping the four finest levels' atomics halves it).  So the
// scatter is designed to issue as few distinct (instruction, segment) pairs
// as possible:
//
//  * wave w owns levels w and 15-w (one coarse + one fine, for balance);
//    lane = (half of the block's samples, level, corner, feature); each lane
//    walks its 128 samples in ray order holding one accumulator for its
//    corner of the current cell;
//  * when the cell changes by delta, the accumulator of old corner c is handed
//    (one ds_bpermute) to the lane of new corner c - delta when that is still
//    a corner of the new cell: an entry shared by consecutive cells is added
//    to once per visit of the ray, not once per cell (tcnn adds it per sample);
//    only corners that leave the cell are issued.  Requests/sample on the
//    bench workload (tools/atomic_sim.py): 34.2 with per-corner run merging,
//    27.2 with the hand-over.
// ---------------------------------------------------------------------------
#define SG_STRIDE 34
#define SC_STREAMS 8         // per wave: (quarter of the block's samples, level) pairs
#define SC_RING 48           // entry records per stream ring (>= 31 pending + 2 steps x 8)

// Finished runs are not issued by the lane that holds them: each of the
// wave's 8 streams (sample quarter, level) compacts its finished runs (ballot
// + mbcnt) into its own LDS ring of (byte offset, f0, f1) entry records and
// issues an atomic instruction when 32 entries (64 dwords) are pending, every
// lane active.  One instruction then covers consecutive samples of ONE level
// of one ray, so entries of the same 64-B segment that leave the cell at
// different steps (a ray moving along x) share one request (tools/atomic_sim.py).
// Ring storage is structure-of-arrays (offsets, f0, f1) so every LDS access
// is a 4-B word.
struct ScatterRing {
    uint32_t* ring;          // this wave's SC_STREAMS x 3 x SC_RING words
    uint32_t head[SC_STREAMS];   // per stream, wave-uniform, in [0, SC_RING)
    uint32_t tail;           // per lane: the tail of this lane's stream, in [0, SC_RING)
};

__device__ __forceinline__ void ring_issue(ScatterRing& R, int s, uint32_t cnt,
                                           __amdgpu_buffer_rsrc_t grad_rs, int dbg) {
    const int lane = rn_lane();
    asm volatile("" ::: "memory");
    if ((uint32_t)lane < 2u * cnt) {
        uint32_t rec = R.head[s] + (lane >> 1);          // < 2 SC_RING: no modulo
        rec = rec >= SC_RING ? rec - SC_RING : rec;
        const uint32_t* base = R.ring + s * 3 * SC_RING;
        const uint32_t off = base[rec] + 4u * (lane & 1);
        const uint32_t v = base[(1 + (lane & 1)) * SC_RING + rec];
        if (rn_dbg(dbg) & 1) asm volatile("" :: "v"(off), "v"(v));
        else __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(__uint_as_float(v), grad_rs,
                                                             (int)off, 0, 0);
    }
    asm volatile("" ::: "memory");
    const uint32_t h = R.head[s] + cnt;
    R.head[s] = h >= SC_RING ? h - SC_RING : h;
}

// append this step's finished runs (lanes with `emit`) to their stream rings;
// no issue here (ring_drain runs every 2 steps: 31 pending + 2 x 8 < SC_RING)
__device__ __forceinline__ void ring_push(ScatterRing& R, bool emit, uint64_t smask, uint32_t off,
                                          float v0, float v1) {
    const uint64_t m = __builtin_amdgcn_ballot_w64(emit) & smask;
    const uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi(hi, __builtin_amdgcn_mbcnt_lo(lo, 0u));
    const int s = rn_lane() >> 3;
    if (emit) {
        uint32_t* base = R.ring + s * 3 * SC_RING;
        uint32_t rec = R.tail + rank;
        rec = rec >= SC_RING ? rec - SC_RING : rec;
        base[rec] = off;
        base[SC_RING + rec] = __float_as_uint(v0);
        base[2 * SC_RING + rec] = __float_as_uint(v1);
    }
    const uint32_t t = R.tail + (uint32_t)(__builtin_popcount(lo) + __builtin_popcount(hi));
    R.tail = t >= SC_RING ? t - SC_RING : t;
}

__device__ __forceinline__ void ring_drain(ScatterRing& R, uint32_t min_cnt,
                                           __amdgpu_buffer_rsrc_t grad_rs, int dbg) {
#pragma unroll
    for (int q = 0; q < SC_STREAMS; ++q) {
        const uint32_t t = __builtin_amdgcn_readlane(R.tail, 8 * q);
        const uint32_t pend = t >= R.head[q] ? t - R.head[q] : t + SC_RING - R.head[q];
        if (pend >= min_cnt && pend > 0u) ring_issue(R, q, pend < 32u ? pend : 32u, grad_rs, dbg);
    }
}

// Walk state of one lane: its entry (coords, index) and the two features'
// accumulated gradient.  Carried across windows by the merged kernel.
struct WalkState {
    uint32_t ex, ey, ez, cur;
    float acc0, acc1;
};

__device__ __forceinline__ void walk_begin(WalkState& W) {
    W.ex = 0xffffffffu; W.ey = 0; W.ez = 0; W.cur = 0; W.acc0 = 0.f; W.acc1 = 0.f;
}

__device__ __forceinline__ LvConst walk_level(const FieldArgs& a, const LvTab& sT) {
    const int lane = rn_lane();
    const int wid = __builtin_amdgcn_readfirstlane((int)threadIdx.x / RN_WAVE);
    const int l = ((lane >> 3) & 1) ? (RN_L - 1 - wid) : wid;
    return lv_const(sT, a.gm, l);
}

// Walk one window of staged rows.  Stream quarter q's samples are rows
// [64q, 64q + nq) of sG/sU (nq per lane: its quarter's count); n0 = the
// largest nq (wave-uniform trip count).
typedef __attribute__((address_space(3))) const float lds_cf;

__device__ __forceinline__ void grid_walk_window(const FieldArgs& a, const LvTab& sT,
                                                 const float* sG_, const float* sU_, int nq, int n0,
                                                 ScatterRing& R, __amdgpu_buffer_rsrc_t grad_rs,
                                                 WalkState& W, int dbg) {
    // 32-bit LDS addressing (generic pointers make the row offsets 64-bit)
    lds_cf* sG = (lds_cf*)sG_;
    lds_cf* sU = (lds_cf*)sU_;
    const int lane = rn_lane();
    const int stream = lane >> 3, quarter = stream >> 1, par = lane & 7;
    const uint32_t px = par & 1, py = (par >> 1) & 1, pz = par >> 2;
    const LvConst lc = walk_level(a, sT);
    const uint64_t smask = 0xffull << (8 * stream);
    constexpr int QN = BWD_WAVES * 8;                     // rows per quarter
    const int s_base = quarter * QN;
    const int wid = __builtin_amdgcn_readfirstlane((int)threadIdx.x / RN_WAVE);
    lds_cf* gcol = sG + 2 * ((stream & 1) ? (RN_L - 1 - wid) : wid);
    typedef float vf4 __attribute__((ext_vector_type(4)));
    typedef float vf2 __attribute__((ext_vector_type(2)));
    typedef __attribute__((address_space(3))) const vf4 lds_cf4;
    typedef __attribute__((address_space(3))) const vf2 lds_cf2;
    // software pipeline: this step's sample row is loaded one step ahead
    vf4 un = *(lds_cf4*)(sU + s_base * 4);
    vf2 gn = *(lds_cf2*)(gcol + s_base * SG_STRIDE);
    for (int j0 = 0; j0 < n0; j0 += 2) {                  // wave-uniform trip count
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
            const int j = j0 + jj;
            const bool act = j < nq;
            const vf4 uc = un;
            const vf2 gc = gn;
            const int nx = s_base + (j + 1 < nq ? j + 1 : 0);
            un = *(lds_cf4*)(sU + nx * 4);
            gn = *(lds_cf2*)(gcol + __umul24((uint32_t)nx, SG_STRIDE));   // u32 offset, not a u64 mad
            const LevelPos p = level_pos(lc.sc, uc.x, uc.y, uc.z);
            // this class's corner of the cell: the one of {g, g+1} with parity p
            const uint32_t cx = (px ^ p.gx) & 1u, cy = (py ^ p.gy) & 1u, cz = (pz ^ p.gz) & 1u;
            const uint32_t X = p.gx + cx, Y = p.gy + cy, Z = p.gz + cz;
            const float w = (cx ? p.fx : 1.0f - p.fx) * (cy ? p.fy : 1.0f - p.fy) *
                            (cz ? p.fz : 1.0f - p.fz);
            const bool same = X == W.ex && Y == W.ey && Z == W.ez;
            ring_push(R, act && !same && W.ex != 0xffffffffu, smask, 8u * (lc.off + W.cur),
                      W.acc0, W.acc1);
            if (act) {
                W.acc0 = (same ? W.acc0 : 0.f) + w * gc.x;
                W.acc1 = (same ? W.acc1 : 0.f) + w * gc.y;
                W.cur = grid_index(lc, X, Y, Z);
                W.ex = X; W.ey = Y; W.ez = Z;
            }
        }
        ring_drain(R, 32u, grad_rs, dbg);
    }
}

// end of a walk: emit the live entry of every lane
__device__ __forceinline__ void walk_end(const FieldArgs& a, const LvTab& sT, ScatterRing& R,
                                         __amdgpu_buffer_rsrc_t grad_rs, WalkState& W, int dbg) {
    const LvConst lc = walk_level(a, sT);
    const uint64_t smask = 0xffull << (8 * (rn_lane() >> 3));
    ring_push(R, W.ex != 0xffffffffu, smask, 8u * (lc.off + W.cur), W.acc0, W.acc1);
    ring_drain(R, 32u, grad_rs, dbg);
    walk_begin(W);
}

// ---------------------------------------------------------------------------
// Row-lane walk of the merged kernel.  Lane = (stream, yz parity class):
// 16 streams per wave = (eighth of the chunk's merged order, level w or
// 15-w), 4 lanes per stream.  A lane tracks the two corners of the current
// cell in its (Y, Z) row (every cell has one corner per parity class
// (X&1, Y&1, Z&1); the lane's row holds the even-X and the odd-X one), so the
// per-sample position, the y/z weights and the row's hash part are computed
// once for two entries (the 8-lane form above computes them per corner).
// Finished entries go to per-stream LDS rings (SoA, W2_RING records) and are
// issued 32 at a time: one instruction = one level of one stretch of rays.
// The rings live in LDS that the MLP phase reuses, so every chunk ends with a
// full drain (walk2_end).
// ---------------------------------------------------------------------------
#define W2_STREAMS 16
#define W2_RING 40          // >= 31 pending + 8 pushed per step
#define W2_RING_WORDS (W2_STREAMS * 3 * W2_RING)   // per wave
#define W2_NONE 0xffffffffu

// The two levels a wave of the merged backward walks: levels a and 15 - a.
// Records per sample grow with the level (C3 replay, tools/records_sim.py:
// 0.20 at level 0 ... 5.58 at level 15), so the pair (0, 15) carries the most
// and (7, 8) the least.  Waves w and w + 4 of a block share a SIMD: waves
// 0-3 take the pairs (0, 15) ... (3, 12) and waves 4-7 the pairs (7, 8) ...
// (4, 11), heaviest with lightest (SIMD issue loads 8.18 / 7.47 / 6.96 / 6.69
// records per sample instead of 8.88 / 7.70 / 6.73 / 5.99 for a = w).
__device__ __forceinline__ int w2_level_a(int wid) { return wid < 4 ? wid : 11 - wid; }

struct Walk2 {
    uint32_t* ring;        // this wave's rings: [stream][3][W2_RING] words
    uint32_t head, tail;   // per lane: its stream's ring head / tail, in [0, W2_RING)
    uint32_t pend;         // per lane: its stream's pending records (tail - head)
    uint32_t ex0, ex1, ey, ez, cur0, cur1;   // even-X / odd-X entries of the row
    float a00, a01, a10, a11;                // their accumulated feature gradients
    // integer mode: the two newest issues, checked for carries one issue late
    int32_t oldA, loA, hiA, oldB, loB, hiB;
    uint32_t offA, offB;
    // fixed-point mode (GM 2): the scales of the wave's two levels (even
    // streams: level wid, odd: 15 - wid; 0 = fp32 atomics for that level) and
    // the largest |record| issued for each, as float bits (NaN/inf included)
    float fxA, fxB;
    uint32_t vmA, vmB;
    // ... and the exact sum of the integer records issued for each (the
    // net-wrap check of rn_grid_fx_fold)
    int64_t sqA, sqB;
    // ... and their position-weighted sum, sum of q * w(element) mod 2^64
    // (fx_weight): two entries that wrap in opposite directions cancel in
    // the plain sum but not in this one
    uint64_t swA, swB;
    // binned mode (GM 4): each level's open page in the pool and its fill,
    // and the levels' first entries (wave-uniform)
    uint32_t pgA, pgB, nA, nB, loffA, loffB;
    bool started;          // the chunk's first step has been walked (wave-uniform)
};

__device__ __forceinline__ void walk2_begin(Walk2& W, uint32_t* ring) {
    W.ring = ring; W.head = 0; W.tail = 0; W.pend = 0;
    W.ex0 = W2_NONE; W.ex1 = W2_NONE; W.ey = 0; W.ez = 0; W.cur0 = 0; W.cur1 = 0;
    W.a00 = W.a01 = W.a10 = W.a11 = 0.f;
    // (vmA/vmB and sqA/sqB are the kernel's: walk2_end re-begins the walk
    // after its last issue, so they are not reset here)
    W.oldA = W.loA = W.hiA = W.oldB = W.loB = W.hiB = 0;
    W.offA = W.offB = 0;
    W.started = false;
}

// Exact integer accumulation of the grid gradient (IG mode).  Each record
// value v becomes q = rint(v * 2^scale_exp) (int64), added as a 32-bit low
// word with a returning atomic; the high word plus any signed overflow of the
// low word (read from the returned old value) goes to a parallel carry array,
// so every entry holds carry * 2^32 + low exactly: sums are order-independent
// (bitwise reproducible) and u32 atomics run 28 % faster than f32 at the
// memory side (profiles/r01/atomic_probe.json).  A carry add is rare.
struct IntGrad {
    __amdgpu_buffer_rsrc_t lo, carry;   // int32 [entries][2] each (built in the kernel)
    float scale;                        // 2^scale_exp (loaded from scale_ptr)
    int32_t* lo_ptr; int32_t* carry_ptr; const float* scale_ptr;
    uint32_t bytes;
    __amdgpu_buffer_rsrc_t fx;          // fixed-point mode (GM 2): FxGrad::acc
    // binned mode (GM 4, rn_bin.h): the page pool the walk appends to
    GbCtl* ctl; uint32_t* page_meta; uint64_t* pages; uint32_t pool_pages;
};

__device__ __forceinline__ void ig_check(int32_t old, int32_t lo, int32_t hi, uint32_t off,
                                         const IntGrad& G) {
    const int32_t nw = (int32_t)((uint32_t)old + (uint32_t)lo);
    const bool ov = ((old ^ nw) & (lo ^ nw)) < 0;
    const int32_t c = hi + (ov ? (lo > 0 ? 1 : -1) : 0);
    if (c != 0) __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(c, G.carry, (int)off, 0, 0);
}

// Fixed-point accumulation of the hashed levels' grid gradient (GM 2, the
// default of the merged backward).  A record v of level l is added as the
// int32 rint(v * 2^e_l) with a NON-returning u32 atomic into `acc` (same
// layout as grid_grad): the memory side serves u32 adds at 26.6 G requests/s
// against 20.9 for f32 (profiles/r01/atomic_probe.json), and the sums are
// exact, so these levels' gradients are bitwise reproducible.  e_l comes from
// the previous step's largest record of the level (rn_grid_fx_fold): that
// record maps to < 2^27 units (2^23 until round 6; FX_TARGET_BITS below),
// leaving 2^4 max-size records of headroom per entry (an entry of a hashed
// level takes ~77 records per C3 step, of mixed sign, and its largest sum
// stays within 2^1.2 of the largest record).  The kernel records this step's
// largest |record| per level; when it reaches 2^30 units (8x growth) or is not
// finite, rn_grid_fx_fold discards the fixed-point sums and the GM 3 launch
// redoes the grid scatter in fp32.
// The first step of a workspace (scale 0) uses fp32 atomics and measures the
// records; the dense levels (few requests, but entries that sum hundreds of
// records) go fixed point from then on with a scale capped by their largest
// entry (k_fx_check).
// An int32 entry can still wrap with every record under 2^30 units (many
// same-sign records on one entry); the kernel therefore also sums each
// level's integer records exactly (int64), and rn_grid_fx_fold sums the
// level's int32 entries exactly: a wrapped entry makes the two differ by a
// multiple of 2^32, which sets the redo flag too.  (A float sum of the
// records is not enough: its rounding reached 2^31 on trained grids.)
struct FxStats {           // rn_grid_fx_fold / rn_field_bwd_merged fx_stats block
    uint32_t vmax[RN_L];   // largest |record| this step (float bits, atomicMax)
    uint32_t emax[RN_L];   // largest |entry| this step, gradient units (float bits; rn_grid_fx_fold)
    int64_t qsum[RN_L];    // sum of the issued integer records
    int64_t esum[RN_L];    // sum of the int32 entries (rn_grid_fx_fold)
    uint64_t wq[RN_L];     // sum of record * fx_weight(element), mod 2^64
    uint64_t we[RN_L];     // sum of entry * fx_weight(element), mod 2^64 (rn_grid_fx_fold)
};
static_assert(sizeof(FxStats) == RN_FX_STATS_BYTES, "FxStats layout (include/radnerf.h)");

// weight of grid-gradient element i (an int32 of the fixed-point table) in the
// position-weighted checksums: its byte offset 4 i, which the walk's issue
// already holds (no multiply on the issue path).  Wraps of +-2^32 on two
// different elements a, b move the weighted sum by 2^34 (a - b) mod 2^64,
// which is 0 only for a = b mod 2^30: never on a table of at most 2^28
// elements (rn_field_bwd_merged refuses fixed point for larger ones).  (Any
// injective weight is linear in the same way for three or more wraps: round
// 5's odd multiplier, (i mod 2^24) * 0x9E3779, cancelled exactly when
// sum(+-i) = 0 mod 2^32, like this one.)  The weights are < 2^30, so the
// walk adds q * w with one signed 32 x 32 -> 64 mad.
__host__ __device__ __forceinline__ uint32_t fx_weight(uint32_t i) { return 4u * i; }

struct FxGrad {
    int32_t* acc;              // int32 [entries][2]
    const float* scale;        // [RN_L] 2^e_l, 0 = fp32 atomics for the level
    uint32_t* vmax;            // FxStats::vmax
    int64_t* qsum;             // FxStats::qsum
    uint64_t* wq;              // FxStats::wq
    const int32_t* redo;       // GM 3: the launch runs only when *redo != 0
    __amdgpu_buffer_rsrc_t rs; // over acc (built in the kernel)
};

__device__ __forceinline__ uint32_t w2_wrap(uint32_t v) { return v >= W2_RING ? v - W2_RING : v; }

// issue up to 32 records of stream s (wave-uniform) as one atomic instruction
// (FULL: exactly 32, every lane issues: no exec-mask region).  ODD = s & 1, a
// template argument: the stream's level (even streams level wid, odd 15 -
// wid) selects its scale, page and statistics registers at compile time (as a
// runtime select the compiler emitted both paths with ~12 register copies of
// the 64-bit sums per issue)
template <int GM, bool ODD, bool FULL = false, bool DEFER = false>
__device__ __forceinline__ void walk2_issue(Walk2& W, int s, uint32_t cnt,
                                            __amdgpu_buffer_rsrc_t grad_rs, const IntGrad& G,
                                            int dbg) {
    const int lane = rn_lane();
    const uint32_t h = __builtin_amdgcn_readlane(W.head, 4 * s);
    constexpr bool odd = ODD;
    // binned (GM 4); GM 5: binned with the even streams' levels (0-7) by fp32
    // atomics, known at compile time -- that instantiation carries no page or
    // record-encoding code (round 6: the renderer's default at scale 16 sends
    // levels [0, 8-9) by fp32 atomics, FusedMLRenderer.bin_f32_levels)
    constexpr bool BIN = GM == 4 || GM == 5;
    constexpr bool F32S = GM == 5 && !ODD;
    // the level's scale as float bits selected on the scalar unit (gfx9 has
    // no scalar float compare: a float test here became a VALU compare + vcc
    // branch per issue)
    const uint32_t scb = GM >= 2 ? (uint32_t)__builtin_amdgcn_readfirstlane(
                                       (int)(odd ? __float_as_uint(W.fxB) : __float_as_uint(W.fxA)))
                                 : 0u;
    const bool fx_lvl = !F32S && (scb << 1) != 0u;   // 2^e_l > 0: fixed point; +-0: fp32 atomics
    const float sc_s = __uint_as_float(scb);
    asm volatile("" ::: "memory");
    if (BIN && fx_lvl) {
        // the level's open page cannot take cnt more records: close it (its
        // level and fill, for the bin pass) and take the pool's next page
        const uint32_t n = odd ? W.nB : W.nA;
        if (n + cnt > GB_PAGE) {                         // wave-uniform
            const uint32_t pg = odd ? W.pgB : W.pgA;
            const int wid = __builtin_amdgcn_readfirstlane((int)threadIdx.x / RN_WAVE);
            const int la = w2_level_a(wid);
            const uint32_t lvl = odd ? RN_L - 1 - la : la;
            uint32_t np = 0u;
            if (lane == 0) {
                if (pg < G.pool_pages) G.page_meta[pg] = lvl | (n << 8);
                np = atomicAdd(&G.ctl->pool_next, 1u);
            }
            np = (uint32_t)__builtin_amdgcn_readlane((int)np, 0);
            if (odd) { W.pgB = np; W.nB = 0u; } else { W.pgA = np; W.nA = 0u; }
        }
    }
    if (GM == 1) {
        // the issue two back has had a whole issue's time to return
        ig_check(W.oldA, W.loA, W.hiA, W.offA, G);
        W.oldA = W.oldB; W.loA = W.loB; W.hiA = W.hiB; W.offA = W.offB;
        W.oldB = 0; W.loB = 0; W.hiB = 0;
    }
    if (FULL || (uint32_t)lane < 2u * cnt) {
        const uint32_t rec = w2_wrap(h + (lane >> 1));
        const uint32_t* base = W.ring + s * 3 * W2_RING;
        const uint32_t w0 = base[rec];
        // byte offset of the lane's feature (GM 4: only the fp32 fallback
        // and the timing branches use it; the page record takes w0)
        const uint32_t off = (BIN ? 8u * ((odd ? W.loffB : W.loffA) + w0) : w0) + 4u * (lane & 1);
        const uint32_t v = base[(1 + (lane & 1)) * W2_RING + rec];
        if (rn_dbg(dbg) & 1) {
            asm volatile("" :: "v"(off), "v"(v));
        } else if (GM == 3 && !fx_lvl) {
            // redo: this level went in with fp32 atomics in the first pass
        } else if (rn_dbg(dbg) & 64) {      // ablation: non-returning i32 adds (timing only)
            (void)__builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(
                (int)(__uint_as_float(v) * 1048576.0f), grad_rs, (int)off, 0, 0);
        } else if (BIN && fx_lvl) {
            // binned: the 32 records go to the level's open page as 32 u64
            // (entry index, q0, q1), one 256-B store: lane 2r writes record
            // r's low word, lane 2r + 1 its high word
            const uint32_t ab = v & 0x7fffffffu;
            if (odd) W.vmB = max(W.vmB, ab); else W.vmA = max(W.vmA, ab);
            // e5m17 (rn_bin.h); a record at or past 2^46 units saturates and
            // vmax flags the step for the fp32 redo
            const uint32_t q = gb_encode_walk(__uint_as_float(v) * sc_s);
            const uint32_t qp = (uint32_t)__builtin_amdgcn_mov_dpp((int)q, 0xb1, 0xf, 0xf, true);   // partner lane ^ 1
            // lane 2r: entry | q0 << 20 (q0 = its own q); lane 2r + 1:
            // q0 >> 12 (the partner's) | q1 << 10 (its own): one shift-or
            // with a per-lane shift and a select, no branch on lane & 1
            // (w0 < the level's size <= 2^GB_IDX_BITS: the walk's hash /
            // dense index is reduced mod the size)
            const bool hi_lane = lane & 1;
            const uint32_t lowbits = hi_lane ? (qp >> 12) & 0x3ffu : w0;
            const uint32_t word = (q << (hi_lane ? 10u : 20u)) | lowbits;
            const uint32_t pg = odd ? W.pgB : W.pgA, n = odd ? W.nB : W.nA;
            uint32_t* dst = reinterpret_cast<uint32_t*>(G.pages + (size_t)pg * GB_PAGE + n) + lane;
            if (pg < G.pool_pages) {
                if (rn_dbg(dbg) & 8) *dst = word;                // (timing only: plain stores)
                else __builtin_nontemporal_store(word, dst);
            }
        } else if (GM == 2) {
            const uint32_t ab = v & 0x7fffffffu;          // |v| bits: NaN / inf order last
            if (odd) W.vmB = max(W.vmB, ab); else W.vmA = max(W.vmA, ab);
            // 2^e_l is a power of two: v * sc is exact; v_cvt_i32_f32 saturates
            // out-of-range values (NaN -> 0): such records are caught by vmax
            // and the step is redone in fp32.  An fp32 level's scale is +-0, so
            // its q is 0 and the sums below do not move: only the atomic
            // differs, and the statistics stay out of the branch (as a branch
            // the compiler copied the 64-bit sums at every issue)
            int q;
            asm("v_cvt_i32_f32 %0, %1" : "=v"(q) : "v"(rintf(__uint_as_float(v) * sc_s)));
            if (fx_lvl)
                (void)__builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(q, G.fx, (int)off, 0, 0);
            else
                __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(__uint_as_float(v), grad_rs,
                                                            (int)off, 0, 0);
            // off = 4 x element = fx_weight(element) < 2^30: one v_mad_i64_i32
            const int64_t qw = (int64_t)q * (int64_t)(int32_t)off;
            if (odd) { W.sqB += (int64_t)q; W.swB += (uint64_t)qw; }
            else { W.sqA += (int64_t)q; W.swA += (uint64_t)qw; }
        } else if (GM == 1) {
            // exact: |v * 2^e| < 2^62 for any finite gradient the scale admits
            const float x = rintf(__uint_as_float(v) * G.scale);
            const long long q = (long long)x;
            const int32_t lo = (int32_t)(uint32_t)(unsigned long long)q;
            W.loB = lo;
            W.hiB = (int32_t)((q - (long long)lo) >> 32);
            W.offB = off;
            W.oldB = __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(lo, G.lo, (int)off, 0, 0);
        } else {
            // fp32 level: still tracked (not GM 5's even streams: the host
            // zeroes those levels' scales every step, so their maxima are unused)
            if (GM == 2 || (BIN && !F32S)) {
                const uint32_t ab = v & 0x7fffffffu;
                if (odd) W.vmB = max(W.vmB, ab); else W.vmA = max(W.vmA, ab);
            }
            __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(__uint_as_float(v), grad_rs,
                                                            (int)off, 0, 0);
        }
    }
    asm volatile("" ::: "memory");
    if (BIN && fx_lvl) {
        if (odd) W.nB += cnt; else W.nA += cnt;
    }
    if (!DEFER) {           // (DEFER: the threshold drain advances every issued ring at once)
        const bool me = (lane >> 2) == s;                 // selects, not a branch
        W.head = me ? w2_wrap(W.head + cnt) : W.head;
        W.pend = me ? W.pend - cnt : W.pend;
    }
}

// integer mode: settle the two outstanding issues (end of a chunk)
__device__ __forceinline__ void walk2_settle(Walk2& W, const IntGrad& G) {
    ig_check(W.oldA, W.loA, W.hiA, W.offA, G);
    ig_check(W.oldB, W.loB, W.hiB, W.offB, G);
    W.oldA = W.loA = W.hiA = W.oldB = W.loB = W.hiB = 0;
}

// issue every stream with >= min_cnt pending (min_cnt 0: drain all)
template <int GM>
__device__ __forceinline__ void walk2_drain(Walk2& W, uint32_t min_cnt,
                                            __amdgpu_buffer_rsrc_t grad_rs, const IntGrad& G,
                                            int dbg) {
    const uint32_t need = min_cnt > 1u ? min_cnt : 1u;
    for (;;) {
        const uint32_t pend = W.pend;
        // lane 0 of each stream's quad (a plain compare's ballot: no
        // bool -> mask round trip)
        const uint64_t m = __builtin_amdgcn_ballot_w64(pend >= need) & 0x1111111111111111ull;
        if (!m) break;
        // even streams (lanes 8k), then odd ones (8k + 4): each loop's level
        // is known at compile time (walk2_issue<ODD>)
        auto run = [&](uint64_t mm, auto odd_c) {
            constexpr bool O = decltype(odd_c)::value;
            while (mm) {
                const int s = __builtin_ctzll(mm) >> 2;
                const uint32_t p = __builtin_amdgcn_readlane(pend, 4 * s);
                if (min_cnt >= 32u)     // threshold drain (constant after inlining): p >= 32
                    walk2_issue<GM, O, true, true>(W, s, 32u, grad_rs, G, dbg);
                else
                    walk2_issue<GM, O>(W, s, p < 32u ? p : 32u, grad_rs, G, dbg);
                mm &= mm - 1;
            }
        };
        run(m & 0x0101010101010101ull, std::integral_constant<bool, false>{});
        run(m & 0x1010101010101010ull, std::integral_constant<bool, true>{});
        if (min_cnt > 0u) {
            // threshold drain: every ring with >= 32 pending issued exactly 32
            // (head / pend of a stream are the same on its 4 lanes), advanced
            // here once instead of by selects after every issue; what remains
            // is < 32
            const bool did = pend >= 32u;
            W.head = did ? w2_wrap(W.head + 32u) : W.head;
            W.pend = did ? pend - 32u : pend;
            break;
        }
    }
}

// append this step's finished entries (up to 2 per lane) to the stream rings,
// lane-major (a lane's even-X and odd-X records adjacent: they share a 64-B
// segment, so an instruction boundary splits them less often; replay of the
// bench samples, tools/atomic_sim2.py: 15.18 -> 14.65 requests/sample)
// Ring word 0 of a record: the byte offset 8 (level offset + entry) of its
// first feature in the grid (GM 4: the entry index within the level, what a
// page record holds)
template <int GM>
__device__ __forceinline__ void walk2_push(Walk2& W, bool e0, bool e1, uint32_t lvl_off) {
    // a stream's 4 lanes are one DPP quad: the lane's first record index is
    // the exclusive quad prefix of the per-lane record counts (two quad_perm
    // steps), the stream's total its lane 3 (ballot + mbcnt + popcount per
    // mask took ~19 VALU operations per step, this ~10; same order)
    const int s = rn_lane() >> 2;
    const uint32_t q = rn_lane() & 3;
    const uint32_t x = (e0 ? 1u : 0u) + (e1 ? 1u : 0u);
    const uint32_t m1 = q >= 1u ? ~0u : 0u, m2 = q >= 2u ? ~0u : 0u;      // loop-invariant
    uint32_t t = x + ((uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x90, 0xf, 0xf, true) & m1);  // [0,0,1,2]
    t += (uint32_t)__builtin_amdgcn_mov_dpp((int)t, 0x40, 0xf, 0xf, true) & m2;         // [0,0,0,1]
    const uint32_t pushed = (uint32_t)__builtin_amdgcn_mov_dpp((int)t, 0xff, 0xf, 0xf, true);  // [3,3,3,3]
    const uint32_t below = t - x;
    uint32_t* base = W.ring + s * 3 * W2_RING;
    // branch-free: a lane with nothing to emit writes the stream's free slot
    // tail + pushed (pending records are <= 31 before the push and <= 39
    // after it, so that slot is outside [head, tail + pushed) of a 40-slot
    // ring; it is overwritten before it is ever read)
    const uint32_t r0 = w2_wrap(W.tail + (e0 ? below : pushed));
    const uint32_t r1 = w2_wrap(W.tail + (e1 ? below + (e0 ? 1u : 0u) : pushed));
    base[r0] = GM >= 4 ? W.cur0 : 8u * (lvl_off + W.cur0);
    base[W2_RING + r0] = __float_as_uint(W.a00);
    base[2 * W2_RING + r0] = __float_as_uint(W.a01);
    base[r1] = GM >= 4 ? W.cur1 : 8u * (lvl_off + W.cur1);
    base[W2_RING + r1] = __float_as_uint(W.a10);
    base[2 * W2_RING + r1] = __float_as_uint(W.a11);
    W.tail = w2_wrap(W.tail + pushed);
    W.pend += pushed;
}

__device__ __forceinline__ LvConst walk2_level(const FieldArgs& a, const LvTab& sT) {
    const int wid = __builtin_amdgcn_readfirstlane((int)threadIdx.x / RN_WAVE);
    const int la = w2_level_a(wid);
    const int l = ((rn_lane() >> 2) & 1) ? (RN_L - 1 - la) : la;
    return lv_const(sT, a.gm, l);
}

// walk one window: the lane's eighth's samples are rows [0, ne) of its
// eighth's staging block sG/sU (per-lane bases; ne per lane: its eighth's
// count; n0 = the largest, wave-uniform; at most WIN)
template <int GM, int WIN = 32>
__device__ __forceinline__ void walk2_window(const FieldArgs& a, const LvTab& sT,
                                             const float* sG_, const float* sU_, int ne, int n0,
                                             __amdgpu_buffer_rsrc_t grad_rs, const IntGrad& G,
                                             Walk2& W, int dbg) {
    lds_cf* sG = (lds_cf*)sG_;
    lds_cf* sU = (lds_cf*)sU_;
    const int lane = rn_lane();
    const int stream = lane >> 2, eighth = stream >> 1;
    const uint32_t py = lane & 1, pz = (lane >> 1) & 1;
    const LvConst lc = walk2_level(a, sT);
    const int wid = __builtin_amdgcn_readfirstlane((int)threadIdx.x / RN_WAVE);
    const int la = w2_level_a(wid);
    lds_cf* gcol = sG + 2 * ((stream & 1) ? (RN_L - 1 - la) : la);
    // sG / sU are this lane's eighth's own block of WIN rows (per-lane bases)
    const int s_base = 0;
    (void)eighth;
    typedef float vf4 __attribute__((ext_vector_type(4)));
    typedef float vf2 __attribute__((ext_vector_type(2)));
    typedef __attribute__((address_space(3))) const vf4 lds_cf4;
    typedef __attribute__((address_space(3))) const vf2 lds_cf2;
    vf4 un = *(lds_cf4*)(sU + s_base * 4);
    vf2 gn = *(lds_cf2*)(gcol + s_base * SG_STRIDE);
    // steps below the wave's smallest count need no per-lane activity test
    // (no exec-mask region): all but a chunk's last window run that form
    int nmin = ne;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) nmin = min(nmin, __shfl_xor(nmin, off));
    // both bounds in SGPRs: scalar loops (a VGPR bound made the compiler run
    // them as divergent loops with exec-mask bookkeeping every step)
    nmin = __builtin_amdgcn_readfirstlane(nmin);
    n0 = __builtin_amdgcn_readfirstlane(n0);
    auto step = [&](int j, auto check) {
        const bool act = decltype(check)::value ? j < ne : true;
        const vf4 uc = un;
        const vf2 gc = gn;
        // the next row, read unconditionally: row ne of a block is the next
        // block's first row or the tail of sW / the rings (always inside the
        // kernel's LDS), read but never used (a clamp to row 0 cost three
        // VALU per step)
        const int nx = s_base + j + 1;
        un = *(lds_cf4*)(sU + nx * 4);
        gn = *(lds_cf2*)(gcol + __umul24((uint32_t)nx, SG_STRIDE));   // u32 offset, not a u64 mad
        const LevelPos p = level_pos(lc.sc, uc.x, uc.y, uc.z);
        const uint32_t c0 = p.gx & 1u;                    // x offset of the even-X corner
        const uint32_t cy = (py ^ p.gy) & 1u, cz = (pz ^ p.gz) & 1u;
        const uint32_t X0 = p.gx + c0, X1 = p.gx + (c0 ^ 1u), Y = p.gy + cy, Z = p.gz + cz;
        const float fxm = 1.0f - p.fx;
        const float wy = cy ? p.fy : 1.0f - p.fy, wz = cz ? p.fz : 1.0f - p.fz;
        // weight = wx * wy * wz in tcnn's dimension order, both corners in
        // packed fp32 (v_pk_mul_f32: the same roundings, half the issues)
        const vf2 wx = {c0 ? p.fx : fxm, c0 ? fxm : p.fx};
        const vf2 w01 = (wx * wy) * wz;
        const bool row = Y == W.ey && Z == W.ez;
        const bool same0 = row && X0 == W.ex0, same1 = row && X1 == W.ex1;
        // W.ex0 / ex1 are W2_NONE (nothing to emit) exactly until the chunk's
        // first walked step (W.started, wave-uniform: a lane active at a step
        // was active at every earlier step of the chunk)
        walk2_push<GM>(W, act && !same0 && W.started, act && !same1 && W.started, lc.off);
        if (act) {
            const vf2 p0 = vf2{same0 ? W.a00 : 0.f, same0 ? W.a01 : 0.f} + w01.x * gc;
            const vf2 p1 = vf2{same1 ? W.a10 : 0.f, same1 ? W.a11 : 0.f} + w01.y * gc;
            W.a00 = p0.x; W.a01 = p0.y; W.a10 = p1.x; W.a11 = p1.y;
            // tcnn grid_index with the row part shared by the two entries;
            // branch-free dense / hashed select (the two levels of a wave differ)
            const uint32_t db = __umul24(Y, lc.res) + __umul24(Z, lc.res2);
            const uint32_t hb = (Y * 2654435761u) ^ (Z * 805459861u);
            const uint32_t d0 = X0 + db, d1 = X1 + db;
            const uint32_t dm = lc.dense ? 0xffffffffu : 0u;
            const uint32_t dd0 = min(d0, d0 - lc.hs), dd1 = min(d1, d1 - lc.hs);   // d < 2 hs
            W.cur0 = (dd0 & dm) | ((X0 ^ hb) & (lc.hs - 1u) & ~dm);
            W.cur1 = (dd1 & dm) | ((X1 ^ hb) & (lc.hs - 1u) & ~dm);
            W.ex0 = X0; W.ex1 = X1; W.ey = Y; W.ez = Z;
        }
        walk2_drain<GM>(W, 32u, grad_rs, G, dbg);
        W.started = true;
    };
    int j = 0;                                            // wave-uniform trip counts
    // two steps per trip: the loop-carried rows and entries stay in their
    // registers (one step per trip copied them back every step)
    for (; j + 1 < nmin; j += 2) {
        step(j, std::integral_constant<bool, false>{});
        step(j + 1, std::integral_constant<bool, false>{});
    }
    for (; j < nmin; ++j) step(j, std::integral_constant<bool, false>{});
    for (; j < n0; ++j) step(j, std::integral_constant<bool, true>{});
}

// end of a chunk: emit every live entry and drain the rings completely
template <int GM>
__device__ __forceinline__ void walk2_end(const FieldArgs& a, const LvTab& sT,
                                          __amdgpu_buffer_rsrc_t grad_rs, const IntGrad& G,
                                          Walk2& W, int dbg) {
    const LvConst lc = walk2_level(a, sT);
    walk2_push<GM>(W, W.ex0 != W2_NONE, W.ex1 != W2_NONE, lc.off);
    walk2_drain<GM>(W, 0u, grad_rs, G, dbg);
    if (GM == 1) walk2_settle(W, G);
    walk2_begin(W, W.ring);
}

// Walk of one wave over the block's 256 samples.  Lane = (stream, parity
// class): stream = (quarter of the samples, level w or 15-w), and each of the
// stream's 8 lanes tracks the current cell's corner of one parity class
// p = (X & 1, Y & 1, Z & 1) (every cell has exactly one corner per class), so
// when the cell moves, the lane's corner either stays the same entry (it is
// shared by the two cells: keep accumulating) or leaves (emit it) -- a lane-
// local test, no data moves between lanes.  Each lane walks its 64 samples in
// ray order holding both features of its entry.
__device__ __forceinline__ void grid_scatter_block(const FieldArgs& a, const LvTab& sT,
                                                   const float* sG, const float* sU, int nblk,
                                                   ScatterRing& R,
                                                   __amdgpu_buffer_rsrc_t grad_rs) {
    constexpr int QN = BWD_WAVES * 8;
    const int quarter = rn_lane() >> 4;
    const int n0 = min(nblk, QN);                         // quarter 0 is the longest
    const int nq = max(0, min(QN, nblk - quarter * QN));
    WalkState W;
    walk_begin(W);
    grid_walk_window(a, sT, sG, sU, nq, n0, R, grad_rs, W, a.dbg);
    walk_end(a, sT, R, grad_rs, W, a.dbg);
}

// dW tile over the 8 waves' images: dY features [ya,+32) x X features [xa,+32).
// Software-pipelined: the four transposed LDS reads of step j + DW_DEPTH - 1
// are issued before step j's MFMA, so each MFMA waits only for its own
// operands (lgkmcnt counts in issue order).  Written as one load per step
// followed by its MFMA, the compiler waited lgkmcnt(0) before every MFMA and
// the 16-step tile took 16 LDS round trips (round 5, field.hip ISA).
// (NS < 16, steps [j0, j0 + NS) only: the balanced-dW timing study, flag 1024)
#define DW_DEPTH 3
template <int NS = 2 * BWD_WAVES>                     // 16 steps of 16 samples
__device__ __forceinline__ f32x16 dw_block_tile(const rn_half* sImg, int ya, int xa, f32x16 acc,
                                                int j0 = 0) {
    half8 ys[DW_DEPTH], xs[DW_DEPTH];
    auto load = [&](int j, half8& y, half8& x) {
        j += j0;
        const rn_half* iy = sImg + (j >> 1) * 2 * RN_IMG_HALFS;
        y = rn_img_read(iy, ya, j & 1);
        x = rn_img_read(iy + RN_IMG_HALFS, xa, j & 1);
    };
#pragma unroll
    for (int j = 0; j < DW_DEPTH - 1; ++j) load(j, ys[j], xs[j]);
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        if (j + DW_DEPTH - 1 < NS)
            load(j + DW_DEPTH - 1, ys[(j + DW_DEPTH - 1) % DW_DEPTH], xs[(j + DW_DEPTH - 1) % DW_DEPTH]);
        acc = rn_mfma(ys[j % DW_DEPTH], xs[j % DW_DEPTH], acc);
    }
    return acc;
}

// flush one owned dW tile (accumulated at scale `sc`) into the global gradient
template <int MODE>
__device__ __forceinline__ void dw_flush(const f32x16& acc, float* dw, int off, int ncols,
                                         int out_base, int in_base, float inv) {
    const int lane = rn_lane(), col = lane & 31, h = lane >> 5;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
        int out;
        if (MODE == DW_PLAIN) out = out_base + row;
        else if (MODE == DW_ROWS_LT3) out = row < 3 ? row : -1;
        else out = row < 16 ? row + 1 : (row == 16 ? 0 : -1);
        if (out >= 0) atomicAdd(dw + off + out * ncols + in_base + col, acc[i] * inv);
    }
}

// flush a wave's owned dW tiles (ownership table in k_field_bwd) into dw
// accA holds rgb-net tiles (at the rgb chain's scale), accB geo-net tiles
// (at the geo chain's scale); a zero scale means "empty"
struct DwScale { float a, b; };

__device__ __forceinline__ void dw_flush_owned(const f32x16& accA, const f32x16& accB, float* dw,
                                               int wid, DwScale sc) {
    const float ia = sc.a != 0.f ? 1.0f / sc.a : 0.f, ib = sc.b != 0.f ? 1.0f / sc.b : 0.f;
    if (wid < 2) {
        if (ia != 0.f) dw_flush<DW_ROWS_LT3>(accA, dw, 9280, 64, 0, 32 * wid, ia);   // rgb3
        if (ib != 0.f) dw_flush<DW_GEO>(accB, dw, 2048, 64, 0, 32 * wid, ib);        // geo2
    } else if (wid < 6) {
        const int mm = (wid - 2) >> 1, nn = (wid - 2) & 1;
        if (ia != 0.f) dw_flush<DW_PLAIN>(accA, dw, 5184, 64, 32 * mm, 32 * nn, ia); // rgb2
        if (wid < 4 && ib != 0.f)
            dw_flush<DW_PLAIN>(accB, dw, 0, 32, 32 * (wid - 2), 0, ib);              // geo1
    } else {
        if (ia != 0.f) dw_flush<DW_PLAIN>(accA, dw, 3136, 32, 32 * (wid - 6), 0, ia); // rgb1
    }
}

// Backward of one block iteration (8 waves x 32-sample tiles, the tiles'
// forward state in `st`): seeds -> block gradient scales -> dX chain on MFMA
// with the block-cooperative dW tiles (accA / accB at cur.a / cur.b, rescaled
// exactly when a scale changes).  Returns dL/dencoding at scale `gscale`
// (rows in MFMA accumulator order); zero_iter: all 256 seeds are zero.
// Two power-of-two scales: the rgb chain (rgb3 -> rgb1) is scaled by the
// block's largest rgb seed, the geo chain (geo2 -> encoding) by the largest
// of all seeds.  With one shared scale, a sub-NeRF whose gate weight is ~0 has
// rgb seeds ~1e-8 of its sigma seeds, and its rgb-net gradients fall below
// f16's range (tcnn's global loss scale flushes them to zero); the rgb-path
// rows of dL/dgeo are brought to the geo scale in fp32 before the f16 cast.
__device__ __forceinline__ f32x16 bwd_window(const FieldArgs& a, const rn_half* sW,
                                             const rn_half* sImg, float* sMax, rn_half* imgY,
                                             rn_half* imgX, FwdState& st, bool valid, int64_t s,
                                             int wid, f32x16& accA, f32x16& accB,
                                             DwScale& cur, bool do_dw, float& gscale_out,
                                             bool& zero_iter_out, bool sync = true,
                                             const float* pre = nullptr) {
    const int lane = rn_lane(), h = lane >> 5;
    const half8 z8 = rn_zero8();
    // timing study only (ablation build, flag 1024; WRONG dW): every layer's
    // dW tiles contracted by all 8 waves, each over its share of the samples
    // (2-tile layers: 4 of the 16 steps, waves w and w + 4 on one SIMD take
    // the same tile), all into the wave's own accumulators -- the MFMA / LDS
    // schedule of a balanced dW ownership without its registers
    const bool bal = rn_dbg(a.dbg) & 1024;
    // ---- seeds (lanes h == 0 own the output rows); `pre`: dL/dsigma and
    // dL/drgb already loaded by the caller (ahead of the forward recompute)
    float o0 = 0.f, o1 = 0.f, o2 = 0.f, gsig = 0.f;
    if (valid && h == 0) {
        const float ds = pre ? pre[0] : a.dsigma[s];
        const float r0 = pre ? pre[1] : a.drgb[3 * s], r1 = pre ? pre[2] : a.drgb[3 * s + 1],
                    r2 = pre ? pre[3] : a.drgb[3 * s + 2];
        const float y0 = sigmoidf(st.out[0]), y1 = sigmoidf(st.out[1]),
                    y2 = sigmoidf(st.out[2]);
        o0 = r0 * (y0 * (1.0f - y0));                    // sigmoid'
        o1 = r1 * (y1 * (1.0f - y1));
        o2 = r2 * (y2 * (1.0f - y2));
        // TruncExp.backward: g * exp(clamp(x, -15, 15))  (custom_functions.py:171-173)
        gsig = ds * expf(fminf(fmaxf(st.g0, -15.f), 15.f));
    }
    float mr = fmaxf(fmaxf(fabsf(o0), fabsf(o1)), fabsf(o2)), mg = fabsf(gsig);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        mr = fmaxf(mr, __shfl_xor(mr, off));
        mg = fmaxf(mg, __shfl_xor(mg, off));
    }
    if (lane == 0) { sMax[2 * wid] = mr; sMax[2 * wid + 1] = mg; }
    if (sync) __syncthreads();                                                    // B0
    float bmr = sMax[0], bmg = sMax[1];
#pragma unroll
    for (int w = 1; w < BWD_WAVES; ++w) { bmr = fmaxf(bmr, sMax[2 * w]); bmg = fmaxf(bmg, sMax[2 * w + 1]); }
    const float bm = fmaxf(bmr, bmg);
    // an iteration whose 256 samples all have zero seeds (samples past the
    // early-termination point of their rays, volumerendering.cu:150) adds
    // nothing to the hash grid: its scatter walk is skipped (an early
    // `continue` of the whole iteration made the compiler spill 190 B/lane)
    const bool zero_iter = bm == 0.f;
    const float gscale = rn_wave_grad_scale(bm);    // geo chain, uniform over the block
    const float rscale = rn_wave_grad_scale(bmr);   // rgb chain (>= gscale)
    if (cur.a != rscale) {                          // exact power-of-two rescales
        accA *= cur.a == 0.f ? 0.f : rscale / cur.a;
        cur.a = rscale;
    }
    if (cur.b != gscale) {
        accB *= cur.b == 0.f ? 0.f : gscale / cur.b;
        cur.b = gscale;
    }
    half8 dO = z8;
    if (h == 0) {
        dO[0] = (rn_half)(o0 * rscale);
        dO[1] = (rn_half)(o1 * rscale);
        dO[2] = (rn_half)(o2 * rscale);
    }
    // ---- layer rgb3: dW (w0, w1) = dO x R2 ; dR2 = Wr3^T dO masked
    if (do_dw) {
        rn_img_write(imgY, 0, dO); rn_img_write(imgY, 1, z8);
#pragma unroll
        for (int q = 0; q < 4; ++q) rn_img_write(imgX, q, st.r2[q]);
    }
    if (sync) __syncthreads();                                                    // B1
    if (do_dw && bal) accA = dw_block_tile<4>(sImg, 0, 32 * (wid & 1), accA, 4 * (wid >> 1));
    else if (do_dw && wid < 2) accA = dw_block_tile(sImg, 0, 32 * wid, accA);
    half8 dr2f[4];
    {
        f32x16 b0 = rn_zero16(), b1 = rn_zero16();
        b0 = rn_mfma(rn_frag(sW, 24), dO, b0);
        b1 = rn_mfma(rn_frag(sW, 25), dO, b1);
        rn_acc_to_frags_masked(b0, st.r2[0], st.r2[1], dr2f[0], dr2f[1]);
        rn_acc_to_frags_masked(b1, st.r2[2], st.r2[3], dr2f[2], dr2f[3]);
    }
    if (sync) __syncthreads();                                                    // B2
    // ---- layer rgb2: dW (w2..w5) = dR2 x R1 ; dR1 = Wr2^T dR2 masked
    if (do_dw) {
#pragma unroll
        for (int q = 0; q < 4; ++q) { rn_img_write(imgY, q, dr2f[q]); rn_img_write(imgX, q, st.r1[q]); }
    }
    if (sync) __syncthreads();                                                    // B3
    if (do_dw && bal)
        accA = dw_block_tile<8>(sImg, 32 * ((wid & 3) >> 1), 32 * (wid & 1), accA, 8 * (wid >> 2));
    else if (do_dw && wid >= 2 && wid < 6)
        accA = dw_block_tile(sImg, 32 * ((wid - 2) >> 1), 32 * ((wid - 2) & 1), accA);
    half8 dr1f[4];
    {
        f32x16 b0 = rn_zero16(), b1 = rn_zero16();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            b0 = rn_mfma(rn_frag(sW, 26 + q), dr2f[q], b0);
            b1 = rn_mfma(rn_frag(sW, 30 + q), dr2f[q], b1);
        }
        rn_acc_to_frags_masked(b0, st.r1[0], st.r1[1], dr1f[0], dr1f[1]);
        rn_acc_to_frags_masked(b1, st.r1[2], st.r1[3], dr1f[2], dr1f[3]);
    }
    if (sync) __syncthreads();                                                    // B4
    // ---- layer rgb1: dW (w6, w7) = dR1 x [SH | geo 1..16] ; dG
    if (do_dw) {
#pragma unroll
        for (int q = 0; q < 4; ++q) rn_img_write(imgY, q, dr1f[q]);
        rn_img_write(imgX, 0, st.sh); rn_img_write(imgX, 1, st.gin);
    }
    if (sync) __syncthreads();                                                    // B5
    if (do_dw && bal) accA = dw_block_tile<4>(sImg, 32 * (wid & 1), 0, accA, 4 * (wid >> 1));
    else if (do_dw && wid >= 6) accA = dw_block_tile(sImg, 32 * (wid - 6), 0, accA);
    half8 dg0, dg1;
    {
        f32x16 b = rn_zero16();
#pragma unroll
        for (int q = 0; q < 4; ++q) b = rn_mfma(rn_frag(sW, 34 + q), dr1f[q], b);
        b *= gscale / rscale;                      // rgb-path rows to the geo scale (exact)
        if (h == 0) b[8] = gsig * gscale;          // row 16 = dL/dh0
        rn_acc_to_frags<false>(b, dg0, dg1);
    }
    if (sync) __syncthreads();                                                    // B6
    // ---- layer geo2: dW (w0, w1) = dG x H1 ; dH1 = Wg2^T dG masked
    if (do_dw) {
        rn_img_write(imgY, 0, dg0); rn_img_write(imgY, 1, dg1);
#pragma unroll
        for (int q = 0; q < 4; ++q) rn_img_write(imgX, q, st.h1[q]);
    }
    if (sync) __syncthreads();                                                    // B7
    if (do_dw && bal) accB = dw_block_tile<4>(sImg, 0, 32 * (wid & 1), accB, 4 * (wid >> 1));
    else if (do_dw && wid < 2) accB = dw_block_tile(sImg, 0, 32 * wid, accB);
    half8 dh1f[4];
    {
        f32x16 b0 = rn_zero16(), b1 = rn_zero16();
        b0 = rn_mfma(rn_frag(sW, 38), dg0, b0); b0 = rn_mfma(rn_frag(sW, 39), dg1, b0);
        b1 = rn_mfma(rn_frag(sW, 40), dg0, b1); b1 = rn_mfma(rn_frag(sW, 41), dg1, b1);
        rn_acc_to_frags_masked(b0, st.h1[0], st.h1[1], dh1f[0], dh1f[1]);
        rn_acc_to_frags_masked(b1, st.h1[2], st.h1[3], dh1f[2], dh1f[3]);
    }
    if (sync) __syncthreads();                                                    // B8
    // ---- layer geo1: dW (w2, w3) = dH1 x E ; dE = Wg1^T dH1
    if (do_dw) {
#pragma unroll
        for (int q = 0; q < 4; ++q) rn_img_write(imgY, q, dh1f[q]);
        rn_img_write(imgX, 0, st.e0); rn_img_write(imgX, 1, st.e1);
    }
    if (sync) __syncthreads();                                                    // B9
    if (do_dw && bal) accB = dw_block_tile<4>(sImg, 32 * (wid & 1), 0, accB, 4 * (wid >> 1));
    else if (do_dw && (wid == 2 || wid == 3)) accB = dw_block_tile(sImg, 32 * (wid - 2), 0, accB);
    f32x16 dE = rn_zero16();
#pragma unroll
    for (int q = 0; q < 4; ++q) dE = rn_mfma(rn_frag(sW, 42 + q), dh1f[q], dE);
    if (sync) __syncthreads();                                                    // B10
    gscale_out = gscale;
    zero_iter_out = zero_iter;
    return dE;
}

template <int MODE, int CACHE>
__global__ void __launch_bounds__(BWD_WAVES * 64)
k_field_bwd(FieldArgs a) {
    __shared__ __attribute__((aligned(16))) rn_half sW[FIELD_FRAGS * RN_FRAG_HALFS];
    __shared__ __attribute__((aligned(16))) rn_half sImg[BWD_WAVES * 2 * RN_IMG_HALFS];
    __shared__ float sMax[2 * BWD_WAVES];
    __shared__ LvTab sT;
    __shared__ uint32_t sRing[BWD_WAVES * SC_STREAMS * 3 * SC_RING];   // scatter rings
    const int k = blockIdx.y;
    rn_block_copy16(sW, a.frags + (size_t)k * FIELD_FRAGS * RN_FRAG_HALFS,
                    FIELD_FRAGS * RN_FRAG_BYTES);
    lv_stage(sT, a.gm);
    __syncthreads();

    int64_t base, n;
    sample_range(a, MODE, k, base, n);
    const int64_t n_tiles = (n + 31) / 32;
    const int64_t n_iters = (n_tiles + BWD_WAVES - 1) / BWD_WAVES;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / RN_WAVE);
    const int lane = rn_lane(), c = lane & 31, h = lane >> 5;
    rn_half* imgY = sImg + wid * 2 * RN_IMG_HALFS;
    rn_half* imgX = imgY + RN_IMG_HALFS;
    const __amdgpu_buffer_rsrc_t grad_rs = rn_rsrc(a.grid_grad, 2 * a.grid_bytes);
    const bool do_dw = !(rn_dbg(a.dbg) & 2);

    // owned dW tiles (ownership table in the header comment above):
    //   w0: r3(n=0), g2(n=0)   w1: r3(n=1), g2(n=1)   w2..w5: r2(m,n)
    //   w2: + g1(m=0)          w3: + g1(m=1)          w6, w7: r1(m)
    f32x16 accA = rn_zero16(), accB = rn_zero16();
    DwScale cur = {0.f, 0.f};   // scales the accumulators are expressed at (0 = empty)

    const bool do_sc = !(rn_dbg(a.dbg) & 4);
    // scatter staging (dL/dfeature rows, unit coords of the iteration's 256
    // samples) reuses the image region, free between B10 and the next B0
    float* sG = reinterpret_cast<float*>(sImg);                        // [256][SG_STRIDE]
    float* sU = sG + BWD_WAVES * 32 * SG_STRIDE;                        // [256][4]
    static_assert(BWD_WAVES * 32 * (SG_STRIDE + 4) * 4 <= BWD_WAVES * 2 * RN_IMG_HALFS * 2,
                  "scatter staging must fit the image region");
    ScatterRing R;
    R.ring = sRing + wid * SC_STREAMS * 3 * SC_RING;
#pragma unroll
    for (int q = 0; q < SC_STREAMS; ++q) R.head[q] = 0;
    R.tail = 0;

    for (int64_t it = blockIdx.x; it < n_iters; it += gridDim.x) {
        rn_lds_order();   // weights stay in LDS: no hoisting of fragment reads
        const int64_t tile = it * BWD_WAVES + wid;
        FwdState st;
        bool valid; int64_t s; float ux, uy, uz;
        tile_forward<MODE, CACHE>(a, sT, sW, base, n, tile, st, valid, s, ux, uy, uz);

        float gscale; bool zero_iter;
        const f32x16 dE = bwd_window(a, sW, sImg, sMax, imgY, imgX, st, valid, s, wid, accA, accB,
                                     cur, do_dw, gscale, zero_iter);

        // ---- hash-grid gradient scatter (grid_scatter_block)
        if (do_sc && !zero_iter) {
            const float ginv = 1.0f / gscale;
            const int srow = wid * 32 + c;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int f = (i & 3) + 8 * (i >> 2) + 4 * h;  // feature
                sG[srow * SG_STRIDE + f] = dE[i] * ginv;
            }
            if (h == 0) { sU[srow * 4 + 0] = ux; sU[srow * 4 + 1] = uy; sU[srow * 4 + 2] = uz; }
            const int64_t rem = n - it * (BWD_WAVES * 32);
            const int nblk = rem < BWD_WAVES * 32 ? (int)rem : BWD_WAVES * 32;
            __syncthreads();
            grid_scatter_block(a, sT, sG, sU, nblk, R, grad_rs);
        }
    }
    if (do_sc) ring_drain(R, 0u, grad_rs, a.dbg);
    // ---- flush the owned dW tiles
    if (do_dw) dw_flush_owned(accA, accB, a.dw + (size_t)k * FIELD_PARAMS, wid, cur);
}

// ---------------------------------------------------------------------------
// Merged backward: the K sub-NeRFs share the hash grid, and the samples of the
// K models on one ray visit the same cells.  k_field_bwd scatters each model's
// samples separately (one stream per (model, ray)); here a block owns a CHUNK
// of rays for all K models and scatters their samples merged in (ray, t)
// order, so consecutive samples of different models share 64-B segments and
// the atomic requests per sample drop (tools/atomic_sim.py on the bench
// workload: per-(model, ray) floor 19.3 -> 12.9 per ray for K = 2).
//
// Per chunk [r0, r1) (grabbed from a guided work queue over rays):
//  1. for each model k (alternating order, so one switch per chunk boundary):
//     switch the block to model k (park the other model's dW accumulators in
//     a per-block global area, reload the weights), then run the MLP backward
//     over model k's samples of the chunk in 8-tile windows (bwd_window) and
//     stage dL/dencoding + unit coords as 144-B rows in the block's scratch;
//  2. walk the chunk's merged order (perm, from rn_bwd_plan) in windows of 256
//     samples: rows -> LDS (sG/sU) -> grid_scatter_block, unchanged.
// The grid gradient is the same sum as k_field_bwd's (float atomics: equal up
// to summation order); dW is identical per model.
// ---------------------------------------------------------------------------
// scratch row (80 B = 20 floats): dE[32] as f16 in the block iteration's
// gradient scale (the dX chain's own range; tcnn's dL/dencoding is f16 too) |
// ux uy uz | 1 / scale (fp32).  Half the 144 B of fp32 rows: the chunk's rows
// stay in L2 for longer chunks.
#define MB_ROW 20
#define MB_WIN 64          // walk window: staged rows per chunk eighth
#define MB_RI_CAP 4096     // merged positions of a chunk with LDS row indices (else per-row perm reads)
#define CH_DESC 20         // chunk descriptor ints (80 B, 16-B aligned)
#define MB_KMAX 8

struct MergeArgs {
    const int32_t* mstart;   // [B + 1] first merged position of ray r; [B] = total
    const int32_t* perm;     // [total] merged position -> sample index
    const int32_t* desc;     // [n_chunks][CH_DESC]: r0, r1, -, -, first sample [8], count [8]
    int32_t* queue;          // [0] bwd ticket, [1] n_chunks, [2] fwd ticket (rn_bwd_plan)
    float* scratch;          // [gridDim.x][rows_cap][MB_ROW]
    float* park;             // [gridDim.x][K][BWD_WAVES][32][64]
    int32_t n_rays, n_models, rows_cap;
};

// wave's dW accumulators <-> its park slot (lane-linear, 32 x 256 B)
__device__ __forceinline__ void dw_park(float* p, const f32x16& A, const f32x16& B) {
    const int lane = rn_lane();
#pragma unroll
    for (int j = 0; j < 16; ++j) { p[j * 64 + lane] = A[j]; p[(16 + j) * 64 + lane] = B[j]; }
}
// (read back past L1 with sc1 buffer loads: nt loads are slow on gfx950)
__device__ __forceinline__ void dw_unpark(const float* p, f32x16& A, f32x16& B) {
    const uint32_t lo = 4u * (uint32_t)rn_lane();
    const __amdgpu_buffer_rsrc_t rs = rn_rsrc(p, 32 * 64 * 4);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        A[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, lo + 256u * j, 0, 16));
        B[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, lo + 256u * (16 + j), 0, 16));
    }
}

// GM: grid-gradient accumulation. 0 fp32 atomics, 1 exact integer with
// carries (IntGrad), 2 fixed point for the hashed levels (FxGrad), 3 the
// fp32 redo of a fixed-point step whose records overflowed the scale (grid
// scatter of the levels that went in as fixed point only, no dW; the launch
// exits at once unless *F.redo is set).
template <int CACHE, bool ABL, int GM>
__global__ void __launch_bounds__(BWD_WAVES * 64)
k_field_bwd_merged(FieldArgs a, MergeArgs m, IntGrad G, FxGrad F) {
    if (GM == 3 && __builtin_nontemporal_load(F.redo) == 0) return;   // uniform: whole grid exits
    if (GM == 1) {
        G.scale = *G.scale_ptr;
        G.lo = rn_rsrc(G.lo_ptr, G.bytes);
        G.carry = rn_rsrc(G.carry_ptr, G.bytes);
    }
    if (GM == 2) G.fx = rn_rsrc(F.acc, 2 * a.grid_bytes);
    // the walk phase stages its windows over the waves' images AND the
    // weights (the weights are reloaded for the next chunk's MLP phase):
    // eighths 0-3 in sImg (then the rings of waves 4-7), eighths 4-7 in sW.
    // (One array for both made the compiler spill 80 VGPRs.)
    __shared__ __attribute__((aligned(16))) rn_half sW[FIELD_FRAGS * RN_FRAG_HALFS];
    __shared__ __attribute__((aligned(16))) rn_half sImg[BWD_WAVES * 2 * RN_IMG_HALFS];
    __shared__ float sMax[2 * BWD_WAVES];
    __shared__ LvTab sT;
    __shared__ uint32_t sRing[BWD_WAVES * SC_STREAMS * 3 * SC_RING];
    __shared__ DwScale sScale[MB_KMAX];         // per model: scales of its parked dW (0 = none)
    // chunk descriptor: r0, r1, then per model: first sample, count, row offset, segment base
    __shared__ int32_t sCh[2 + 4 * MB_KMAX];
    // the walk's scratch-row index of each merged position of the chunk
    __shared__ uint16_t sRowIdx[MB_RI_CAP];
    const int K = m.n_models, B = m.n_rays;
    lv_stage(sT, a.gm);
    if (threadIdx.x < MB_KMAX) sScale[threadIdx.x] = DwScale{0.f, 0.f};

    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / RN_WAVE);
    const int lvA = w2_level_a(wid);             // this wave's walk levels: lvA, 15 - lvA
    const int lane = rn_lane(), c = lane & 31, h = lane >> 5;
    rn_half* imgY = sImg + wid * 2 * RN_IMG_HALFS;
    rn_half* imgX = imgY + RN_IMG_HALFS;
    const __amdgpu_buffer_rsrc_t grad_rs = rn_rsrc(a.grid_grad, 2 * a.grid_bytes);
    const int dbg = ABL ? a.dbg : 0;      // ablation flags (tools/ablate.py) only in ABL builds
    const bool do_dw = !(rn_dbg(dbg) & 2) && GM != 3;
    // fixed point: this wave's two levels' scales (wave-uniform) and maxima
    float fxA = 0.f, fxB = 0.f;
    uint32_t vmA = 0u, vmB = 0u;
    int64_t sqA = 0, sqB = 0;
    uint64_t swA = 0, swB = 0;
    // binned mode: this wave's open pages (none yet: the first issue takes one)
    uint32_t pgA = 0xffffffffu, pgB = 0xffffffffu, nA = GB_PAGE, nB = GB_PAGE;
    if (GM >= 2) {
        fxA = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(F.scale[lvA])));
        fxB = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(F.scale[RN_L - 1 - lvA])));
    }
    const bool do_sc = !(rn_dbg(dbg) & 4);
    // walk windows of MB_WIN rows per eighth: each window's staging loads
    // wait (vmcnt, in issue order) for the atomics the previous window issued,
    // so fewer, longer windows wait less often (round 3: 32 -> 64)
    // one eighth's staging block: MB_WIN rows of dL/dE (SG_STRIDE floats)
    // then MB_WIN unit coords + 1/scale (4 floats)
    constexpr int EB = MB_WIN * (SG_STRIDE + 4);         // floats per eighth
    auto eighth_g = [&](int e) -> float* {
        return e < 4 ? reinterpret_cast<float*>(sImg) + e * EB
                     : reinterpret_cast<float*>(sW) + (e - 4) * EB;
    };
    // walk rings: waves 0-3 in sRing, waves 4-7 in sImg past eighths 0-3
    // (free during the scatter phase; drained every chunk)
    static_assert(4 * W2_RING_WORDS * 4 <= BWD_WAVES * SC_STREAMS * 3 * SC_RING * 4, "rings");
    static_assert(4 * EB * 4 + 4 * W2_RING_WORDS * 4 <= BWD_WAVES * 2 * RN_IMG_HALFS * 2,
                  "eighths 0-3 + rings in the image region");
    static_assert(4 * EB * 4 <= FIELD_FRAGS * RN_FRAG_HALFS * 2, "eighths 4-7 in the weights");
    uint32_t* ring2 = wid < 4 ? sRing + wid * W2_RING_WORDS
                              : reinterpret_cast<uint32_t*>(sImg) + 4 * EB +
                                    (wid - 4) * W2_RING_WORDS;
    // this lane's walk eighth (stream = lane >> 2, eighth = stream >> 1)
    float* const wG = eighth_g(rn_lane() >> 3);
    float* const wU = wG + MB_WIN * SG_STRIDE;
    bool sw_ok = false;                          // sW holds model cur_k's weights

    f32x16 accA = rn_zero16(), accB = rn_zero16();
    DwScale cur = {0.f, 0.f};
    int cur_k = -1;
    // (ablation build, flag 4096) summed wave cycles: [0] MLP phase, [1]
    // window staging, [2] walk, [3] chunk tails; inside the MLP phase [4]
    // model switches (park / unpark / weights), [5] forward recompute, [6]
    // bwd_window, [7] row stores
    uint64_t cyc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    float* park = m.park + (size_t)blockIdx.x * K * BWD_WAVES * 2048 + wid * 2048;
    float* rows = m.scratch + (size_t)blockIdx.x * m.rows_cap * MB_ROW;
    const __amdgpu_buffer_rsrc_t rows_rs = rn_rsrc(rows, (uint32_t)m.rows_cap * MB_ROW * 4u);
    int n_local = 0;
    int ticket = 0, n_chunks = 0;
    if (threadIdx.x == 0) { n_chunks = m.queue[1]; ticket = atomicAdd(m.queue, 1); }
    if (threadIdx.x < K) sCh[2 + 3 * MB_KMAX + threadIdx.x] = a.seg_base[threadIdx.x];

    for (;;) {
        __syncthreads();                         // previous chunk done with sCh / LDS
        if (threadIdx.x == 0) {
            // this chunk's descriptor (one 80-B load; its ticket was taken
            // during the previous chunk) and the next chunk's ticket
            const int ch = ticket;
            ticket = atomicAdd(m.queue, 1);
            int4 d[CH_DESC / 4];
            if (ch < n_chunks) {
#pragma unroll
                for (int q = 0; q < CH_DESC / 4; ++q)
                    d[q] = reinterpret_cast<const int4*>(m.desc + (size_t)ch * CH_DESC)[q];
            }
            const int32_t* di = reinterpret_cast<const int32_t*>(d);
            sCh[0] = ch < n_chunks ? di[0] : B; sCh[1] = ch < n_chunks ? di[1] : B;
            int roff = 0;
            for (int k = 0; k < K; ++k) {
                const int nk = ch < n_chunks ? di[4 + MB_KMAX + k] : 0;
                sCh[2 + k] = di[4 + k]; sCh[2 + MB_KMAX + k] = nk;
                sCh[2 + 2 * MB_KMAX + k] = roff;
                roff += nk;
            }
        }
        __syncthreads();
        const int r0 = sCh[0], r1 = sCh[1];
        if (r0 >= B) break;
        const bool rev = n_local & 1;
        ++n_local;
        // the chunk's rays into LDS (the walk rings' area, free until the
        // walk): the MLP tiles look a sample's ray up there
        constexpr int RAYS_LDS = BWD_WAVES * SC_STREAMS * 3 * SC_RING / 6;
        const int nr_lds = r1 - r0 <= RAYS_LDS ? r1 - r0 : 0;
        float* sRays = reinterpret_cast<float*>(sRing);
        for (int i = threadIdx.x; i < 6 * nr_lds; i += blockDim.x) {
            const int q = i / 6, cc = i - 6 * q;
            sRays[i] = cc < 3 ? a.rays_o[3 * (r0 + q) + cc] : a.rays_d[3 * (r0 + q) + cc - 3];
        }
        __syncthreads();

        // ---- 1. MLP backward per model, rows staged in the block's scratch
        const bool prof = ABL && (rn_dbg(dbg) & 4096);
        uint64_t tp0 = prof ? __builtin_amdgcn_s_memtime() : 0;
        for (int kk = 0; kk < K; ++kk) {
            const int k = rev ? K - 1 - kk : kk;
            const int a_k = sCh[2 + k], n_k = sCh[2 + MB_KMAX + k], roff = sCh[2 + 2 * MB_KMAX + k];
            if (n_k == 0) continue;
            uint64_t ts0 = prof ? __builtin_amdgcn_s_memtime() : 0;
            if (k != cur_k || !sw_ok) {
                // model k's weights and (k != cur_k) its parked dW tiles are
                // loaded first, then the current model's tiles are parked:
                // vmcnt counts in issue order, so loads issued after the
                // park's stores waited for them (a model switch took ~10 %
                // of the MLP phase at K = 8).  A model never parked has
                // scale 0 and its loaded tiles are dropped.
                constexpr int WV = (FIELD_FRAGS * RN_FRAG_BYTES / 16 + BWD_WAVES * RN_WAVE - 1) /
                                   (BWD_WAVES * RN_WAVE);
                int4 wv[WV];
                const int4* wsrc =
                    reinterpret_cast<const int4*>(a.frags + (size_t)k * FIELD_FRAGS * RN_FRAG_HALFS);
#pragma unroll
                for (int q = 0; q < WV; ++q) {
                    const int i = threadIdx.x + q * BWD_WAVES * RN_WAVE;
                    wv[q] = i < FIELD_FRAGS * RN_FRAG_BYTES / 16 ? wsrc[i] : int4{0, 0, 0, 0};
                }
                const bool sw_k = k != cur_k;
                const DwScale nsc = sw_k ? sScale[k] : cur;
                f32x16 nA = accA, nB = accB;
                if (sw_k) dw_unpark(park + (size_t)k * BWD_WAVES * 2048, nA, nB);
                __syncthreads();                 // every wave done with sW
                if (sw_k && cur_k >= 0) {
                    dw_park(park + (size_t)cur_k * BWD_WAVES * 2048, accA, accB);
                    if (threadIdx.x == 0) sScale[cur_k] = cur;
                }
                int4* wdst = reinterpret_cast<int4*>(sW);
#pragma unroll
                for (int q = 0; q < WV; ++q) {
                    const int i = threadIdx.x + q * BWD_WAVES * RN_WAVE;
                    if (i < FIELD_FRAGS * RN_FRAG_BYTES / 16) wdst[i] = wv[q];
                }
                __syncthreads();
                if (sw_k) {
                    cur = nsc;
                    const bool live = nsc.a != 0.f || nsc.b != 0.f;
                    accA = live ? nA : rn_zero16();
                    accB = live ? nB : rn_zero16();
                    cur_k = k;
                }
            }
            sw_ok = true;
            if (prof) { const uint64_t t = __builtin_amdgcn_s_memtime(); cyc[4] += t - ts0; ts0 = t; }
            for (int w0 = 0; w0 < n_k; w0 += BWD_WAVES * 32) {
                rn_lds_order();
                const int i = w0 + wid * 32 + c;
                const bool valid = i < n_k;
                // ablation 256: every tile reads the chunk's first 32 samples
                // (cache-resident inputs; timing only)
                const int64_t s = a_k + (valid ? ((rn_dbg(dbg) & 256) ? (i & 31) : i) : 0);
                FwdState st;
                float ux, uy, uz;
                // the backward seeds, loaded ahead of the forward recompute
                // (their latency hides behind its MFMAs)
                float pre[4] = {0.f, 0.f, 0.f, 0.f};
                if (valid && h == 0) {
                    pre[0] = a.dsigma[s];
                    pre[1] = a.drgb[3 * s]; pre[2] = a.drgb[3 * s + 1]; pre[3] = a.drgb[3 * s + 2];
                }
                tile_forward_rays<CACHE>(a, sT, sW, s, valid,
                                         CACHE == CACHE_READ ? cache_slot(a, s) : nullptr, sRays,
                                         r0, nr_lds, st, ux, uy, uz);
                if (prof) {
                    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                    const uint64_t t = __builtin_amdgcn_s_memtime(); cyc[5] += t - ts0; ts0 = t;
                }
                float gscale; bool zero_iter;
                // ablation 512: no block barriers in the MLP phase (wrong
                // results; timing of the barrier cost only)
                const f32x16 dE = bwd_window(a, sW, sImg, sMax, imgY, imgX, st, valid, s, wid,
                                             accA, accB, cur, do_dw, gscale, zero_iter,
                                             !(rn_dbg(dbg) & 512), pre);
                if (prof) { const uint64_t t = __builtin_amdgcn_s_memtime(); cyc[6] += t - ts0; ts0 = t; }
                if (valid) {
                    const float ginv = zero_iter ? 0.f : 1.0f / gscale;
                    float* row = rows + (size_t)(roff + i) * MB_ROW;
                    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
                    h4* rh = reinterpret_cast<h4*>(row);
#pragma unroll
                    for (int g = 0; g < 4; ++g)     // features 8g + 4h .. +3 = dE[4g .. 4g+3]
                        rh[2 * g + h] = h4{(_Float16)dE[4 * g], (_Float16)dE[4 * g + 1],
                                           (_Float16)dE[4 * g + 2], (_Float16)dE[4 * g + 3]};
                    if (h == 0) *reinterpret_cast<float4*>(row + 16) = make_float4(ux, uy, uz, ginv);
                }
                if (prof) { const uint64_t t = __builtin_amdgcn_s_memtime(); cyc[7] += t - ts0; ts0 = t; }
            }
        }
        if (prof) { const uint64_t t = __builtin_amdgcn_s_memtime(); cyc[0] += t - tp0; tp0 = t; }
        if (!do_sc) continue;

        // ---- 2. scatter in merged (ray, t) order
        const int p_base = m.mstart[r0], n_p = m.mstart[r1] - p_base;
        // scratch row of merged position p: the sample's model k from the
        // segment bases (branch-free, K <= 8), its row offset in the chunk
        auto row_of = [&](int p) -> int {
            const int smp = m.perm[p_base + p];
            int k = 0;
#pragma unroll
            for (int kq = 1; kq < MB_KMAX; ++kq)
                k = (kq < K && smp >= sCh[2 + 3 * MB_KMAX + kq]) ? kq : k;
            return sCh[2 + 2 * MB_KMAX + k] + (smp - sCh[2 + k]);
        };
        // the chunk's row indices in LDS, built once with coalesced perm reads
        // before the walk issues anything: a window's staging then reads them
        // from LDS instead of loading perm per row (a global load that waited,
        // vmcnt in issue order, for every atomic / page store the wave had
        // issued before it).  A chunk longer than the table reads perm per row.
        const bool ri_ok = n_p <= MB_RI_CAP;                // block-uniform
        if (ri_ok) {
            // all of a thread's perm loads in flight together (a plain loop
            // waited for each one)
            constexpr int RI_PER = MB_RI_CAP / (BWD_WAVES * RN_WAVE);
            int smp[RI_PER];
#pragma unroll
            for (int q = 0; q < RI_PER; ++q) {
                const int p = threadIdx.x + q * BWD_WAVES * RN_WAVE;
                smp[q] = p < n_p ? m.perm[p_base + p] : 0;
            }
#pragma unroll
            for (int q = 0; q < RI_PER; ++q) {
                const int p = threadIdx.x + q * BWD_WAVES * RN_WAVE;
                int k = 0;
#pragma unroll
                for (int kq = 1; kq < MB_KMAX; ++kq)
                    k = (kq < K && smp[q] >= sCh[2 + 3 * MB_KMAX + kq]) ? kq : k;
                if (p < n_p) sRowIdx[p] = (uint16_t)(sCh[2 + 2 * MB_KMAX + k] + (smp[q] - sCh[2 + k]));
            }
        }
        __builtin_amdgcn_s_waitcnt(0x0070);     // vmcnt(0): this wave's rows are in L2
        __syncthreads();
        // the chunk's merged order is cut into 8 contiguous eighths, one per
        // stream eighth; each window stages the next 32 rows of every eighth
        // and the walks carry their state across windows (no restart per window)
        const int E = (n_p + 7) >> 3;
        const int elen_lane = max(0, min(E, n_p - (rn_lane() >> 3) * E));   // walk eighth
        Walk2 W;
        walk2_begin(W, ring2);
        W.fxA = fxA; W.fxB = fxB; W.vmA = vmA; W.vmB = vmB; W.sqA = sqA; W.sqB = sqB;
        W.swA = swA; W.swB = swB;
        W.pgA = pgA; W.pgB = pgB; W.nA = nA; W.nB = nB;
        W.loffA = sT.off[lvA]; W.loffB = sT.off[RN_L - 1 - lvA];
        sw_ok = false;                           // the staging overwrites sW
        for (int w0 = 0; w0 < E; w0 += MB_WIN) {
          int nz = 0;
#pragma unroll 1
          for (int pass = 0; pass < MB_WIN / 32; ++pass) {
            // wave e stages eighth e's rows [w0, w0 + MB_WIN), 32 per pass
            const int half = threadIdx.x & 1;
            const int e = wid, jj = pass * 32 + ((threadIdx.x >> 1) & 31);
            float* const sG = eighth_g(e);               // wave-uniform
            float* const sU = sG + MB_WIN * SG_STRIDE;
            const int j = jj;                            // row of the eighth's block
            const int elen = max(0, min(E, n_p - e * E));
            if (w0 + jj < elen) {
                const int row_i = ri_ok ? (int)sRowIdx[e * E + w0 + jj] : row_of(e * E + w0 + jj);
                // rows were written by other waves of this block: read past L1
                // with sc1 buffer loads (L2-served; the nt loads used before cost
                // field_bwd 0.09 ms at C3, profiles/r03/rowab_*_r1.json)
                typedef float nf4 __attribute__((ext_vector_type(4)));
                typedef _Float16 h8 __attribute__((ext_vector_type(8)));
                const uint32_t rb = (uint32_t)row_i * (MB_ROW * 4u);
                const nf4 u = __builtin_bit_cast(nf4, __builtin_amdgcn_raw_buffer_load_b128(
                    rows_rs, rb + 64u, 0, 16));
                float* dst = sG + j * SG_STRIDE + 16 * half;
                typedef uint32_t u4v __attribute__((ext_vector_type(4)));
                // both 16-B halves of the row's dL/dE loaded before either is
                // used (one round trip per row)
                u4v raw[2];
#pragma unroll
                for (int qq = 0; qq < 2; ++qq)
                    raw[qq] = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(
                        rows_rs, rb + 16u * (2u * half + qq), 0, 16));
                uint32_t bits = 0u;
#pragma unroll
                for (int qq = 0; qq < 2; ++qq) {
                    const h8 v = __builtin_bit_cast(h8, raw[qq]);
                    bits |= (raw[qq].x | raw[qq].y) | (raw[qq].z | raw[qq].w);
#pragma unroll
                    for (int e2 = 0; e2 < 8; e2 += 2) {
                        const float a0 = (float)v[e2] * u.w, a1 = (float)v[e2 + 1] * u.w;
                        *reinterpret_cast<float2*>(dst + 8 * qq + e2) = make_float2(a0, a1);
                    }
                }
                // any non-zero row value (sign bits masked) with a non-zero
                // 1/scale: a superset of "some staged product is non-zero"
                // (only an fp32 underflow of the product differs, and walking
                // a window of zeros adds nothing); per-element tests of the
                // products compiled to ~60 VALU per row half
                nz |= ((bits & 0x7fff7fffu) != 0u) & (u.w != 0.f);
                // both lanes of the row store the same coordinates (no
                // lane-parity branch)
                *reinterpret_cast<nf4*>(sU + j * 4) = u;
            }
          }
            // a window whose rows are all zero (rays past early termination)
            // adds nothing; skipping it keeps the walk state valid (entries
            // are identified by their coordinates)
            const bool live_w = __syncthreads_or(nz);
            if (prof) { const uint64_t t = __builtin_amdgcn_s_memtime(); cyc[1] += t - tp0; tp0 = t; }
            if (live_w && !(rn_dbg(dbg) & 32)) {
                const int ne = max(0, min(MB_WIN, elen_lane - w0));
                const int n0 = max(0, min(MB_WIN, min(E, n_p) - w0));
                walk2_window<GM, MB_WIN>(a, sT, wG, wU, ne, n0, grad_rs, G, W, dbg);
            }
            __syncthreads();
            if (prof) { const uint64_t t = __builtin_amdgcn_s_memtime(); cyc[2] += t - tp0; tp0 = t; }
        }
        walk2_end<GM>(a, sT, grad_rs, G, W, dbg);
        if (prof) { const uint64_t t = __builtin_amdgcn_s_memtime(); cyc[3] += t - tp0; tp0 = t; }
        vmA = W.vmA; vmB = W.vmB; sqA = W.sqA; sqB = W.sqB;
        swA = W.swA; swB = W.swB;
        pgA = W.pgA; pgB = W.pgB; nA = W.nA; nB = W.nB;
        __syncthreads();                         // rings (image region) drained
    }
    if (ABL && (rn_dbg(dbg) & 4096) && rn_lane() == 0) {
#pragma unroll
        for (int q = 0; q < 8; ++q) atomicAdd(g_rn_cyc + q, (unsigned long long)cyc[q]);
    }
    if (GM >= 4 && rn_lane() == 0) {             // close this wave's open pages
        if (pgA < G.pool_pages) G.page_meta[pgA] = (uint32_t)lvA | (nA << 8);
        if (pgB < G.pool_pages) G.page_meta[pgB] = (uint32_t)(RN_L - 1 - lvA) | (nB << 8);
    }
    if (GM == 2 || GM >= 4) {                    // this step's largest |record| per level
        vmA = rn_wave_max_u32(vmA);
        vmB = rn_wave_max_u32(vmB);
        int64_t dA = sqA, dB = sqB;
        uint64_t eA = swA, eB = swB;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            dA += __shfl_xor(dA, off);
            dB += __shfl_xor(dB, off);
            eA += __shfl_xor(eA, off);
            eB += __shfl_xor(eB, off);
        }
        if (rn_lane() == 0) {
            if (vmA) atomicMax(F.vmax + lvA, vmA);
            if (vmB) atomicMax(F.vmax + RN_L - 1 - lvA, vmB);
            if (dA != 0) atomicAdd(reinterpret_cast<unsigned long long*>(F.qsum + lvA),
                                   (unsigned long long)dA);
            if (dB != 0) atomicAdd(reinterpret_cast<unsigned long long*>(F.qsum + RN_L - 1 - lvA),
                                   (unsigned long long)dB);
            if (eA != 0) atomicAdd(reinterpret_cast<unsigned long long*>(F.wq + lvA), eA);
            if (eB != 0) atomicAdd(reinterpret_cast<unsigned long long*>(F.wq + RN_L - 1 - lvA), eB);
        }
    }
    // ---- flush every model's dW (the current one from registers)
    if (do_dw) {
        for (int k = 0; k < K; ++k) {
            DwScale sc = sScale[k];
            f32x16 A, Bm;
            if (k == cur_k) { sc = cur; A = accA; Bm = accB; }
            else if (sc.a != 0.f || sc.b != 0.f) dw_unpark(park + (size_t)k * BWD_WAVES * 2048, A, Bm);
            if (sc.a != 0.f || sc.b != 0.f)
                dw_flush_owned(A, Bm, a.dw + (size_t)k * FIELD_PARAMS, wid, sc);
        }
    }
}

// ---------------------------------------------------------------------------
// Merged forward: blocks take the plan's chunks (whole rays) and evaluate the
// K models' tiles of a chunk interleaved (tile i of model 0, tile i of model
// 1, ...), so the models' samples of the same rays are gathered close in time
// by the same CU: the second model's corners hit L1/L2 lines the first one
// fetched (the fine levels otherwise miss L2 for every sample).  With
// K <= FM_LDS_K the K models' forward fragments sit in LDS (dynamic, K x
// 24 KB); with more (GW), the MLP tiles read them from global memory (L2).
// Same outputs as k_field_fwd (per-sample arithmetic is identical).
// ---------------------------------------------------------------------------
#define FM_KMAX 8
#define FM_LDS_K 4

template <int CACHE, bool ENC_M, bool GW>
__global__ void __launch_bounds__(1024)
k_field_fwd_merged(FieldArgs a, MergeArgs m) {
    extern __shared__ __attribute__((aligned(16))) rn_half sWm[];   // [K][24 frags]
    __shared__ LvTab sT;
    __shared__ int32_t sCh[2][2 + 2 * FM_KMAX];      // this and the previous chunk
    const int K = m.n_models, B = m.n_rays;
    if (!GW) {
        for (int k = 0; k < K; ++k)
            rn_block_copy16(sWm + (size_t)k * FIELD_FWD_FRAGS * RN_FRAG_HALFS,
                            a.frags + (size_t)k * FIELD_FRAGS * RN_FRAG_HALFS,
                            FIELD_FWD_FRAGS * RN_FRAG_BYTES);
    }
    lv_stage(sT, a.gm);
    const int waves = blockDim.x / RN_WAVE;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / RN_WAVE);
    const int lane = rn_lane(), c = lane & 31, h = lane >> 5;
    int ticket = 0, n_chunks = 0;
    if (threadIdx.x == 0) { n_chunks = m.queue[1]; ticket = atomicAdd(m.queue + 2, 1); }

    // per-model MLP tile u of chunk descriptor ch (tile i of model 0, tile i
    // of model 1, ...); false: past the end
    auto mlp_tile = [&](const int32_t* ch, int u) {
        const int k = u % K, t = u / K;
        const int n_k = ch[2 + FM_KMAX + k];
        if (t * 32 >= n_k) return;                           // wave-uniform
        rn_lds_order();
        const int i = t * 32 + c;
        const bool valid = i < n_k;
        const int64_t s = ch[2 + k] + (valid ? i : 0);
        FwdState st;
        float ux, uy, uz;
        constexpr int TC = ENC_M ? CACHE_READ_NT : CACHE;
        const rn_half* W = GW ? a.frags + (size_t)k * FIELD_FRAGS * RN_FRAG_HALFS
                              : sWm + (size_t)k * FIELD_FWD_FRAGS * RN_FRAG_HALFS;
        tile_forward_s<1, TC>(a, sT, W, s, valid, TC != CACHE_NONE ? cache_slot(a, s) : nullptr,
                              st, ux, uy, uz);
        if (valid && h == 0) {
            a.sigma[s] = expf(st.g0);
            a.rgb[3 * s + 0] = sigmoidf(st.out[0]);
            a.rgb[3 * s + 1] = sigmoidf(st.out[1]);
            a.rgb[3 * s + 2] = sigmoidf(st.out[2]);
        }
    };
    auto mlp_tiles = [&](const int32_t* ch) {
        int max_t = 0;
        for (int k = 0; k < K; ++k) max_t = max(max_t, (ch[2 + FM_KMAX + k] + 31) >> 5);
        return max_t * K;
    };

    bool prev_live = false;
    for (int it = 0;; ++it) {
        int32_t* cur = sCh[it & 1];
        const int32_t* prev = sCh[(it & 1) ^ 1];
        __syncthreads();
        if (threadIdx.x == 0) {
            const int ch = ticket;
            ticket = atomicAdd(m.queue + 2, 1);           // the next chunk's, ahead
            int4 d[CH_DESC / 4];
            if (ch < n_chunks) {
#pragma unroll
                for (int q = 0; q < CH_DESC / 4; ++q)
                    d[q] = reinterpret_cast<const int4*>(m.desc + (size_t)ch * CH_DESC)[q];
            }
            const int32_t* di = reinterpret_cast<const int32_t*>(d);
            cur[0] = ch < n_chunks ? di[0] : B;
            cur[1] = ch < n_chunks ? di[1] : B;
            for (int k = 0; k < K; ++k) {
                cur[2 + k] = di[4 + k];
                cur[2 + FM_KMAX + k] = ch < n_chunks ? di[4 + MB_KMAX + k] : 0;
            }
        }
        __syncthreads();
        const bool live = cur[0] < B;
        if (!ENC_M) {
            if (!live) break;
            const int nt = mlp_tiles(cur);
            for (int u = wid; u < nt; u += waves) mlp_tile(cur, u);
            continue;
        }
        // Merged-order encoding, software-pipelined over chunks: iteration it
        // encodes chunk it in merged (ray, t, model) order into the encoding
        // cache -- a tile mixes the sub-NeRFs of one ray stretch, so its
        // corners share more lines (tools/fwd_lines_sim.py: 20.9 vs 28.2 lines
        // per sample) -- and runs the per-model MLP tiles of chunk it - 1,
        // whose encodings the barrier above published; one work list, no
        // barrier between the two kinds of tile.
        if (!live && !prev_live) break;
        int p_base = 0, n_p = 0;
        if (live) { p_base = m.mstart[cur[0]]; n_p = m.mstart[cur[1]] - p_base; }
        const int nA = (n_p + 31) >> 5;
        const int nB = prev_live ? mlp_tiles(prev) : 0;
        for (int u = wid; u < nA + nB; u += waves) {
            if (u >= nA) { mlp_tile(prev, u - nA); continue; }
            const int q = u * 32 + c;
            const bool valid = q < n_p;
            const int64_t s = m.perm[p_base + (valid ? q : 0)];
            float x, y, z, dx, dy, dz;
            load_sample<1>(a, s, x, y, z, dx, dy, dz);
            const float ux = unit_coord(x, a.xyz_min[0], a.extent[0]);
            const float uy = unit_coord(y, a.xyz_min[1], a.extent[1]);
            const float uz = unit_coord(z, a.xyz_min[2], a.extent[2]);
            half8 e0, e1;
            encode_lane(a, sT, rn_rsrc(a.grid, a.grid_bytes), h, ux, uy, uz, valid, e0, e1);
            if (valid) { half8* fc = cache_slot(a, s); fc[0] = e0; fc[1] = e1; }
        }
        prev_live = live;
    }
}


// ---------------------------------------------------------------------------
// Level-partitioned forward (round 3, after a probe: tools/enc_probe.py).
// The merged forward gathers all sixteen levels of a sample on one CU, so
// every XCD's 4 MB L2 faces the whole 23 MB table and the fine levels miss
// it for nearly every sample (27 fabric requests per sample at C5).  Here
// the encoding is split by level instead:
//   1. k_enc_prep: per merged position p the sample's unit coordinates and
//      index (16 B), computed once (bit-identical to load_sample<1>);
//   2. k_field_encode_levels: block b encodes levels g and 15 - g, g = b % 8,
//      for every sample (one level after the other).  Workgroups are dispatched to the XCDs round-robin
//      (a rotation that varies by dispatch: measured, group g ran on XCD
//      g - 1 for all its blocks), so each XCD gathers from two levels' tables
//      only; correctness does not depend on the mapping.  Output: one f16x2
//      plane per level, planes[L][s] (bit-identical to encode_lane);
//   3. k_field_mlp_planes: the MLP tiles per model read the 8 levels of each
//      lane from the planes, write sigma / rgb and the encoding cache (tile
//      layout) that the backward and the input-gradient kernels read.
// Static splits, no ticket queues (a per-XCD ticket word serialised at
// ~100 ns per ticket: 1.9 ms at C3).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
k_enc_prep(FieldArgs a, MergeArgs m, float4* __restrict__ prep) {
    const int P = m.mstart[m.n_rays];
    for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < P; p += gridDim.x * blockDim.x) {
        const int s = m.perm[p];
        float x, y, z, dx, dy, dz;
        load_sample<1>(a, s, x, y, z, dx, dy, dz);
        prep[p] = make_float4(unit_coord(x, a.xyz_min[0], a.extent[0]),
                              unit_coord(y, a.xyz_min[1], a.extent[1]),
                              unit_coord(z, a.xyz_min[2], a.extent[2]), __int_as_float(s));
    }
}

__global__ void __launch_bounds__(256)
k_field_encode_levels(FieldArgs a, MergeArgs m, const float4* __restrict__ prep,
                      int32_t* __restrict__ xq, uint64_t pairing) {
    __shared__ LvTab sT;
    lv_stage(sT, a.gm);
    __syncthreads();
    const int g = blockIdx.x & 7;
    if (xq && threadIdx.x == 0) {           // probe: group g's blocks per XCD, its span
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
        atomicAdd(xq + 8 * g + (int)(xcc & 7u), 1);
        atomicMin(reinterpret_cast<unsigned long long*>(xq + 64) + g,
                  (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
    // group g's levels: byte g of `pairing` (low nibble la, high lb)
    const int la = (int)((pairing >> (8 * g)) & 15u), lb = (int)((pairing >> (8 * g + 4)) & 15u);
    const int P = m.mstart[m.n_rays];
    const int nt = (P + 31) >> 5;
    const int nb = (int)(gridDim.x >> 3), j = (int)(blockIdx.x >> 3);
    const int t0 = (int)((int64_t)nt * j / nb), t1 = (int)((int64_t)nt * (j + 1) / nb);
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), waves = blockDim.x >> 6;
    const int lane = rn_lane(), c = lane & 31, h = lane >> 5;
    const __amdgpu_buffer_rsrc_t rs = rn_rsrc(a.grid, a.grid_bytes);
    const LvConst LA = lv_const_uniform(sT, a.gm, la), LB = lv_const_uniform(sT, a.gm, lb);
    // level la over the block's tiles, then level lb: the XCD's blocks run in
    // step, so its L2 holds one level's table at a time (two hashed levels at
    // once, 4 MB, filled the whole L2).  A wave takes two tiles per pass.
#pragma unroll 1
    for (int ph = 0; ph < 2; ++ph) {
        const LvConst& LC = ph ? LB : LA;
        uint32_t* const out = const_cast<uint32_t*>(a.planes) + (size_t)(ph ? lb : la) * a.plane_stride;
        for (int t = t0 + 2 * wid; t < t1; t += 2 * waves) {
            const bool v0 = t * 32 + c < P;
            const bool v1 = t + 1 < t1 && (t + 1) * 32 + c < P;
            const bool valid = h ? v1 : v0;
            const int p = (t + h) * 32 + c;
            const float4 q = prep[valid ? p : 0];
            const uint32_t v = encode_tiles(a, rs, h, LC, q.x, q.y, q.z, v0, v1);
            if (valid) __builtin_nontemporal_store(v, out + __float_as_int(q.w));
        }
    }
    if (xq) {
        __syncthreads();
        if (threadIdx.x == 0)
            atomicMax(reinterpret_cast<unsigned long long*>(xq + 80) + g,
                      (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
}

// MLP tiles of the K models (tile u of the flat list: model k's 32 samples
// from seg_base[k] + 32 t).  Block b takes a contiguous range of the list,
// which spans one or two models at the bench sizes; their forward fragments
// are staged in LDS, FM_LDS_K models at a time.
__global__ void __launch_bounds__(1024)
k_field_mlp_planes(FieldArgs a, int K) {
    extern __shared__ __attribute__((aligned(16))) rn_half sWm[];   // [<= FM_LDS_K][24 frags]
    __shared__ LvTab sT;
    // the K segments (first sample, count), read once: per tile they were a
    // global round trip ahead of the tile's dependent loads
    __shared__ int32_t sSeg[2][FM_KMAX];
    lv_stage(sT, a.gm);
    if (threadIdx.x < K) {
        sSeg[0][threadIdx.x] = a.seg_base[threadIdx.x];
        sSeg[1][threadIdx.x] = a.seg_count[threadIdx.x];
    }
    int first[FM_KMAX + 1];
    first[0] = 0;
    for (int k = 0; k < K; ++k)
        first[k + 1] = first[k] + ((__builtin_amdgcn_readfirstlane(a.seg_count[k]) + 31) >> 5);
    const int T = first[K];
    const int u0 = (int)((int64_t)T * blockIdx.x / gridDim.x);
    const int u1 = (int)((int64_t)T * (blockIdx.x + 1) / gridDim.x);
    if (u0 >= u1) return;                                   // block-uniform
    int k_lo = 0, k_hi = 0;
    for (int k = 0; k < K; ++k) {
        if (first[k + 1] <= u0) k_lo = k + 1;
        if (first[k] < u1) k_hi = k;
    }
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), waves = blockDim.x >> 6;
    const int lane = rn_lane(), c = lane & 31, h = lane >> 5;
    for (int kb = k_lo; kb <= k_hi; kb += FM_LDS_K) {
        const int ke = min(k_hi, kb + FM_LDS_K - 1);
        __syncthreads();                                    // previous models' tiles done
        for (int k = kb; k <= ke; ++k)
            rn_block_copy16(sWm + (size_t)(k - kb) * FIELD_FWD_FRAGS * RN_FRAG_HALFS,
                            a.frags + (size_t)k * FIELD_FRAGS * RN_FRAG_HALFS,
                            FIELD_FWD_FRAGS * RN_FRAG_BYTES);
        __syncthreads();
        const int ua = max(u0, first[kb]), ub = min(u1, first[ke + 1]);
        for (int u = ua + wid; u < ub; u += waves) {
            int k = kb;
            while (k < ke && u >= first[k + 1]) ++k;
            const int t = u - first[k];
            const int n_k = sSeg[1][k];
            const int i = t * 32 + c;
            const bool valid = i < n_k;
            const int64_t s = sSeg[0][k] + (valid ? i : 0);
            FwdState st;
            float ux, uy, uz;
            rn_lds_order();
            tile_forward_s<1, CACHE_PLANES>(a, sT, sWm + (size_t)(k - kb) * FIELD_FWD_FRAGS * RN_FRAG_HALFS,
                                            s, valid, a.feat ? cache_slot(a, s) : nullptr, st,
                                            ux, uy, uz);
            if (valid && h == 0) {
                a.sigma[s] = expf(st.g0);
                a.rgb[3 * s + 0] = sigmoidf(st.out[0]);
                a.rgb[3 * s + 1] = sigmoidf(st.out[1]);
                a.rgb[3 * s + 2] = sigmoidf(st.out[2]);
            }
        }
    }
}


// Integer-mode scale: 2^(26 - e) with 2^(e-1) <= M < 2^e, M the largest
// backward seed of the step (|dL/dsigma * sigma|, |dL/drgb|), so a seed-sized
// contribution is ~2^26 units; larger ones carry exactly.
__global__ void __launch_bounds__(256)
k_seed_max(const int32_t* __restrict__ seg_base, const int32_t* __restrict__ seg_count,
           const float* __restrict__ sigma, const float* __restrict__ dsigma,
           const float* __restrict__ drgb, uint32_t* __restrict__ mbits) {
    const int k = blockIdx.y;
    const int64_t base = seg_base[k], n = seg_count[k];
    float mx = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = base + i;
        mx = fmaxf(mx, fabsf(dsigma[s] * sigma[s]));
        mx = fmaxf(mx, fmaxf(fabsf(drgb[3 * s]), fmaxf(fabsf(drgb[3 * s + 1]), fabsf(drgb[3 * s + 2]))));
    }
    mx = rn_wave_max(mx);
    if (rn_lane() == 0 && mx > 0.f && isfinite(mx)) atomicMax(mbits, __float_as_uint(mx));
}

__global__ void k_seed_scale(const uint32_t* __restrict__ mbits, float* __restrict__ scale) {
    const float m = __uint_as_float(*mbits);
    float sc = 1.0f;
    if (m > 0.f) {
        int e;
        frexpf(m, &e);                   // m = f * 2^e, f in [0.5, 1)
        sc = scalbnf(1.0f, max(-100, min(100, 26 - e)));
    }
    *scale = sc;
}

// grid_grad += (carry * 2^32 + lo) / scale; lo = carry = 0 for the next step
__global__ void __launch_bounds__(256)
k_igrad_to_f32(int64_t n, int32_t* __restrict__ lo, int32_t* __restrict__ carry,
               const float* __restrict__ scale, float* __restrict__ grad) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = ((double)carry[i] * 4294967296.0 + (double)lo[i]) / (double)*scale;
    grad[i] += (float)v;
    lo[i] = 0;
    carry[i] = 0;
}

// Exact per-level sum of the int32 entries (int64), for the net-wrap check,
// and the level's largest |entry| in gradient units (the next step's scale
// keeps it in range): from the int32 entries of a fixed-point level, from
// grid_grad for a level that went in as fp32 this step (the first step; an
// upper bound when the caller accumulates several steps into grid_grad).
__global__ void __launch_bounds__(256)
k_fx_esum(GridMeta gm, const float* __restrict__ scale, const int32_t* __restrict__ acc,
          const float* __restrict__ grad, FxStats* __restrict__ st) {
    const int l = blockIdx.y;
    const float sc = scale[l];
    typedef int vi4 __attribute__((ext_vector_type(4)));
    const int64_t e0 = 2 * (int64_t)gm.offset[l], n4 = (2 * (int64_t)gm.hsize[l]) >> 2;
    int64_t s = 0;
    uint64_t ws = 0;                 // sum of entry * fx_weight(element), mod 2^64
    uint32_t mx = 0u;           // fixed point: |int|; fp32 level: |float| bits
    auto uabs = [](int x) { return x < 0 ? 0u - (uint32_t)x : (uint32_t)x; };
    if (sc != 0.f) {
        const vi4* a4 = reinterpret_cast<const vi4*>(acc + e0);
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
             i += (int64_t)gridDim.x * blockDim.x) {
            const vi4 v = __builtin_nontemporal_load(a4 + i);
            s += (int64_t)v.x + v.y + v.z + v.w;
            const uint32_t el = (uint32_t)(e0 + 4 * i);
            ws += (uint64_t)((int64_t)v.x * (int64_t)fx_weight(el)) +
                  (uint64_t)((int64_t)v.y * (int64_t)fx_weight(el + 1)) +
                  (uint64_t)((int64_t)v.z * (int64_t)fx_weight(el + 2)) +
                  (uint64_t)((int64_t)v.w * (int64_t)fx_weight(el + 3));
            mx = max(max(mx, max(uabs(v.x), uabs(v.y))), max(uabs(v.z), uabs(v.w)));
        }
    } else {
        const vi4* g4 = reinterpret_cast<const vi4*>(grad + e0);
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
             i += (int64_t)gridDim.x * blockDim.x) {
            const vi4 v = __builtin_nontemporal_load(g4 + i);
            mx = max(max(mx, max((uint32_t)v.x & 0x7fffffffu, (uint32_t)v.y & 0x7fffffffu)),
                     max((uint32_t)v.z & 0x7fffffffu, (uint32_t)v.w & 0x7fffffffu));
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        s += __shfl_xor(s, off);
        ws += __shfl_xor(ws, off);
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, off));
    }
    // one atomic per block (per-wave atomics on the level words serialised:
    // 107 us for 16k of them)
    __shared__ int64_t sW[4];
    __shared__ uint64_t sWw[4];
    __shared__ uint32_t sM[4];
    const int w = threadIdx.x / RN_WAVE;
    if (rn_lane() == 0) { sW[w] = s; sWw[w] = ws; sM[w] = mx; }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int64_t t = (sW[0] + sW[1]) + (sW[2] + sW[3]);
        const uint64_t tw = (sWw[0] + sWw[1]) + (sWw[2] + sWw[3]);
        if (tw != 0) atomicAdd(reinterpret_cast<unsigned long long*>(st->we + l), tw);
        uint32_t m = max(max(sM[0], sM[1]), max(sM[2], sM[3]));
        if (sc != 0.f) m = __float_as_uint((float)m / sc);     // units -> gradient units
        if (t != 0) atomicAdd(reinterpret_cast<unsigned long long*>(st->esum + l), (unsigned long long)t);
        if (m != 0u && m < 0x7f800000u) atomicMax(st->emax + l, m);
    }
}

// Fixed-point step bookkeeping (one wave): redo flag of this step, the next
// step's per-level scales from this step's largest records, statistics reset.
// Scale 2^(FX_TARGET_BITS - e) with |record| < 2^e: the largest record maps
// to < 2^27 units.  A level whose largest record reached 2^30 units under the
// current scale (8x growth since the step the scale came from), or a
// non-finite one, or whose entries wrapped (entry sum != record sum), sets the
// redo flag: rn_grid_fx_fold then discards the fixed-point sums and the GM 3
// launch recomputes the grid gradient in fp32.
// Headroom measured on C3 over 12 Adam steps (tools/fx_diag.py): the largest
// |entry| of a hashed level stays within 2^1.2 of its largest record, so at
// 2^27 units it sits ~2^3 below the int32 range.  A dense (coarse) level's
// entry sums up to hundreds of records, so its scale is also capped by this
// step's largest |entry|: it maps to < 2^29 units (2^2 of headroom for growth;
// the first step's entries are read from the fp32 grid_grad); a dense level
// with no entry measured maps its largest record to < 2^14 units.
// Why these units (round 6; tools/fx_units_probe.py,
// profiles/r06/fxunits/): FusedAdam's eps 1e-15 turns any non-zero gradient
// into an lr-sized step, so an entry below half a unit (flushed to 0) moves
// the update as much as a wrong sign.  C3, 3 Adam steps, largest per-level
// update difference from fp32 (fp32 with the rays reversed: <= 0.07 %):
// 2048 rays 2.66 % at (23, 28, 28) -> 1.14 % at (27, 29, 30); 8192 rays 1.02
// -> 0.38 %; flushed entries 0.031 -> 0.005 %; no step redone in 1,150
// probe and training steps; 1000 training steps end within 0.03 dB of fp32
// either way.  (26, 30, 30) redid one of 1000 training steps (entry cap too
// close to 2^31).
#ifndef FX_TARGET_BITS              // (-D overrides: unit studies, tools/fx_units_probe.py)
#define FX_TARGET_BITS 27
#endif
#ifndef FX_ENTRY_BITS
#define FX_ENTRY_BITS 29
#endif
#define FX_DENSE_FIRST_BITS 14
#ifndef FX_GROWTH_BITS
#define FX_GROWTH_BITS 30
#endif
#define FX_GROWTH_UNITS ((float)(1u << FX_GROWTH_BITS))   // 2^30
// Binned mode (ctl != NULL, rn_grid_binned_fold): records are e5m17 (rn_bin.h),
// summed exactly in int64, so there is no entry cap and no wrap check; the
// largest record maps to < 2^GB_TARGET_BITS = 2^38 units (256x headroom below
// 2^46, the first value e5m17 cannot hold: a record that reaches it sets the
// redo flag -- the bar is exact, every record below it is representable), and
// so does a pool overflow (the walk ran out of pages) or a fault word the bin
// pass set (inputs out of range).
__global__ void __launch_bounds__(64)
k_fx_check(uint32_t hashed_mask, const float* __restrict__ scale_cur,
           float* __restrict__ scale_next, FxStats* __restrict__ stats,
           int32_t* __restrict__ redo, const GbCtl* __restrict__ ctl, uint32_t pool_pages) {
    const int l = threadIdx.x;
    uint32_t* vmax = stats->vmax;
    const bool binned = ctl != nullptr;
    // pool overflow, or inputs the bin pass refused (GbCtl::fault)
    bool bad = binned && l == 0 && (ctl->pool_next > pool_pages || ctl->fault != 0u);
    const float growth = binned ? GB_GROWTH_UNITS : FX_GROWTH_UNITS;
    if (l < RN_L) {
        // net wrap of an int32 entry: the entries' exact sum differs from the
        // records' exact sum (by a multiple of 2^32)
        // (and the position-weighted sums: opposite wraps cancel only in the plain one)
        if (!binned && scale_cur[l] != 0.f &&
            (stats->esum[l] != stats->qsum[l] || stats->we[l] != stats->wq[l]))
            bad = true;
        stats->esum[l] = 0;
        stats->qsum[l] = 0;
        stats->we[l] = 0;
        stats->wq[l] = 0;
        const uint32_t vb = vmax[l];
        const float sc = scale_cur[l];
        const uint32_t em = stats->emax[l];
        float nx = sc;                                   // no records this step: keep
        if (vb >= 0x7f800000u) {                         // inf / NaN record
            nx = 0.f;
            bad = bad || sc != 0.f;
        } else if (vb != 0u) {
            const float v = __uint_as_float(vb);
            bad = bad || (sc != 0.f && v * sc >= growth);
            int e;
            frexpf(v, &e);                               // v < 2^e
            int bits = (binned ? GB_TARGET_BITS : FX_TARGET_BITS) - e;
            if (binned) {
                // int64 sums: no entry cap
            } else if (em != 0u) {                       // the largest entry stays < 2^29 units
                int ee;
                frexpf(__uint_as_float(em), &ee);
                bits = min(bits, FX_ENTRY_BITS - ee);
            } else if (!((hashed_mask >> l) & 1u)) {     // dense level, no entry measured
                bits = FX_DENSE_FIRST_BITS - e;
            }
            nx = scalbnf(1.0f, max(-126, min(126, bits)));
        }
        scale_next[l] = nx;
        vmax[l] = 0u;
        stats->emax[l] = 0u;
    }
    const uint64_t b = __builtin_amdgcn_ballot_w64(bad);
    if (l == 0) *redo = b ? 1 : 0;
}

// grid_grad += acc * 2^-e_l over the fixed-point levels' entries (elements
// [e0, e1), 16-B aligned), acc = 0; with the redo flag set the sums are only
// cleared (the fp32 redo adds the step's gradient instead).
__global__ void __launch_bounds__(256)
k_fx_fold(int64_t e0, int64_t e1, GridMeta gm, const float* __restrict__ scale,
          int32_t* __restrict__ acc, float* __restrict__ grad, const int32_t* __restrict__ redo) {
    __shared__ uint32_t sOff[RN_L];
    __shared__ float sInv[RN_L];
    if (threadIdx.x < RN_L) {
        sOff[threadIdx.x] = gm.offset[threadIdx.x];
        const float sc = scale[threadIdx.x];
        sInv[threadIdx.x] = sc != 0.f ? 1.0f / sc : 0.f;     // exact: powers of two
    }
    __syncthreads();
    const bool discard = *redo != 0;
    const int64_t n4 = (e1 - e0) >> 2;
    typedef int vi4 __attribute__((ext_vector_type(4)));
    vi4* a4 = reinterpret_cast<vi4*>(acc + e0);
    float4* g4 = reinterpret_cast<float4*>(grad + e0);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * blockDim.x) {
        const vi4 v = __builtin_nontemporal_load(a4 + i);
        if ((v.x | v.y | v.z | v.w) == 0) continue;
        __builtin_nontemporal_store(vi4{0, 0, 0, 0}, a4 + i);
        if (discard) continue;
        const uint32_t ent = (uint32_t)((e0 + 4 * i) >> 1);
        int l = 0;
#pragma unroll
        for (int k = 1; k < RN_L; ++k) l = ent >= sOff[k] ? k : l;
        const float inv = sInv[l];
        float4 g = g4[i];
        g.x += (float)v.x * inv; g.y += (float)v.y * inv;
        g.z += (float)v.z * inv; g.w += (float)v.w * inv;
        g4[i] = g;
    }
}

// Merged order of the K models' samples per ray (ray-major, then t, ties by
// model): perm[mstart[r] + rank] = sample.  One wave per ray; each sample's
// rank = its index in its (model, ray) run + the samples of the other models
// of the ray that precede it (binary search; t increases along a run).  The
// ray's K runs are staged in the wave's LDS slice when they fit (always for
// K = 2), so the searches are LDS reads instead of dependent global loads.
#define PLAN_WAVES 4
#define PLAN_LDS 2048      // floats per wave

// Stage one ray's K runs of t (and, with ids, each sample's position in the
// concatenation) into the wave's LDS slice: position i of the concatenated
// runs [bnd[k], bnd[k+1]) is sample off[k] + i - bnd[k].  Positions are dealt
// over the lanes with PLAN_UNR loads in flight per lane (a loop per run, one
// load then its store, waited for each load: 16 round trips per ray at K = 8,
// and k_bwd_plan_multi took 0.139 ms at C5).  bnd / off are wave-uniform.
#define PLAN_UNR 8

// The level-partitioned forward's per-position input (k_enc_prep's float4:
// unit coordinates, sample id), written by the plan as it places each sample
// (rn_bwd_plan with `prep`): the plan has the sample's t in LDS and its ray,
// so the separate pass that re-read perm, ts and the ray (C3 0.03 ms) goes.
// Arithmetic as load_sample<1> + unit_coord (bit-identical).
struct PlanPrep {
    float4* prep;             // null: the plan writes perm only
    const float* rays_o; const float* rays_d;
    float mn[3], ext[3];
    // 1 / extent when every extent is a power of two (scale 0.5: 1, scale 16:
    // 32): x / ext and x * (1 / ext) are then the same float, and the three
    // IEEE divisions per sample leave the merge's serial chain; 0 otherwise
    float inv[3];
};
struct RayPos { float o[3], d[3]; };
__device__ __forceinline__ RayPos plan_ray(const PlanPrep& P, int r) {
    RayPos q;
#pragma unroll
    for (int c = 0; c < 3; ++c) { q.o[c] = P.rays_o[3 * r + c]; q.d[c] = P.rays_d[3 * r + c]; }
    return q;
}
__device__ __forceinline__ void plan_prep_write(const PlanPrep& P, const RayPos& q, int pos,
                                                float t, int s) {
    const float x = fmaf(t, q.d[0], q.o[0]), y = fmaf(t, q.d[1], q.o[1]), z = fmaf(t, q.d[2], q.o[2]);
    auto u = [&](float v, int c) {
        return P.inv[0] != 0.f ? fminf(fmaxf((v - P.mn[c]) * P.inv[c], 0.0f), 1.0f)
                               : unit_coord(v, P.mn[c], P.ext[c]);
    };
    P.prep[pos] = make_float4(u(x, 0), u(y, 1), u(z, 2), __int_as_float(s));
}

// Ray r's run of each model (count, first sample) and its merged start ms.
// r is wave-uniform (the wave id read back as a scalar), and every model's
// words load unconditionally (index clamped to K - 1, zeroed after): scalar
// loads issued together.  (With the wave id a vector value and each load
// under k < K, the 2K counts / offsets became vector loads waited for one by
// one: ~16 round trips per ray at K = 8.)
__device__ __forceinline__ void plan_ray_runs(int K, int B, int r, const int32_t* __restrict__ counts,
                                              const int32_t* __restrict__ offsets,
                                              const int32_t* __restrict__ seg_base, int* cnt,
                                              int* off, int& ms) {
    int c[MB_KMAX], o[MB_KMAX], sb[MB_KMAX];
#pragma unroll
    for (int k = 0; k < MB_KMAX; ++k) {
        const int kk = k < K ? k : K - 1;
        c[k] = counts[kk * B + r]; o[k] = offsets[kk * B + r]; sb[k] = seg_base[kk];
    }
    ms = 0;
#pragma unroll
    for (int k = 0; k < MB_KMAX; ++k) {
        cnt[k] = k < K ? c[k] : 0;
        off[k] = k < K ? o[k] : 0;
        ms += k < K ? o[k] - sb[k] : 0;
    }
}
__device__ __forceinline__ void plan_stage(int K, int tot_r, const int* bnd, const int* off,
                                           const float* __restrict__ ts, float* st, uint16_t* si) {
    const int lane = rn_lane();
    for (int i0 = 0; i0 < tot_r; i0 += RN_WAVE * PLAN_UNR) {
        float v[PLAN_UNR];
#pragma unroll
        for (int u = 0; u < PLAN_UNR; ++u) {
            const int i = i0 + u * RN_WAVE + lane;
            int base = off[0];                    // off[k] - bnd[k] of i's run (bnd[0] = 0)
#pragma unroll
            for (int kq = 1; kq < MB_KMAX; ++kq)
                base = (kq < K && i >= bnd[kq]) ? off[kq] - bnd[kq] : base;
            v[u] = i < tot_r ? ts[base + i] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < PLAN_UNR; ++u) {
            const int i = i0 + u * RN_WAVE + lane;
            if (i < tot_r) {
                st[i] = v[u];
                if (si) si[i] = (uint16_t)i;
            }
        }
    }
}

__global__ void __launch_bounds__(PLAN_WAVES * 64)
k_bwd_plan(int B, int K, const int32_t* __restrict__ counts, const int32_t* __restrict__ offsets,
           const int32_t* __restrict__ seg_base, const int32_t* __restrict__ seg_count,
           const float* __restrict__ ts, int32_t* __restrict__ mstart, int32_t* __restrict__ perm,
           PlanPrep P) {
    __shared__ float sT[PLAN_WAVES][PLAN_LDS];
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / RN_WAVE);
    const int r = blockIdx.x * PLAN_WAVES + wid;
    if (r >= B) return;                      // wave-uniform; no block barrier below
    const int lane = rn_lane();
    int ms = 0, tot_r = 0;
    int cnt[MB_KMAX], off[MB_KMAX], loc[MB_KMAX];
    plan_ray_runs(K, B, r, counts, offsets, seg_base, cnt, off, ms);
#pragma unroll
    for (int k = 0; k < MB_KMAX; ++k) { loc[k] = tot_r; tot_r += cnt[k]; }
    if (lane == 0) {
        mstart[r] = ms;
        if (r == 0) {
            int tot = 0;
            for (int k = 0; k < K; ++k) tot += seg_count[k];
            mstart[B] = tot;
        }
    }
    const bool staged = tot_r <= PLAN_LDS;
    float* st = sT[wid];
    const RayPos rq = P.prep ? plan_ray(P, r) : RayPos{};
    if (staged) {
        plan_stage(K, tot_r, loc, off, ts, st, nullptr);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
    if (K == 2 && staged) {
        // merge path: lane j emits merged positions [j L, (j+1) L); it finds
        // how many of them come from model 0 by a binary search on its
        // diagonal (model 0 first on equal t, as below), then merges serially
        // -- ~log2(n) + L dependent LDS reads per lane instead of a search
        // per sample (C3: 0.064 -> 0.040 ms with k_bwd_chunks)
        const float* A = st + loc[0];
        const float* Bv = st + loc[1];
        const int nA = cnt[0], nB = cnt[1], n = nA + nB;
        const int L = (n + RN_WAVE - 1) / RN_WAVE;
        const int d = min(lane * L, n);
        int lo = max(0, d - nB), hi = min(d, nA);
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (A[mid] <= Bv[d - 1 - mid]) lo = mid + 1; else hi = mid;
        }
        int a = lo, b = d - lo;
        const int e = min(d + L, n);
        for (int q = d; q < e; ++q) {
            const bool takeA = a < nA && (b >= nB || A[a] <= Bv[b]);
            const int smp = takeA ? off[0] + a : off[1] + b;
            perm[ms + q] = smp;
            if (P.prep) plan_prep_write(P, rq, ms + q, takeA ? A[a] : Bv[b], smp);
            a += takeA ? 1 : 0;
            b += takeA ? 0 : 1;
        }
        return;
    }
    for (int k = 0; k < K; ++k) {
        for (int i = lane; i < cnt[k]; i += RN_WAVE) {
            const float t = staged ? st[loc[k] + i] : ts[off[k] + i];
            int pos = i;
            for (int k2 = 0; k2 < K; ++k2) {
                if (k2 == k) continue;
                int lo = 0, hi = cnt[k2];        // count of t2 < t (k2 > k) or t2 <= t (k2 < k)
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    const float t2 = staged ? st[loc[k2] + mid] : ts[off[k2] + mid];
                    if (t2 < t || (k2 < k && t2 == t)) lo = mid + 1; else hi = mid;
                }
                pos += lo;
            }
            perm[ms + pos] = off[k] + i;
            if (P.prep) plan_prep_write(P, rq, ms + pos, t, off[k] + i);
        }
    }
}

// The same merged order for K > 2 by a merge tree in LDS: the ray's K runs
// (staged with their sample indices) are merged pairwise, log2(K) levels; each
// pair is merged by the whole wave with merge path (lane j: a diagonal binary
// search, then L serial steps).  Runs are merged in model order and the left
// run wins ties, so the result is ordered by (t, model) like k_bwd_plan's
// ranks.  ~log2(n) + n/64 dependent LDS reads per lane and level instead of
// (K-1) binary searches per sample (C5: K = 8, ~760 samples per ray).
#define PLANM_WAVES 2
#define PLANM_LDS 2048     // samples per wave

// Sample ids in LDS are u16 positions in the ray's staged runs (model k's run
// starts at kb[k]); the last level maps them to global sample indices
// (ko[k] + id - kb[k]).  u16 ids take a block to 48 KB of LDS: 3 blocks (6
// waves) per CU instead of 2, for a latency-bound merge.
__device__ __forceinline__ void merge_pair_wave(const float* tA, const uint16_t* iA, int nA,
                                                const float* tB, const uint16_t* iB, int nB,
                                                float* to, uint16_t* io, int32_t* gout,
                                                const int* kb, const int* ko, int K,
                                                const PlanPrep& P, const RayPos& rq, int gpos) {
    const int lane = rn_lane();
    const int n = nA + nB;
    const int L = (n + RN_WAVE - 1) / RN_WAVE;
    const int d = min(lane * L, n);
    int lo = max(0, d - nB), hi = min(d, nA);
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (tA[mid] <= tB[d - 1 - mid]) lo = mid + 1; else hi = mid;
    }
    int a = lo, b = d - lo;
    const int e = min(d + L, n);
    for (int q = d; q < e; ++q) {
        // both heads' t and ids read together (one LDS round trip per step;
        // as selects of the addresses, the compare, the id and the output t
        // were three).  a = nA / b = nB read one past their run, inside the
        // wave's slice, and are not used
        const float ta = tA[a], tb = tB[b];
        const int ja = iA[a], jb = iB[b];
        const bool takeA = a < nA && (b >= nB || ta <= tb);
        const int idx = takeA ? ja : jb;
        if (gout) {
            int base = ko[0];
#pragma unroll
            for (int j = 1; j < MB_KMAX; ++j)
                if (j < K && idx >= kb[j]) base = ko[j] - kb[j];
            gout[q] = base + idx;
            if (P.prep) plan_prep_write(P, rq, gpos + q, takeA ? ta : tb, base + idx);
        } else {
            to[q] = takeA ? ta : tb;
            io[q] = (uint16_t)idx;
        }
        a += takeA ? 1 : 0;
        b += takeA ? 0 : 1;
    }
}

__global__ void __launch_bounds__(PLANM_WAVES * 64)
k_bwd_plan_multi(int B, int K, const int32_t* __restrict__ counts,
                 const int32_t* __restrict__ offsets, const int32_t* __restrict__ seg_base,
                 const int32_t* __restrict__ seg_count, const float* __restrict__ ts,
                 int32_t* __restrict__ mstart, int32_t* __restrict__ perm, PlanPrep P) {
    // (+2: a merge step reads one past the last run)
    __shared__ float sT[PLANM_WAVES][2][PLANM_LDS + 2];
    __shared__ uint16_t sI[PLANM_WAVES][2][PLANM_LDS + 2];
    static_assert(PLANM_LDS <= 65536, "u16 sample ids");
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / RN_WAVE);
    const int r = blockIdx.x * PLANM_WAVES + wid;
    if (r >= B) return;                      // wave-uniform; no block barrier below
    const int lane = rn_lane();
    int ms = 0, tot_r = 0;
    int bnd[MB_KMAX + 1], off[MB_KMAX], cnt[MB_KMAX];
    plan_ray_runs(K, B, r, counts, offsets, seg_base, cnt, off, ms);
#pragma unroll
    for (int k = 0; k < MB_KMAX; ++k) { bnd[k] = tot_r; tot_r += cnt[k]; }
    bnd[MB_KMAX] = tot_r;
    const RayPos rq = P.prep ? plan_ray(P, r) : RayPos{};
    if (lane == 0) {
        mstart[r] = ms;
        if (r == 0) {
            int tot = 0;
            for (int k = 0; k < K; ++k) tot += seg_count[k];
            mstart[B] = tot;
        }
    }
    if (tot_r > PLANM_LDS) {
        // (rays longer than the LDS slice: rank by binary searches in global memory)
        for (int k = 0; k < K; ++k) {
            const int ck = bnd[k + 1] - bnd[k];
            for (int i = lane; i < ck; i += RN_WAVE) {
                const float t = ts[off[k] + i];
                int pos = i;
                for (int k2 = 0; k2 < K; ++k2) {
                    if (k2 == k) continue;
                    int lo = 0, hi = bnd[k2 + 1] - bnd[k2];
                    while (lo < hi) {
                        const int mid = (lo + hi) >> 1;
                        const float t2 = ts[off[k2] + mid];
                        if (t2 < t || (k2 < k && t2 == t)) lo = mid + 1; else hi = mid;
                    }
                    pos += lo;
                }
                perm[ms + pos] = off[k] + i;
                if (P.prep) plan_prep_write(P, rq, ms + pos, t, off[k] + i);
            }
        }
        return;
    }
    int cur = 0;
    int kb[MB_KMAX];                          // the models' runs (bnd is merged below)
#pragma unroll
    for (int k = 0; k < MB_KMAX; ++k) kb[k] = k < K ? bnd[k] : 0;
    plan_stage(K, tot_r, bnd, off, ts, sT[wid][0], sI[wid][0]);
    int nr = K;
    while (true) {
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        const bool last = nr <= 2;
        const float* ts_ = sT[wid][cur];
        const uint16_t* is_ = sI[wid][cur];
        for (int p = 0; 2 * p < nr; ++p) {
            const int a0 = bnd[2 * p], a1 = bnd[min(2 * p + 1, nr)], b1 = bnd[min(2 * p + 2, nr)];
            merge_pair_wave(ts_ + a0, is_ + a0, a1 - a0, ts_ + a1, is_ + a1, b1 - a1,
                            sT[wid][cur ^ 1] + a0, sI[wid][cur ^ 1] + a0,
                            nullptr, kb, off, K, P, rq, ms + a0);
        }
        if (last) {
            // the merged order is in LDS like every level's: perm (and the
            // level forward's input) go out in position order, coalesced and
            // off the merge's serial chain (written from inside it, each
            // lane's stores were L positions apart)
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            const float* to = sT[wid][cur ^ 1];
            const uint16_t* io = sI[wid][cur ^ 1];
            for (int q = lane; q < tot_r; q += RN_WAVE) {
                const int idx = io[q];
                int base = off[0];
#pragma unroll
                for (int jk = 1; jk < MB_KMAX; ++jk)
                    if (jk < K && idx >= kb[jk]) base = off[jk] - kb[jk];
                perm[ms + q] = base + idx;
                if (P.prep) plan_prep_write(P, rq, ms + q, to[q], base + idx);
            }
            return;
        }
        // runs after this level: boundaries of the merged pairs
        const int nn = (nr + 1) / 2;
        for (int p = 0; p < nn; ++p) bnd[p] = bnd[2 * p];
        bnd[nn] = bnd[nr];
        nr = nn;
        cur ^= 1;
    }
}

// Chunk schedule of the merged backward over the merged positions [0, total):
// big chunks for the first 15/16 of the work, then chunks of min_chunk (a short
// tail: blocks finish together).  With `blocks` > 0 the big chunks are a
// multiple of the persistent blocks in number, each <= max_chunk positions
// (size ceil(main / (blocks m)), m = ceil(main / (blocks max_chunk))): every
// block takes m of them.  A count just past a multiple (C4 at 2560: 534 big
// chunks for 256 blocks) left a few blocks one big chunk behind the rest, a
// tail the min_chunk phase was too small to hide (C4 485 vs 523 M samples/s
// at 2560 vs 3072).  Chunk c holds the rays whose merged start lies in
// [bound(c), bound(c+1)), so it is whole rays of at most max_chunk + K *
// max_samples samples (possibly none).
struct ChunkPlan {
    int head_n, head, max_chunk, min_chunk, c1, n;
    // first merged position of head chunk c (c <= head_n): head chunk c holds
    // ~head (c + 1) / head_n positions, a ramp from ~0 to head
    __host__ __device__ int hbound(int c) const {
        return head_n > 0 ? (int)(((int64_t)head * c * (c + 1)) / (2 * (int64_t)head_n)) : 0;
    }
    __host__ __device__ int bound(int c) const {
        const int H = hbound(head_n);
        if (c < head_n) return hbound(c);
        if (c <= c1) return H + (c - head_n) * max_chunk;
        return H + (c1 - head_n) * max_chunk + (c - c1) * min_chunk;
    }
};

// head_n chunks ramping from ~0 to `head` samples first (one per block): the
// blocks' first MLP phases end at staggered times, so the walks' requests
// reach the memory-side atomic units spread out instead of all at once after
// one full chunk's MLP phase, and the blocks stay out of phase after.  A ramp
// to max_chunk: C3 1183.4 -> 1189.2 M samples/s (field_bwd 2.995 -> 2.973
// ms), C2 853.7 -> 862.3; head chunks of one size (rounds 2 and 5) changed
// nothing, and at scale 16 a ramp to max_chunk / 2 lost 2-5 % (the big chunks,
// only ~2 per block there, get shorter); profiles/r06/headramp/.  Then
// max_chunk up to 15/16 of the work, then min_chunk (round 6: a tail of 1/16
// instead of 1/8, with its chunks sized by shape on the host: C3 1191 -> 1194,
// C4 653 -> 658, C5 789 -> 791; no tail at all lost 1 %; profiles/r06/tail/)
__host__ __device__ __forceinline__ ChunkPlan chunk_plan(int total, int head_n, int head,
                                                         int max_chunk, int min_chunk, int blocks) {
    ChunkPlan p;
    p.head = head; p.max_chunk = max_chunk; p.min_chunk = min_chunk;
#ifndef RN_TAIL_SHIFT              // (timing studies: -D overrides the tail's share, 2^-shift)
#define RN_TAIL_SHIFT 4
#endif
    const int main_end = total - (RN_TAIL_SHIFT < 31 ? total >> RN_TAIL_SHIFT : 0);
    // the ramp takes ~head (head_n + 1) / 2 positions: none if that is past the main part
    p.head_n = head > 0 && (int64_t)head * (head_n + 1) / 2 <= main_end ? head_n : 0;
    const int H = p.hbound(p.head_n);
    if (blocks > 0 && main_end > H) {
        const int64_t main = main_end - H, per = (int64_t)blocks * max_chunk;
        const int64_t m = (main + per - 1) / per;
        const int64_t sz = (main + (int64_t)blocks * m - 1) / ((int64_t)blocks * m);
        p.max_chunk = (int)(sz < min_chunk ? min_chunk : (sz > max_chunk ? max_chunk : sz));
    }
    p.c1 = p.head_n + (main_end > H ? (main_end - H) / p.max_chunk : 0);
    const int rest = total - p.bound(p.c1);
    p.n = p.c1 + (rest > 0 ? (rest + min_chunk - 1) / min_chunk : 0);
    return p;
}

__global__ void __launch_bounds__(256)
k_bwd_chunks(int B, int K, const int32_t* __restrict__ mstart,
             const int32_t* __restrict__ offsets, const int32_t* __restrict__ seg_base,
             const int32_t* __restrict__ seg_count, int head_n, int head, int max_chunk,
             int min_chunk, int blocks, int cap_chunks, int32_t* __restrict__ chunk_first,
             int32_t* __restrict__ desc, int32_t* __restrict__ queue) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    const int total = mstart[B];
    const ChunkPlan p = chunk_plan(total, head_n, head, max_chunk, min_chunk, blocks);
    const int n = min(p.n, cap_chunks);
    if (c == 0) { queue[0] = 0; queue[1] = n; queue[2] = 0; }
    if (c > n) return;
    if (c == n) { chunk_first[c] = B; return; }
    // first ray with mstart >= bound, for this chunk and the next
    int first[2];
    for (int e = 0; e < 2; ++e) {
        if (c + e == n) { first[e] = B; continue; }
        const int bound = p.bound(c + e);
        int lo = 0, hi = B;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (mstart[mid] < bound) lo = mid + 1; else hi = mid;
        }
        first[e] = lo;
    }
    chunk_first[c] = first[0];
    // descriptor: the chunk's sample range per model (the blocks read it with
    // one 80-B load per ticket)
    int32_t* d = desc + (size_t)c * CH_DESC;
    const int r0 = first[0], r1 = first[1];
    d[0] = r0; d[1] = r1; d[2] = 0; d[3] = 0;
    for (int k = 0; k < MB_KMAX; ++k) {
        int a0 = 0, cnt = 0;
        if (k < K && r0 < B) {
            a0 = offsets[k * B + r0];
            const int a1 = r1 < B ? offsets[k * B + r1] : seg_base[k] + seg_count[k];
            cnt = a1 - a0;
        }
        d[4 + k] = a0; d[4 + MB_KMAX + k] = cnt;
    }
}

// dst[k][i] = idx[i] >= 0 ? f16(src[k][idx[i]]) : 0
__global__ void __launch_bounds__(256)
k_pack_f16(int64_t n, int K, int64_t src_stride, int64_t dst_stride, const float* __restrict__ src,
           const int32_t* __restrict__ idx, rn_half* __restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int k = blockIdx.y;
    const int32_t j = idx[i];
    dst[k * dst_stride + i] = j >= 0 ? (rn_half)src[k * src_stride + j] : (rn_half)0.f;
}

__global__ void __launch_bounds__(256)
k_to_f16(int64_t n, const float* __restrict__ src, rn_half* __restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    dst[i] = (rn_half)src[i];
}

inline int nblk(int64_t n, int t) { return (int)((n + t - 1) / t); }

}  // namespace

extern "C" {

void rn_set_debug_flags(int flags) { g_field_dbg = flags; }
}  // extern "C"
int rn_debug_flags_internal() { return rn_dbg(g_field_dbg); }   // 0 in librn.so
extern "C" {

int rn_set_level_pairing(uint64_t pairing) {
    if (pairing != 0) {
        uint32_t seen = 0;
        for (int i = 0; i < 16; ++i) seen |= 1u << ((pairing >> (4 * i)) & 15u);
        RN_CHECK_ARG(seen == 0xffffu, "pairing: every level exactly once");
    }
    g_level_pairing = pairing;
    return 0;
}

/* ablation builds: read and clear the per-phase cycle counters (8 x u64) */
int rn_debug_cycles(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rn_cyc), sizeof(unsigned long long) * 8, 0,
                            hipMemcpyDeviceToHost) != hipSuccess)
        return 2;
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_rn_cyc), z, sizeof(z), 0, hipMemcpyHostToDevice) != hipSuccess)
        return 2;
    return 0;
}

int rn_pack_f16(const float* src, int64_t src_stride, const int32_t* index, int64_t n,
                int32_t n_models, int64_t dst_stride, void* dst, void* stream) {
    RN_CHECK_ARG(n >= 0 && n_models >= 1, "bad sizes");
    if (n == 0) return 0;
    RN_CHECK_ARG(src && index && dst, "null pointer");
    dim3 grid(nblk(n, 256), n_models);
    k_pack_f16<<<grid, 256, 0, (hipStream_t)stream>>>(n, n_models, src_stride, dst_stride, src,
                                                       index, (rn_half*)dst);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_to_f16(const float* src, int64_t n, void* dst, void* stream) {
    RN_CHECK_ARG(n >= 0, "bad size");
    if (n == 0) return 0;
    RN_CHECK_ARG(src && dst, "null pointer");
    k_to_f16<<<nblk(n, 256), 256, 0, (hipStream_t)stream>>>(n, src, (rn_half*)dst);
    RN_CHECK_LAUNCH();
    return 0;
}

// hash-grid level table (offsets/hsize/res/scale: 16 entries each)
int rn_field_fwd(const float* xyzs, const float* dirs, int64_t n_samples, const float* ts,
                 const int32_t* ray_of, const float* rays_o, const float* rays_d,
                 const int32_t* seg_base, const int32_t* seg_count, int32_t n_models,
                 const void* grid_f16, const uint32_t* level_offset, const uint32_t* level_hsize,
                 const uint32_t* level_res, const float* level_scale, const float* xyz_min,
                 const float* extent, const void* frags, float* sigma, float* rgb,
                 void* feat_cache, int32_t blocks_per_model, void* stream) {
    RN_CHECK_ARG(n_models >= 1 && n_samples >= 0 && blocks_per_model >= 1, "bad sizes");
    RN_CHECK_ARG(grid_f16 && level_offset && level_hsize && level_res && level_scale && xyz_min &&
                 extent && frags && sigma && rgb, "null pointer");
    FieldArgs a{};
    fill_args(a, xyz_min, extent, level_offset, level_hsize, level_res, level_scale);
    a.grid = (const rn_half*)grid_f16; a.frags = (const rn_half*)frags;
    a.sigma = sigma; a.rgb = rgb; a.feat = (rn_half*)feat_cache;
    a.dbg = rn_dbg(g_field_dbg);
    dim3 grid(blocks_per_model, n_models);
    if (xyzs) {
        RN_CHECK_ARG(dirs && n_models == 1, "xyz mode needs dirs and a single model");
        if (n_samples == 0) return 0;
        a.xyzs = xyzs; a.dirs = dirs; a.n_fixed = n_samples;
        if (feat_cache) k_field_fwd<0, CACHE_WRITE><<<grid, 256, 0, (hipStream_t)stream>>>(a);
        else k_field_fwd<0, CACHE_NONE><<<grid, 256, 0, (hipStream_t)stream>>>(a);
    } else {
        RN_CHECK_ARG(ts && ray_of && rays_o && rays_d && seg_base && seg_count,
                     "compact mode needs ts/ray_of/rays/segments");
        a.ts = ts; a.ray_of = ray_of; a.rays_o = rays_o; a.rays_d = rays_d;
        a.seg_base = seg_base; a.seg_count = seg_count;
        if (feat_cache) k_field_fwd<1, CACHE_WRITE><<<grid, 256, 0, (hipStream_t)stream>>>(a);
        else k_field_fwd<1, CACHE_NONE><<<grid, 256, 0, (hipStream_t)stream>>>(a);
    }
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_field_bwd(const float* xyzs, const float* dirs, int64_t n_samples, const float* ts,
                 const int32_t* ray_of, const float* rays_o, const float* rays_d,
                 const int32_t* seg_base, const int32_t* seg_count, int32_t n_models,
                 const void* grid_f16, const uint32_t* level_offset, const uint32_t* level_hsize,
                 const uint32_t* level_res, const float* level_scale, const float* xyz_min,
                 const float* extent, const void* frags, const float* dL_dsigma,
                 const float* dL_drgb, float* grid_grad, float* dw, const void* feat_cache,
                 int32_t blocks_per_model, void* stream) {
    RN_CHECK_ARG(n_models >= 1 && n_samples >= 0 && blocks_per_model >= 1, "bad sizes");
    RN_CHECK_ARG(grid_f16 && level_offset && level_hsize && level_res && level_scale && xyz_min &&
                 extent && frags && dL_dsigma && dL_drgb && grid_grad && dw, "null pointer");
    FieldArgs a{};
    fill_args(a, xyz_min, extent, level_offset, level_hsize, level_res, level_scale);
    a.dbg = rn_dbg(g_field_dbg);
    a.grid = (const rn_half*)grid_f16; a.frags = (const rn_half*)frags;
    a.dsigma = dL_dsigma; a.drgb = dL_drgb; a.grid_grad = grid_grad; a.dw = dw;
    a.feat = (rn_half*)feat_cache;
    dim3 grid(blocks_per_model, n_models);
    if (xyzs) {
        RN_CHECK_ARG(dirs && n_models == 1, "xyz mode needs dirs and a single model");
        if (n_samples == 0) return 0;
        a.xyzs = xyzs; a.dirs = dirs; a.n_fixed = n_samples;
        if (feat_cache) k_field_bwd<0, CACHE_READ><<<grid, BWD_WAVES * 64, 0, (hipStream_t)stream>>>(a);
        else k_field_bwd<0, CACHE_NONE><<<grid, BWD_WAVES * 64, 0, (hipStream_t)stream>>>(a);
    } else {
        RN_CHECK_ARG(ts && ray_of && rays_o && rays_d && seg_base && seg_count,
                     "compact mode needs ts/ray_of/rays/segments");
        a.ts = ts; a.ray_of = ray_of; a.rays_o = rays_o; a.rays_d = rays_d;
        a.seg_base = seg_base; a.seg_count = seg_count;
        if (feat_cache) k_field_bwd<1, CACHE_READ><<<grid, BWD_WAVES * 64, 0, (hipStream_t)stream>>>(a);
        else k_field_bwd<1, CACHE_NONE><<<grid, BWD_WAVES * 64, 0, (hipStream_t)stream>>>(a);
    }
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_bwd_plan(const int32_t* counts, const int32_t* offsets, const int32_t* seg_base,
                const int32_t* seg_count, const float* ts, int64_t n_rays, int32_t n_models,
                int32_t head_chunks, int32_t head_size, int32_t max_chunk, int32_t min_chunk,
                int32_t balance_blocks, int32_t cap_chunks, int32_t* mstart, int32_t* perm,
                int32_t* chunk_first, int32_t* chunk_desc, int32_t* queue, const float* rays_o,
                const float* rays_d, const float* xyz_min, const float* extent, float* prep,
                void* stream) {
    RN_CHECK_ARG(n_rays >= 1 && n_models >= 1 && n_models <= MB_KMAX, "bad sizes");
    RN_CHECK_ARG(max_chunk >= min_chunk && min_chunk >= 1 && cap_chunks >= 1 && head_chunks >= 0 &&
                 head_size >= 0 && head_size <= max_chunk && balance_blocks >= 0,
                 "bad chunk sizes");
    RN_CHECK_ARG(counts && offsets && seg_base && seg_count && ts && mstart && perm &&
                 chunk_first && chunk_desc && queue, "null pointer");
    RN_CHECK_ARG(!prep || (rays_o && rays_d && xyz_min && extent), "null pointer (prep)");
    PlanPrep P{};
    P.prep = (float4*)prep; P.rays_o = rays_o; P.rays_d = rays_d;
    if (prep) {
        bool pow2 = true;
        for (int c = 0; c < 3; ++c) {
            P.mn[c] = xyz_min[c]; P.ext[c] = extent[c];
            int e;
            pow2 = pow2 && extent[c] > 0.f && std::frexp(extent[c], &e) == 0.5f &&
                   e > -120 && e < 120;
        }
        for (int c = 0; c < 3; ++c) P.inv[c] = pow2 ? 1.0f / extent[c] : 0.f;
    }
    if (n_models > 2)
        k_bwd_plan_multi<<<nblk(n_rays, PLANM_WAVES), PLANM_WAVES * 64, 0, (hipStream_t)stream>>>(
            (int)n_rays, n_models, counts, offsets, seg_base, seg_count, ts, mstart, perm, P);
    else
        k_bwd_plan<<<nblk(n_rays, PLAN_WAVES), PLAN_WAVES * 64, 0, (hipStream_t)stream>>>(
            (int)n_rays, n_models, counts, offsets, seg_base, seg_count, ts, mstart, perm, P);
    RN_CHECK_LAUNCH();
    k_bwd_chunks<<<nblk(cap_chunks + 1, 256), 256, 0, (hipStream_t)stream>>>(
        (int)n_rays, n_models, mstart, offsets, seg_base, seg_count, head_chunks, head_size,
        max_chunk, min_chunk, balance_blocks, cap_chunks, chunk_first, chunk_desc, queue);
    RN_CHECK_LAUNCH();
    return 0;
}

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
                        void* stream) {
    RN_CHECK_ARG(!igrad_lo || (igrad_carry && igrad_scale), "integer mode needs carry and scale");
    RN_CHECK_ARG(fx_mode == 0 || fx_mode == 2 || fx_mode == 3 || fx_mode == 4 || fx_mode == 5,
                 "fx_mode: 0, 2, 3, 4 or 5");
    const bool binned = fx_mode == 4 || fx_mode == 5;
    RN_CHECK_ARG(fx_mode != 2 || (fx_acc && fx_scale && fx_stats && feat_cache),
                 "fixed-point mode needs acc, scale, stats and the encoding cache");
    RN_CHECK_ARG(!binned || (fx_scale && fx_stats && feat_cache && gb_ctl && gb_page_meta &&
                                  gb_pages && gb_pool_pages >= 1),
                 "binned mode needs scale, stats, the encoding cache and the page pool");
    for (int l = 0; binned && l < RN_L; ++l)
        RN_CHECK_ARG(level_hsize[l] <= (1u << GB_IDX_BITS) &&
                     level_hsize[l] <= ((uint32_t)GB_MAX_BINS << GB_SLICE_BITS),
                     "binned mode: a level has more than 2^20 entries");
    RN_CHECK_ARG(fx_mode != 3 || (fx_redo && fx_scale && feat_cache),
                 "fixed-point redo needs the redo flag, the step's scales and the encoding cache");
    RN_CHECK_ARG(!(igrad_lo && fx_mode), "integer and fixed-point modes are exclusive");
    RN_CHECK_ARG(n_rays >= 1 && n_models >= 1 && n_models <= MB_KMAX && blocks >= 1 &&
                 max_samples >= 1 && max_chunk >= 1, "bad sizes");
    RN_CHECK_ARG(scratch_rows >= (int64_t)max_chunk + (int64_t)n_models * max_samples,
                 "scratch_rows must be >= max_chunk + n_models * max_samples");
    RN_CHECK_ARG(ts && ray_of && rays_o && rays_d && seg_base && seg_count && mstart &&
                 perm && chunk_desc && queue && grid_f16 && level_offset && level_hsize && level_res &&
                 level_scale && xyz_min && extent && frags && dL_dsigma && dL_drgb && grid_grad &&
                 dw && scratch && park, "null pointer");
    // fixed point: the wrap checksum's element weights 4 i (fx_weight) stay
    // injective and below 2^30 up to 2^28 elements
    RN_CHECK_ARG(fx_mode != 2 ||
                 2ull * ((uint64_t)level_offset[RN_L - 1] + level_hsize[RN_L - 1]) <= (1ull << 28),
                 "fixed-point mode: the grid has more than 2^28 gradient elements");
    FieldArgs a{};
    fill_args(a, xyz_min, extent, level_offset, level_hsize, level_res, level_scale);
    a.dbg = rn_dbg(g_field_dbg);
    a.grid = (const rn_half*)grid_f16; a.frags = (const rn_half*)frags;
    a.dsigma = dL_dsigma; a.drgb = dL_drgb; a.grid_grad = grid_grad; a.dw = dw;
    a.feat = (rn_half*)feat_cache;
    a.ts = ts; a.ray_of = ray_of; a.rays_o = rays_o; a.rays_d = rays_d;
    a.seg_base = seg_base; a.seg_count = seg_count;
    MergeArgs m{};
    m.mstart = mstart; m.perm = perm; m.desc = chunk_desc;
    m.queue = queue;
    m.scratch = scratch; m.park = park;
    m.n_rays = (int)n_rays; m.n_models = n_models; m.rows_cap = (int)scratch_rows;
    hipStream_t st = (hipStream_t)stream;
    // the ticket is reset per launch, so a backward can be re-run on one plan
    if (hipMemsetAsync(queue, 0, sizeof(int32_t), st) != hipSuccess) {
        rn_set_error("%s: ticket reset failed", __func__);
        return 2;
    }
    IntGrad G{};
    if (igrad_lo) {
        G.bytes = 2 * a.grid_bytes;            // int32 arrays, same size as the f32 grad
        G.lo_ptr = igrad_lo; G.carry_ptr = igrad_carry; G.scale_ptr = igrad_scale;
    }
    if (binned) {
        if (hipMemsetAsync(gb_ctl, 0, GB_CTL_RESET_BYTES, st) != hipSuccess) {
            rn_set_error("%s: page pool reset failed", __func__);
            return 2;
        }
        G.ctl = (GbCtl*)gb_ctl; G.page_meta = gb_page_meta; G.pages = gb_pages;
        G.pool_pages = (uint32_t)gb_pool_pages;
    }
    FxGrad F{};
    F.acc = fx_acc; F.scale = fx_scale; F.redo = fx_redo;
    if (fx_stats) {
        F.vmax = reinterpret_cast<FxStats*>(fx_stats)->vmax;
        F.qsum = reinterpret_cast<FxStats*>(fx_stats)->qsum;
        F.wq = reinterpret_cast<FxStats*>(fx_stats)->wq;
    }
    const dim3 blk(BWD_WAVES * 64);
    if constexpr (RN_ABL) {                     // timing studies (librn_abl.so only)
        if (a.dbg && (binned || fx_mode == 2 || (fx_mode == 0 && !igrad_lo))) {
            if (fx_mode == 5) k_field_bwd_merged<CACHE_READ, true, 5><<<blocks, blk, 0, st>>>(a, m, G, F);
            else if (fx_mode == 4) k_field_bwd_merged<CACHE_READ, true, 4><<<blocks, blk, 0, st>>>(a, m, G, F);
            else if (fx_mode == 2) k_field_bwd_merged<CACHE_READ, true, 2><<<blocks, blk, 0, st>>>(a, m, G, F);
            else if (feat_cache) k_field_bwd_merged<CACHE_READ, true, 0><<<blocks, blk, 0, st>>>(a, m, G, F);
            else k_field_bwd_merged<CACHE_NONE, true, 0><<<blocks, blk, 0, st>>>(a, m, G, F);
            RN_CHECK_LAUNCH();
            return 0;
        }
    }
    if (fx_mode == 5) {
        k_field_bwd_merged<CACHE_READ, false, 5><<<blocks, blk, 0, st>>>(a, m, G, F);
    } else if (fx_mode == 4) {
        k_field_bwd_merged<CACHE_READ, false, 4><<<blocks, blk, 0, st>>>(a, m, G, F);
    } else if (fx_mode == 2) {
        k_field_bwd_merged<CACHE_READ, false, 2><<<blocks, blk, 0, st>>>(a, m, G, F);
    } else if (fx_mode == 3) {
        k_field_bwd_merged<CACHE_READ, false, 3><<<blocks, blk, 0, st>>>(a, m, G, F);
    } else if (igrad_lo) {
        if (feat_cache) k_field_bwd_merged<CACHE_READ, false, 1><<<blocks, blk, 0, st>>>(a, m, G, F);
        else k_field_bwd_merged<CACHE_NONE, false, 1><<<blocks, blk, 0, st>>>(a, m, G, F);
    } else {
        if (feat_cache) k_field_bwd_merged<CACHE_READ, false, 0><<<blocks, blk, 0, st>>>(a, m, G, F);
        else k_field_bwd_merged<CACHE_NONE, false, 0><<<blocks, blk, 0, st>>>(a, m, G, F);
    }
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_field_fwd_merged(const float* ts, const int32_t* ray_of, const float* rays_o,
                        const float* rays_d, const int32_t* seg_base, const int32_t* seg_count,
                        const int32_t* chunk_desc, int32_t* queue,
                        int64_t n_rays, int32_t n_models, const void* grid_f16,
                        const uint32_t* level_offset, const uint32_t* level_hsize,
                        const uint32_t* level_res, const float* level_scale,
                        const float* xyz_min, const float* extent, const void* frags,
                        float* sigma, float* rgb, void* feat_cache, const int32_t* mstart,
                        const int32_t* perm, int32_t blocks, int32_t threads, void* stream) {
    RN_CHECK_ARG(n_rays >= 1 && n_models >= 1 && n_models <= FM_KMAX && blocks >= 1,
                 "bad sizes (n_models <= 8)");
    RN_CHECK_ARG(threads >= 64 && threads <= 1024 && threads % 64 == 0, "threads: 64..1024, waves");
    RN_CHECK_ARG(ts && ray_of && rays_o && rays_d && seg_base && seg_count &&
                 chunk_desc && queue && grid_f16 && level_offset && level_hsize && level_res &&
                 level_scale && xyz_min && extent && frags && sigma && rgb, "null pointer");
    RN_CHECK_ARG(!(mstart || perm) || (mstart && perm && feat_cache),
                 "merged-order encoding needs mstart, perm and the encoding cache");
    FieldArgs a{};
    fill_args(a, xyz_min, extent, level_offset, level_hsize, level_res, level_scale);
    a.dbg = rn_dbg(g_field_dbg);
    a.grid = (const rn_half*)grid_f16; a.frags = (const rn_half*)frags;
    a.sigma = sigma; a.rgb = rgb; a.feat = (rn_half*)feat_cache;
    a.ts = ts; a.ray_of = ray_of; a.rays_o = rays_o; a.rays_d = rays_d;
    a.seg_base = seg_base; a.seg_count = seg_count;
    MergeArgs m{};
    m.desc = chunk_desc; m.queue = queue;
    m.mstart = mstart; m.perm = perm;
    m.n_rays = (int)n_rays; m.n_models = n_models;
    const bool gw = n_models > FM_LDS_K;
    const size_t lds = gw ? 0 : (size_t)n_models * FIELD_FWD_FRAGS * RN_FRAG_BYTES;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(queue + 2, 0, sizeof(int32_t), st) != hipSuccess) {
        rn_set_error("%s: ticket reset failed", __func__);
        return 2;
    }
#define RN_FM_LAUNCH(C, E)                                                                     \
    do {                                                                                       \
        if (gw) k_field_fwd_merged<C, E, true><<<blocks, threads, 0, st>>>(a, m);              \
        else k_field_fwd_merged<C, E, false><<<blocks, threads, lds, st>>>(a, m);              \
    } while (0)
    if (mstart) RN_FM_LAUNCH(CACHE_WRITE, true);
    else if (feat_cache) RN_FM_LAUNCH(CACHE_WRITE, false);
    else RN_FM_LAUNCH(CACHE_NONE, false);
#undef RN_FM_LAUNCH
    RN_CHECK_LAUNCH();
    return 0;
}

/* level-partitioned merged forward (k_enc_prep + k_field_encode_levels +
   k_field_mlp_planes): the same outputs and encoding cache as
   rn_field_fwd_merged with the merged-order encoding.  planes: 16 x
   plane_stride u32 (plane_stride >= every sample index + 1); prep: 16 B per
   merged sample; xq (optional probe): 96 int32, [8 g + x] += blocks of level
   group g that ran on XCD x, then u64 [32 + g] first start and [40 + g] last
   end of group g's blocks (s_memrealtime, 100 MHz). */
int rn_field_fwd_levels(const float* ts, const int32_t* ray_of, const float* rays_o,
                        const float* rays_d, const int32_t* seg_base, const int32_t* seg_count,
                        int64_t n_rays, int32_t n_models, const void* grid_f16,
                        const uint32_t* level_offset, const uint32_t* level_hsize,
                        const uint32_t* level_res, const float* level_scale,
                        const float* xyz_min, const float* extent, const void* frags,
                        float* sigma, float* rgb, void* feat_cache, const int32_t* mstart,
                        const int32_t* perm, uint32_t* planes, int64_t plane_stride, void* prep,
                        int32_t prep_ready, int32_t enc_blocks, int32_t mlp_blocks, int32_t* xq,
                        void* stream) {
    RN_CHECK_ARG(n_rays >= 1 && n_models >= 1 && n_models <= FM_KMAX && plane_stride >= 1,
                 "bad sizes (n_models <= 8)");
    RN_CHECK_ARG(enc_blocks >= 8 && enc_blocks % 8 == 0 && mlp_blocks >= 1,
                 "bad launch (enc_blocks: a multiple of 8)");
    RN_CHECK_ARG(ts && ray_of && rays_o && rays_d && seg_base && seg_count && grid_f16 &&
                 level_offset && level_hsize && level_res && level_scale && xyz_min && extent &&
                 frags && sigma && rgb && mstart && perm && planes && prep, "null pointer");
    FieldArgs a{};
    fill_args(a, xyz_min, extent, level_offset, level_hsize, level_res, level_scale);
    a.dbg = rn_dbg(g_field_dbg);
    a.grid = (const rn_half*)grid_f16; a.frags = (const rn_half*)frags;
    a.sigma = sigma; a.rgb = rgb; a.feat = (rn_half*)feat_cache;
    a.planes = planes; a.plane_stride = plane_stride;
    a.ts = ts; a.ray_of = ray_of; a.rays_o = rays_o; a.rays_d = rays_d;
    a.seg_base = seg_base; a.seg_count = seg_count;
    MergeArgs m{};
    m.mstart = mstart; m.perm = perm; m.n_rays = (int)n_rays; m.n_models = n_models;
    hipStream_t st = (hipStream_t)stream;
    if (xq && (hipMemsetAsync(xq, 0, 64 * sizeof(int32_t), st) != hipSuccess ||
               hipMemsetAsync(xq + 64, 0xff, 16 * sizeof(int32_t), st) != hipSuccess ||
               hipMemsetAsync(xq + 80, 0, 16 * sizeof(int32_t), st) != hipSuccess)) {
        rn_set_error("%s: probe reset failed", __func__);
        return 2;
    }
    // (prep_ready: rn_bwd_plan wrote the per-position input as it placed the samples)
    if (!prep_ready) k_enc_prep<<<1024, 256, 0, st>>>(a, m, (float4*)prep);
    // level groups: (g, 15 - g) unless a study set another pairing (each level
    // exactly once: checked on the host)
    uint64_t pairing = g_level_pairing;
    if (pairing == 0)
        for (int g = 0; g < 8; ++g) pairing |= (uint64_t)(g | ((RN_L - 1 - g) << 4)) << (8 * g);
    k_field_encode_levels<<<enc_blocks, 256, 0, st>>>(a, m, (const float4*)prep, xq, pairing);
    k_field_mlp_planes<<<mlp_blocks, 1024,
                         (size_t)min(n_models, FM_LDS_K) * FIELD_FWD_FRAGS * RN_FRAG_BYTES, st>>>(
        a, n_models);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_seed_scale(const int32_t* seg_base, const int32_t* seg_count, int32_t n_models,
                  const float* sigma, const float* dL_dsigma, const float* dL_drgb,
                  uint32_t* work, float* scale, void* stream) {
    RN_CHECK_ARG(n_models >= 1, "bad sizes");
    RN_CHECK_ARG(seg_base && seg_count && sigma && dL_dsigma && dL_drgb && work && scale,
                 "null pointer");
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(work, 0, sizeof(uint32_t), st) != hipSuccess) {
        rn_set_error("%s: memset failed", __func__);
        return 2;
    }
    k_seed_max<<<dim3(256, n_models), 256, 0, st>>>(seg_base, seg_count, sigma, dL_dsigma,
                                                     dL_drgb, work);
    RN_CHECK_LAUNCH();
    k_seed_scale<<<1, 1, 0, st>>>(work, scale);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_grid_fx_fold(const uint32_t* level_offset, const uint32_t* level_hsize,
                    const uint32_t* level_res, int32_t* fx_acc, const float* fx_scale_cur,
                    float* fx_scale_next, uint32_t* fx_vmax, int32_t* fx_redo, float* grid_grad,
                    void* stream) {
    RN_CHECK_ARG(level_offset && level_hsize && level_res && fx_acc && fx_scale_cur &&
                 fx_scale_next && fx_vmax && fx_redo && grid_grad, "null pointer");
    RN_CHECK_ARG(fx_scale_cur != fx_scale_next, "scale_cur and scale_next must differ");
    GridMeta gm{};
    uint32_t hashed = 0;
    for (int l = 0; l < RN_L; ++l) {
        gm.offset[l] = level_offset[l]; gm.hsize[l] = level_hsize[l]; gm.res[l] = level_res[l];
        const uint64_t r = level_res[l];
        if (r * r * r > (uint64_t)level_hsize[l]) hashed |= 1u << l;
        RN_CHECK_ARG(level_offset[l] % 8 == 0, "level offsets must be multiples of 8 entries");
    }
    hipStream_t st = (hipStream_t)stream;
    FxStats* stats = reinterpret_cast<FxStats*>(fx_vmax);
    k_fx_esum<<<dim3(128, RN_L), 256, 0, st>>>(gm, fx_scale_cur, fx_acc, grid_grad, stats);
    k_fx_check<<<1, 64, 0, st>>>(hashed, fx_scale_cur, fx_scale_next, stats, fx_redo, nullptr, 0u);
    RN_CHECK_LAUNCH();
    {   // every level (dense ones go fixed point from their second step)
        const int64_t e0 = 2 * (int64_t)level_offset[0];
        const int64_t e1 = 2 * ((int64_t)level_offset[RN_L - 1] + level_hsize[RN_L - 1]);
        RN_CHECK_ARG(e1 % 4 == 0, "table size must be a multiple of 2 entries");
        const int64_t n4 = (e1 - e0) / 4;
        const int nb = (int)std::min<int64_t>(2048, (n4 + 255) / 256);
        k_fx_fold<<<nb > 0 ? nb : 1, 256, 0, st>>>(e0, e1, gm, fx_scale_cur, fx_acc, grid_grad,
                                                    fx_redo);
        RN_CHECK_LAUNCH();
    }
    return 0;
}

}  // extern "C"

int rn_fx_check_binned(const float* fx_scale_cur, float* fx_scale_next, uint32_t* fx_stats,
                       int32_t* fx_redo, const void* ctl, uint32_t pool_pages, void* stream) {
    k_fx_check<<<1, 64, 0, (hipStream_t)stream>>>(0u, fx_scale_cur, fx_scale_next,
                                                  reinterpret_cast<FxStats*>(fx_stats), fx_redo,
                                                  (const GbCtl*)ctl, pool_pages);
    RN_CHECK_LAUNCH();
    return 0;
}

extern "C" {

int rn_igrad_to_f32(int64_t n, int32_t* igrad_lo, int32_t* igrad_carry, const float* scale,
                    float* grid_grad, void* stream) {
    RN_CHECK_ARG(n >= 0, "bad size");
    if (n == 0) return 0;
    RN_CHECK_ARG(igrad_lo && igrad_carry && scale && grid_grad, "null pointer");
    k_igrad_to_f32<<<nblk(n, 256), 256, 0, (hipStream_t)stream>>>(n, igrad_lo, igrad_carry, scale,
                                                                   grid_grad);
    RN_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
