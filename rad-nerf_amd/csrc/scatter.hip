// Binned grid-gradient scatter, passes 2 and 3 (the merged backward's walk,
// field.hip GM 4, is pass 1: it appends each level's records to pages).
//
//   k_grid_bin  one workgroup per page: counting sort of the page's records
//               by slice of the page's level (gb_slice_bits: 64-4096 entries)
//               in LDS, the sorted page written back coalesced, plus each
//               slice's run (start, count) and the page's entry in its level's
//               page list;
//   k_grid_sum  one workgroup per slice: the slice's runs of every page of
//               its level added into an int64 copy of the slice in LDS
//               (ds_add_u64: exact and order-free), then
//               grid_grad += acc * 2^-e_l once per touched entry.
//
// The bin pass reads and writes 8 B per record in whole pages, the sum pass
// reads each run's lines (runs of ~64 records at the hashed levels, longer at
// the dense ones), against the 64-B memory-side request per 1.84 records of
// the atomic form.  See rn_bin.h for the formats.
// Reference: the tcnn grid-encoding backward (hash-grid parameter gradient)
// behind /root/reference/models/networks.py:300-328.
#include "rn_common.h"
#include "rn_field.h"
#include "rn_bin.h"

// timing studies only (ablation bit 21): per-phase wave cycles of k_grid_sum
// summed over waves ([0] LDS zero + barrier, [1] first run fetch, [2] run
// loop, [3] write-back), [4] waves, [5] groups, [6] earliest wave start and
// [7] latest wave end (s_memrealtime, 100 MHz)
__device__ unsigned long long g_gb_cyc[8];

namespace {

// record loads of the sum pass: plain loads (0.729 -> 0.717 ms at C5 against
// non-temporal ones); the bin pass keeps non-temporal loads of its pages (read
// once: 1.107 vs 1.21 ms with plain loads; profiles/r05/ab/ab_ntld_*)
__device__ __forceinline__ uint64_t gb_ld(const uint64_t* p) { return *p; }


#define GB_SUM_THREADS 1024

// THREADS per page; PF: the next page's records are loaded (all 8192, the
// fill is not known yet) while this one is sorted
template <int THREADS, bool PF>
__global__ void __launch_bounds__(THREADS, THREADS / 128)   // two workgroups per CU
k_grid_bin(GbPool P, bool rotate) {
    constexpr int PT = GB_PAGE / THREADS;
    __shared__ uint64_t sRec[GB_PAGE];
    __shared__ uint32_t sHist[GB_MAX_BINS];
    const int tid = threadIdx.x, lane = rn_lane(), wid = tid / RN_WAVE;
    const uint32_t np = min(__builtin_nontemporal_load(&P.ctl->pool_next), P.pool_pages);
    uint64_t r[PT];
    auto load_page = [&](uint32_t pg, uint64_t* dst, uint32_t n) {
        const uint64_t* src = P.pages_in + (size_t)pg * GB_PAGE;
#pragma unroll
        for (int j = 0; j < PT; ++j) {
            const uint32_t i = tid + THREADS * j;
            dst[j] = i < n ? __builtin_nontemporal_load(src + i) : 0ull;
        }
    };
    if (PF && blockIdx.x < np) load_page(blockIdx.x, r, GB_PAGE);
    for (uint32_t p = blockIdx.x; p < np; p += gridDim.x) {
        const uint32_t meta = P.page_meta[p];
        uint32_t l = meta & 0xffu, n = meta >> 8;
        if (l >= RN_L || n > GB_PAGE) {                 // a corrupt meta: refuse the page
            if (tid == 0) atomicOr(&P.ctl->fault, GB_FAULT_META);
            l = 0u; n = 0u;
        }
        const uint32_t hs = P.hsize[l];
        for (int i = tid; i < GB_MAX_BINS; i += THREADS) sHist[i] = 0u;
        __syncthreads();
        if (!PF) load_page(p, r, n);
        uint64_t rn[PF ? PT : 1];
        if (PF && p + gridDim.x < np) load_page(p + gridDim.x, rn, GB_PAGE);
        uint32_t key[PT];
        const uint32_t sb = P.slice_bits[l];
        bool bad_idx = false;
#pragma unroll
        for (int j = 0; j < PT; ++j) {
            const uint32_t i = tid + THREADS * j;
            key[j] = ~0u;
            if (i < n) {
                const uint32_t e = gb_idx(r[j]);
                // an index outside the level would bin past its slices (and
                // past sHist): refused, and the step is redone
                if (e < hs) {
                    const uint32_t b = e >> sb;
                    key[j] = (b << 16) | atomicAdd(&sHist[b], 1u);
                } else {
                    bad_idx = true;
                }
            }
        }
        if (__builtin_amdgcn_ballot_w64(bad_idx) != 0ull && lane == 0)
            atomicOr(&P.ctl->fault, GB_FAULT_INDEX);
        __syncthreads();
        if (wid == 0) {
            // exclusive scan of the bins, GB_BPL per lane, in an order rotated
            // by the page (bin (j + rot) mod 256 is laid out j-th): slice b's
            // run sits at a different offset of every page, so the sum pass's
            // reads of one slice (one run per page) spread over the memory
            // channels instead of repeating one offset at a 64-KB stride
            constexpr int GB_BPL = GB_MAX_BINS / 64;
            const uint32_t rot = rotate ? (p * 97u) & (GB_MAX_BINS - 1u) : 0u;
            uint32_t h[GB_BPL], tot = 0u;
#pragma unroll
            for (int k = 0; k < GB_BPL; ++k) {
                h[k] = sHist[(GB_BPL * lane + k + rot) & (GB_MAX_BINS - 1u)];
                tot += h[k];
            }
            uint32_t incl = tot;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t o = (uint32_t)__shfl_up((int)incl, off);
                incl += lane >= off ? o : 0u;
            }
            uint32_t s0 = incl - tot;
            uint32_t* d = P.desc + (size_t)p * GB_MAX_BINS;
#pragma unroll
            for (int k = 0; k < GB_BPL; ++k) {
                const uint32_t bin = (GB_BPL * lane + k + rot) & (GB_MAX_BINS - 1u);
                d[bin] = s0 | (h[k] << 16);
                sHist[bin] = s0;
                s0 += h[k];
            }
            if (lane == 0 && n > 0) {
                const uint32_t slot = atomicAdd(&P.ctl->level_npages[l], 1u);
                if (slot < P.pool_pages) P.level_pages[(size_t)l * P.pool_pages + slot] = p;
                else atomicOr(&P.ctl->fault, GB_FAULT_LIST);     // a control block not reset
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PT; ++j) {
            const uint32_t i = tid + THREADS * j;
            if (i < n && key[j] != ~0u) sRec[sHist[key[j] >> 16] + (key[j] & 0xffffu)] = r[j];
        }
        __syncthreads();
        uint64_t* dst = P.pages_out + (size_t)p * GB_PAGE;
#pragma unroll 4
        for (uint32_t i = tid; i < n; i += THREADS) __builtin_nontemporal_store(sRec[i], dst + i);
        if (PF) {
#pragma unroll
            for (int j = 0; j < PT; ++j) r[j] = rn[j];
        }
    }
}

struct GbSumArgs {
    uint32_t first[RN_L + 1];     // first slice of the q-th level in launch order (level 15 - q)
    uint32_t off[RN_L], hs[RN_L];
};

// ABL (timing studies only, tools/bin_probe.py): 1 no LDS adds (records
// XOR-folded into a register)
template <int ABL>
__device__ __forceinline__ void gb_add(int64_t* acc, uint64_t r, uint64_t& fold, uint32_t emask) {
    const uint32_t e = gb_idx(r) & emask;
    if (ABL == 1) {
        fold ^= r;
    } else {
        __hip_atomic_fetch_add(acc + 2 * e, gb_v0(r), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(acc + 2 * e + 1, gb_v1(r), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

#define GB_RUNS 8                 // runs of one wave in flight (up to 2 loads each)
static_assert(GB_RUNS == 8, "k_grid_sum deals pages to the waves in groups of 8 lanes");

// Record loads are issued by the run's lanes only (exec-masked): the pass
// fetches the lines a run covers and nothing past it.  Full-lane loads
// (clamped into the page, the tail dropped in registers) took 0.92 against
// 0.70 ms at C5's volume (profiles/r04/binprobe/binprobe_full_v.json,
// bis4).  What made the first versions of this pass slow (4.1-4.6 ms) was
// one workgroup: level 0 at scale 16 was a single 4096-entry slice taking all
// 1M of its records, with one dependent load per 64 records (binprobe_full_s
// vs _t: the long-run loads 8 in flight, 1.95 ms; vs _u: per-level slice
// sizes, gb_slice_bits, 0.94 ms).
template <int ABL, bool PROF = false, int BIS = 0>
__global__ void __launch_bounds__(GB_SUM_THREADS, 8)   // two workgroups per CU
k_grid_sum(GbPool P, GbSumArgs s, const float* __restrict__ scale, const int32_t* __restrict__ redo,
           float* __restrict__ grad) {
    extern __shared__ int64_t acc[];               // [GB_SLICE][2], then the group counter
    uint64_t tp = PROF ? __builtin_amdgcn_s_memtime() : 0, cyc[4] = {0, 0, 0, 0}, ngrp = 0;
    const uint64_t rt0 = PROF ? __builtin_amdgcn_s_memrealtime() : 0;
    if (redo && __builtin_nontemporal_load(redo) != 0) return;   // the fp32 redo replaces the step
    int q = 0;
#pragma unroll
    for (int k = 1; k < RN_L; ++k) q = blockIdx.x >= s.first[k] ? k : q;
    const int l = RN_L - 1 - q;
    const uint32_t b = blockIdx.x - s.first[q];
    const uint32_t npg = min(__builtin_nontemporal_load(&P.ctl->level_npages[l]), P.pool_pages);
    const float sc = scale[l];
    if (npg == 0u || sc == 0.f) return;            // no records (an fp32 level went in by atomics)
    const int tid = threadIdx.x, lane = rn_lane();
    const uint32_t sbits = P.slice_bits[l], emask = (1u << sbits) - 1u;
    for (int i = tid; i < (2 << sbits); i += GB_SUM_THREADS) acc[i] = 0;
    if (tid == 0) *reinterpret_cast<uint32_t*>(acc + 2 * GB_SLICE) = 0u;   // the group counter
    __syncthreads();
    auto stamp = [&](int ph) {
        if (PROF) { const uint64_t t = __builtin_amdgcn_s_memtime(); cyc[ph] += t - tp; tp = t; }
    };
    stamp(0);
    const uint32_t* lp = P.level_pages + (size_t)l * P.pool_pages;
    // Each wave takes groups of 8 pages of the level's list from a workgroup
    // counter (lanes 0-7 hold a group's runs of this slice: page, start |
    // count << 16) and loads the next group's runs while it sums this one.
    // Dealing the groups statically (wave w: groups w, w + 16, ...) left ~20 %
    // of the waves' time at the final barrier, waiting for the slowest wave
    // (memory latency varies from group to group): at 1/8 of C5's volume
    // 0.139 -> 0.118 ms, at the full volume 0.74 -> 0.73-0.74 ms
    // (profiles/r04/binprobe/binprobe_{fp,full}_dy*.json).  The
    // slices of a level walk its page list from different starting points
    // (slice b at b / nslices of the list).
    const uint32_t nsl = s.first[q + 1] - s.first[q];
    const uint32_t start = (uint32_t)(((uint64_t)b * npg) / nsl);
    uint64_t fold = 0ull;
    // the runs of one group of 8 pages: lanes k0 .. k0 + 7 of (pgc, dc)
    auto sum_group = [&](uint32_t pgc, uint32_t dc, int k0) {
        ngrp += PROF ? 1 : 0;
        uint64_t r0[GB_RUNS], r1[GB_RUNS];
        uint32_t cnt[GB_RUNS], st[GB_RUNS];
        const uint64_t* pgp[GB_RUNS];
#pragma unroll
        for (int j = 0; j < GB_RUNS; ++j) {
            const uint32_t dk = (uint32_t)__builtin_amdgcn_readlane((int)dc, k0 + j);
            const uint32_t pk = (uint32_t)__builtin_amdgcn_readlane((int)pgc, k0 + j);
            // BIS (timing bisection only, full-lane loads): 1 load every run,
            // 2 and fold every lane, 3 every run 64 records, 4 as built
            // before round 4's exec-masked loads
            cnt[j] = BIS == 3 ? 64u : dk >> 16;
            st[j] = dk & 0xffffu;
            pgp[j] = P.pages_out + (size_t)pk * GB_PAGE;
            r0[j] = 0ull; r1[j] = 0ull;
            if (BIS == 0) {                                 // the run's lanes only
                if ((uint32_t)lane < cnt[j])
                    r0[j] = gb_ld(pgp[j] + st[j] + lane);
                if ((uint32_t)lane + 64u < cnt[j])
                    r1[j] = gb_ld(pgp[j] + st[j] + 64u + lane);
            } else {                                        // full-lane loads (timing)
                if (BIS != 4 || cnt[j] != 0u)
                    r0[j] = gb_ld(pgp[j] + min(st[j] + lane, GB_PAGE - 1u));
                if (cnt[j] > 64u)
                    r1[j] = gb_ld(pgp[j] + min(st[j] + 64u + lane, GB_PAGE - 1u));
            }
        }
#pragma unroll
        for (int j = 0; j < GB_RUNS; ++j) {
            if (BIS == 2 || (uint32_t)lane < cnt[j]) gb_add<ABL>(acc, r0[j], fold, emask);
            if ((uint32_t)lane + 64u < cnt[j]) gb_add<ABL>(acc, r1[j], fold, emask);
            // the rest of a run over 128 records (the coarse levels' runs are
            // long): 8 full-lane loads in flight per step
            for (uint32_t o = 128u; o < cnt[j]; o += 8u * 64u) {
                uint64_t rr[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    rr[u] = 0ull;
                    if (BIS == 0 ? o + 64u * u + lane < cnt[j] : o + 64u * u < cnt[j])
                        rr[u] = gb_ld(
                            pgp[j] + min(st[j] + o + 64u * u + lane, GB_PAGE - 1u));
                }
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (o + 64u * u + lane < cnt[j]) gb_add<ABL>(acc, rr[u], fold, emask);
            }
        }
    };
    {
        uint32_t* ctr = reinterpret_cast<uint32_t*>(acc + 2 * GB_SLICE);
        const uint32_t ngr = (npg + GB_RUNS - 1u) / GB_RUNS;
        auto grab = [&]() -> uint32_t {
            uint32_t x = 0u;
            if (lane == 0) x = atomicAdd(ctr, 1u);
            return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
        };
        auto group_runs = [&](uint32_t g, uint32_t& pg, uint32_t& d) {
            uint32_t i = g * GB_RUNS + (uint32_t)(lane & 7);
            pg = 0u; d = 0u;
            if (lane < GB_RUNS && g < ngr && i < npg) {
                i += start;
                i = i >= npg ? i - npg : i;
                pg = lp[i];
                // a page id outside the pool or a run past its page (the bin
                // pass writes neither): skipped, and the fault word says so
                const bool pg_ok = pg < P.pool_pages;
                d = pg_ok ? P.desc[(size_t)pg * GB_MAX_BINS + b] : 0u;
                if (!pg_ok || (d & 0xffffu) + (d >> 16) > GB_PAGE) {
                    atomicOr(&P.ctl->fault, GB_FAULT_RUN);
                    atomicOr(&P.ctl->sum_fault, GB_FAULT_RUN);     // sticky: read by the host
                    pg = 0u; d = 0u;
                }
            }
        };
        uint32_t g = grab(), pg, d;
        group_runs(g, pg, d);
        if (PROF) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); stamp(1); }
        while (g < ngr) {                               // wave-uniform
            const uint32_t pgc = pg, dc = d;
            const uint32_t gn = grab();
            group_runs(gn, pg, d);
            sum_group(pgc, dc, 0);
            g = gn;
        }
    }
    stamp(2);
    __syncthreads();
    if (ABL == 1 && fold == 0x0123456789abcdefull) acc[0] = 1;    // keeps the loads
    const float inv = 1.0f / sc;                   // exact: a power of two
    const uint32_t e0 = b << sbits;
    const uint32_t ne = min(1u << sbits, s.hs[l] - e0);
    float2* g = reinterpret_cast<float2*>(grad) + (size_t)s.off[l] + e0;
    for (uint32_t e = tid; e < ne; e += GB_SUM_THREADS) {
        const int64_t a0 = acc[2 * e], a1 = acc[2 * e + 1];
        if ((a0 | a1) == 0) continue;
        float2 v = g[e];
        v.x += (float)a0 * inv;
        v.y += (float)a1 * inv;
        g[e] = v;
    }
    if (PROF) {
        stamp(3);
        if (lane == 0) {
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) atomicAdd(g_gb_cyc + qq, (unsigned long long)cyc[qq]);
            atomicAdd(g_gb_cyc + 4, 1ull);
            atomicAdd(g_gb_cyc + 5, (unsigned long long)ngrp);
            atomicMin(g_gb_cyc + 6, (unsigned long long)rt0);
            atomicMax(g_gb_cyc + 7, (unsigned long long)__builtin_amdgcn_s_memrealtime());
        }
    }
}

}  // namespace

extern "C" {

int rn_debug_gb_cycles(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_gb_cyc), sizeof(unsigned long long) * 8, 0,
                            hipMemcpyDeviceToHost) != hipSuccess)
        return 2;
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, ~0ull, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_gb_cyc), z, sizeof(z), 0, hipMemcpyHostToDevice) != hipSuccess)
        return 2;
    return 0;
}

int rn_grid_bin_layout(int32_t* out) {
    RN_CHECK_ARG(out, "null pointer");
    out[0] = GB_PAGE; out[1] = GB_MAX_BINS; out[2] = (int32_t)GB_SLICE;
    out[3] = (int32_t)sizeof(GbCtl); out[4] = GB_IDX_BITS; out[5] = GB_V_BITS;
    out[6] = GB_M_BITS; out[7] = GB_TARGET_BITS;
    return 0;
}

int rn_grid_slice_bits(const uint32_t* level_hsize, int32_t* out) {
    RN_CHECK_ARG(level_hsize && out, "null pointer");
    for (int l = 0; l < RN_L; ++l) {
        RN_CHECK_ARG(level_hsize[l] >= 1 && level_hsize[l] <= (1u << GB_IDX_BITS),
                     "level too large for binning");
        out[l] = (int32_t)gb_slice_bits(level_hsize[l]);
    }
    return 0;
}

int rn_grid_record_encode(const float* x, int64_t n, uint32_t* out) {
    RN_CHECK_ARG(n >= 0, "bad size");
    RN_CHECK_ARG(n == 0 || (x && out), "null pointer");
    for (int64_t i = 0; i < n; ++i) out[i] = gb_encode(x[i]);
    return 0;
}

int rn_grid_record_decode(const uint32_t* f, int64_t n, int64_t* out) {
    RN_CHECK_ARG(n >= 0, "bad size");
    RN_CHECK_ARG(n == 0 || (f && out), "null pointer");
    for (int64_t i = 0; i < n; ++i) out[i] = gb_decode(f[i]);
    return 0;
}

int rn_grid_bin(const uint32_t* level_hsize, void* ctl, const uint32_t* page_meta,
                const uint64_t* pages_in, uint64_t* pages_out, uint32_t* desc,
                uint32_t* level_pages, int32_t pool_pages, int32_t blocks, void* stream) {
    RN_CHECK_ARG(level_hsize && ctl && page_meta && pages_in && pages_out && desc && level_pages,
                 "null pointer");
    RN_CHECK_ARG(pool_pages >= 1 && blocks >= 1, "bad sizes");
    GbPool P{};
    for (int l = 0; l < RN_L; ++l) {
        RN_CHECK_ARG(level_hsize[l] >= 1 && level_hsize[l] <= (GB_MAX_BINS << GB_SLICE_BITS) &&
                         level_hsize[l] <= (1u << GB_IDX_BITS), "level too large for binning");
        P.slice_bits[l] = (uint8_t)gb_slice_bits(level_hsize[l]);
        P.hsize[l] = level_hsize[l];
    }
    P.ctl = (GbCtl*)ctl; P.page_meta = (uint32_t*)page_meta; P.pages_in = (uint64_t*)pages_in;
    P.pages_out = pages_out; P.desc = desc; P.level_pages = level_pages;
    P.pool_pages = (uint32_t)pool_pages;
    // (timing studies only: bit 20 no per-page rotation of the run layout;
    // bits 22-23 the variant: 1 = 512 threads with the next page prefetched,
    // 2 = 256 threads)
    const int dbg = rn_debug_flags_internal();       // 0 in librn.so
    const bool rotate = !((dbg >> 20) & 1);
    const int var = (dbg >> 22) & 3;
    hipStream_t st = (hipStream_t)stream;
    bool done = false;
    if constexpr (RN_ABL) {
        done = var == 1 || var == 2;
        if (var == 1) k_grid_bin<512, true><<<blocks, 512, 0, st>>>(P, rotate);
        else if (var == 2) k_grid_bin<256, false><<<blocks, 256, 0, st>>>(P, rotate);
    }
    if (!done) k_grid_bin<1024, false><<<blocks, 1024, 0, st>>>(P, rotate);
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_grid_sum(const uint32_t* level_offset, const uint32_t* level_hsize, const void* ctl,
                const uint32_t* desc, const uint32_t* level_pages, const uint64_t* pages_out,
                int32_t pool_pages, const float* fx_scale, const int32_t* redo, float* grid_grad,
                int32_t level_lo, int32_t level_hi, void* stream) {
    RN_CHECK_ARG(level_offset && level_hsize && ctl && desc && level_pages && pages_out &&
                 fx_scale && grid_grad, "null pointer");
    RN_CHECK_ARG(pool_pages >= 1, "bad sizes");
    RN_CHECK_ARG(level_lo >= 0 && level_lo <= level_hi && level_hi <= RN_L,
                 "levels: 0 <= level_lo <= level_hi <= 16");
    GbSumArgs s{};
    uint32_t total = 0;
    for (int q = 0; q < RN_L; ++q) {            // the finest (heaviest) levels first
        const int l = RN_L - 1 - q;
        RN_CHECK_ARG(level_hsize[l] >= 1 && level_hsize[l] <= (GB_MAX_BINS << GB_SLICE_BITS) &&
                         level_hsize[l] <= (1u << GB_IDX_BITS), "level too large for binning");
        s.first[q] = total;
        const uint32_t sb = gb_slice_bits(level_hsize[l]);
        // levels outside [level_lo, level_hi) get no workgroups (an empty
        // range of blockIdx: the kernel's level search never lands on them)
        if (l >= level_lo && l < level_hi) total += (level_hsize[l] + (1u << sb) - 1) >> sb;
    }
    s.first[RN_L] = total;
    if (total == 0) return 0;
    for (int l = 0; l < RN_L; ++l) { s.off[l] = level_offset[l]; s.hs[l] = level_hsize[l]; }
    GbPool P{};
    P.ctl = (GbCtl*)ctl; P.desc = (uint32_t*)desc; P.level_pages = (uint32_t*)level_pages;
    P.pages_out = (uint64_t*)pages_out; P.pool_pages = (uint32_t)pool_pages;
    for (int l = 0; l < RN_L; ++l) P.slice_bits[l] = (uint8_t)gb_slice_bits(level_hsize[l]);
    const size_t lds = (size_t)GB_SLICE * 2 * sizeof(int64_t) + 16;   // + the group counter
    // ablations (timing studies only): bit 16 no LDS adds, bit 21 per-phase cycles
    const int dbg = rn_debug_flags_internal() >> 16;   // 0 in librn.so
    hipStream_t st = (hipStream_t)stream;
#define GB_SUM_LAUNCH(A, PR, BI) \
    k_grid_sum<A, PR, BI><<<total, GB_SUM_THREADS, lds, st>>>(P, s, fx_scale, redo, grid_grad)
    bool done = false;
    if constexpr (RN_ABL) {
        done = true;
        if (dbg & 32) GB_SUM_LAUNCH(0, true, 0);
        else if ((dbg & 1) && (dbg & 0x1c)) {    // bits 18-20 with 16: bisection (timing)
            const int bis = (dbg >> 2) & 7;
            if (bis == 1) GB_SUM_LAUNCH(1, false, 1);
            else if (bis == 2) GB_SUM_LAUNCH(1, false, 2);
            else if (bis == 3) GB_SUM_LAUNCH(1, false, 3);
            else GB_SUM_LAUNCH(0, false, 4);
        }
        else if (dbg & 1) GB_SUM_LAUNCH(1, false, 0);
        else done = false;
    }
    if (!done) GB_SUM_LAUNCH(0, false, 0);
#undef GB_SUM_LAUNCH
    RN_CHECK_LAUNCH();
    return 0;
}

int rn_grid_bin_check(const uint32_t* level_hsize, void* ctl, const uint32_t* page_meta,
                      const uint64_t* pages_in, uint64_t* pages_out, uint32_t* desc,
                      uint32_t* level_pages, int32_t pool_pages, const float* fx_scale_cur,
                      float* fx_scale_next, uint32_t* fx_stats, int32_t* fx_redo, void* stream) {
    RN_CHECK_ARG(fx_scale_cur && fx_scale_next && fx_stats && fx_redo, "null pointer");
    RN_CHECK_ARG(fx_scale_cur != fx_scale_next, "scale_cur and scale_next must differ");
    int st = rn_grid_bin(level_hsize, ctl, page_meta, pages_in, pages_out, desc, level_pages, pool_pages,
                         2048, stream);
    if (st) return st;
    return rn_fx_check_binned(fx_scale_cur, fx_scale_next, fx_stats, fx_redo, ctl,
                              (uint32_t)pool_pages, stream);
}

int rn_grid_binned_fold(const uint32_t* level_offset, const uint32_t* level_hsize, void* ctl,
                        const uint32_t* page_meta, const uint64_t* pages_in, uint64_t* pages_out,
                        uint32_t* desc, uint32_t* level_pages, int32_t pool_pages,
                        const float* fx_scale_cur, float* fx_scale_next, uint32_t* fx_stats,
                        int32_t* fx_redo, float* grid_grad, void* stream) {
    const int st = rn_grid_bin_check(level_hsize, ctl, page_meta, pages_in, pages_out, desc,
                                     level_pages, pool_pages, fx_scale_cur, fx_scale_next, fx_stats,
                                     fx_redo, stream);
    if (st) return st;
    return rn_grid_sum(level_offset, level_hsize, ctl, desc, level_pages, pages_out, pool_pages,
                       fx_scale_cur, fx_redo, grid_grad, 0, RN_L, stream);
}

}  // extern "C"
