"""Fused Rad-NeRF training render: the whole hot path of ml_render
(models/ml_rendering.py:11-78 + :158-202) for all K sub-NeRFs as a fixed
chain of HIP launches with no host synchronisation:

  forward : gate_fwd (side stream) | ml_march_count (single pass, staged)
            -> scan_segments -> ml_compact
            -> field_fwd (all K models, compact samples) -> ml_composite_fw
            -> ml_combine_fw
  backward: ml_combine_bw -> ml_composite_bw -> field_bwd -> gate_bwd

Sample buffers are sized for the worst case (B*K*max_samples, + alignment),
so sample counts never have to be read back; every kernel consumes the
device-side counts.  Outputs equal the unfused drop-in path (rendering.py)
for the same noise (tests/test_gpu_parity.py).
"""
import collections

import torch

from . import layout as LY
from ._lib import lib

MAX_SAMPLES = 1024
NEAR_DISTANCE = 0.01
SEG_ALIGN = 128
FX_STATS_BYTES = 640      # include/radnerf.h RN_FX_STATS_BYTES


# GbCtl (csrc/rn_bin.h) words read back after each binned backward: pool_next
# (word 0) ... sum_fault (word 18, sticky across steps)
GB_SUM_FAULT = 18
GB_CTL_READ = GB_SUM_FAULT + 1


def clamp_split(split_level):
    """The binned fold's level cut for the data-parallel hook schedule, in
    [0, 15]: levels [cut, 16) are summed first and handed to
    after_grid_levels, then [0, cut).  0 sums the whole grid at once; 16
    would leave the first sum empty and release the grid before any level
    was summed, so it is clamped to 15."""
    return max(0, min(15, int(split_level)))


def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


# per (device, stream): forward scratch shared by every workspace (level_buffers)
_LEVEL_SCRATCH = {}


class Workspace:
    """Persistent device buffers for one (B, K) configuration."""

    def __init__(self, n_rays, n_models, device, max_samples=MAX_SAMPLES, capacity=None):
        B, K = n_rays, n_models
        self.B, self.K, self.device = B, K, device
        cap = capacity or (B * K * max_samples + SEG_ALIGN * K)
        self.capacity = cap
        f = dict(device=device, dtype=torch.float32)
        i = dict(device=device, dtype=torch.int32)
        self.counts = torch.empty(K, B, **i)
        self.offsets = torch.empty(K, B, **i)
        self.seg = torch.zeros(2 * K + 2, **i)      # seg_base[K] | seg_count[K] | meta[2]
        self.used = torch.empty(K, B, **i)
        self.ts = torch.empty(cap, **f)
        self.deltas = torch.empty(cap, **f)
        self.ray_of = torch.empty(cap, **i)
        self.sigma = torch.empty(cap, **f)
        self.rgb = torch.empty(cap, 3, **f)
        self.ws = torch.empty(cap, **f)
        self.dsigma = torch.empty(cap, **f)
        self.drgb = torch.empty(cap, 3, **f)
        self.opacity_k = torch.empty(K, B, **f)
        self.depth_k = torch.empty(K, B, **f)
        self.rgb_k = torch.empty(K, B, 3, **f)
        self.dgate = torch.empty(B, K, **f)
        # single-pass march staging: max_samples slots per (model, ray)
        self.stage_ts = torch.empty(K * B * max_samples, **f)
        self.stage_dt = torch.empty(K * B * max_samples, **f)
        # field fwd -> bwd encoding cache: 32 f16 per sample slot (64 B)
        self.feat = torch.empty((cap + 31) // 32 * 32, 32, device=device, dtype=torch.float16)
        # merged backward (rn_bwd_plan): per-ray merged starts, merged order, queue head
        self.mstart = torch.empty(B + 1, **i)
        self.perm = torch.empty(cap, **i)
        self.queue = torch.zeros(3, **i)
        self._bwd_scratch = None
        self._chunks = None
        self.generation = 0         # forwards run through this workspace (_MLRenderFn)

    def chunk_list(self, max_chunk, min_chunk, head_chunks=0, balance_blocks=0):
        """rn_bwd_plan's chunk list, sized for the workspace capacity."""
        # include/radnerf.h's bound (the tail after the last big chunk can
        # hold up to max_chunk more samples in min_chunk pieces)
        cap = (head_chunks + self.capacity // max_chunk + self.capacity // (8 * min_chunk) +
               max_chunk // min_chunk + 3 + balance_blocks)
        if self._chunks is None or self._chunks.numel() < cap + 1:
            self._chunks = torch.empty(cap + 1, device=self.device, dtype=torch.int32)
            self._chunk_desc = torch.empty(cap + 1, 20, device=self.device, dtype=torch.int32)
        return cap, self._chunks

    def level_buffers(self, stream=None):
        """rn_field_fwd_levels' per-level encoding planes (16 x f16x2 per
        sample slot, 64 B) and merged-order unit coordinates (16 B).  They are
        scratch of one forward (written by the encode, read by the MLP
        tiles), so the workspaces of a device share one pair per stream,
        grown to the largest (80 B per slot in every workspace
        was ~40 % of a workspace)."""
        rows = self.feat.shape[0]
        key = (str(self.device), int(stream) if stream is not None else 0)
        cur = _LEVEL_SCRATCH.get(key)
        if cur is None or cur[0].shape[1] < rows:
            cur = (torch.empty(16, rows, device=self.device, dtype=torch.int32),
                   torch.empty(rows, 4, device=self.device, dtype=torch.float32))
            _LEVEL_SCRATCH[key] = cur
        return cur

    def fx_buffers(self, n, device):
        """Fixed-point grid-gradient state (rn_grid_fx_fold): int32 sums (n,
        zero between steps), per-level scales (2, 16) (current / next, swapped
        by fx_i each step; zeros = fp32 until the first step has measured the
        records), the per-level statistics block (FX_STATS_BYTES: record
        maxima, plain and weighted record / entry sums; include/radnerf.h)
        and the redo flag."""
        if getattr(self, "_fx", None) is None or self._fx[0].numel() != n:
            z = dict(device=device, dtype=torch.int32)
            self._fx = (torch.zeros(n, **z), torch.zeros(2, 16, device=device),
                        torch.zeros(FX_STATS_BYTES // 4, **z), torch.zeros(1, **z))
            self.fx_i = 0
        return self._fx

    def bin_pool(self, pages):
        """Page pool of the binned grid-gradient scatter (fx_mode 4,
        rn_grid_binned_fold; csrc/rn_bin.h): control block, page levels /
        fills, the pages (u64 records; the bin pass sorts each page in place),
        per-page slice runs, per-level page lists (a step that overflows the
        pool is redone in fp32; _bin_pool grows it from the counts the
        backwards read back)."""
        b = getattr(self, "_bin", None)
        if b is None or b["pages"] < pages:
            lay = lib().bin_layout()
            i = dict(device=self.device, dtype=torch.int32)
            self._bin = b = dict(
                pages=pages, page=lay["page"],
                ctl=torch.zeros(lay["ctl_bytes"] // 4, **i),
                meta=torch.zeros(pages, **i),
                recs=torch.empty(pages * lay["page"], device=self.device, dtype=torch.int64),
                desc=torch.empty(pages * lay["bins"], **i),
                lpages=torch.empty(16 * pages, **i))
        return b

    def bwd_scratch(self, blocks, max_chunk, max_samples=MAX_SAMPLES):
        """Per-block row scratch and dW park area of rn_field_bwd_merged."""
        rows = max_chunk + self.K * max_samples
        key = (blocks, rows)
        if self._bwd_scratch is None or self._bwd_scratch[0] != key:
            f = dict(device=self.device, dtype=torch.float32)
            self._bwd_scratch = (key, torch.empty(blocks * rows * 20, **f),
                                 torch.empty(blocks * self.K * 8 * 2048, **f))
        return rows, self._bwd_scratch[1], self._bwd_scratch[2]

    @property
    def seg_base(self):
        return self.seg[: self.K]

    @property
    def seg_count(self):
        return self.seg[self.K: 2 * self.K]

    @property
    def meta(self):
        return self.seg[2 * self.K:]

    def n_samples(self):
        """Total marched samples (reads back: diagnostics only)."""
        return int(self.meta[1].item())


class FusedMLRenderer:
    """Owns the workspace and runs the fused forward / backward chains."""

    def __init__(self, model, gating_net, n_rays, device=None, fwd_blocks=None, bwd_blocks=None,
                 capacity=None):
        self.model, self.gate = model, gating_net
        self.device = device or model.mlp_params.device
        self.ws = Workspace(n_rays, model.size, self.device, capacity=capacity)
        K = model.size
        bf = [getattr(model, f"density_bitfield_{i}") for i in range(K)]
        self.bitfield_bytes = bf[0].numel()
        self.fwd_blocks = fwd_blocks or max(1, 2048 // K)
        self.bwd_blocks = bwd_blocks or max(1, 256 // K)
        self.feat_cache = True      # field fwd stores the encoding, bwd skips the re-gather
        # backward scatters the K models' grid gradients merged per ray
        # (rn_field_bwd_merged); False: one model per block (rn_field_bwd)
        # (K = 1 too: its row-lane walk beats the per-model kernel, step 3.60 vs
        # 3.74 ms, profiles/r01/step_variants_k1.json)
        self.merged_bwd = 1 <= model.size <= 8      # rn_field_bwd_merged: K <= 8
        # forward evaluating the K models' tiles of a chunk interleaved
        # (rn_field_fwd_merged, K <= 8; bit-exact with rn_field_fwd).  One
        # block per CU keeps a chunk's rays in that CU's L1, so the second
        # model's corners hit lines the first fetched: C3 1.12 ms vs 1.30 ms
        # before the merged-order encode (tools/fwd_blocks_sweep.py; 2 blocks
        # per CU 1.17, 3 x 4 waves 1.35)
        # (K > 4: the MLP fragments are read from global memory instead of LDS)
        # (K = 1: the per-model kernel, 3.72 vs 3.74 ms per step)
        self.merged_fwd = 1 < model.size <= 8
        # merged forward: encode each chunk in merged (ray, t, model) order
        # first (tiles mixing the sub-NeRFs of a ray stretch share more grid
        # lines: 20.9 vs 28.2 per sample, tools/fwd_lines_sim.py), then the
        # per-model MLP tiles read the encoding cache.  C3: field_fwd 1.095 ->
        # 1.03 ms.  One sub-NeRF has nothing to interleave.
        self.merged_encode = model.size > 1
        self.merged_fwd_blocks = 256
        # 16 waves: with the merged-order encode, C3 step 5.13 ms vs 5.16 at 8
        # (tools/step_variants.py, profiles/r01/step_variants_fwd_shape.json)
        self.merged_fwd_threads = 1024
        # level-partitioned forward (rn_field_fwd_levels): each XCD encodes two
        # levels of every sample, so its L2 holds two levels' tables instead of
        # sixteen; bit-exact with the merged forward (tools/enc_probe.py).
        # bench.py A/B (profiles/r03/lv_*_a1.json): C2 802 -> 853, C3 1098 ->
        # 1139, C4 401 -> 450, C5 513 -> 549 M samples/s.  Needs the plan's
        # merged order (rn_bwd_plan runs with the merged backward or forward).
        self.level_fwd = self.merged_bwd or self.merged_fwd
        # the plan writes the level forward's per-position input (no prep pass)
        self.plan_prep = True
        self.level_enc_blocks = 4096
        self.level_mlp_blocks = 256
        self.merged_blocks = 256
        # chunk of merged samples per queue ticket: 1024 keeps a block's staged
        # rows L2-resident (C3 sweep: 768 3.94, 1024 3.88, 2048 3.92, 4096 4.05,
        # 8192 4.50 ms)
        # Small steps want more, smaller chunks (at least a few per block): C1
        # (K = 1, 1024 rays) 1024 -> 256 is 0.707 -> 0.618 ms per step, C2
        # (K = 1, 8192 rays) 512 = 1024 (tools/step_variants.py, r02)
        rk = n_rays * model.size
        self.max_chunk = 256 if rk <= 1024 else (512 if rk <= 4096 else 1024)
        # with the fixed-point scatter (cheaper requests) longer chunks pay at
        # scale 0.5 with several sub-NeRFs (fewer end-of-chunk ring flushes):
        # C3 step 1024 5.02, 1280 4.94, 1536 4.89, 1792 4.92 ms; K = 8 at
        # scale 16 (C5 per GPU) 1024 12.36, 2048 12.23 ms; K = 4 at scale 16
        # (C4 per GPU) keeps 1024 (3.82 vs 3.92 at 1536); K = 1 (C2) 512-1024
        # within 0.6 % (tools/step_variants.py, profiles/r02/step_variants_fx_chunk.json)
        # Round 5, with the big chunks balanced over the blocks (balance_chunks
        # below): longer chunks pay at K >= 4 (fewer model switches -- park /
        # unpark dW, reload weights -- and ring drains per sample): C5 per GPU
        # 2048 645, 4096 664, 6144 670, 8192 671-675; C4 1024 512, 2048 533,
        # 3072 535, 4096 537, 6144 422; C3 1024 1136, 1536 1158, 2048 1148
        # (profiles/r05/chunk3/); after the walk-step work of late round 5:
        # C5 6144 728, 8192 730, 12288 734.6, 16384 734.2; C4 3072 591, 4096
        # 589, 6144 468; C3 1024 1172, 1536 1182, 2048 1177 (profiles/r05/chunk5/)
        if model.size >= 8 and rk > 4096:
            self.max_chunk = 12288
        elif model.size >= 4 and rk > 4096 and float(model.scale) > 0.5:
            self.max_chunk = 4096
        elif model.size >= 2 and rk > 4096 and float(model.scale) <= 0.5:
            self.max_chunk = 1536
        # exact integer accumulation of the grid gradient (rn_seed_scale +
        # returning u32 atomics with carries + rn_igrad_to_f32): bitwise
        # reproducible grid gradients, but each issue waits for the previous
        # one's return (the compiler's vmcnt(0)): 4.33 vs 3.81 ms on C3, so the
        # default stays fp32 atomics
        self.int_grad = False
        # fixed-point accumulation of the hashed levels' grid gradient (u32
        # adds, scale from the previous step's largest record, fp32 redo on
        # overflow; rn_grid_fx_fold): field_bwd C3 3.76 -> 3.50 ms, C4 per
        # GPU 3.29 -> 2.60, C5 10.54 -> 8.59 (tools/ablate.py, r02).  The
        # first backward of a workspace runs fp32 (no scale yet).  Its
        # bookkeeping (entry sums, check, fold over the whole table: 0.06 ms,
        # + 0.011 ms for the redo launch) is per step, not per sample: at C1's
        # 1024 rays x 1 sub-NeRF fp32 atomics win (494 vs 462 M samples/s),
        # from C2's 8192 rays on fixed point does (C2 800 vs 696, C3 1078 vs
        # 998; tools/gpu/fx_small.sh, profiles/r03/fx_small_r03.jsonl)
        self.grid_fx = rk > 1024
        # binned ("store and sum") scatter of the fixed-point records at scale
        # 16 (fx_mode 4 + rn_grid_binned_fold): the walk appends records to
        # pages with plain stores, a bin pass sorts each page by 4096-entry
        # slice, a sum pass adds each slice in LDS (int64, exact) -- instead
        # of memory-side atomics, which were 45 % of C5's field_bwd
        # (DESIGN §4 "Binned scatter")
        self.grid_bin = self.grid_fx and float(model.scale) > 0.5
        # binned mode: the coarse levels [0, n) go in by fp32 atomics instead
        # of page records.  A coarse record shares its 64-B request with its
        # neighbours (dense levels, the first hashed ones) and the walk hides
        # those atomics, while a page record costs 24 B of bin + sum traffic
        # (round 6, tools/level_bin_probe.py, profiles/r06/level_bin/): all
        # binned -> levels [0, n) fp32: C5 738 -> 763 M samples/s per GPU at
        # n = 9, C4 599 -> 640 at n = 8 (beyond, the atomics bind).  Those
        # levels' sums are then fp32 in arrival order (the fine levels' stay
        # exact int64); exact int64 sums with u64 atomics were measured too
        # and lost to fp32 (16-B entries double the requests of an x-pair;
        # DESIGN §4)
        self.bin_f32_levels = (9 if model.size >= 8 else 8) if self.grid_bin else 0
        # the int32 form's wrap checksums weight gradient element i by 4 i
        # (field.hip fx_weight), injective up to 2^28 elements: a larger table
        # (none of the reference's configs: 16 levels x 2^19 entries x 2
        # features = 2^24) keeps fp32 atomics unless it is binned (no checksum)
        if not self.grid_bin and model.xyz_encoder.params.numel() > (1 << 28):
            self.grid_fx = False
        # initial pool: records per (ray, sub-NeRF) at scale 16 (C5's replay:
        # 63.5 records x 95 samples; tools/records_sim.py), x 1.15
        self.bin_records_per_pair = 6912
        # the tail's chunks (the last 1/16 of the merged positions; 1/8 until
        # late round 6, where these sweeps ran): small
        # enough for the blocks to finish together, large enough that a
        # chunk's fixed cost -- K model switches (weights, parked dW) and ring
        # flushes -- stays small.  Round 6, interleaved (profiles/r06/minchunk/):
        # C3 256 1182, 384 1189, 512 1188, 768 1179; C5 512 774, 1024 782,
        # 2048 780, 3072 789, 3584 786, 4096 781; C4 512 649, 640 648, 768 642,
        # 1024 651.5, 2048 623; the pinned rank 512 581, 1024 578, 2048 578.
        # (At C5 3072 leaves ~250 tail chunks, at most one per block; the
        # optimum moves with the step's size, so the rule holds from the
        # measured ray counts up.)
        self.min_chunk = 512
        if float(model.scale) > 0.5:
            if model.size >= 8 and n_rays >= 8192:
                # with the 1/16 tail: 1536 791 vs 3072 784 (profiles/r06/tail/)
                self.min_chunk = 1536
            # (K = 4: 1024 won with the 1/8 tail; with 1/16, 512: 658 vs 653)
        # hash levels whose grid gradient goes in by fp32 atomics instead of
        # fixed point (int32 or binned): () = none, every level an exact
        # integer sum (bitwise reproducible).  (3, ..., 8) at C3 brings the
        # per-entry 3-step Adam difference from fp32 from 1.1 % to 0.3 %
        # (levels 3-8 hold most of the int32 form's flushed entries) at the
        # cost of those levels' reproducibility (bench.py
        # --fx-f32-levels)
        self.fx_f32_levels = ()
        # head chunks: the first chunk of each block ramps from ~0 to
        # head_chunk merged samples (rn_bwd_plan), so the blocks' walks start
        # staggered instead of all after one full MLP phase.  Round 6
        # (profiles/r06/headramp/, interleaved): a ramp to max_chunk at scale
        # 0.5, C3 1183.4 -> 1189.2 M samples/s, C2 853.7 -> 862.3, C1 within
        # noise (then 256); at scale 16 a ramp to max_chunk / 2 cost C4 650 ->
        # 617 and C5 773 -> 762 (only ~2 big chunks per block, which get
        # shorter), so none there.  (Head chunks of one size, rounds 2 and 5,
        # changed nothing.)
        self.head_chunk = self.max_chunk if float(model.scale) <= 0.5 and rk > 1024 else 0
        # big chunks a multiple of the persistent blocks in number (rn_bwd_plan
        # balance_blocks): every block takes the same number of them
        self.balance_chunks = True
        # gate backward on this process (pinned.PinnedMLRenderer: rank 0 only),
        # and where: "field" side stream beside field_bwd, "early" side stream
        # beside composite_bw, "main" in line before field_bwd
        self.gate_grad_here = True
        # "early": beside composite_bw, before field_bwd's persistent blocks
        # occupy every CU (beside field_bwd it waited for them: its events
        # spanned 1.3-3.7 ms for a 0.09 ms kernel).  C3 step: early 5.037,
        # field 5.045, main 5.117 ms (tools/step_variants.py, r02)
        self.gate_bwd_at = "early"
        # input gradients (dL/drays_o, dL/drays_d) in backward(): set by
        # _MLRenderFn when the rays require grad (--optimize_ext)
        self.input_grad = False
        # called right after the merged field_bwd launch (stream order), when
        # the MLP gradient is final (data-parallel early all-reduce)
        self.after_field_bwd = None
        # called (stream order) when the grid gradient of levels
        # [grid_split_level, 16) -- the tail of the flat table, the fine hashed
        # levels -- is final, with grid_split_level as argument; the binned
        # fold then sums levels [0, grid_split_level), so a data-parallel
        # caller's collective of the fine levels overlaps it.  With the int32
        # fold (one short pass over every level) it is called with 0 after the
        # fold and the redo launch, when the whole table is final.
        self.after_grid_levels = None
        self.grid_split_level = 8
        # record HIP events around every launch (True) or the named ones (a set)
        self.trace = False
        self.events = {}

    def _ev(self, name, L_call, *args, stream=None):
        """Launch through librn; with tracing on (for this kernel), bracket it
        with events on the launch stream (bench.py's per-kernel timing)."""
        if not self.trace or (self.trace is not True and name not in self.trace):
            return L_call(*args)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        L_call(*args)
        b.record(stream)
        self.events.setdefault(name, []).append((a, b))

    def _ev_open(self, name):
        """start one event span over several launches (closed by _ev_close)"""
        if not self.trace or (self.trace is not True and name not in self.trace):
            return None
        a = torch.cuda.Event(enable_timing=True)
        a.record()
        return (name, a)

    def _ev_close(self, span):
        if span is not None:
            b = torch.cuda.Event(enable_timing=True)
            b.record()
            self.events.setdefault(span[0], []).append((span[1], b))

    def _side(self, dev):
        """Side stream for the gate MLP: it runs beside the march (forward) and
        beside field_bwd (backward), joined back before its outputs are used."""
        if getattr(self, "_side_stream", None) is None:
            self._side_stream = torch.cuda.Stream(dev)
        return self._side_stream

    def _f32_level_index(self, dev):
        key = (tuple(sorted(int(l) for l in self.fx_f32_levels)), str(dev))
        if getattr(self, "_f32_idx", (None,))[0] != key:
            if any(not 0 <= l < 16 for l in key[0]):
                raise ValueError(f"fx_f32_levels: hash levels are 0..15, got {key[0]}")
            self._f32_idx = (key, torch.tensor(key[0], dtype=torch.int64, device=dev))
        return self._f32_idx[1]

    def kernel_times_ms(self):
        """{kernel: [ms per launch]} of the traced launches (synchronises)."""
        torch.cuda.synchronize()
        return {k: [a.elapsed_time(b) for a, b in v] for k, v in self.events.items()}

    def bitfields(self):
        K = self.model.size
        bf = [getattr(self.model, f"density_bitfield_{i}") for i in range(K)]
        if all(b.data_ptr() == bf[0].data_ptr() + i * self.bitfield_bytes for i, b in enumerate(bf)):
            return bf[0]
        self._bf = torch.stack(bf).contiguous()
        return self._bf

    # ------------------------------------------------------------------ forward
    def forward(self, rays_o, rays_d, gate_in2, noise, bg, T_threshold=1e-4,
                exp_step_factor=0.0):
        m, g, w, L = self.model, self.gate, self.ws, lib()
        B, K, G = rays_o.shape[0], m.size, g.out_dim     # K rendered here, G gated
        assert B == w.B and noise.shape == (K, B)
        st = _stream(rays_o.device)
        out_gate = torch.empty(B, G, device=rays_o.device)
        imp = torch.zeros(G, device=rays_o.device)
        side = self._side(rays_o.device)
        main = torch.cuda.current_stream(rays_o.device)
        if G == 1:
            # softmax over one sub-NeRF is exactly 1 (and its gradient exactly
            # 0): single-NGP configs C1 / C2 skip the gate MLP
            out_gate.fill_(1.0)
            imp.fill_(float(B))
            side.wait_stream(main)
        else:
            frags = g.packed_frags()          # (re)packed on the main stream
            side.wait_stream(main)
            self._ev("gate_fwd", L.gate_fwd, rays_o.data_ptr(), gate_in2.data_ptr(), 3, B, G,
                     frags.data_ptr(), out_gate.data_ptr(), imp.data_ptr(),
                     max(1, min(256, (B + 127) // 128)), side.cuda_stream, stream=side)
        bits = self.bitfields()
        march = (rays_o.data_ptr(), rays_d.data_ptr(), m.center.data_ptr(),
                 m.half_size.data_ptr(), NEAR_DISTANCE, noise.data_ptr(), bits.data_ptr(),
                 self.bitfield_bytes, K, m.cascades, float(m.scale), float(exp_step_factor),
                 m.grid_size, MAX_SAMPLES, B)
        # single pass: march once into per-(model, ray) staging slots, scan the
        # counts, compact (the two-pass form re-marches every ray instead)
        self._ev("march", L.ml_march_count, *march, w.counts.data_ptr(),
                 w.stage_ts.data_ptr(), w.stage_dt.data_ptr(), st)
        self._ev("scan", L.scan_segments, w.counts.data_ptr(), K, B, SEG_ALIGN,
                 w.offsets.data_ptr(), w.seg_base.data_ptr(), w.seg_count.data_ptr(),
                 w.meta.data_ptr(), st)
        self._ev("compact", L.ml_compact, w.counts.data_ptr(), w.offsets.data_ptr(), B, K,
                 MAX_SAMPLES, w.stage_ts.data_ptr(), w.stage_dt.data_ptr(), w.ts.data_ptr(),
                 w.deltas.data_ptr(), w.ray_of.data_ptr(), st)
        if self.merged_bwd or self.merged_fwd:
            # the plan also writes the level forward's per-position input
            self._plan(st, rays_o, rays_d if self.level_fwd and self.plan_prep else None)
        self._field(True, rays_o, rays_d, st)
        self._ev("composite_fw", L.ml_composite_fw, w.sigma.data_ptr(), w.rgb.data_ptr(), w.deltas.data_ptr(),
                          w.ts.data_ptr(), w.counts.data_ptr(), w.offsets.data_ptr(), B, K,
                          float(T_threshold), w.used.data_ptr(), w.opacity_k.data_ptr(),
                          w.depth_k.data_ptr(), w.rgb_k.data_ptr(), w.ws.data_ptr(), st)
        # per-ray outputs of all G gated sub-NeRFs (here: the K rendered ones;
        # pinned.PinnedMLRenderer gathers them from every rank)
        ok, dk, rk = self._gather_model_outputs()
        rgb = torch.empty(B, 3, device=rays_o.device)
        opacity = torch.empty(B, device=rays_o.device)
        depth = torch.empty(B, G, device=rays_o.device)
        main.wait_stream(side)            # gate output joins here
        out_gate.record_stream(side)
        imp.record_stream(side)
        self._ev("combine_fw", L.ml_combine_fw, out_gate.data_ptr(), ok.data_ptr(), dk.data_ptr(),
                        rk.data_ptr(), bg.data_ptr(), B, G, rgb.data_ptr(),
                        opacity.data_ptr(), depth.data_ptr(), st)
        return rgb, opacity, depth, out_gate, imp

    def _gather_model_outputs(self):
        """(opacity, depth, rgb) per (sub-NeRF, ray) of every gated sub-NeRF,
        after this step's composite (forward)."""
        return self._model_outputs()

    def _model_outputs(self):
        """The same, as the forward left them (backward)."""
        w = self.ws
        return w.opacity_k, w.depth_k, w.rgb_k

    def _local_cols(self, x):
        """Columns of a (B, G) per-ray tensor that belong to the rendered sub-NeRFs."""
        return x

    def _plan(self, st, rays_o=None, rays_d=None):
        """Merged (ray, t) order + chunk schedule of this step's samples
        (rn_bwd_plan), shared by the merged forward and backward; with the
        rays (forward, level-partitioned encode) also the encode's
        per-position input, so rn_field_fwd_levels skips its prep pass."""
        w, L, m = self.ws, lib(), self.model
        prep = w.level_buffers(st)[1] if rays_d is not None else None
        self._min_chunk = min(self.min_chunk, self.max_chunk)
        head_n = self.merged_blocks if self.head_chunk else 0
        head = min(self.head_chunk, self.max_chunk)
        bal = self.merged_blocks if self.balance_chunks else 0
        self._cap_chunks, self._chunks = w.chunk_list(self.max_chunk, self._min_chunk, head_n, bal)
        self._ev("bwd_plan", L.bwd_plan, w.counts.data_ptr(), w.offsets.data_ptr(),
                 w.seg_base.data_ptr(), w.seg_count.data_ptr(), w.ts.data_ptr(), w.B, w.K,
                 head_n, head, self.max_chunk, self._min_chunk, bal, self._cap_chunks,
                 w.mstart.data_ptr(), w.perm.data_ptr(), self._chunks.data_ptr(),
                 w._chunk_desc.data_ptr(), w.queue.data_ptr(),
                 None if prep is None else rays_o.data_ptr(),
                 None if prep is None else rays_d.data_ptr(),
                 None if prep is None else m._h_min.ctypes.data,
                 None if prep is None else m._h_ext.ctypes.data,
                 None if prep is None else prep.data_ptr(), st)
        self._plan_key = (self.max_chunk, self._min_chunk, head_n, head, bal)
        self._prep_ready = prep is not None

    def _field(self, fwd, rays_o, rays_d, st, grid_grad=None, dw=None):
        m, w, L = self.model, self.ws, lib()
        lo, lh, lr, ls = m.xyz_encoder.level_ptrs()
        common = (None, None, 0, w.ts.data_ptr(), w.ray_of.data_ptr(), rays_o.data_ptr(),
                  rays_d.data_ptr(), w.seg_base.data_ptr(), w.seg_count.data_ptr(), m.size,
                  m.xyz_encoder.params_f16().data_ptr(), lo, lh, lr, ls, m._h_min.ctypes.data,
                  m._h_ext.ctypes.data, m.packed_frags().data_ptr())
        if fwd and self.level_fwd and (self.merged_bwd or self.merged_fwd):
            planes, prep = w.level_buffers(st)
            self._ev("field_fwd", L.field_fwd_levels, w.ts.data_ptr(), w.ray_of.data_ptr(),
                     rays_o.data_ptr(), rays_d.data_ptr(), w.seg_base.data_ptr(),
                     w.seg_count.data_ptr(), w.B, m.size, *common[10:], w.sigma.data_ptr(),
                     w.rgb.data_ptr(), w.feat.data_ptr(), w.mstart.data_ptr(), w.perm.data_ptr(),
                     planes.data_ptr(), planes.shape[1], prep.data_ptr(),
                     int(getattr(self, "_prep_ready", False)), self.level_enc_blocks,
                     self.level_mlp_blocks, None, st)
            self._prep_ready = False
        elif fwd and self.merged_fwd:
            self._ev("field_fwd", L.field_fwd_merged, w.ts.data_ptr(), w.ray_of.data_ptr(),
                     rays_o.data_ptr(), rays_d.data_ptr(), w.seg_base.data_ptr(),
                     w.seg_count.data_ptr(), w._chunk_desc.data_ptr(),
                     w.queue.data_ptr(), w.B, m.size, *common[10:], w.sigma.data_ptr(),
                     w.rgb.data_ptr(), w.feat.data_ptr() if self.feat_cache else None,
                     *((w.mstart.data_ptr(), w.perm.data_ptr())
                       if self.feat_cache and self.merged_encode else (None, None)),
                     self.merged_fwd_blocks, self.merged_fwd_threads, st)
        elif fwd:
            self._ev("field_fwd", L.field_fwd, *common, w.sigma.data_ptr(), w.rgb.data_ptr(),
                     w.feat.data_ptr() if self.feat_cache else None, self.fwd_blocks, st)
        elif self.merged_bwd:
            rows, scratch, park = w.bwd_scratch(self.merged_blocks, self.max_chunk)
            if getattr(self, "_plan_key", None) != (
                    self.max_chunk, min(self.min_chunk, self.max_chunk),
                    self.merged_blocks if self.head_chunk else 0,
                    min(self.head_chunk, self.max_chunk),
                    self.merged_blocks if self.balance_chunks else 0):
                self._plan(st)      # chunk sizes changed since the forward
            chunks = self._chunks
            ig = (None, None, None)
            fx = (None, None, None, None, 0)
            gb = (None, None, None, 0)
            use_fx = self.grid_fx and self.feat_cache and not self.int_grad
            use_bin = use_fx and self.grid_bin
            if use_fx:
                acc, scales, stats, redo = w.fx_buffers(grid_grad.numel(), grid_grad.device)
                cur, nxt = scales[w.fx_i], scales[1 - w.fx_i]
                if self.fx_f32_levels:
                    # these levels go in by fp32 atomics this step (a zero
                    # scale selects the kernel's per-level fp32 path)
                    cur.index_fill_(0, self._f32_level_index(cur.device), 0.0)
                n32 = max(0, min(16, int(self.bin_f32_levels))) if use_bin else 0
                if n32:
                    cur[:n32].zero_()           # binned mode: coarse levels by fp32 atomics
                fx = (acc.data_ptr(), cur.data_ptr(), stats.data_ptr(), None, 2)
            if use_bin:
                pool = self._bin_pool(w)
                # fx_mode 5: levels 0-7 (the walk's even streams) are fp32 by
                # construction, so that walk carries no page code for them
                fx = (None, cur.data_ptr(), stats.data_ptr(), None, 5 if n32 >= 8 else 4)
                gb = (pool["ctl"].data_ptr(), pool["meta"].data_ptr(), pool["recs"].data_ptr(),
                      pool["pages"])
            if self.int_grad:
                n_g = grid_grad.numel()
                if getattr(w, "_igrad", None) is None or w._igrad[0].numel() != n_g:
                    z = dict(device=grid_grad.device, dtype=torch.int32)
                    w._igrad = (torch.zeros(n_g, **z), torch.zeros(n_g, **z),
                                torch.ones(1, device=grid_grad.device),
                                torch.zeros(1, **z))
                lo, carry, scale, work = w._igrad
                self._ev("seed_scale", L.seed_scale, w.seg_base.data_ptr(),
                         w.seg_count.data_ptr(), m.size, w.sigma.data_ptr(), w.dsigma.data_ptr(),
                         w.drgb.data_ptr(), work.data_ptr(), scale.data_ptr(), st)
                ig = (lo.data_ptr(), carry.data_ptr(), scale.data_ptr())
            self._ev("field_bwd", L.field_bwd_merged, w.ts.data_ptr(), w.ray_of.data_ptr(),
                     rays_o.data_ptr(), rays_d.data_ptr(), w.seg_base.data_ptr(),
                     w.seg_count.data_ptr(), w.mstart.data_ptr(),
                     w.perm.data_ptr(), w._chunk_desc.data_ptr(), w.queue.data_ptr(), w.B, m.size,
                     MAX_SAMPLES,
                     *common[10:], w.dsigma.data_ptr(), w.drgb.data_ptr(), grid_grad.data_ptr(),
                     dw.data_ptr(), w.feat.data_ptr() if self.feat_cache else None,
                     scratch.data_ptr(), rows, park.data_ptr(), self.max_chunk,
                     self.merged_blocks, *ig, *fx, *gb, st)
            if self.after_field_bwd is not None:
                # the MLP gradient (dW) is final here; the grid gradient only
                # after the fold / bin + sum below: a data-parallel caller
                # starts the MLP / gate all-reduce now (bench.py)
                self.after_field_bwd()
            def fx_redo():
                # the fp32 redo of a flagged step's grid scatter: exits at once
                # unless the fold / check set the flag (no host synchronisation)
                self._ev("fx_redo", L.field_bwd_merged, w.ts.data_ptr(), w.ray_of.data_ptr(),
                         rays_o.data_ptr(), rays_d.data_ptr(), w.seg_base.data_ptr(),
                         w.seg_count.data_ptr(), w.mstart.data_ptr(),
                         w.perm.data_ptr(), w._chunk_desc.data_ptr(), w.queue.data_ptr(), w.B,
                         m.size, MAX_SAMPLES, *common[10:], w.dsigma.data_ptr(), w.drgb.data_ptr(),
                         grid_grad.data_ptr(), dw.data_ptr(), w.feat.data_ptr(),
                         scratch.data_ptr(), rows, park.data_ptr(), self.max_chunk,
                         self.merged_blocks, None, None, None, None, cur.data_ptr(), None,
                         redo.data_ptr(), 3, None, None, None, 0, st)

            if use_bin:
                # bin the pages and check the step (a record past e5m17's
                # range, a pool overflow or a refused input flags it for the
                # fp32 redo), run the redo launch (the sums exit when flagged,
                # so it can go first), then sum the fine levels, hand them to
                # after_grid_levels (their all-reduce overlaps the rest) and sum
                # the coarse levels
                span = self._ev_open("fx_bin")
                L.grid_bin_check(lh, pool["ctl"].data_ptr(), pool["meta"].data_ptr(),
                                 pool["recs"].data_ptr(), pool["recs"].data_ptr(),
                                 pool["desc"].data_ptr(), pool["lpages"].data_ptr(), pool["pages"],
                                 cur.data_ptr(), nxt.data_ptr(), stats.data_ptr(),
                                 redo.data_ptr(), st)
                self._ev_close(span)
                # the pages this backward took, read back without a sync
                # (_bin_pool reads it BIN_LAG backwards later)
                seen = self._bin_seen(w)
                # pool_next and the sum passes' sticky fault word (GbCtl)
                seen[0].copy_(pool["ctl"][:GB_CTL_READ], non_blocking=True)
                seen[1].record(torch.cuda.current_stream(grid_grad.device))
                fx_redo()
                span = self._ev_open("fx_sum")
                # a split of 16 would hand the whole grid over before any level
                # is summed: the cut lies in [0, 15]
                split = clamp_split(self.grid_split_level) if self.after_grid_levels else 0
                sums = ((split, 16), (0, split)) if split > 0 else ((0, 16),)
                for i, (l0, l1) in enumerate(sums):
                    L.grid_sum(lo, lh, pool["ctl"].data_ptr(), pool["desc"].data_ptr(),
                               pool["lpages"].data_ptr(), pool["recs"].data_ptr(), pool["pages"],
                               cur.data_ptr(), redo.data_ptr(), grid_grad.data_ptr(), l0, l1, st)
                    if i == 0 and split > 0:
                        self.after_grid_levels(split)
                self._ev_close(span)
                if split == 0 and self.after_grid_levels is not None:
                    self.after_grid_levels(0)
                w.fx_i ^= 1
            elif use_fx:
                # fold the fixed-point sums into grid_grad (or flag the step for
                # the fp32 redo), next step's scales; then the redo launch
                self._ev("fx_fold", L.grid_fx_fold, lo, lh, lr, acc.data_ptr(), cur.data_ptr(),
                         nxt.data_ptr(), stats.data_ptr(), redo.data_ptr(), grid_grad.data_ptr(),
                         st)
                fx_redo()
                if self.after_grid_levels is not None:
                    self.after_grid_levels(0)
                w.fx_i ^= 1
            if self.int_grad:
                self._ev("igrad_to_f32", L.igrad_to_f32, grid_grad.numel(), ig[0], ig[1], ig[2],
                         grid_grad.data_ptr(), st)
            if not (use_bin or use_fx) and self.after_grid_levels is not None:
                # fp32 atomics: final after field_bwd (int_grad: after its
                # conversion into grid_grad)
                self.after_grid_levels(0)
        else:
            self._ev("field_bwd", L.field_bwd, *common, w.dsigma.data_ptr(),
                     w.drgb.data_ptr(), grid_grad.data_ptr(), dw.data_ptr(),
                     w.feat.data_ptr() if self.feat_cache else None, self.bwd_blocks, st)

    # pool growth reads the page count of the binned backward this many
    # backwards back, waiting for it if needed (reading whichever
    # count had arrived made the pool size -- and so which steps after an
    # overflow were binned and which redone in fp32 -- depend on host timing)
    BIN_LAG = 2

    def _bin_seen(self, w):
        """the next of BIN_LAG + 1 pinned (count, event) slots, in turn"""
        ring = getattr(w, "_bin_ring", None)
        if ring is None:
            ring = w._bin_ring = [[torch.zeros(GB_CTL_READ, dtype=torch.int32, pin_memory=True),
                                   None, -1] for _ in range(self.BIN_LAG + 1)]
            w._bin_n = 0
        slot = ring[w._bin_n % len(ring)]
        slot[1] = torch.cuda.Event()
        slot[2] = w._bin_n
        w._bin_n += 1
        return slot

    def _bin_pool(self, w):
        """The page pool for this backward: sized from the records per (ray,
        sub-NeRF) at first, then grown when the binned backward BIN_LAG
        backwards back took more than 7/8 of it (its count, read back
        asynchronously, is waited for here: a function of the step sequence,
        not of how far the host runs ahead)."""
        lay = lib().bin_layout()
        b = getattr(w, "_bin", None)
        if b is None:
            # every wave keeps one page per level open (2 per wave of each
            # persistent block), so a step fills pages only partly at small sizes
            need = (-(-self.bin_records_per_pair * w.B * w.K // lay["page"]) +
                    2 * 8 * self.merged_blocks)
        else:
            need = b["pages"]
            ring = getattr(w, "_bin_ring", None)
            n = getattr(w, "_bin_n", 0) - self.BIN_LAG
            if ring is not None and n >= 0:
                slot = ring[n % len(ring)]
                if slot[2] == n and slot[1] is not None:
                    slot[1].synchronize()
                    if int(slot[0][GB_SUM_FAULT]) != 0:
                        raise RuntimeError(
                            "binned grid scatter: a sum pass refused a page run (GbCtl "
                            f"sum_fault {int(slot[0][GB_SUM_FAULT]):#x}) at or before the "
                            f"backward {self.BIN_LAG} steps back; that step's grid gradient "
                            "is incomplete (the page pool or its descriptors were corrupted)")
                    used = int(slot[0][0])
                    if used * 8 > need * 7:      # above 7/8: grow to 1.5x what was used
                        need = used * 3 // 2 + 64
        return w.bin_pool(need)

    # ----------------------------------------------------------------- backward
    def backward(self, rays_o, rays_d, gate_in2, gate, bg, dL_drgb, dL_dopacity, dL_ddepth,
                 dL_dgate_ext=None, T_threshold=1e-4, grid_grad=None, mlp_grad=None,
                 gate_grad=None):
        """Accumulates into grid_grad / mlp_grad / gate_grad (zero-initialised
        by the caller or allocated here) and returns them."""
        m, g, w, L = self.model, self.gate, self.ws, lib()
        B, K, G = rays_o.shape[0], m.size, g.out_dim
        dev = rays_o.device
        st = _stream(dev)
        grid_grad = torch.zeros_like(m.xyz_encoder.params) if grid_grad is None else grid_grad
        mlp_grad = torch.zeros_like(m.mlp_params) if mlp_grad is None else mlp_grad
        gate_grad = torch.zeros_like(g.params) if gate_grad is None else gate_grad
        ok, _, rk = self._model_outputs()
        dgate = self._dgate(B, G)
        self._ev("combine_bw", L.ml_combine_bw, dL_drgb.data_ptr(), dL_dopacity.data_ptr(),
                 ok.data_ptr(), rk.data_ptr(), bg.data_ptr(), B, G, dgate.data_ptr(), st)
        if dL_dgate_ext is not None:
            dgate.add_(dL_dgate_ext)
        side = self._side(dev)
        main = torch.cuda.current_stream(dev)

        gate_dx = self._gate_dinput(B, dev) if self.input_grad else None
        gate_dfr = g.packed_dinput_frags() if gate_dx is not None and G > 1 else None
        if gate_dx is not None and not self.gate_grad_here:
            gate_dx.zero_()             # no gate backward on this process

        def gate_bwd(stream):
            if G == 1:              # d softmax over one model = 0: nothing to add
                if gate_dx is not None:
                    gate_dx.zero_()
                return
            frags = g.packed_frags()
            if stream is side:
                side.wait_stream(main)
            self._ev("gate_bwd", L.gate_bwd, rays_o.data_ptr(), gate_in2.data_ptr(), 3, B, G,
                     frags.data_ptr(), dgate.data_ptr(), gate_grad.data_ptr(),
                     gate_grad.numel(), None if gate_dfr is None else gate_dfr.data_ptr(),
                     None if gate_dx is None else gate_dx.data_ptr(),
                     max(1, min(128, (B + 127) // 128)), stream.cuda_stream, stream=stream)

        # gate backward: it only needs dL/dgate (combine_bw)
        gate_at = self.gate_bwd_at if self.gate_grad_here else None
        if gate_at == "early":          # side stream, beside composite_bw
            gate_bwd(side)
        gate_k = self._local_cols(gate)
        ddepth_k = None if dL_ddepth is None else self._local_cols(dL_ddepth)
        self._ev("composite_bw", L.ml_composite_bw, dL_drgb.data_ptr(), dL_dopacity.data_ptr(),
                          None if ddepth_k is None else ddepth_k.data_ptr(), gate_k.data_ptr(),
                          bg.data_ptr(), w.sigma.data_ptr(), w.rgb.data_ptr(),
                          w.deltas.data_ptr(), w.ts.data_ptr(), w.counts.data_ptr(),
                          w.offsets.data_ptr(), w.opacity_k.data_ptr(), w.depth_k.data_ptr(),
                          w.rgb_k.data_ptr(), B, K, float(T_threshold), w.dsigma.data_ptr(),
                          w.drgb.data_ptr(), st)
        if gate_at == "field":          # side stream, beside field_bwd
            gate_bwd(side)
        elif gate_at == "main":         # in line, before field_bwd
            gate_bwd(main)
        self._field(False, rays_o, rays_d, st, grid_grad, mlp_grad)
        if self.input_grad:
            self._input_grads(rays_o, rays_d, st)
        if gate_at in ("early", "field"):
            main.wait_stream(side)
            gate_grad.record_stream(side)
            if gate_dx is not None:
                gate_dx.record_stream(side)
        return grid_grad, mlp_grad, gate_grad

    def _gate_dinput(self, B, dev):
        w = self.ws
        if getattr(w, "gate_dx", None) is None or w.gate_dx.shape[0] != B:
            w.gate_dx = torch.empty(B, 6, device=dev)
        return w.gate_dx

    def _input_grads(self, rays_o, rays_d, st):
        """dL/drays_o, dL/drays_d through the field and the march (the path
        --optimize_ext differentiates, train_ml.py:90-93): rn_field_dinput over
        the compact samples of all K sub-NeRFs, then rn_ml_march_bw sums each
        ray's samples (custom_functions.py:102-112).  The gate's own input
        gradient is in ws.gate_dx ((B, 6): rays_o | second gate input)."""
        m, w, L = self.model, self.ws, lib()
        if getattr(w, "dxyz", None) is None:
            w.dxyz = torch.empty(w.capacity, 3, device=w.device)
            w.ddir = torch.empty(w.capacity, 3, device=w.device)
            w.drays_o = torch.empty(w.B, 3, device=w.device)
            w.drays_d = torch.empty(w.B, 3, device=w.device)
        lo, lh, lr, ls = m.xyz_encoder.level_ptrs()
        self._ev("field_dinput", L.field_dinput, None, None, 0, w.ts.data_ptr(),
                 w.ray_of.data_ptr(), rays_o.data_ptr(), rays_d.data_ptr(),
                 w.seg_base.data_ptr(), w.seg_count.data_ptr(), m.size,
                 m.xyz_encoder.params_f16().data_ptr(), lo, lh, lr, ls, m._h_min.ctypes.data,
                 m._h_ext.ctypes.data, m.packed_frags().data_ptr(),
                 m.packed_dinput_frags().data_ptr(), w.dsigma.data_ptr(), w.drgb.data_ptr(),
                 w.feat.data_ptr() if self.feat_cache else None, w.dxyz.data_ptr(),
                 w.ddir.data_ptr(), self.fwd_blocks, st)
        self._ev("march_bw", L.ml_march_bw, w.counts.data_ptr(), w.offsets.data_ptr(), w.B, m.size,
                 w.ts.data_ptr(), w.dxyz.data_ptr(), w.ddir.data_ptr(), w.drays_o.data_ptr(),
                 w.drays_d.data_ptr(), st)

    def _dgate(self, B, G):
        return self.ws.dgate

    # --------------------------------------------------------------- train step
    def train_step(self, rays_o, rays_d, gate_in2, target_rgb, noise, bg, lambda_opacity=1e-3,
                   lambda_cv_importance=0.0, lambda_depth_mutual=0.0, T_threshold=1e-4,
                   exp_step_factor=0.0, grid_grad=None, mlp_grad=None, gate_grad=None):
        """render -> NeRFLoss -> backward of train_ml.py:179-192 as one launch
        chain: the fused loss kernel writes the backward seeds directly.
        Returns ({term: mean}, (grid_grad, mlp_grad, gate_grad)); gradients are
        accumulated into the given buffers (zero them first)."""
        from .losses import fused_nerf_loss
        rgb, opacity, depth, gate, imp = self.forward(rays_o, rays_d, gate_in2, noise, bg,
                                                      T_threshold, exp_step_factor)
        terms, (d_rgb, d_op, d_depth, d_gate) = fused_nerf_loss(
            rgb, target_rgb, opacity, depth, gate, imp, lambda_opacity, lambda_cv_importance,
            lambda_depth_mutual)
        grads = self.backward(rays_o, rays_d, gate_in2, gate, bg, d_rgb, d_op, d_depth, d_gate,
                              T_threshold, grid_grad, mlp_grad, gate_grad)
        return terms, grads


class _MLRenderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, grid_params, mlp_params, gate_params, renderer, rays_o, rays_d, gate_in2,
                noise, bg, T_threshold, esf):
        rgb, opacity, depth, gate, imp = renderer.forward(rays_o, rays_d, gate_in2, noise, bg,
                                                          T_threshold, esf)
        # the backward reads this step's samples from the renderer's workspace:
        # stamp it, so a second forward through the same workspace before this
        # backward is caught instead of silently differentiating the wrong step
        renderer.ws.generation += 1
        ctx.generation = renderer.ws.generation
        ctx.renderer = renderer
        ctx.save_for_backward(rays_o, rays_d, gate_in2, gate, bg)
        ctx.T = T_threshold
        return rgb, opacity, depth, gate

    @staticmethod
    def backward(ctx, d_rgb, d_op, d_depth, d_gate):
        rays_o, rays_d, gate_in2, gate, bg = ctx.saved_tensors
        if ctx.renderer.ws.generation != ctx.generation:
            raise RuntimeError(
                "ml_render_fused: the renderer's workspace was reused by another forward "
                "(same model, gate and batch size) before this backward; run the backward "
                "first, or render the other batch under torch.no_grad()")
        B, K = gate.shape
        dev = rays_o.device
        z = lambda *s: torch.zeros(*s, device=dev)
        d_rgb = z(B, 3) if d_rgb is None else d_rgb.float().contiguous()
        d_op = z(B) if d_op is None else d_op.float().contiguous()
        d_depth = None if d_depth is None else d_depth.float().contiguous()
        d_gate = None if d_gate is None else d_gate.float().contiguous()
        r = ctx.renderer
        need_o, need_d, need_2 = ctx.needs_input_grad[4:7]
        r.input_grad = bool(need_o or need_d or need_2)
        try:
            gg, mg, ag = r.backward(rays_o, rays_d, gate_in2, gate, bg, d_rgb, d_op, d_depth,
                                    d_gate, ctx.T)
        finally:
            input_grad, r.input_grad = r.input_grad, False
        do = dd = d2 = None
        if input_grad:
            w = r.ws
            do = w.drays_o + w.gate_dx[:, 0:3] if need_o else None
            dd = w.drays_d.clone() if need_d else None
            d2 = w.gate_dx[:, 3:6].contiguous() if need_2 else None
        return gg, mg, ag, None, do, dd, d2, None, None, None, None


class _GradNotSupported(torch.autograd.Function):
    """Identity on an output the fused chain computes but does not
    differentiate (independent_rgbs, render()'s ws): it stays on the autograd
    graph (anchored to a parameter), and a loss that reaches it raises at
    backward time instead of silently contributing no gradient."""

    @staticmethod
    def forward(ctx, x, anchor, what):
        ctx.what = what
        return x.clone()

    @staticmethod
    def backward(ctx, g, _g_anchor=None):
        raise RuntimeError(
            f"{ctx.what}: the fused training render does not back-propagate through this "
            "output; render with fused=False to differentiate it")


def grad_unsupported(x, anchors, what):
    """x as a graph output whose backward raises (see _GradNotSupported),
    anchored to the first of `anchors` (a tensor or a sequence of them) that
    requires grad; x itself (detached) when autograd is off or none does."""
    if torch.is_tensor(anchors):
        anchors = (anchors,)
    if torch.is_grad_enabled():
        for anchor in anchors:
            if anchor.requires_grad:
                return _GradNotSupported.apply(x, anchor, what)
    return x


_RENDERERS = collections.OrderedDict()
# a workspace holds 1024 sample slots per (ray, sub-NeRF) at ~124 B each (t, dt,
# ray, sigma, rgb, ws, their gradients, staging, the 64-B encoding cache, the
# merged order): ~0.13 GB per 1k rays x sub-NeRFs; the level-partitioned
# forward's planes (80 B per slot) and the binned scatter's page pool are
# shared per device and stream / sized to the records: keep a few workspaces
MAX_RENDERERS = 4


def get_renderer(model, gating_net, n_rays, grad=True):
    """The cached renderer (and workspace) of (model, gate, batch size).
    Renders without autograd (grad=False) get their own workspace, so a
    logging / validation render between a forward and its backward does not
    overwrite the samples the backward reads.  Least recently used entries
    beyond MAX_RENDERERS are dropped (their workspaces freed)."""
    key = (id(model), id(gating_net), n_rays, str(model.mlp_params.device), bool(grad))
    r = _RENDERERS.get(key)
    if r is None or r.model is not model or r.gate is not gating_net:
        r = FusedMLRenderer(model, gating_net, n_rays)
        _RENDERERS[key] = r
    _RENDERERS.move_to_end(key)
    while len(_RENDERERS) > MAX_RENDERERS:
        _RENDERERS.popitem(last=False)
    return r


def release_renderers():
    """Drop every cached renderer and its device workspace (and the shared
    forward scratch)."""
    _RENDERERS.clear()
    _LEVEL_SCRATCH.clear()


def ml_render_fused(model, gating_net, rays_o, rays_d, imgs_d, warmup=False, **kwargs):
    """Same result dict as ml_rendering.ml_render (train mode)."""
    rays_o, rays_d = rays_o.float().contiguous(), rays_d.float().contiguous()
    second = imgs_d.float().contiguous() if gating_net.type == "image" else rays_d
    B, K, dev = rays_o.shape[0], model.size, rays_o.device
    esf = float(kwargs.get("exp_step_factor", 0.0))
    noise = kwargs.get("noise")
    if noise is None:
        noise = torch.rand(K, B, device=dev)
    if esf == 0:
        bg = torch.ones(3, device=dev)
    elif kwargs.get("random_bg", False):
        bg = torch.rand(3, device=dev)
    else:
        bg = torch.zeros(3, device=dev)
    r = get_renderer(model, gating_net, B, grad=torch.is_grad_enabled())
    rgb, opacity, depth, gate = _MLRenderFn.apply(
        model.xyz_encoder.params, model.mlp_params, gating_net.params, r, rays_o, rays_d, second,
        noise.contiguous(), bg, float(kwargs.get("T_threshold", 1e-4)), esf)
    w = r.ws
    # each sub-NeRF's own colour (ml_rendering.py:65,73): values only -- a loss
    # on them raises at backward (the fused backward seeds the combined rgb)
    anchors = (model.mlp_params, model.xyz_encoder.params, gating_net.params)
    singles = [grad_unsupported(w.rgb_k[i] + bg * (1 - w.opacity_k[i])[:, None],
                                anchors, "ml_render independent_rgbs")
               for i in range(K)]
    return {"rgb": rgb, "independent_rgbs": singles, "depth": depth, "opacity": opacity,
            "gating_code": gate, "gating_importance": gate.sum(0)}
