"""CPU: the merged backward's chunk schedule (field.hip chunk_plan, restated
on the host in test_gpu_ml._chunk_bounds) never needs more chunk slots than
include/radnerf.h's cap_chunks bound, which Workspace.chunk_list allocates
(the old bound lacked the tail that the last big chunk can leave
to min_chunk pieces, and k_bwd_chunks truncates silently past the cap)."""
import numpy as np

from test_gpu_ml import _chunk_bounds


def header_cap(total, head_n, max_chunk, min_chunk, blocks):
    return (head_n + total // max_chunk + total // (8 * min_chunk) + max_chunk // min_chunk + 3 +
            blocks)


def test_chunk_count_within_documented_cap():
    rng = np.random.default_rng(0)
    worst = 0.0
    for _ in range(3000):
        max_chunk = int(rng.choice([256, 512, 1024, 1536, 2560, 4096, 8192, 12288]))
        min_chunk = int(rng.choice([256, 512, 1024, 3072])) if max_chunk >= 512 else 256
        min_chunk = min(min_chunk, max_chunk)
        blocks = int(rng.choice([0, 37, 128, 256]))
        head = int(rng.choice([0, 256, 512]))
        head_n = blocks if head else 0
        total = int(rng.integers(0, 20_000_000)) if rng.random() < 0.5 else int(rng.integers(0, 40000))
        bounds, _, _, _ = _chunk_bounds(total, head_n, head, max_chunk, min_chunk, blocks)
        cap = header_cap(total, head_n, max_chunk, min_chunk, blocks)
        assert len(bounds) <= cap, (total, head_n, head, max_chunk, min_chunk, blocks, len(bounds), cap)
        worst = max(worst, len(bounds) / cap)
    assert worst > 0.5          # the bound is not vacuous
