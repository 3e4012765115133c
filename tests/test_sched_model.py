"""CPU: the mixed-key scheduler's chunk plan (tools/sched_model.py, rule for rule as
nebula_amd/csrc/sched.hpp / sched.hip) on the BASELINE configs' key and size mixes and on random
batches: every packet in exactly one chunk, one key and one size class per chunk, no chunk wider
than a wave, short classes never run at more lanes than they have blocks, the front and tail
ranges inside the workspace bounds the engine allocates (sched_max_chunks / sched_max_short), and
C3's lane utilisation as DESIGN.md §3.2 states it. The GPU tests check the ciphertexts these plans
produce (tests/test_gpu_parity.py); this pins the plan's own arithmetic."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)
import sched_model as M  # noqa: E402
from nebula_amd import workload as W  # noqa: E402


def _check(key_id, aad_len, length, max_keys, split_cls=M.SPLIT_TAIL_CLASS):
    n = len(key_id)
    chunks = M.plan(key_id, aad_len, length, max_keys, split_cls)
    seen = np.concatenate([c.packets for c in chunks]) if chunks else np.zeros(0, np.int64)
    assert np.array_equal(np.sort(seen), np.arange(n)), "every packet in exactly one chunk"
    cls = M.size_class(aad_len, length)
    key = np.where(key_id < max_keys, key_id, max_keys)
    nblk = M.blocks(aad_len, length)
    for c in chunks:
        assert (key[c.packets] == c.key).all() and (cls[c.packets] == c.cls).all()
        lpp = 1 << c.lg
        if c.kind == "front":
            assert c.lg == 2 and 1 <= len(c.packets) <= M.groups(c.cls) * M.CHUNK_PKTS
        else:
            assert c.lg in (3, 4) and 1 <= len(c.packets) * lpp <= M.WAVE
            assert c.kind == ("long" if M.tail_long(c.cls, c.lg) else "short")
            # capped for short classes: at 2**lg lanes the shortest class-cls packet has a block per lane
            assert (c.cls, c.lg) not in ((0, 3), (0, 4), (1, 4))
            assert nblk[c.packets].max() > lpp // 2 or c.cls == 0
    nfront = sum(c.kind == "front" for c in chunks)
    nlong = sum(c.kind == "long" for c in chunks)
    nshort = sum(c.kind == "short" for c in chunks)
    # the engine sizes the workspace for max(n, 64 Ki) packets (engine.cpp sched_reserve); the bound
    # must hold for n itself, so the fronts (from 0 up) never meet the long tails (from the top down)
    assert nfront + nlong <= M.max_chunks(n, max_keys)
    assert nshort <= M.max_short(n, max_keys)
    return chunks, nblk


@pytest.mark.parametrize("idx", [2, 4])
def test_baseline_mixed_configs(idx):
    """C3 (4096 keys, 64 Ki × 1300 B) and C5 (4096 keys, 1 Mi IMIX) at full size."""
    n, sizes, ratio = (65536, (1300,), (1,)) if idx == 2 else (1 << 20, (90, 576, 1300), (7, 4, 1))
    kid = W.key_ids(n, 4096)
    lens = W.payload_lens(n, sizes, ratio)
    aad = np.full(n, 16, np.uint32)
    chunks, nblk = _check(kid, aad, lens, 4096)
    if idx == 2:
        # C3: Poisson(16) packets per key; with the 8/16-lane tails 86.7% of the lane-rounds carry a
        # block; the round-4 split of 9-12 packet tails would make it 89.4%
        used = int(nblk.sum())
        spent = sum(M.lane_rounds(c, nblk) for c in chunks)
        assert abs(used / spent - 0.867) < 0.005
        fronts = sum(c.kind == "front" for c in chunks)
        tails = len(chunks) - fronts
        # ≈ 16 fronts and 7 tails per workgroup on 256 CUs (the wave timeline)
        assert 15 <= fronts / 256 <= 17 and 6 <= tails / 256 <= 8
        split, _ = _check(kid, aad, lens, 4096, split_cls=M.EXPERIMENT_SPLIT_CLASS)
        assert abs(used / sum(M.lane_rounds(c, nblk) for c in split) - 0.894) < 0.005


def test_random_batches():
    rng = np.random.default_rng(7)
    for _ in range(40):
        n = int(rng.integers(1, 3000))
        max_keys = int(rng.choice([1, 3, 17, 64, 300]))
        kid = rng.integers(0, max_keys + 2, n).astype(np.uint32)  # some keys outside the table
        length = rng.choice([0, 1, 15, 16, 17, 90, 576, 1300, 1500, 9000, 65000], n).astype(np.uint32)
        aad = rng.choice([0, 16, 1348], n, p=[0.1, 0.8, 0.1]).astype(np.uint32)
        _check(kid, aad, length, max_keys)


def test_bin_tail_shapes():
    """One bin of c packets, c = 1..40: c // 16 full groups, then a 9-15 packet tail as a partial
    4-lane group, a 5-8 packet tail at 8 lanes, a 1-4 packet tail at 16 (1300-B packets); with the
    experiment's split, a 9-12 packet tail as 8 packets at 8 lanes and the rest at 16."""
    for split_cls in (M.SPLIT_TAIL_CLASS, M.EXPERIMENT_SPLIT_CLASS):
        for c in range(1, 41):
            kid = np.zeros(c, np.uint32)
            chunks, _ = _check(kid, np.full(c, 16, np.uint32), np.full(c, 1300, np.uint32), 4, split_cls)
            t = c % 16
            lo = 13 if split_cls < 99 else 9
            front = [len(x.packets) for x in chunks if x.kind == "front"]
            back = [(len(x.packets), x.lg) for x in chunks if x.kind != "front"]
            assert sum(front) == c // 16 * 16 + (t if t >= lo else 0)
            if t == 0 or t >= lo:
                assert back == []
            elif t >= 9:
                assert back == [(8, 3), (t - 8, 4)]
            else:
                assert back == [(t, 4 if t <= 4 else 3)]
