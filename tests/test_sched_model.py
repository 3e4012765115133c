"""CPU: the mixed-key scheduler's chunk plan (tools/sched_model.py, rule for rule as
nebula_amd/csrc/sched.hpp / sched_body.hpp) on the BASELINE configs' key and size mixes and on random
batches: every packet in exactly one chunk, one key per chunk, segment 0 of one size class and
segment 1 (packets riding in a leftover group's free slots) of a smaller class, no chunk wider than
a wave, short classes never run at more lanes than they have blocks, the chunks inside the
workspace bound the engine allocates (sched_max_chunks, and each cost bucket's capacity), the
buckets ordered longest first, and C3's lane utilisation as DESIGN.md §3.2 states it. The GPU tests
check the ciphertexts these plans produce (tests/test_gpu_parity.py); this pins the plan's own
arithmetic."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)
import sched_model as M  # noqa: E402
from nebula_amd import workload as W  # noqa: E402


def _check(key_id, aad_len, length, max_keys, max_groups=8):
    n = len(key_id)
    chunks = M.plan(key_id, aad_len, length, max_keys, max_groups)
    seen = np.concatenate([c.packets for c in chunks]) if chunks else np.zeros(0, np.int64)
    assert np.array_equal(np.sort(seen), np.arange(n)), "every packet in exactly one chunk"
    cls = M.size_class(aad_len, length)
    key = np.where(key_id < max_keys, key_id, max_keys)
    nblk = M.blocks(aad_len, length)
    for c in chunks:
        assert (key[c.packets] == c.key).all()
        seg0, seg1 = c.packets[:c.count0], c.packets[c.count0:]
        assert len(seg0) >= 1 and (cls[seg0] == c.cls).all()
        assert (cls[seg1] < c.cls).all(), "absorbed packets come from a smaller class"
        assert len(c.packets) <= 255 and len(seg1) <= 15  # the record's 8-bit counts
        lpp = 1 << c.lg
        if c.kind == "front":
            assert c.lg == 2 and 1 <= len(c.packets) <= M.groups(c.cls) * M.CHUNK_PKTS
            assert len(seg1) == 0 or len(c.packets) <= M.CHUNK_PKTS  # a leftover group only
        else:
            assert c.lg in (3, 4) and 1 <= len(c.packets) * lpp <= M.WAVE
            # capped for short classes: at 2**lg lanes the shortest class-cls packet has a block per lane
            assert (c.cls, c.lg) not in ((0, 3), (0, 4), (1, 4))
            assert nblk[seg0].max() > lpp // 2 or c.cls == 0
        # an absorbed packet needs no more rounds than segment 0's class allows at these lanes
        if len(seg1):
            assert ((nblk[seg1] + lpp - 1) // lpp).max() <= ((4 << c.cls) + lpp - 1) // lpp
    # the engine sizes the workspace for max(n, 64 Ki) packets (engine.cpp sched_reserve); the bound
    # must hold for n itself: all chunks, and so every bucket, within max_chunks
    assert len(chunks) <= M.max_chunks(n, max_keys)
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
        # block; one size class, so nothing is absorbed
        used = int(nblk.sum())
        spent = sum(M.lane_rounds(c, nblk) for c in chunks)
        assert abs(used / spent - 0.867) < 0.005
        fronts = sum(c.kind == "front" for c in chunks)
        tails = len(chunks) - fronts
        # ≈ 16 fronts and 7 tails per workgroup on 256 CUs (the wave timeline)
        assert 15 <= fronts / 256 <= 17 and 6 <= tails / 256 <= 8
        # longest first: the 21-round fronts, then 8-lane tails (11 rounds), then 16-lane (6)
        assert [c.bucket for c in chunks if c.kind == "front"] == [0] * fronts
        assert {(c.lg, c.bucket) for c in chunks if c.kind == "tail"} == {(3, 1), (4, 3)}


def test_c5_shard_absorbs_leftovers():
    """C5's 8-GPU shard (131 072 IMIX packets over 4096 keys, 32 per key): a key's leftover groups
    take the next smaller class's leftover packets, which removes chunks and lane-rounds against
    planning each (class, key) bin alone."""
    full = W.config(4, scale=1.0 / 8)
    d = full.desc
    chunks, nblk = _check(d["key_id"], d["aad_len"], d["len"], 4096)
    absorbed = sum(len(c.packets) - c.count0 for c in chunks)
    assert absorbed > 0.04 * len(d)
    spent = sum(M.lane_rounds(c, nblk) for c in chunks) // M.WAVE
    assert len(chunks) < 14000 and spent < 68000  # per-bin plans: 14 564 chunks, ≈ 73 000 wave-rounds


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
    """One bin of c packets, c = 1..40: c // 16 full groups, then a 9-15 packet leftover as a partial
    4-lane group, a 5-8 packet leftover at 8 lanes, a 1-4 packet leftover at 16 (1300-B packets)."""
    for c in range(1, 41):
        kid = np.zeros(c, np.uint32)
        chunks, _ = _check(kid, np.full(c, 16, np.uint32), np.full(c, 1300, np.uint32), 4)
        t = c % 16
        front = [len(x.packets) for x in chunks if x.kind == "front"]
        back = [(len(x.packets), x.lg) for x in chunks if x.kind != "front"]
        assert sum(front) == c // 16 * 16 + (t if t >= 9 else 0)
        if t == 0 or t >= 9:
            assert back == []
        else:
            assert back == [(t, 4 if t <= 4 else 3)]


def test_small_batch_front_groups():
    """Below NEB_KNOB_SMALL_BATCH packets per wave (C5's shard by tunnel: 512 keys, 256 packets each)
    every front chunk holds one group; the leftovers are planned as without the cap. (Here the tunnel
    shard of a 131 072-packet IMIX batch: 512 keys, 32 packets each.)"""
    d = W.shard_by_key(W.config(4, scale=1.0 / 8), 0, 8).desc
    plain, _ = _check(d["key_id"], d["aad_len"], d["len"], 4096)
    fine, _ = _check(d["key_id"], d["aad_len"], d["len"], 4096, max_groups=1)
    assert max(len(c.packets) for c in fine if c.kind == "front") == M.CHUNK_PKTS
    multi = sum(len(c.packets) // M.CHUNK_PKTS - 1 for c in plain if c.kind == "front" and c.count0 > M.CHUNK_PKTS)
    assert multi > 0 and len(fine) == len(plain) + multi


def test_leftover_absorption_rules():
    """3 large (1300 B) + 6 medium (576 B) + 2 small (90 B) packets of one key: the large leftover
    at 16 lanes takes 1 medium packet, the 5 remaining medium packets at 8 lanes take 3 small ones
    (the 2 there are), so the key runs 2 chunks instead of 3."""
    lens = np.array([1300] * 3 + [576] * 6 + [90] * 2, np.uint32)
    kid = np.zeros(len(lens), np.uint32)
    chunks, _ = _check(kid, np.full(len(lens), 16, np.uint32), lens, 4)
    shapes = sorted((c.cls, c.lg, c.count0, len(c.packets) - c.count0) for c in chunks)
    assert shapes == [(4, 3, 5, 2), (5, 4, 3, 1)]
