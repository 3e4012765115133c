"""GPU parity: the gfx950 kernels through the C ABI against the oracle, bit-exact.

Batches are the BASELINE.json configs (full C1; C2-C5 at sizes the oracle finishes in seconds),
the committed golden digests, edge shapes (empty payload / AAD, partial blocks, long AAD GMAC-only
relay, jumbo), failure semantics (tampered CT / tag / AAD / counter -> status 1 and zeroed payload,
exhausted counter -> status 2, wrong key -> status 3), and at full C2 size the size-independent
round-trip property seal -> open == identity with every tag distinct.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from nebula_amd import _lib as L
from nebula_amd import workload as W

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def run_device(engine, b, seal=True, arena=None, key_hint="auto", desc=None):
    from nebula_amd.batch import DeviceBatch, install_keys

    ciphers = install_keys(engine, b)
    try:
        db = DeviceBatch(engine, b, ciphers)
        if arena is not None:
            import torch
            db.arena.copy_(torch.from_numpy(arena))
        if desc is not None:
            import torch
            d = desc.copy()
            slots = np.array([c.key_id for c in ciphers], np.uint32)
            d["key_id"] = np.where(desc["key_id"] < len(slots), slots[np.minimum(desc["key_id"], len(slots) - 1)],
                                   desc["key_id"])
            db.desc.copy_(torch.from_numpy(d.view(np.uint8)))
        if key_hint != "auto":
            db.key_hint = key_hint
        (db.seal if seal else db.open)()
        import torch
        torch.cuda.synchronize()
        return db.arena_host(), db.status_host()
    finally:
        for c in ciphers:
            c.destroy()


def oracle_seal(oracle_mod, b, arena=None):
    a = (b.arena if arena is None else arena).copy()
    st = oracle_mod.batch(b.alg, 0, b.keys, b.desc, a)
    return a, st


def oracle_open(oracle_mod, b, arena):
    a = arena.copy()
    st = oracle_mod.batch(b.alg, 1, b.keys, b.desc, a)
    return a, st


@pytest.mark.parametrize("name", ["c1_aesgcm_1key_1024x1300", "c3_aesgcm_4096keys_512x1300",
                                  "c4_chachapoly_4096keys_512x1300", "c5_aesgcm_imix_4096keys_2048"])
def test_golden_batches(engine, name):
    import make_golden

    meta = json.load(open(os.path.join(GOLD, "batches.json")))[name]
    b = make_golden.BATCHES[name]()
    arena, st = run_device(engine, b, seal=True)
    assert (st == 0).all()
    assert hashlib.sha256(arena.tobytes()).hexdigest() == meta["sealed_sha256"]
    # and back
    opened, st2 = run_device(engine, b, seal=False, arena=arena)
    assert (st2 == 0).all()
    exp = b.arena.copy()
    slots_o, slots_e = opened.reshape(b.n, b.stride), exp.reshape(b.n, b.stride)
    for i in range(b.n):
        ln = int(b.desc["len"][i])
        assert np.array_equal(slots_o[i, :16 + ln], slots_e[i, :16 + ln])


@pytest.mark.parametrize("cfg,scale", [(1, 1 / 64), (2, 1 / 64), (3, 1 / 64), (4, 1 / 512)])
def test_configs_scaled_vs_oracle(engine, oracle_mod, cfg, scale):
    b = W.config(cfg, scale)
    ref, st_ref = oracle_seal(oracle_mod, b)
    got, st = run_device(engine, b, seal=True)
    assert (st == 0).all() and (st_ref == 0).all()
    assert np.array_equal(got, ref)
    ref_o, _ = oracle_open(oracle_mod, b, ref)
    got_o, st_o = run_device(engine, b, seal=False, arena=ref)
    assert (st_o == 0).all()
    assert np.array_equal(got_o, ref_o)


@pytest.mark.parametrize("alg,n,nkeys,sizes,ratio", [
    # C3's density (Poisson(16) packets per key): full 16-packet groups, 9-15 packet partial groups
    # and 8/16-lane tails, each key's chunk with the permuted final
    (L.ALG_AESGCM, 4096, 256, (1300,), (1,)),
    # IMIX with a few keys: bins of hundreds of packets, so the short classes run front chunks of
    # 4-8 groups one after another on one staging of the key's tables
    (L.ALG_AESGCM, 16384, 16, (90, 576, 1300), (7, 4, 1)),
    # every size class, both sides of each class boundary (1-128 blocks at 4 lanes per packet)
    (L.ALG_AESGCM, 6000, 24, (0, 1, 16, 17, 48, 49, 112, 113, 240, 241, 496, 497, 1008, 1009, 2032, 2033),
     (1,) * 16),
    (L.ALG_CHACHAPOLY, 4096, 256, (1300,), (1,)),
])
def test_mixed_key_density_vs_oracle(engine, oracle_mod, alg, n, nkeys, sizes, ratio):
    """Mixed-key batches at the densities where the chunk shapes differ (sched.hpp): the result is
    bit-exact against the oracle, seal and open."""
    b = W.make_batch(alg, n, nkeys, sizes=sizes, ratio=ratio, seed=n ^ nkeys, name="density")
    ref, st_ref = oracle_seal(oracle_mod, b)
    got, st = run_device(engine, b, seal=True)
    assert (st == 0).all() and (st_ref == 0).all()
    assert np.array_equal(got, ref)
    ref_o, _ = oracle_open(oracle_mod, b, ref)
    got_o, st_o = run_device(engine, b, seal=False, arena=ref)
    assert (st_o == 0).all()
    assert np.array_equal(got_o, ref_o)


# the three counting layouts of the mixed-key scheduler (sched.hip), forced by its per-batch knobs
# (NEB_KNOB_SUB_BINS_FROM, NEB_KNOB_TILE_BINS_FROM): one count word per bin, kSubBins words, or the
# per-tile LDS histograms with a scan over the tiles (4-21 tiles here; the engine's 8192 key slots
# make the 65 544-bin, 128 KiB-LDS case)
NEVER = 4000000000
BINNING = {"one_word": (NEVER, NEVER), "subbins": (0, NEVER), "tiles": (NEVER, 0)}


@pytest.mark.parametrize("path", sorted(BINNING))
@pytest.mark.parametrize("n,nkeys,sizes,ratio", [
    (4096, 256, (1300,), (1,)),
    (6000, 24, (0, 1, 16, 17, 48, 49, 112, 113, 240, 241, 496, 497, 1008, 1009, 2032, 2033), (1,) * 16),
    # IMIX over 1000 keys, 21 sub-bin workgroups' worth
    (21000, 1000, (90, 576, 1300), (7, 4, 1)),
])
def test_binning_paths_vs_oracle(engine, oracle_mod, knobs, path, n, nkeys, sizes, ratio):
    knobs(L.KNOB_SUB_BINS_FROM, BINNING[path][0])
    knobs(L.KNOB_TILE_BINS_FROM, BINNING[path][1])
    b = W.make_batch(L.ALG_AESGCM, n, nkeys, sizes=sizes, ratio=ratio, seed=n ^ nkeys ^ 0x5EED, name="binning")
    ref, st_ref = oracle_seal(oracle_mod, b)
    for rep in range(2):  # twice: each path leaves its counters and bins clear for the next batch
        got, st = run_device(engine, b, seal=True)
        assert (st == 0).all() and (st_ref == 0).all()
        assert np.array_equal(got, ref)
    ref_o, _ = oracle_open(oracle_mod, b, ref)
    got_o, st_o = run_device(engine, b, seal=False, arena=ref)
    assert (st_o == 0).all()
    assert np.array_equal(got_o, ref_o)


@pytest.mark.parametrize("max_keys", [1024, 4096])
def test_tile_binning_lds_rows_vs_oracle(oracle_mod, knobs, max_keys):
    """The tile binning (sched.hip) on engines with 1024 and 4096 key slots (8200 / 32 776 bins,
    against the shared 8192-slot engine's 65 544): the counting pass's per-tile LDS histogram at
    these sizes, the scan over the tiles, and the scatter reading each tile's bin offsets from its
    row of tpre in global memory. An IMIX batch over 1000 keys in 21 tiles, seal twice and open."""
    from nebula_amd import Engine

    knobs(L.KNOB_TILE_BINS_FROM, 0)
    e = Engine(0, max_keys=max_keys)
    try:
        b = W.make_batch(L.ALG_AESGCM, 21000, 1000, sizes=(90, 576, 1300), ratio=(7, 4, 1), seed=0x711E5,
                         name="tiles")
        ref, st_ref = oracle_seal(oracle_mod, b)
        for rep in range(2):
            got, st = run_device(e, b, seal=True)
            assert (st == 0).all() and (st_ref == 0).all()
            assert np.array_equal(got, ref)
        ref_o, _ = oracle_open(oracle_mod, b, ref)
        got_o, st_o = run_device(e, b, seal=False, arena=ref)
        assert (st_o == 0).all()
        assert np.array_equal(got_o, ref_o)
    finally:
        e.close()


def _edge_batch(alg, lens, alens, nkeys=3, seed=99):
    rng = np.random.default_rng(seed)
    n = len(lens)
    keys = rng.integers(0, 256, 32 * nkeys, dtype=np.uint8)
    offs, pos = [], 0
    for ln, al in zip(lens, alens):
        aad_off = pos
        src = (aad_off + al + 15) // 16 * 16
        offs.append((aad_off, src))
        pos = (src + ln + 16 + 63) // 64 * 64
    arena = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    desc = np.zeros(n, L.DESC_DTYPE)
    for i, ((a, s), ln, al) in enumerate(zip(offs, lens, alens)):
        desc[i] = (s, s, a, int(rng.integers(0, 2**63)), ln, al, i % nkeys, 0)
    return W.Batch(alg, keys, np.zeros(nkeys, np.uint32), desc, arena, 0, "edge")


EDGE_LENS = [0, 1, 15, 16, 17, 31, 32, 33, 63, 64, 65, 255, 256, 257, 1299, 1300, 1301, 4096, 9001]


@pytest.mark.parametrize("alg", [L.ALG_AESGCM, L.ALG_CHACHAPOLY])
def test_edge_shapes(engine, oracle_mod, alg):
    lens, alens = [], []
    for ln in EDGE_LENS:
        for al in (0, 1, 16, 17, 40):
            lens.append(ln)
            alens.append(al)
    # GMAC-only relay: empty payload, AAD = whole inner packet (connection_state.go:121-148)
    lens += [0, 0]
    alens += [1348, 9033]
    b = _edge_batch(alg, lens, alens)
    ref, _ = oracle_seal(oracle_mod, b)
    got, st = run_device(engine, b, seal=True)
    assert (st == 0).all()
    assert np.array_equal(got, ref)
    ref_o, _ = oracle_open(oracle_mod, b, ref)
    got_o, st_o = run_device(engine, b, seal=False, arena=ref)
    assert (st_o == 0).all()
    assert np.array_equal(got_o, ref_o)


@pytest.mark.parametrize("nkeys", [1, 2])
@pytest.mark.parametrize("lens", [[1300, 4064, 17], [4065, 1300], [1048545, 100], [1048544, 0]])
def test_counter_cache_tiers(engine, oracle_mod, nkeys, lens):
    """The AES-CTR round-1/2 caching tiers are chosen per wave by the largest block counter:
    below 2^8 (payload <= 4064 B), below 2^16 (<= 1048544 B), else the full cipher. Each batch
    puts packets on both sides of a boundary into one wave; nkeys 1 = single-key kernel,
    2 = the chunked mixed-key kernel."""
    b = _edge_batch(L.ALG_AESGCM, lens, [16] * len(lens), nkeys=nkeys, seed=len(lens) * 7 + lens[0])
    ref, _ = oracle_seal(oracle_mod, b)
    got, st = run_device(engine, b, seal=True)
    assert (st == 0).all()
    assert np.array_equal(got, ref)
    ref_o, _ = oracle_open(oracle_mod, b, ref)
    got_o, st_o = run_device(engine, b, seal=False, arena=ref)
    assert (st_o == 0).all()
    assert np.array_equal(got_o, ref_o)


@pytest.mark.parametrize("alg", [L.ALG_AESGCM, L.ALG_CHACHAPOLY])
def test_unaligned_offsets(engine, oracle_mod, alg):
    """Descriptors may point anywhere (Go slices): odd AAD / payload offsets, out-of-place."""
    rng = np.random.default_rng(5)
    n = 40
    keys = rng.integers(0, 256, 64, dtype=np.uint8)
    arena = rng.integers(0, 256, n * 3000, dtype=np.uint8)
    desc = np.zeros(n, L.DESC_DTYPE)
    for i in range(n):
        base = i * 3000
        ln = int(rng.integers(0, 1400))
        al = int(rng.integers(0, 40))
        a = base + int(rng.integers(0, 7))
        s = a + al + int(rng.integers(0, 5))
        dst = s if i % 2 else base + 1500 + int(rng.integers(0, 3))
        desc[i] = (s, dst, a, int(rng.integers(0, 2**63)), ln, al, i % 2, 0)
    b = W.Batch(alg, keys, np.zeros(2, np.uint32), desc, arena, 0, "unaligned")
    ref, _ = oracle_seal(oracle_mod, b)
    got, st = run_device(engine, b, seal=True)
    assert (st == 0).all()
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("alg,nkeys", [(L.ALG_AESGCM, 1), (L.ALG_AESGCM, 8), (L.ALG_CHACHAPOLY, 8)])
def test_aligned_dst_skewed_src(engine, oracle_mod, alg, nkeys):
    """Out-of-place with 16-byte aligned destinations and sources at every byte skew: whole waves of
    dword-aligned sources (one dwordx4 per block), whole waves of byte-skewed ones and mixed waves
    (two aligned blocks and a shift), as a TX segment's payload inside its TUN read is read."""
    rng = np.random.default_rng(17 + nkeys)
    n = 16 * 24
    keys = rng.integers(0, 256, 32 * nkeys, dtype=np.uint8)
    stride = 3072
    arena = rng.integers(0, 256, n * stride, dtype=np.uint8)
    desc = np.zeros(n, L.DESC_DTYPE)
    for i in range(n):
        w = i // 16
        skew = 0 if w < 4 else (4 * (w % 4) if w < 8 else (3 + 4 * (w % 3) if w < 12 else int(rng.integers(0, 16))))
        base = i * stride
        ln = int(rng.choice([1300, 1448, 577, 16, 15]))
        src = base + 32 + skew
        dst = base + 1536
        desc[i] = (src, dst, base, int(rng.integers(0, 2**62)), ln, 16, i % nkeys, 0)
    b = W.Batch(alg, keys, np.zeros(nkeys, np.uint32), desc, arena, 0, "skewed-src")
    ref, _ = oracle_seal(oracle_mod, b)
    got, st = run_device(engine, b, seal=True)
    assert (st == 0).all()
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("shift", [1, 4, 8])
@pytest.mark.parametrize("alg,nkeys", [(L.ALG_AESGCM, 1), (L.ALG_AESGCM, 16), (L.ALG_CHACHAPOLY, 16)])
def test_unaligned_arena_base(engine, oracle_mod, alg, nkeys, shift):
    """The device arena itself may start at any byte address (a torch view, a Go slice): aligned
    descriptor offsets then no longer mean aligned addresses, and the kernels must not take their
    16-byte vector fast paths on them."""
    import torch

    from nebula_amd.batch import DeviceBatch, install_keys

    b = W.make_batch(alg, 512, nkeys, sizes=(90, 576, 1300), ratio=(1, 1, 2), name="shifted")
    ciphers = install_keys(engine, b)
    try:
        db = DeviceBatch(engine, b, ciphers)
        big = torch.zeros(b.arena.nbytes + 16, dtype=torch.uint8, device=db.dev)
        db.arena = big[shift:shift + b.arena.nbytes]
        db.arena.copy_(torch.from_numpy(b.arena))
        assert db.arena.data_ptr() % 16 == shift % 16
        db.seal()
        torch.cuda.synchronize()
        ref, _ = oracle_seal(oracle_mod, b)
        assert (db.status_host() == 0).all()
        assert np.array_equal(db.arena_host(), ref)
        db.open()
        torch.cuda.synchronize()
        ref_o, _ = oracle_open(oracle_mod, b, ref)
        assert (db.status_host() == 0).all()
        assert np.array_equal(db.arena_host(), ref_o)
        assert not big[:shift].any() and not big[shift + b.arena.nbytes:].any()  # nothing outside
    finally:
        for c in ciphers:
            c.destroy()


@pytest.mark.parametrize("alg", [L.ALG_AESGCM, L.ALG_CHACHAPOLY])
def test_auth_failures_zero_payload_only(engine, oracle_mod, alg):
    b = W.make_batch(alg, 64, 4, name="tamper")
    sealed, _ = oracle_seal(oracle_mod, b)
    t = sealed.copy()
    d = b.desc
    victims = {3: "ct", 10: "tag", 17: "aad", 33: "ct-last-byte"}
    t[int(d["src_off"][3]) + 5] ^= 0x80
    t[int(d["src_off"][10]) + int(d["len"][10]) + 7] ^= 1
    t[int(d["aad_off"][17]) + 12] ^= 4
    t[int(d["src_off"][33]) + int(d["len"][33]) - 1] ^= 1
    desc = d.copy()
    desc["counter"][50] += 1  # wrong nonce
    victims[50] = "nonce"
    got, st = run_device(engine, b, seal=False, arena=t, desc=desc)
    exp_fail = sorted(victims)
    assert sorted(np.flatnonzero(st == L.STATUS_AUTH_FAILED).tolist()) == exp_fail
    assert (st[[i for i in range(64) if i not in victims]] == 0).all()
    for i in exp_fail:
        s, ln = int(d["src_off"][i]), int(d["len"][i])
        assert not got[s:s + ln].any(), victims[i]
        a = int(d["aad_off"][i])
        assert np.array_equal(got[a:a + 16], t[a:a + 16])          # header untouched
        assert np.array_equal(got[s + ln:s + ln + 16], t[s + ln:s + ln + 16])  # tag untouched
        nxt = a + b.stride
        assert np.array_equal(got[s + ln + 16:nxt], t[s + ln + 16:nxt])  # neighbour untouched


@pytest.mark.parametrize("alg", [L.ALG_AESGCM, L.ALG_CHACHAPOLY])
def test_exhausted_counter_and_bad_key(engine, oracle_mod, alg):
    b = W.make_batch(alg, 16, 2, name="ex")
    desc = b.desc.copy()
    desc["counter"][2] = L.REJECT_AFTER_MESSAGES
    desc["counter"][3] = L.REJECT_AFTER_MESSAGES - 1
    desc["key_id"][5] = 7000  # not installed
    got, st = run_device(engine, b, seal=True, desc=desc)
    assert st[2] == L.STATUS_EXHAUSTED and st[5] == L.STATUS_BAD_KEY
    assert (np.delete(st, [2, 5]) == 0).all()
    s = int(desc["src_off"][2])
    assert np.array_equal(got[s:s + 1316], b.arena[s:s + 1316])  # nothing written
    b2 = W.Batch(alg, b.keys, b.remote_index, desc, b.arena, b.stride, "ex")
    ref, _ = oracle_seal(oracle_mod, W.Batch(alg, b.keys, b.remote_index, desc[[3]], b.arena, b.stride, "x"))
    s3 = int(desc["src_off"][3])
    assert np.array_equal(got[s3:s3 + 1316], ref[s3:s3 + 1316])
    del b2


def test_key_hint_mismatch_flags_bad_key(engine):
    b = W.make_batch(L.ALG_AESGCM, 8, 2, name="hint")
    from nebula_amd.batch import DeviceBatch, install_keys
    import torch

    ciphers = install_keys(engine, b)
    try:
        db = DeviceBatch(engine, b, ciphers)
        db.key_hint = ciphers[0].key_id
        db.seal()
        torch.cuda.synchronize()
        st = db.status_host()
        kid = b.desc["key_id"]
        assert (st[kid == 0] == 0).all() and (st[kid == 1] == L.STATUS_BAD_KEY).all()
    finally:
        for c in ciphers:
            c.destroy()


def test_full_c2_roundtrip_property(engine):
    """Full 64 Ki x 1300 B (BASELINE configs[1]): open(seal(x)) == x, all tags distinct, and the
    sealed digest matches the oracle on a strided sample of packets."""
    import torch
    from nebula_amd.batch import DeviceBatch, install_keys

    b = W.config(1)
    ciphers = install_keys(engine, b)
    try:
        db = DeviceBatch(engine, b, ciphers)
        db.seal()
        torch.cuda.synchronize()
        assert (db.status_host() == 0).all()
        sealed = db.arena_host()
        tags = sealed.reshape(b.n, b.stride)[:, 16 + 1300:32 + 1300]
        assert len({t.tobytes() for t in tags}) == b.n
        db.open()
        torch.cuda.synchronize()
        assert (db.status_host() == 0).all()
        opened = db.arena_host().reshape(b.n, b.stride)
        assert np.array_equal(opened[:, :16 + 1300], b.arena.reshape(b.n, b.stride)[:, :16 + 1300])
    finally:
        for c in ciphers:
            c.destroy()
    import oracle

    idx = np.arange(0, b.n, 257)
    sub = W.Batch(b.alg, b.keys, b.remote_index, b.desc[idx], b.arena, b.stride, "sample")
    ref = b.arena.copy()
    oracle.batch(sub.alg, 0, sub.keys, sub.desc, ref)
    s2, r2 = sealed.reshape(b.n, b.stride), ref.reshape(b.n, b.stride)
    assert np.array_equal(s2[idx], r2[idx])


@pytest.mark.parametrize("extra", [1, 37, 4 * 16 * 64 + 5, 30001])
def test_single_key_partial_last_pass(engine, oracle_mod, extra):
    """One key, a batch just past one pass of the single-key kernel's waves (64 Ki packets on one
    MI355X): the packets of the partial last pass go to the tail kernel (64 lanes per packet, a grid
    of at most two workgroups per CU striding over them: 30001 takes 8 strides). Every
    packet, ragged sizes, sealed and opened, bit-exact against the oracle."""
    import torch
    from nebula_amd.batch import DeviceBatch, install_keys

    n = 65536 + extra
    b = W.make_batch(L.ALG_AESGCM, n, 1, sizes=(0, 1, 16, 17, 95, 130, 257), ratio=(1, 1, 1, 1, 2, 2, 1),
                     seed=97 + extra, name="tail")
    ref, _ = oracle_seal(oracle_mod, b)
    ciphers = install_keys(engine, b)
    try:
        db = DeviceBatch(engine, b, ciphers)
        db.seal()
        torch.cuda.synchronize()
        assert (db.status_host() == 0).all()
        assert np.array_equal(db.arena_host(), ref)
        db.open()
        torch.cuda.synchronize()
        assert (db.status_host() == 0).all()
        ref_o, _ = oracle_open(oracle_mod, b, ref)
        assert np.array_equal(db.arena_host(), ref_o)
    finally:
        for c in ciphers:
            c.destroy()


@pytest.mark.parametrize("arena_kind", ["pinned", "pageable"])
@pytest.mark.parametrize("alg", [L.ALG_AESGCM, L.ALG_CHACHAPOLY])
def test_host_pipeline_matches_device(engine, oracle_mod, alg, arena_kind):
    """neb_*_batch_host: a pinned arena runs zero-copy (the kernels on host memory), a pageable one
    through the staged H2D -> kernel -> D2H pipeline; both equal the oracle byte for byte."""
    from nebula_amd.batch import PinnedBuffer, host_batch, install_keys, slot_desc

    b = W.make_batch(alg, 20000, 64, sizes=(90, 576, 1300), ratio=(7, 4, 1), name="host")
    ciphers = install_keys(engine, b)
    buf = None
    try:
        d = slot_desc(b, ciphers)
        if arena_kind == "pinned":
            buf = PinnedBuffer(b.arena.nbytes)
            arena = buf.array
            arena[:] = b.arena
        else:
            arena = b.arena.copy()
        st = host_batch(engine, alg, False, d, arena)
        assert (st == 0).all()
        ref, _ = oracle_seal(oracle_mod, b)
        assert np.array_equal(arena, ref)
        st = host_batch(engine, alg, True, d, arena)
        assert (st == 0).all()
        ref_o, _ = oracle_open(oracle_mod, b, ref)
        assert np.array_equal(arena, ref_o)
    finally:
        if buf is not None:
            buf.free()
        for c in ciphers:
            c.destroy()


@pytest.mark.parametrize("mode", ["zc", "dma"])
def test_host_modes_shuffled_descriptors(engine, oracle_mod, mode, knobs):
    """Both host paths (zero-copy, hipMemcpyAsync staging) on a pinned arena with
    the descriptors in random order: pipeline chunks then cover overlapping arena spans, which the
    engine must retire in order (each chunk copies its whole span back). Also an arena that starts
    one byte past a 16-byte boundary (the kernels touch only aligned host arenas: DMA staging)."""
    from nebula_amd.batch import PinnedBuffer, host_batch, install_keys, slot_desc

    knobs(L.KNOB_HOST_MODE, 1 if mode == "dma" else 0)
    b = W.make_batch(L.ALG_AESGCM, 20000, 64, sizes=(90, 576, 1300), ratio=(7, 4, 1), name="shuffled")
    ciphers = install_keys(engine, b)
    buf = PinnedBuffer(b.arena.nbytes + 16)
    try:
        d = slot_desc(b, ciphers)
        perm = np.random.default_rng(7).permutation(b.n)
        dp = d[perm]
        ref, _ = oracle_seal(oracle_mod, b)
        ref_o, _ = oracle_open(oracle_mod, b, ref)
        for shift in (0, 1):
            arena = buf.array[shift:shift + b.arena.nbytes]
            arena[:] = b.arena
            st = host_batch(engine, b.alg, False, dp, arena)
            assert (st == 0).all()
            assert np.array_equal(arena, ref), (mode, shift)
            st = host_batch(engine, b.alg, True, dp, arena)
            assert (st == 0).all()
            assert np.array_equal(arena, ref_o), (mode, shift)
    finally:
        buf.free()
        for c in ciphers:
            c.destroy()


def test_host_zero_copy_rejects_out_of_bounds(engine):
    """A descriptor past the pinned arena is refused before any kernel touches host memory."""
    from nebula_amd.batch import PinnedBuffer, host_batch, install_keys, slot_desc

    b = W.make_batch(L.ALG_AESGCM, 64, 1, name="oob")
    ciphers = install_keys(engine, b)
    buf = PinnedBuffer(b.arena.nbytes)
    try:
        buf.array[:] = b.arena
        d = slot_desc(b, ciphers)
        d["len"][-1] = b.stride * 4  # runs past the end of the arena
        with pytest.raises(Exception):
            host_batch(engine, b.alg, False, d, buf.array)
        assert np.array_equal(buf.array, b.arena)  # nothing was written
    finally:
        buf.free()
        for c in ciphers:
            c.destroy()


WRAP = 2**64 - 16  # an offset whose sum with any length wraps around 2^64


@pytest.mark.parametrize("mode", ["zc", "dma"])
@pytest.mark.parametrize("case", ["src_wrap", "dst_wrap", "aad_wrap", "past_end"])
def test_host_rejects_invalid_descriptor_untouched(engine, mode, case, knobs):
    """A host batch with one bad descriptor — an offset near 2^64 whose end wraps around, or a
    length past the arena — is refused before anything is copied or launched, in every host mode.
    The bad descriptor is the last of a 20000-packet batch, so the staged modes would otherwise
    have sealed their first chunks in place already."""
    from nebula_amd.batch import PinnedBuffer, host_batch, install_keys, slot_desc

    knobs(L.KNOB_HOST_MODE, 1 if mode == "dma" else 0)
    b = W.make_batch(L.ALG_AESGCM, 20000, 4, sizes=(90, 576, 1300), ratio=(7, 4, 1), name="wrap")
    ciphers = install_keys(engine, b)
    buf = PinnedBuffer(b.arena.nbytes)
    try:
        buf.array[:] = b.arena
        d = slot_desc(b, ciphers)
        if case == "past_end":
            d["len"][-1] = b.stride * 4
        else:
            d[case.split("_")[0] + "_off"][-1] = WRAP
        for open_ in (False, True):
            with pytest.raises(Exception):
                host_batch(engine, b.alg, open_, d, buf.array)
            assert np.array_equal(buf.array, b.arena), (mode, case, open_)
    finally:
        buf.free()
        for c in ciphers:
            c.destroy()


@pytest.mark.parametrize("cfg", [1, 2])
def test_cipher_destroy_waits_for_queued_batches(engine, oracle_mod, cfg):
    """neb_cipher_destroy right after an asynchronous seal was enqueued behind other work on the
    caller's stream: the batch still runs with the installed key (destroy waits for it), so the
    output equals the oracle; the slot is free afterwards. Single key (its key-use event bound to
    the batch's last kernel) and mixed keys (the scheduler workspace's event)."""
    import torch

    from nebula_amd.batch import DeviceBatch, install_keys

    b = W.config(cfg, 1 / 16)
    ref, _ = oracle_seal(oracle_mod, b)
    ciphers = install_keys(engine, b)
    db = DeviceBatch(engine, b, ciphers)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        x = torch.randn(4096, 4096, device="cuda")
        for _ in range(8):  # a few ms of work ahead of the seal on the same stream
            x = x @ x
            x = x / x.norm()
        db.seal(stream=s.cuda_stream)
    slot = ciphers[0].key_id
    ciphers[0].destroy()
    s.synchronize()
    assert (db.status_host() == 0).all()
    assert np.array_equal(db.arena_host(), ref)
    from nebula_amd.noiseutil import CipherAESGCM
    again = CipherAESGCM.Cipher(engine, bytes(range(32)))  # the freed slot is handed out again
    try:
        assert again.key_id == slot
    finally:
        again.destroy()
        for c in ciphers[1:]:
            c.destroy()


@pytest.mark.parametrize("alg,nkeys", [(L.ALG_AESGCM, 1), (L.ALG_AESGCM, 64), (L.ALG_CHACHAPOLY, 64)])
def test_relay_gmac_batches(engine, oracle_mod, alg, nkeys):
    """GMAC-only relay packets (VerifyRelay, connection_state.go:121-148; the relay seal at
    inside.go:491): every wave is AAD-only, so the kernels skip the AES in all rounds but the
    length block's (E_K(J0)); ChaCha20-Poly1305 relay packets are Poly1305 over the AD. A pure
    relay batch, then relay packets mixed into ordinary ones
    (waves where some lanes need keystream), sealed and opened bit-exact against the oracle; a
    flipped AD bit fails only its own packet."""
    rb = W.relay_batch(alg, 3000, nkeys, seed=314)
    ref, _ = oracle_seal(oracle_mod, rb)
    got, st = run_device(engine, rb, seal=True)
    assert (st == 0).all()
    assert np.array_equal(got, ref)
    ref_o, _ = oracle_open(oracle_mod, rb, ref)
    got_o, st_o = run_device(engine, rb, seal=False, arena=ref)
    assert (st_o == 0).all()
    assert np.array_equal(got_o, ref_o)
    bad = ref.copy()
    bad[int(rb.desc["aad_off"][17]) + 700] ^= 0x10
    _, st_b = run_device(engine, rb, seal=False, arena=bad)
    assert st_b[17] == L.STATUS_AUTH_FAILED and (np.delete(st_b, 17) == 0).all()
    # mixed: relay and 1300-B packets interleaved in one batch
    lens = [1300 if i % 3 else 0 for i in range(600)]
    alens = [16 if i % 3 else 1348 for i in range(600)]
    mb = _edge_batch(alg, lens, alens, nkeys=nkeys, seed=316)
    ref, _ = oracle_seal(oracle_mod, mb)
    got, st = run_device(engine, mb, seal=True)
    assert (st == 0).all()
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("name", ["c2_full", "c3_full", "c4_full", "c5_full"])
def test_full_size_batches_match_oracle_digests(engine, name):
    """Every BASELINE.json GPU config at full size (C2/C3/C4: 64 Ki x 1300 B, 1 and 4096 keys, both
    ciphers; C5: 1 Mi IMIX packets over 4096 keys on one GPU): the whole sealed arena and the whole
    opened arena hash to the digests the plain-C oracle and OpenSSL EVP agreed on
    (tests/golden/full_digests.json, make_golden.py). Seal and open through the device batch path."""
    import hashlib
    import time

    import torch
    from nebula_amd.batch import DeviceBatch, install_keys
    import make_golden

    meta = json.load(open(os.path.join(GOLD, "full_digests.json")))[name]
    t0 = time.time()
    b = make_golden.FULL[name]()
    assert (b.n, b.nkeys, b.alg, b.stride) == (meta["n"], meta["nkeys"], meta["alg"], meta["stride"])
    assert hashlib.sha256(b.arena.tobytes()).hexdigest() == meta["plain_sha256"]
    ciphers = install_keys(engine, b)
    try:
        db = DeviceBatch(engine, b, ciphers)
        db.seal()
        torch.cuda.synchronize()
        assert (db.status_host() == 0).all()
        assert hashlib.sha256(db.arena_host().tobytes()).hexdigest() == meta["sealed_sha256"]
        db.open()
        torch.cuda.synchronize()
        assert (db.status_host() == 0).all()
        assert hashlib.sha256(db.arena_host().tobytes()).hexdigest() == meta["opened_sha256"]
    finally:
        for c in ciphers:
            c.destroy()
    print(f"{name}: {b.n} packets, {time.time() - t0:.1f} s")


_C5 = {}


@pytest.mark.parametrize("by,rank", [("key", 0), ("range", 7)])
def test_c5_gpu_shard_vs_oracle(engine, oracle_mod, by, rank):
    """One GPU's part of C5 over 8 GPUs at full size (131 072 IMIX packets): the tunnels with
    key_id mod 8 = rank (the bench's split: 512 keys, ≈ 256 packets each, one 16-packet group per
    front chunk below NEB_KNOB_SMALL_BATCH) and the contiguous range (4096 keys, 32 each: leftover
    groups taking smaller classes' packets). Sealed arena byte for byte against the oracle, opened
    back to the plaintext. (The byte-serial oracle takes ≈ 20 s per shard.)"""
    if "b" not in _C5:
        _C5["b"] = W.config(4)
    b = (W.shard_by_key if by == "key" else W.shard)(_C5["b"], rank, 8)
    assert 120000 < b.n < 142000
    ref, st_ref = oracle_seal(oracle_mod, b)
    got, st = run_device(engine, b, seal=True)
    assert (st == 0).all() and (st_ref == 0).all()
    assert np.array_equal(got, ref)
    opened, st_o = run_device(engine, b, seal=False, arena=got)
    assert (st_o == 0).all()
    used = np.arange(b.stride)[None, :] < 16 + b.desc["len"][:, None].astype(np.int64)  # header + payload
    assert np.array_equal(opened.reshape(b.n, b.stride)[used], b.arena.reshape(b.n, b.stride)[used])
