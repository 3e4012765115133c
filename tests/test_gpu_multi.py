"""GPU: one batch over several engines (contiguous packet shards, one host thread and
stream per engine, no collective) — in one process (neb_*_batch_host_multi, neb_*_batch_sharded;
two engines on the one GPU of the test box stand in for two GPUs) and in two processes (the
bench.py --gpus N layout, both ranks on the one GPU). The union of the shards must equal the oracle
over the whole batch, byte for byte."""
import os
import socket

import numpy as np
import pytest

from nebula_amd import _lib as L
from nebula_amd import workload as W

pytestmark = pytest.mark.gpu


def _engines_with_keys(b, m):
    from nebula_amd.batch import install_keys_multi
    from nebula_amd.noiseutil import Engine

    engines = [Engine(0, max_keys=256) for _ in range(m)]
    ciphers = install_keys_multi(engines, b)
    ids = [[c.key_id for c in cs] for cs in ciphers]
    assert all(x == ids[0] for x in ids), "keys must sit at the same key_ids on every engine"
    return engines, ciphers


def _close(engines, ciphers):
    for cs in ciphers:
        for c in cs:
            c.destroy()
    for e in engines:
        e.close()


@pytest.mark.parametrize("alg,nkeys", [(L.ALG_AESGCM, 1), (L.ALG_AESGCM, 37), (L.ALG_CHACHAPOLY, 37)])
def test_host_multi_two_engines_two_threads(oracle_mod, alg, nkeys):
    from nebula_amd.batch import PinnedBuffer, slot_desc
    from nebula_amd.shard import host_batch_multi

    b = W.make_batch(alg, 9001, nkeys, sizes=(90, 576, 1300), ratio=(7, 4, 1), seed=nkeys, name="multi")
    ref = b.arena.copy()
    assert (oracle_mod.batch(alg, 0, b.keys, b.desc, ref) == 0).all()
    engines, ciphers = _engines_with_keys(b, 2)
    buf = PinnedBuffer(b.arena.nbytes)
    try:
        d = slot_desc(b, ciphers[0])
        hint = d["key_id"][0] if nkeys == 1 else L.KEYS_MIXED
        for arena in (buf.array, b.arena.copy()):  # pinned (zero-copy) and pageable (staged)
            arena[:] = b.arena
            assert (host_batch_multi(engines, alg, False, d, arena, hint) == 0).all()
            assert np.array_equal(arena, ref)
            assert (host_batch_multi(engines, alg, True, d, arena, hint) == 0).all()
            exp = ref.copy()
            oracle_mod.batch(alg, 1, b.keys, b.desc, exp)
            assert np.array_equal(arena, exp)
    finally:
        buf.free()
        _close(engines, ciphers)


@pytest.mark.parametrize("m", [2, 3])
def test_sharded_device_batch(oracle_mod, m):
    import torch

    from nebula_amd.shard import ShardedDevice

    b = W.make_batch(L.ALG_AESGCM, 20000, 64, sizes=(90, 576, 1300), ratio=(7, 4, 1), seed=m, name="sharded")
    ref = b.arena.copy()
    assert (oracle_mod.batch(b.alg, 0, b.keys, b.desc, ref) == 0).all()
    engines, ciphers = _engines_with_keys(b, m)
    try:
        sd = ShardedDevice(engines, b, ciphers)
        sd.run(False)
        torch.cuda.synchronize()
        assert all((s == 0).all() for s in sd.statuses())
        assert np.array_equal(np.concatenate(sd.arenas()), ref)
        sd.run(True)
        exp = ref.copy()
        oracle_mod.batch(b.alg, 1, b.keys, b.desc, exp)
        assert np.array_equal(np.concatenate(sd.arenas()), exp)
    finally:
        _close(engines, ciphers)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch

    from nebula_amd import shard as S
    from nebula_amd import workload as W2
    from nebula_amd.batch import DeviceBatch, install_keys
    from nebula_amd.noiseutil import Engine

    ctrl = S.Control(world)
    full = W2.config(4, 1 / 64)  # C5's shape, scaled: each rank its contiguous shard
    part = W2.shard(full, rank, world)
    eng = Engine(0, 4096)
    cs = install_keys(eng, part)
    db = DeviceBatch(eng, part, cs)
    ctrl.barrier()
    db.seal()
    torch.cuda.synchronize()
    np.save(os.path.join(outdir, f"sealed{rank}.npy"), db.arena_host())
    np.save(os.path.join(outdir, f"status{rank}.npy"), db.status_host())
    ctrl.barrier()
    for c in cs:
        c.destroy()
    eng.close()


def test_two_processes_one_gpu_weak_shards(oracle_mod, tmp_path):
    """The bench.py --gpus N layout rehearsed on one GPU: two ranks (gloo control plane), each an
    engine sealing its contiguous shard of C5's IMIX shape; the shards' union equals the oracle."""
    import torch.multiprocessing as mp

    world = 2
    mp.spawn(_rank, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    full = W.config(4, 1 / 64)
    ref = full.arena.copy()
    assert (oracle_mod.batch(full.alg, 0, full.keys, full.desc, ref) == 0).all()
    got = np.concatenate([np.load(tmp_path / f"sealed{r}.npy") for r in range(world)])
    assert all((np.load(tmp_path / f"status{r}.npy") == 0).all() for r in range(world))
    assert np.array_equal(got, ref)


def _diverge(engines, ciphers, j, alg):
    """Engine 1's slot of key j destroyed and reinstalled with another key (it lands in the same
    slot): a tunnel whose key differs between engines, which the multi-engine calls must refuse."""
    from nebula_amd.noiseutil import CipherAESGCM, CipherChaChaPoly

    cf = CipherAESGCM if alg == L.ALG_AESGCM else CipherChaChaPoly
    slot = ciphers[1][j].key_id
    ciphers[1][j].destroy()
    ciphers[1][j] = cf.Cipher(engines[1], bytes(range(100, 132)))
    assert ciphers[1][j].key_id == slot
    return slot


@pytest.mark.parametrize("alg,nkeys", [(L.ALG_AESGCM, 1), (L.ALG_AESGCM, 37), (L.ALG_CHACHAPOLY, 37)])
def test_host_multi_diverged_key_is_bad_key(oracle_mod, alg, nkeys):
    """A key slot that holds another install on engine 1 than on engine 0: the packets of shard 1
    that use it get NEB_STATUS_BAD_KEY and stay untouched (never sealed with the other key); every
    other packet equals the oracle. Pinned (zero-copy) and pageable (staged) arenas."""
    from nebula_amd.batch import PinnedBuffer, slot_desc
    from nebula_amd.shard import host_batch_multi

    b = W.make_batch(alg, 4000, nkeys, sizes=(90, 576, 1300), ratio=(7, 4, 1), seed=5 + nkeys, name="fence")
    ref = b.arena.copy()
    assert (oracle_mod.batch(alg, 0, b.keys, b.desc, ref) == 0).all()
    engines, ciphers = _engines_with_keys(b, 2)
    buf = PinnedBuffer(b.arena.nbytes)
    try:
        j = 3 % nkeys
        slot = _diverge(engines, ciphers, j, alg)
        d = slot_desc(b, ciphers[0])
        hint = slot if nkeys == 1 else L.KEYS_MIXED
        n = len(d)
        bad = np.zeros(n, bool)
        bad[n // 2:] = b.desc["key_id"][n // 2:] == j  # shard 1 = the second half
        assert bad.any()
        rows = b.arena.reshape(n, b.stride)
        for arena in (buf.array, b.arena.copy()):
            arena[:] = b.arena
            st = host_batch_multi(engines, alg, False, d, arena, hint)
            assert (st[bad] == L.STATUS_BAD_KEY).all() and (st[~bad] == 0).all()
            # the call returned NEB_OK; the calling thread's last error says which engine was fenced
            assert L.lib().neb_last_error().decode().startswith("key fence: engine 1 ")
            got = arena.reshape(n, b.stride)
            assert np.array_equal(got[bad], rows[bad]), "a refused packet was touched"
            assert np.array_equal(got[~bad], ref.reshape(n, b.stride)[~bad])
    finally:
        buf.free()
        _close(engines, ciphers)


@pytest.mark.parametrize("nkeys", [1, 64])
def test_sharded_diverged_key_is_bad_key(oracle_mod, nkeys):
    import torch

    from nebula_amd.shard import ShardedDevice

    b = W.make_batch(L.ALG_AESGCM, 6000, nkeys, sizes=(90, 576, 1300), ratio=(7, 4, 1), seed=11, name="fence")
    ref = b.arena.copy()
    assert (oracle_mod.batch(b.alg, 0, b.keys, b.desc, ref) == 0).all()
    engines, ciphers = _engines_with_keys(b, 2)
    try:
        j = 5 % nkeys
        _diverge(engines, ciphers, j, b.alg)
        sd = ShardedDevice(engines, b, ciphers)
        sd.run(False)
        torch.cuda.synchronize()
        st = sd.statuses()
        n0 = len(st[0])
        bad1 = b.desc["key_id"][n0:] == j
        assert (st[0] == 0).all()
        assert (st[1][bad1] == L.STATUS_BAD_KEY).all() and (st[1][~bad1] == 0).all()
        a0, a1 = sd.arenas()
        assert np.array_equal(a0, ref[:a0.size])
        r1 = ref[a0.size:].reshape(-1, b.stride)
        g1 = a1.reshape(-1, b.stride)
        assert np.array_equal(g1[~bad1], r1[~bad1])
        assert np.array_equal(g1[bad1], b.arena[a0.size:].reshape(-1, b.stride)[bad1])
    finally:
        _close(engines, ciphers)


def test_host_multi_staged_overlapping_spans(oracle_mod):
    """Packed, unaligned packets (stride 1341 B, not a multiple of 16) with shuffled descriptors in a
    pageable arena: each shard's staged span covers bytes of the other's packets, so the shards must
    not copy their spans back over each other (they run one after another)."""
    from nebula_amd.batch import slot_desc
    from nebula_amd.shard import host_batch_multi

    alg = L.ALG_AESGCM
    b = W.make_batch(alg, 3000, 17, seed=21, name="packed")
    n, ln = b.n, 1300
    stride = 16 + ln + 16 + 9
    arena = np.zeros(n * stride + 7, np.uint8)
    src = b.arena.reshape(n, b.stride)
    base = 7 + np.arange(n, dtype=np.uint64) * np.uint64(stride)
    for i in range(n):
        o = int(base[i])
        arena[o:o + 16 + ln] = src[i, :16 + ln]
    d = b.desc.copy()
    d["aad_off"] = base
    d["src_off"] = base + np.uint64(16)
    d["dst_off"] = base + np.uint64(16)
    perm = np.random.default_rng(3).permutation(n)
    d = d[perm]
    ref = arena.copy()
    assert (oracle_mod.batch(alg, 0, b.keys, d, ref) == 0).all()
    engines, ciphers = _engines_with_keys(b, 2)
    try:
        dd = slot_desc(W.Batch(alg, b.keys, b.remote_index, d, arena, stride, "packed"), ciphers[0])
        a = arena.copy()
        assert (host_batch_multi(engines, alg, False, dd, a, L.KEYS_MIXED) == 0).all()
        assert np.array_equal(a, ref)
        assert (host_batch_multi(engines, alg, True, dd, a, L.KEYS_MIXED) == 0).all()
        exp = ref.copy()
        oracle_mod.batch(alg, 1, b.keys, d, exp)
        assert np.array_equal(a, exp)
    finally:
        _close(engines, ciphers)


def test_cipher_create_multi_all_or_nothing():
    """neb_cipher_create_multi takes the lowest slot free on every engine and reserves it on all."""
    from nebula_amd.noiseutil import CipherAESGCM, Engine

    engines = [Engine(0, max_keys=8) for _ in range(3)]
    try:
        a = CipherAESGCM.Cipher(engines[1], bytes(32))  # slot 0 taken on engine 1 only
        ms = CipherAESGCM.CipherMulti(engines, bytes(range(32)))
        assert [c.key_id for c in ms] == [1, 1, 1]
        with pytest.raises(L.NebError):
            CipherAESGCM.CipherMulti([engines[0], engines[0]], bytes(32))  # an engine twice
        fill = [CipherAESGCM.Cipher(engines[2], bytes([i] * 32)) for i in range(7)]  # engine 2 full
        with pytest.raises(L.NebError) as ei:
            CipherAESGCM.CipherMulti(engines, bytes(32))
        assert ei.value.rc == L.ERR_NO_KEY_SLOT
        assert sorted(c.key_id for c in CipherAESGCM.CipherBatch(engines[0], [bytes(32)] * 2)) == [0, 2]
        for c in [a] + ms + fill:
            c.destroy()
    finally:
        for e in engines:
            e.close()
