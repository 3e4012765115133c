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
    from nebula_amd.batch import install_keys
    from nebula_amd.noiseutil import Engine

    engines = [Engine(0, max_keys=256) for _ in range(m)]
    ciphers = [install_keys(e, b) for e in engines]
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
