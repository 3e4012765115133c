"""CPU, world_size 2 over gloo: the multi-GPU sharding of bench.py / nebula_amd.shard.

Each rank takes its contiguous shard of a (scaled) C5 IMIX batch, seals it with the oracle, and
the union of the shards must equal sealing the whole batch: rebased offsets, no packet lost or
duplicated, no exchange needed. The control plane (barrier, max of timings) runs over gloo.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    import oracle
    from nebula_amd import shard as S
    from nebula_amd import workload as W

    ctrl = S.Control(world)
    full = W.make_batch(1, 1000, 64, sizes=(90, 576, 1300), ratio=(7, 4, 1), name="dist")
    part = W.shard(full, rank, world)
    lo, hi = S.shard_range(full.n, rank, world)
    assert part.n == hi - lo
    st = oracle.batch(part.alg, 0, part.keys, part.desc, part.arena)
    assert (st == 0).all()
    dt = S.timed(ctrl, lambda: None)
    t_max = ctrl.max(float(rank + 1))
    n_sum = ctrl.sum(float(part.n))
    np.save(os.path.join(out, f"shard{rank}.npy"), part.arena)
    with open(os.path.join(out, f"meta{rank}.txt"), "w") as f:
        f.write(f"{lo} {hi} {t_max} {n_sum} {dt >= 0}")
    ctrl.dist.destroy_process_group()


def test_two_rank_shards_cover_batch_exactly(tmp_path, oracle_mod):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    from nebula_amd import workload as W

    full = W.make_batch(1, 1000, 64, sizes=(90, 576, 1300), ratio=(7, 4, 1), name="dist")
    ref = full.arena.copy()
    oracle_mod.batch(1, 0, full.keys, full.desc, ref)
    got = np.concatenate([np.load(tmp_path / f"shard{r}.npy") for r in range(world)])
    assert np.array_equal(got, ref)
    metas = [open(tmp_path / f"meta{r}.txt").read().split() for r in range(world)]
    assert int(metas[0][0]) == 0 and int(metas[0][1]) == int(metas[1][0]) and int(metas[1][1]) == full.n
    assert float(metas[0][2]) == float(metas[1][2]) == 2.0      # max over ranks
    assert float(metas[0][3]) == float(full.n)                   # sum of shard sizes


@pytest.mark.parametrize("n,world", [(65536, 8), (1 << 20, 8), (7, 4), (1, 2)])
def test_shard_ranges_tile(n, world):
    from nebula_amd.shard import shard_range

    prev = 0
    for r in range(world):
        lo, hi = shard_range(n, r, world)
        assert lo == prev and hi >= lo
        prev = hi
    assert prev == n
