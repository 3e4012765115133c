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


@pytest.mark.parametrize("world", [2, 3, 8])
def test_tunnel_shards_partition_batch(oracle_mod, world):
    """bench.py's default C5 sharding (`--shard-by key`, workload.shard_by_key): rank r takes the
    tunnels with key_id mod world == r. Every packet lands in exactly one shard, every tunnel's
    packets in one shard and in batch order, and sealing each shard with the oracle gives the
    bytes sealing the whole batch gives at those packets' slots (rebased offsets)."""
    from nebula_amd import workload as W

    full = W.make_batch(1, 1500, 37, sizes=(90, 576, 1300), ratio=(7, 4, 1), name="tunnels")
    ref = full.arena.copy()
    assert (oracle_mod.batch(1, 0, full.keys, full.desc, ref) == 0).all()
    ref_slots = ref.reshape(full.n, full.stride)
    seen = np.zeros(full.n, np.int64)
    for r in range(world):
        part = W.shard_by_key(full, r, world)
        idx = np.flatnonzero(full.desc["key_id"] % world == r)
        assert part.n == len(idx) and (part.desc["key_id"] % world == r).all()
        assert np.array_equal(part.desc["counter"], full.desc["counter"][idx])  # batch order kept
        seen[idx] += 1
        got = part.arena.copy()
        assert (oracle_mod.batch(1, 0, part.keys, part.desc, got) == 0).all()
        assert np.array_equal(got.reshape(part.n, part.stride), ref_slots[idx])
    assert (seen == 1).all()


@pytest.mark.parametrize("n,world", [(65536, 8), (1 << 20, 8), (7, 4), (1, 2)])
def test_shard_ranges_tile(n, world):
    from nebula_amd.shard import shard_range

    prev = 0
    for r in range(world):
        lo, hi = shard_range(n, r, world)
        assert lo == prev and hi >= lo
        prev = hi
    assert prev == n


def _run_bench(args, env_extra=None, timeout=240):
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *args], env=env, capture_output=True,
                       text=True, timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, (json.loads(lines[-1]) if lines else None), r.stderr


def test_bench_bare_gpus2_starts_two_ranks():
    """`python bench.py --gpus 2` with no launcher starts two rank processes itself (gloo control
    plane), and the one JSON line aggregates both ranks: n_gpus 2, the max of the ranks' times, the
    sum of their bytes, and per-GPU / aggregate bandwidth over both ranks' kernel times."""
    rc, res, err = _run_bench(["--gpus", "2", "--stub", "--steps", "3", "--warmup", "1"])
    assert rc == 0, err
    assert res["n_gpus"] == 2 and "rank processes" in res["launcher"]
    assert res["ms_per_step"] == pytest.approx(2.0)             # max over ranks: rank 1's 2 ms
    assert res["value"] == pytest.approx(2.0 / 0.002)           # 2 x 1 GiB over 2 ms
    pg, ag = res["roofline"]["per_gpu"], res["roofline"]["aggregate"]
    assert pg["ranks"] == 2 and pg["achieved_max"] == pytest.approx(1000.0) and pg["achieved_min"] == pytest.approx(500.0)
    assert ag["achieved"] == pytest.approx(1500.0) and ag["frac"] == pytest.approx(1500.0 / 16000.0, abs=1e-4)


def test_bench_bare_gpus4_starts_four_ranks():
    """The self-launch at world size 4 (the driver's 1-2-4-8 sweep, a stub worker per rank): n_gpus 4,
    the slowest rank's time, every rank's bytes and kernel bandwidth in the per-GPU min / max and the
    aggregate over 4 devices."""
    rc, res, err = _run_bench(["--gpus", "4", "--stub", "--steps", "2", "--warmup", "1"])
    assert rc == 0, err
    assert res["n_gpus"] == 4 and "4 rank processes" in res["launcher"]
    assert res["ms_per_step"] == pytest.approx(4.0)             # max over ranks: rank 3's 4 ms
    assert res["value"] == pytest.approx(4.0 / 0.004)           # 4 x 1 GiB over 4 ms
    pg, ag = res["roofline"]["per_gpu"], res["roofline"]["aggregate"]
    assert pg["ranks"] == 4 and pg["achieved_max"] == pytest.approx(1000.0) and pg["achieved_min"] == pytest.approx(250.0)
    assert ag["devices"] == 4 and ag["peak"] == pytest.approx(32000.0)
    assert ag["achieved"] == pytest.approx(1000.0 + 500.0 + 1000.0 / 3 + 250.0, abs=0.01)  # (rounded to 0.01)


def test_bench_under_launcher_env_runs_one_rank_per_process():
    """Under a launcher (WORLD_SIZE already set) bench.py is one rank and does not spawn; a lone
    rank with WORLD_SIZE=1 and --gpus 1 prints its own line."""
    rc, res, err = _run_bench(["--gpus", "1", "--stub"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc == 0, err
    assert res["n_gpus"] == 1 and "launcher" not in res


def test_bench_failed_rank_fails_the_run():
    """A rank that dies makes the whole run exit non-zero with no JSON line (never a one-GPU line
    for an N-GPU request)."""
    rc, res, err = _run_bench(["--gpus", "2", "--stub"], {"NEB_BENCH_STUB_FAIL": "1"})
    assert rc != 0 and res is None
