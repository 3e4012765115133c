"""GPU: the batched receive path (neb_rx_open_batch_host — ConnectionState.Decrypt over a whole
recvmmsg flush, connection_state.go:99-119) against the oracle's packet-by-packet receive loop
(oracle/replay_oracle.py rx_sequential + oracle AEAD): statuses, every arena byte (refused packets
untouched, forged ones zeroed, accepted ones decrypted in place), window state and counters."""
import contextlib
import os
import random

import numpy as np
import pytest

from nebula_amd import _lib as L

pytestmark = pytest.mark.gpu

SLOT = 16 + 1400 + 16


def _build(oracle_mod, alg, keys, arrivals, seed, lens=None):
    """arrivals: [(tunnel, counter, forged)] -> (arena, desc (tunnel index in key_id), payloads)."""
    rng = random.Random(seed)
    lens = lens or [0, 1, 15, 16, 17, 100, 576, 1300, 1400]
    n = len(arrivals)
    arena = np.zeros(n * SLOT, np.uint8)
    desc = np.zeros(n, dtype=L.DESC_DTYPE)
    pts = []
    for i, (t, ctr, forged) in enumerate(arrivals):
        ln = rng.choice(lens) if i % 5 else lens[-2]
        pt = bytes(rng.getrandbits(8) for _ in range(ln))
        hdr = oracle_mod.header_encode(1, 1, 0, 0x1000 + t, ctr)
        ct = bytearray(oracle_mod.seal(alg, keys[t], oracle_mod.nonce(alg, ctr), hdr, pt))
        if forged:
            ct[rng.randrange(len(ct))] ^= 1 << rng.randrange(8)
        base = i * SLOT
        arena[base:base + 16] = np.frombuffer(hdr, np.uint8)
        arena[base + 16:base + 16 + len(ct)] = np.frombuffer(bytes(ct), np.uint8)
        desc[i] = (base + 16, base + 16, base, ctr, ln, 16, t, 0)
        pts.append(pt)
    return arena, desc, pts


def _expected(oracle_mod, R, alg, keys, arrivals, arena, pts, window_len, seeds, installed):
    wins = {t: R.Bits(window_len) for t in range(len(keys)) if t in seeds}
    for t, mi in seeds.items():
        for i in range(1, mi + 1):
            wins[t].update(i)
    verdicts = [(L.STATUS_OK if not forged else L.STATUS_AUTH_FAILED) if t in installed else L.STATUS_BAD_KEY
                for (t, _, forged) in arrivals]
    st, dec = R.rx_sequential(wins, [a[0] for a in arrivals], [a[1] for a in arrivals], verdicts)
    exp = arena.copy()
    for i, ((t, ctr, forged), s, d) in enumerate(zip(arrivals, st, dec)):
        if not d or verdicts[i] == L.STATUS_BAD_KEY:
            continue
        base = i * SLOT + 16
        ln = len(pts[i])
        exp[base:base + ln] = 0 if forged else np.frombuffer(pts[i], np.uint8)
    return st, exp, wins


def _run(engine, oracle_mod, alg, arrivals, ntunnels=3, window_len=8192, seeds=None, installed=None, seed=1,
         lens=None, device=False, strict=False, count=None, hint=False, knobs=()):
    """hint: the device receive is told the batch's one tunnel key (key_hint = the first arrival's
    slot), so its open runs the single-key kernels' RX instantiations; knobs: (knob, value) pairs set
    around the receive."""
    import replay_oracle as R
    from nebula_amd.connection_state import Bits, rx_open_batch
    from nebula_amd.noiseutil import CipherAESGCM, CipherChaChaPoly

    rng = random.Random(seed * 31 + alg)
    keys = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(ntunnels)]
    seeds = {t: 2 for t in range(ntunnels)} if seeds is None else seeds
    installed = set(range(ntunnels)) if installed is None else installed
    cf = CipherAESGCM if alg == L.ALG_AESGCM else CipherChaChaPoly
    ciphers = {t: cf.Cipher(engine, keys[t]) for t in installed}
    # tunnels whose key is not installed get a slot id from the top of the table (never allocated here)
    slot_of = {t: (ciphers[t].key_id if t in ciphers else engine.max_keys - 1 - t) for t in range(ntunnels)}
    try:
        arena, desc, pts = _build(oracle_mod, alg, keys, arrivals, seed, lens)
        exp_status, exp_arena, owins = _expected(oracle_mod, R, alg, keys, arrivals, arena, pts, window_len, seeds,
                                                 installed)
        windows = [None] * engine.max_keys
        ewins = {}
        for t, mi in seeds.items():
            w = Bits(window_len)
            for i in range(1, mi + 1):
                w.Update(i)
            ewins[t] = w
            windows[slot_of[t]] = w
        d = desc.copy()
        d["key_id"] = [slot_of[int(t)] for t in desc["key_id"]]
        if device:  # neb_rx_open_batch: the batch and the windows in device memory
            import torch

            from nebula_amd.connection_state import DeviceWindows, rx_open_batch_device
            dev = torch.device("cuda", engine.device)
            if count == "fit":  # just the slots in use
                count = max(slot_of.values()) + 1
            dw = DeviceWindows(engine, count or engine.max_keys, window_len)
            try:
                for t, w in ewins.items():
                    dw.load(slot_of[t], w)
                d_desc = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
                d_arena = torch.from_numpy(arena).to(dev)
                d_status = torch.full((len(d),), -1, dtype=torch.int32, device=dev)
                key_hint = slot_of[arrivals[0][0]] if hint else L.KEYS_MIXED
                # strict: the parallel form only: the call fails if any window needs the host
                with contextlib.ExitStack() as knob_stack:
                    knob_stack.enter_context(L.knob(L.KNOB_RX_STRICT, 1 if strict else 0))
                    for k, v in knobs:
                        knob_stack.enter_context(L.knob(k, v))
                    rx_open_batch_device(engine, alg, dw, d_desc, d_arena, d_status, key_hint=key_hint)
                torch.cuda.synchronize()
                got = d_status.cpu().numpy()
                arena[:] = d_arena.cpu().numpy()
                for t, w in ewins.items():
                    dw.store(slot_of[t], w)
            finally:
                dw.destroy()
        else:
            got = rx_open_batch(engine, alg, windows, d, arena)
        assert got.tolist() == exp_status
        assert np.array_equal(arena, exp_arena)
        for t, w in ewins.items():
            o = owins[t]
            assert (w.current, w.lost, w.dupe, w.out_of_window) == (o.current, o.lost, o.dupe, o.out_of_window)
            assert [bool(x) for x in w.snapshot()] == o.snapshot()
        return got
    finally:
        for c in ciphers.values():
            c.destroy()


ARRIVALS = [
    (0, 3, False), (0, 4, False), (1, 3, False), (0, 5, False),
    (0, 4, False),                      # duplicate inside the batch: refused, never decrypted
    (1, 5, False), (1, 4, False),       # reorder inside the window: accepted
    (0, 7, True), (0, 7, False),        # forged copy first, genuine second: forged zeroed, genuine accepted
    (0, 6, False), (0, 6, False),       # duplicate
    (2, 3, True), (2, 3, True), (2, 3, False),  # two forgeries then the genuine one
    (1, 2, False),                      # handshake counter: pre-marked seen (connection_state.go:70-72)
    (0, 9003, False), (0, 10, False),   # jump past the window, then a stale counter: out of window
    (1, 4, False),                      # replay of an accepted packet
    (0, 9002, False), (0, 9003, True),  # in-window backfill; forged duplicate of the current counter
]


@pytest.mark.parametrize("device", [False, True])
@pytest.mark.parametrize("alg", [L.ALG_AESGCM, L.ALG_CHACHAPOLY])
def test_rx_batch_matches_sequential_decrypt(engine, oracle_mod, alg, device):
    st = _run(engine, oracle_mod, alg, ARRIVALS, device=device)
    assert (st == L.STATUS_REPLAY).sum() >= 5 and (st == L.STATUS_AUTH_FAILED).sum() >= 3


@pytest.mark.parametrize("device", [False, True])
def test_rx_batch_missing_window_and_key(engine, oracle_mod, device):
    """Tunnel 2 has no window (no ConnectionState): BAD_KEY, untouched. Tunnel 1's key is not
    installed: its window passes the packet, the engine refuses the key, the window is not updated."""
    arr = [(0, 3, False), (2, 3, False), (1, 3, False), (1, 4, False), (0, 4, False)]
    st = _run(engine, oracle_mod, L.ALG_AESGCM, arr, seeds={0: 2, 1: 2}, installed={0, 2}, device=device)
    assert st.tolist() == [0, L.STATUS_BAD_KEY, L.STATUS_BAD_KEY, L.STATUS_BAD_KEY, 0]


def _random_arrivals(rng, n, ntun, forge, jump=40):
    cur = [2] * ntun
    arr = []
    for _ in range(n):
        t = rng.randrange(ntun)
        r = rng.random()
        if r < 0.6:
            cur[t] += 1 + (rng.random() < 0.1) * rng.randrange(1, jump)
            c = cur[t]
        elif r < 0.85:
            c = max(1, cur[t] - rng.randrange(0, 80))
        else:
            c = cur[t] + rng.randrange(1, 30)
        arr.append((t, c, rng.random() < forge))
    return arr


@pytest.mark.parametrize("device", [False, True])
def test_rx_batch_random_traffic(engine, oracle_mod, device):
    """A long random receive stream over 8 tunnels and a small window: loss, reordering, jumps,
    replays and forgeries, checked packet by packet against the sequential oracle."""
    if device:
        arr = _random_arrivals(random.Random(7), 3000, 8, 0.05)
        _run(engine, oracle_mod, L.ALG_AESGCM, arr, ntunnels=8, window_len=64, seed=3, device=True)
        return
    rng = random.Random(7)
    cur = [2] * 8
    arr = []
    for _ in range(3000):
        t = rng.randrange(8)
        r = rng.random()
        if r < 0.6:
            cur[t] += 1 + (rng.random() < 0.1) * rng.randrange(1, 40)
            c = cur[t]
        elif r < 0.85:
            c = max(1, cur[t] - rng.randrange(0, 80))
        else:
            c = cur[t] + rng.randrange(1, 30)
        arr.append((t, c, rng.random() < 0.05))
    _run(engine, oracle_mod, L.ALG_AESGCM, arr, ntunnels=8, window_len=64, seed=3)


@pytest.mark.parametrize("device", [False, True])
def test_rx_batch_large(engine, oracle_mod, device):
    """A 20 000-packet receive batch over 6 tunnels (the host pool's per-window split; on the
    device, windows with forgeries take the exact sequential finish): duplicates, replays and
    forged-then-genuine copies."""
    rng = random.Random(13)
    cur = [2] * 6
    arr = []
    for k in range(20000):
        t = rng.randrange(6)
        r = rng.random()
        if r < 0.7:
            cur[t] += 1 + (rng.random() < 0.05) * rng.randrange(1, 300)
            c = cur[t]
        elif r < 0.9:
            c = max(1, cur[t] - rng.randrange(0, 120))
        else:
            c = cur[t] + rng.randrange(1, 50)
        arr.append((t, c, rng.random() < 0.04))
        if k % 8192 == 8191:  # a forged copy just before a boundary, its genuine twin just after
            cur[t] += 1
            arr.append((t, cur[t], True))
            arr.append((t, cur[t], False))
    _run(engine, oracle_mod, L.ALG_AESGCM, arr, ntunnels=6, window_len=256, seed=5, lens=[0, 1, 16, 40, 100],
         device=device)


def _one_tunnel_arrivals(rng, n, forge):
    arr = _random_arrivals(rng, n, 1, forge)
    arr += [(0, c, False) for (_, c, f) in arr[:50] if not f]  # replays of accepted packets: REPLAY, untouched
    return arr


@pytest.mark.parametrize("n,grid", [(700, 0), (20000, 0), (20000, 3)])
@pytest.mark.parametrize("forge", [0.0, 0.03])
def test_rx_device_single_key_hint(engine, oracle_mod, n, grid, forge):
    """A one-tunnel receive told its key (key_hint): the open runs the single-key kernels' RX
    instantiations behind the admission mask — gcm_single_tail_kernel<RX> for a small batch,
    gcm_single_kernel<RX> for a large one, and (grid capped at 3 workgroups, NEB_KNOB_SINGLE_MAX_GRID)
    both, the tail taking the partial last pass. A refused packet must keep its REPLAY status and its
    bytes; forged packets, replays of accepted ones and in-batch duplicates included."""
    rng = random.Random(n * 7 + grid + int(forge * 100))
    arr = _one_tunnel_arrivals(rng, n, forge)
    knobs = [(L.KNOB_SINGLE_MAX_GRID, grid)] if grid else []
    st = _run(engine, oracle_mod, L.ALG_AESGCM, arr, ntunnels=1, window_len=1024, seed=21, lens=[0, 16, 90, 600],
              device=True, hint=True, knobs=knobs, strict=forge == 0.0)
    assert (st == L.STATUS_REPLAY).sum() >= 50
    if forge:
        assert (st == L.STATUS_AUTH_FAILED).sum() > 0


@pytest.mark.parametrize("n", [3000, 20000])
def test_rx_device_mixed_key_unprebinned(engine, oracle_mod, n):
    """A mixed-key receive binned by the open itself (NEB_KNOB_SUB_BINS_FROM 0: as a batch past the
    sub-bin threshold is, instead of prebinned by the plan's launches): gcm_chunk_kernel<open, RX>
    with the admission mask read per packet. Replays, duplicates and forgeries over 8 tunnels against
    the sequential oracle; refused packets untouched."""
    rng = random.Random(n)
    arr = _random_arrivals(rng, n, 8, 0.04)
    st = _run(engine, oracle_mod, L.ALG_AESGCM, arr, ntunnels=8, window_len=128, seed=23, lens=[0, 16, 90, 600, 1300],
              device=True, knobs=[(L.KNOB_SUB_BINS_FROM, 0)])
    assert (st == L.STATUS_REPLAY).sum() > 0 and (st == L.STATUS_AUTH_FAILED).sum() > 0


@pytest.mark.parametrize("length", [1, 64, 256, 8192])
def test_rx_device_parallel_form(engine, oracle_mod, length):
    """Device windows, no forgeries: every window finishes on the device's parallel form (prefix
    maxima, first occurrences, per-slot bitmap and lost counts), over warmup, steady state, jumps
    past the window, reordering and in-batch duplicates."""
    rng = random.Random(length)
    arr = _random_arrivals(rng, 6000, 5, 0.0, jump=3 * length + 2)
    _run(engine, oracle_mod, L.ALG_AESGCM, arr, ntunnels=5, window_len=length, seed=9, lens=[0, 16, 60],
         seeds={0: 2, 1: 2, 2: 2, 3: 2, 4: 2}, device=True, strict=True)


@pytest.mark.parametrize("count", ["fit", 40000])
def test_rx_device_sort_passes(engine, oracle_mod, count):
    """The stable sort by window in one pass (a window set of fewer than 256 slots: keys of at most
    8 bits) and in three (40 000 slots: 16-bit keys), then the parallel form."""
    rng = random.Random(5)
    arr = _random_arrivals(rng, 5000, 6, 0.0, jump=200)
    _run(engine, oracle_mod, L.ALG_AESGCM, arr, ntunnels=6, window_len=1024, seed=11, lens=[0, 16, 60],
         device=True, strict=True, count=count)


def test_rx_device_one_big_window(engine, oracle_mod):
    """One tunnel, 20 000 packets in one window run (the C2 shape): the parallel form only."""
    rng = random.Random(77)
    arr = _random_arrivals(rng, 20000, 1, 0.0)
    _run(engine, oracle_mod, L.ALG_CHACHAPOLY, arr, ntunnels=1, window_len=8192, seed=4, lens=[0, 16, 90],
         device=True, strict=True)


def test_rx_device_lookback_timeout_moves_no_window(engine, oracle_mod):
    """A device receive whose scan lookback times out fails the batch (NEB_ERR_HIP) and moves no
    window: neither the scan blocks that finished (their finals came from a partial prefix) nor the
    failed one (its packets were never opened, so their counters are unauthenticated) commit
    anything. Forced with the fault-injection spin limit 0 (every scan block that starts inside a
    run and has to wait fails); the same batch then passes with the default limit, against the
    oracle."""
    import torch

    from nebula_amd.connection_state import Bits, DeviceWindows, rx_open_batch_device
    from nebula_amd.noiseutil import CipherAESGCM

    rng = random.Random(21)
    arr = _random_arrivals(rng, 3000, 4, 0.0)  # runs of ~750 packets: most scan blocks start mid-run
    keys = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(4)]
    ciphers = [CipherAESGCM.Cipher(engine, k) for k in keys]
    dev = torch.device("cuda", engine.device)
    try:
        arena, desc, _ = _build(oracle_mod, L.ALG_AESGCM, keys, arr, 3, lens=[0, 16, 60])
        desc["key_id"] = [ciphers[int(t)].key_id for t in desc["key_id"]]
        dw = DeviceWindows(engine, engine.max_keys, 1024)
        try:
            before = {}
            for c in ciphers:
                w = Bits(1024)
                w.Update(1)
                w.Update(2)
                dw.load(c.key_id, w)
                before[c.key_id] = (w.current, w.lost, w.dupe, w.out_of_window, list(w.snapshot()))
            d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
            d_arena = torch.from_numpy(arena).to(dev)
            d_status = torch.full((len(desc),), -1, dtype=torch.int32, device=dev)
            dw.set_spin_limit(0)
            with pytest.raises(L.NebError) as ei:
                rx_open_batch_device(engine, L.ALG_AESGCM, dw, d_desc, d_arena, d_status)
            assert ei.value.rc == L.ERR_HIP
            torch.cuda.synchronize()
            for c in ciphers:
                w = Bits(1024)
                dw.store(c.key_id, w)
                assert (w.current, w.lost, w.dupe, w.out_of_window, list(w.snapshot())) == before[c.key_id]
            # the windows are intact: the same batch (fresh arena) goes through with the default limit
            dw.set_spin_limit(1 << 20)
            d_arena.copy_(torch.from_numpy(arena).to(dev))
            rx_open_batch_device(engine, L.ALG_AESGCM, dw, d_desc, d_arena, d_status)
            torch.cuda.synchronize()
            assert (d_status.cpu().numpy() != -1).all()
        finally:
            dw.destroy()
    finally:
        for c in ciphers:
            c.destroy()
    # and the full check of that batch against the oracle, on fresh windows
    _run(engine, oracle_mod, L.ALG_AESGCM, arr, ntunnels=4, window_len=1024, seed=3, lens=[0, 16, 60], device=True)


def test_rx_device_counters_near_wrap(engine, oracle_mod):
    """Counters at and beyond 2^62 (a window's current and packets near 2^64): those windows take
    the exact sequential path on the host, the others the parallel form, in one batch."""
    big = 1 << 62
    arr = [(0, 3, False), (1, big + 5, False), (1, big + 3, False), (1, big + 5, False),
           (2, 2**64 - 3, False), (2, 2**64 - 1, True), (2, 2**64 - 1, False), (2, 5, False),
           (0, 4, False), (0, 4, False), (1, big - 1, False)]
    _run(engine, oracle_mod, L.ALG_AESGCM, arr, device=True)


@pytest.mark.parametrize("device", [False, True])
def test_rx_forged_far_counter_costs_one_round(engine, oracle_mod, capfd, device):
    """A forged packet with a counter far ahead of its window, then hundreds of genuine ones: the
    simulation (every tag assumed to verify) holds the genuine ones back, the forgery fails, and
    the real pass must open them all in one more batch, not one open per packet."""
    arr = [(0, 5 + 100000, True)] + [(0, 3 + k, False) for k in range(400)] + [(1, 3, False)]
    arr += [(0, 3 + 200000, True)] + [(0, 403 + k, False) for k in range(100)]
    os.environ["NEB_RX_STATS"] = "1"
    try:
        _run(engine, oracle_mod, L.ALG_AESGCM, arr, ntunnels=2, window_len=8192, seed=6, lens=[0, 16, 100],
             device=device)
    finally:
        os.environ.pop("NEB_RX_STATS", None)
    err = capfd.readouterr().err
    lines = [ln for ln in err.splitlines() if ln.startswith("rx exact:")]
    assert lines, err
    import re
    rounds, opens = map(int, re.search(r"(\d+) rounds, (\d+) extra opens", lines[-1]).groups())
    assert rounds <= 3 and opens <= 2, lines[-1]


@pytest.mark.parametrize("order", ["increasing", "decreasing"])
@pytest.mark.parametrize("device", [False, True])
def test_rx_interleaved_forgeries_bounded_rounds(engine, oracle_mod, capfd, device, order):
    """Forged packets with counters far ahead, each followed by a run of genuine ones (F1, P.., F2,
    P.., ...): every forgery holds back the genuine packets after it in the simulation. The exact
    pass must still finish in at most two extra batches (the second verifies everything left out of
    place), with results identical to the sequential loop: refused packets untouched, accepted ones
    decrypted, forged ones that pass their window zeroed."""
    arr, nxt = [], 3
    for m in range(40):
        far = 10**6 + (m if order == "increasing" else 40 - m) * 10**5
        arr.append((0, far, True))
        for _ in range(8):
            arr.append((0, nxt, False))
            nxt += 1
        if m % 7 == 3:
            arr.append((0, nxt - 2, False))  # an in-batch replay too
    arr.append((1, 3, False))
    os.environ["NEB_RX_STATS"] = "1"
    try:
        _run(engine, oracle_mod, L.ALG_AESGCM, arr, ntunnels=2, window_len=8192, seed=8, lens=[0, 16, 100],
             device=device)
    finally:
        os.environ.pop("NEB_RX_STATS", None)
    err = capfd.readouterr().err
    lines = [ln for ln in err.splitlines() if ln.startswith("rx exact:")]
    assert lines, err
    import re
    rounds, opens = map(int, re.search(r"(\d+) rounds, (\d+) extra opens", lines[-1]).groups())
    assert rounds <= 3 and opens <= 2, lines[-1]


def test_rx_batch_invalid_descriptor_touches_nothing(engine, oracle_mod):
    """A receive batch with a descriptor whose offset wraps around 2^64 is refused before any
    window moves or any packet is opened."""
    from nebula_amd.connection_state import Bits, rx_open_batch
    from nebula_amd.noiseutil import CipherAESGCM

    keys = [bytes(range(32))]
    arrivals = [(0, c, False) for c in range(3, 40)]
    arena, desc, _ = _build(oracle_mod, L.ALG_AESGCM, keys, arrivals, 5)
    c = CipherAESGCM.Cipher(engine, keys[0])
    try:
        w = Bits(8192)
        w.Update(1)
        w.Update(2)
        windows = [None] * engine.max_keys
        windows[c.key_id] = w
        d = desc.copy()
        d["key_id"] = c.key_id
        d["aad_off"][-1] = 2**64 - 8
        before = arena.copy()
        with pytest.raises(Exception):
            rx_open_batch(engine, L.ALG_AESGCM, windows, d, arena)
        assert np.array_equal(arena, before)
        assert (w.current, w.lost, w.dupe, w.out_of_window) == (2, 0, 0, 0)
    finally:
        c.destroy()


def test_device_windows_api_errors(engine):
    """neb_dwindows_* and neb_rx_open_batch refuse what Bits / the host call refuse: a length that
    is not a power of two, a slot out of range, a host window of another length, storing an absent
    slot, a bad algorithm, a window set of another engine."""
    import ctypes as C

    from nebula_amd.connection_state import Bits, DeviceWindows
    from nebula_amd.noiseutil import Engine

    lib = L.lib()
    h = C.c_void_p()
    assert lib.neb_dwindows_create(engine.handle, 4, 1000, C.byref(h)) == L.ERR_INVALID
    assert lib.neb_dwindows_create(engine.handle, 0, 1024, C.byref(h)) == L.ERR_INVALID
    dw = DeviceWindows(engine, 4, 1024)
    try:
        w = Bits(1024)
        w.Update(5)
        assert lib.neb_dwindows_load(dw.handle, 4, w.handle) == L.ERR_INVALID       # slot out of range
        assert lib.neb_dwindows_load(dw.handle, 0, Bits(2048).handle) == L.ERR_INVALID  # other length
        assert lib.neb_dwindows_store(dw.handle, 1, w.handle) == L.ERR_INVALID      # absent slot
        dw.load(1, w)
        back = Bits(1024)
        dw.store(1, back)
        assert back.current == 5 and back.snapshot() == w.snapshot()
        dw.load(1, None)
        assert lib.neb_dwindows_store(dw.handle, 1, back.handle) == L.ERR_INVALID
        assert lib.neb_rx_open_batch(engine.handle, 7, dw.handle, None, 0, None, None, L.KEYS_MIXED, None) == \
            L.ERR_INVALID
        assert lib.neb_rx_open_batch(engine.handle, L.ALG_AESGCM, dw.handle, None, 0, None, None, L.KEYS_MIXED,
                                     None) == L.OK  # empty batch
        other = Engine(engine.device, 16)
        try:
            assert lib.neb_rx_open_batch(other.handle, L.ALG_AESGCM, dw.handle, None, 0, None, None, L.KEYS_MIXED,
                                         None) == L.ERR_INVALID
        finally:
            other.close()
    finally:
        dw.destroy()


@pytest.mark.parametrize("strict", [False, True])
def test_rx_device_batches_one_and_many_windows(engine, oracle_mod, strict):
    """Consecutive batches on one device window set, alternating between batches whose packets all
    name one window (run order = arrival order: the sort writes the identity) and batches that name
    several — including one whose only other window is its last packet's, one whose first packet
    names an absent window, and one that names only an absent window. Per-packet receive is
    sequential, so the batches together must equal the oracle's loop over their concatenation."""
    import replay_oracle as R
    import torch

    from nebula_amd.connection_state import Bits, DeviceWindows, rx_open_batch_device
    from nebula_amd.noiseutil import CipherAESGCM

    rng = random.Random(404)
    ntun, wl = 3, 1024
    keys = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(ntun)]
    installed = {0, 1}  # tunnel 2: no key and no window
    nxt = {0: 3, 1: 3, 2: 3}

    def batch(tuns, n):
        out = []
        for _ in range(n):
            t = rng.choice(tuns)
            c = nxt[t] + rng.choice([0, 0, 1, 2]) - (1 if rng.random() < 0.1 else 0)
            nxt[t] = max(nxt[t], c + 1)
            out.append((t, c, not strict and rng.random() < 0.03))
        return out

    batches = [batch([0, 1], 300), batch([0], 500), batch([0], 200) + [(1, nxt[1], False)], batch([1], 400)]
    if not strict:  # packets of an absent window (the strict mode's parallel form refuses a batch with them)
        batches += [[(2, 3, False)] + batch([0], 100), batch([2], 50), batch([0, 1, 2], 300)]
    batches += [batch([1], 250), batch([0, 1], 100)]
    arrivals = [a for b in batches for a in b]
    ciphers = {t: CipherAESGCM.Cipher(engine, keys[t]) for t in installed}
    slot_of = {t: (ciphers[t].key_id if t in ciphers else engine.max_keys - 1 - t) for t in range(ntun)}
    dw = None
    try:
        arena, desc, pts = _build(oracle_mod, L.ALG_AESGCM, keys, arrivals, 9, [0, 16, 40, 1300])
        seeds = {0: 2, 1: 2}
        exp_status, exp_arena, owins = _expected(oracle_mod, R, L.ALG_AESGCM, keys, arrivals, arena, pts, wl, seeds,
                                                 installed)
        d = desc.copy()
        d["key_id"] = [slot_of[int(t)] for t in desc["key_id"]]
        dev = torch.device("cuda", engine.device)
        dw = DeviceWindows(engine, engine.max_keys, wl)
        ewins = {}
        for t, mi in seeds.items():
            w = Bits(wl)
            for i in range(1, mi + 1):
                w.Update(i)
            ewins[t] = w
            dw.load(slot_of[t], w)
        d_arena = torch.from_numpy(arena).to(dev)
        got = []
        a = 0
        for b in batches:
            dd = torch.from_numpy(d[a:a + len(b)].view(np.uint8).copy()).to(dev)
            st = torch.full((len(b),), -1, dtype=torch.int32, device=dev)
            with L.knob(L.KNOB_RX_STRICT, 1 if strict else 0):
                rx_open_batch_device(engine, L.ALG_AESGCM, dw, dd, d_arena, st)
            got += st.cpu().tolist()
            a += len(b)
        assert got == exp_status
        assert np.array_equal(d_arena.cpu().numpy(), exp_arena)
        for t, w in ewins.items():
            dw.store(slot_of[t], w)
            o = owins[t]
            assert (w.current, w.lost, w.dupe, w.out_of_window) == (o.current, o.lost, o.dupe, o.out_of_window)
            assert [bool(x) for x in w.snapshot()] == o.snapshot()
    finally:
        if dw is not None:
            dw.destroy()
        for c in ciphers.values():
            c.destroy()


def test_rx_concurrent_receives_on_one_engine(engine, oracle_mod):
    """Two threads receive on one engine at once (Nebula's `routines` listenOut loops share one
    engine): pinned arenas, so both take the piped zero-copy path through the engine's shared
    staging buffers, and the second batch is larger, so its call reallocates them. Every call's
    statuses, arena bytes and windows equal the sequential oracle's (the verdicts are copied out of
    the shared staging before it is released)."""
    import threading

    import replay_oracle as R
    from nebula_amd.batch import PinnedBuffer
    from nebula_amd.connection_state import Bits, rx_open_batch
    from nebula_amd.noiseutil import CipherAESGCM

    rng = random.Random(21)
    jobs = []
    for j, n in enumerate([1500, 6000, 2500, 9000]):
        keys = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(2)]
        arr = _random_arrivals(random.Random(100 + j), n, 2, 0.03)
        arena, desc, pts = _build(oracle_mod, L.ALG_AESGCM, keys, arr, 30 + j, lens=[0, 16, 100, 576])
        st, exp, owins = _expected(oracle_mod, R, L.ALG_AESGCM, keys, arr, arena, pts, 1024, {0: 2, 1: 2}, {0, 1})
        ciphers = [CipherAESGCM.Cipher(engine, k) for k in keys]
        buf = PinnedBuffer(arena.nbytes)
        buf.array[:] = arena
        wins = [None] * engine.max_keys
        ew = []
        for t, c in enumerate(ciphers):
            w = Bits(1024)
            w.Update(1)
            w.Update(2)
            wins[c.key_id] = w
            ew.append(w)
        d = desc.copy()
        d["key_id"] = [ciphers[int(t)].key_id for t in desc["key_id"]]
        jobs.append(dict(d=d, buf=buf, wins=wins, ew=ew, st=st, exp=exp, owins=owins, ciphers=ciphers))
    results = [None] * len(jobs)

    def work(j):
        jb = jobs[j]
        results[j] = rx_open_batch(engine, L.ALG_AESGCM, jb["wins"], jb["d"], jb["buf"].array)

    try:
        for rep in range(2):
            ths = [threading.Thread(target=work, args=(j,)) for j in (2 * rep, 2 * rep + 1)]
            for t in ths:
                t.start()
            for t in ths:
                t.join()
        for j, jb in enumerate(jobs):
            assert results[j].tolist() == jb["st"], j
            assert np.array_equal(jb["buf"].array, jb["exp"]), j
            for t, w in enumerate(jb["ew"]):
                o = jb["owins"][t]
                assert (w.current, w.lost, w.dupe, w.out_of_window) == (o.current, o.lost, o.dupe, o.out_of_window)
    finally:
        for jb in jobs:
            jb["buf"].free()
            for c in jb["ciphers"]:
                c.destroy()


def _wire_batch(oracle_mod, alg, keys, seed=3, n_rand=600):
    """Wire packets of every kind readOutsidePackets meets (outside.go:30-133): messages, relayed
    messages (GMAC over the AD), encrypted control types, unencrypted types, bad versions and
    subtypes, runts, packets with no tunnel, forgeries, replays, a header whose counter was edited.
    Returns (arena, packets [(off, len, tunnel or None)], plaintexts)."""
    rng = random.Random(seed)
    SL = 1600
    items = []
    ctr = {t: 2 for t in range(len(keys))}

    def sealed(t, typ, sub, c, pt, relay=False):
        hdr = bytes([(1 << 4) | typ, sub, 0, 0]) + (0x1000 + t).to_bytes(4, "big") + c.to_bytes(8, "big")
        nb = oracle_mod.nonce(alg, c)
        if relay:
            ad = hdr + pt
            return ad + oracle_mod.seal(alg, keys[t], nb, ad, b"")
        return hdr + oracle_mod.seal(alg, keys[t], nb, hdr, pt)

    fixed = []
    for t in range(len(keys)):
        for typ, sub in ((1, 0), (1, 1), (4, 0), (4, 1), (6, 0), (3, 0), (5, 0)):
            ctr[t] += 1
            pt = bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 16, 100, 1300])))
            fixed.append((sealed(t, typ, sub, ctr[t], pt, relay=(typ, sub) == (1, 1)), t))
    hs = bytes([0x10, 0, 0, 0]) + bytes(60)           # handshake IXPSK0: left to the control plane
    fixed += [(hs, 0), (bytes([0x12, 0]) + bytes(40), 1)]  # recv error
    fixed += [(bytes([0x21, 0]) + bytes(40), 0)]        # version 2
    fixed += [(bytes([0x11, 2]) + bytes(40), 0), (bytes([0x10, 1]) + bytes(40), 0), (bytes([0x17, 0]) + bytes(40), 0)]
    fixed += [(b"", 0), (b"\x11", 0), (bytes([0x11, 0]) + bytes(13), 0)]  # runts (< 16: no header)
    ctr[0] += 1
    short = sealed(0, 1, 0, ctr[0], b"")[:31]             # a header and 15 bytes: under 16 + 16
    fixed += [(short, 0)]
    ctr[1] += 1
    fixed += [(sealed(1, 1, 0, ctr[1], b"no tunnel"), None)]
    ctr[2] += 1
    edited = bytearray(sealed(2, 1, 0, ctr[2], b"x" * 200))
    edited[15] ^= 1                                        # counter edited in flight: wrong nonce, wrong AD
    fixed += [(bytes(edited), 2)]
    # random traffic: messages, forgeries, replays of earlier packets
    sent = []
    for _ in range(n_rand):
        t = rng.randrange(len(keys))
        r = rng.random()
        if r < 0.15 and sent:
            fixed.append(rng.choice(sent))
            continue
        ctr[t] += 1 + (rng.random() < 0.1) * rng.randrange(1, 30)
        relay = rng.random() < 0.1
        pkt = bytearray(sealed(t, 1, 1 if relay else 0, ctr[t], bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 20, 576]))),
                               relay=relay))
        if rng.random() < 0.05:
            pkt[rng.randrange(16, len(pkt))] ^= 1 << rng.randrange(8)
        fixed.append((bytes(pkt), t))
        sent.append((bytes(pkt), t))
    rng.shuffle(fixed)
    arena = np.zeros(len(fixed) * SL, np.uint8)
    packets = []
    for i, (pkt, t) in enumerate(fixed):
        arena[i * SL:i * SL + len(pkt)] = np.frombuffer(pkt, np.uint8)
        packets.append((i * SL, len(pkt), t))
    return arena, packets


def _wire_expected(oracle_mod, R, alg, keys, arena, packets, window_len, own=frozenset()):
    wins = {t: R.Bits(window_len) for t in range(len(keys))}
    for w in wins.values():
        w.update(1)
        w.update(2)
    exp = arena.copy()
    status = []
    for i, (off, ln, t) in enumerate(packets):
        pkt = bytes(arena[off:off + ln])
        st, go = R.read_outside_gate(pkt, t is not None, i in own)
        if st is not None:
            status.append(st)
            continue
        kind, c = go
        w = wins[t]
        if not w.check(c):
            status.append(R.REPLAY)
            continue
        nb = oracle_mod.nonce(alg, c)
        if kind == "relay":
            ok = oracle_mod.open_(alg, keys[t], nb, pkt[:ln - 16], pkt[ln - 16:]) is not None
        else:
            pt = oracle_mod.open_(alg, keys[t], nb, pkt[:16], pkt[16:])
            ok = pt is not None
            exp[off + 16:off + ln - 16] = np.frombuffer(pt, np.uint8) if ok else 0
        if not ok:
            status.append(R.AUTH_FAILED)
            continue
        status.append(R.OK if w.update(c) else R.REPLAY)
    return status, exp, wins


@pytest.mark.parametrize("device", [False, True])
@pytest.mark.parametrize("alg", [L.ALG_AESGCM, L.ALG_CHACHAPOLY])
def test_rx_wire_gate_matches_read_outside_packets(engine, oracle_mod, alg, device):
    """neb_rx_open_wire_batch[_host]: the header parse, version / subtype / size checks and the
    header's counter as nonce on the engine's side, then Decrypt or VerifyRelay — statuses, every
    arena byte and the windows equal the oracle's readOutsidePackets loop (oracle/replay_oracle.py
    read_outside_gate + the sequential receive)."""
    import replay_oracle as R
    from nebula_amd.connection_state import (Bits, DeviceWindows, rx_open_wire_batch,
                                             rx_open_wire_batch_device)
    from nebula_amd.noiseutil import CipherAESGCM, CipherChaChaPoly

    rng = random.Random(alg * 5 + device)
    keys = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(3)]
    arena, packets = _wire_batch(oracle_mod, alg, keys, seed=alg + 2 * device)
    # the caller's double-encryption check (outside.go:66-74) refuses every 17th datagram
    own = frozenset(i for i in range(3, len(packets), 17) if packets[i][2] is not None)
    exp_status, exp_arena, owins = _wire_expected(oracle_mod, R, alg, keys, arena, packets, 256, own)
    cf = CipherAESGCM if alg == L.ALG_AESGCM else CipherChaChaPoly
    ciphers = [cf.Cipher(engine, k) for k in keys]
    try:
        pk = np.zeros(len(packets), L.RX_PACKET_DTYPE)
        for i, (off, ln, t) in enumerate(packets):
            pk[i] = (off, ln | (0x80000000 if i in own else 0), ciphers[t].key_id if t is not None else L.KEYS_MIXED)
        ewins = []
        for c in ciphers:
            w = Bits(256)
            w.Update(1)
            w.Update(2)
            ewins.append(w)
        if device:
            import torch
            dev = torch.device("cuda", engine.device)
            dw = DeviceWindows(engine, engine.max_keys, 256)
            try:
                for c, w in zip(ciphers, ewins):
                    dw.load(c.key_id, w)
                d_pk = torch.from_numpy(pk.view(np.uint8).copy()).to(dev)
                d_arena = torch.from_numpy(arena).to(dev)
                d_status = torch.full((len(pk),), -1, dtype=torch.int32, device=dev)
                rx_open_wire_batch_device(engine, alg, dw, d_pk, d_arena, d_status)
                torch.cuda.synchronize()
                got = d_status.cpu().numpy()
                arena = d_arena.cpu().numpy()
                for c, w in zip(ciphers, ewins):
                    dw.store(c.key_id, w)
            finally:
                dw.destroy()
        else:
            windows = [None] * engine.max_keys
            for c, w in zip(ciphers, ewins):
                windows[c.key_id] = w
            got = rx_open_wire_batch(engine, alg, windows, pk, arena)
        assert got.tolist() == exp_status
        assert np.array_equal(arena, exp_arena)
        for t, w in enumerate(ewins):
            o = owins[t]
            assert (w.current, w.lost, w.dupe, w.out_of_window) == (o.current, o.lost, o.dupe, o.out_of_window)
        kinds = set(exp_status)
        assert {R.OK, R.INVALID, R.NOT_MESSAGE, R.BAD_KEY, R.REPLAY, R.AUTH_FAILED} <= kinds, kinds
    finally:
        for c in ciphers:
            c.destroy()
