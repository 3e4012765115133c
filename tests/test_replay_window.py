"""CPU: the anti-replay window (nebula.Bits, bits.go) — oracle and engine against the reference's
own bits_test.go scenarios (tests/golden/replay_window.json), engine against oracle on long random
sequences, and the ConnectionState counter rules (connection_state_test.go:84-160)."""
import json
import os
import random

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "replay_window.json")))
M64 = (1 << 64) - 1


def run_scenario(sc, new):
    w = None
    for op in sc["ops"]:
        k = op[0]
        where = (sc["name"], op)
        if k == "new":
            w = new(op[1])
        elif k == "reset":
            w.reset_counters()
        elif k == "check":
            assert w.check(op[1]) == op[2], where
        elif k == "update":
            assert w.update(op[1]) == op[2], where
        elif k == "check_range":
            for i in range(op[1], op[2] + 1):
                assert w.check(i) == op[3], (where, i)
        elif k == "update_range":
            for i in range(op[1], op[2] + 1):
                assert w.update(i) == op[3], (where, i)
        elif k == "check_update_range":
            for i in range(op[1], op[2] + 1):
                assert w.check(i) == op[3] and w.update(i) == op[3], (where, i)
        elif k == "current":
            assert w.current == op[1], where
        elif k == "snapshot":
            assert [int(x) for x in w.snapshot()] == op[1], where
        elif k == "lost":
            assert w.lost == op[1], where
        elif k == "dupe":
            assert w.dupe == op[1], where
        elif k == "oow":
            assert w.out_of_window == op[1], where
        else:
            raise KeyError(k)


class LibWindow:
    """Adapter: the engine's window with the oracle's method names."""

    def __init__(self, length):
        from nebula_amd.connection_state import Bits

        self.b = Bits(length)
        self.length = length

    def check(self, i):
        return self.b.Check(i)

    def update(self, i):
        return self.b.Update(i)

    def reset_counters(self):
        self.b.reset_counters()

    def snapshot(self):
        return self.b.snapshot()

    def __getattr__(self, name):
        return getattr(self.b, name)


@pytest.fixture(scope="module")
def R():
    import replay_oracle

    return replay_oracle


@pytest.mark.parametrize("sc", FIX["scenarios"], ids=[s["name"] for s in FIX["scenarios"]])
def test_oracle_matches_reference_scenarios(sc, R):
    run_scenario(sc, R.Bits)


@pytest.mark.parametrize("sc", FIX["scenarios"], ids=[s["name"] for s in FIX["scenarios"]])
def test_engine_window_matches_reference_scenarios(sc):
    run_scenario(sc, LibWindow)


def test_window_lengths(R):
    from nebula_amd.connection_state import Bits

    for bad in FIX["invalid_lengths"]:
        with pytest.raises(ValueError):
            Bits(bad)
        with pytest.raises(ValueError):
            R.Bits(bad)
    for good in FIX["valid_lengths"]:
        assert Bits(good).length == good


def _random_ops(rng, length, n, base):
    """Arrival patterns of a receive path: in order, reordering inside the window, duplicates,
    jumps of up to a few windows, stale counters, and counter 0."""
    cur = base
    ops = []
    for _ in range(n):
        r = rng.random()
        if r < 0.45:
            cur = (cur + 1) & M64
            c = cur
        elif r < 0.65:
            c = (cur - rng.randrange(0, 2 * length + 2)) & M64
        elif r < 0.75:
            c = cur
        elif r < 0.9:
            cur = (cur + rng.randrange(2, 3 * length + 3)) & M64
            c = cur
        elif r < 0.95:
            c = (cur + rng.randrange(1, length + 1)) & M64
        else:
            c = rng.choice([0, 1, length, length + 1, M64, M64 - 1])
        ops.append((rng.random() < 0.5, c))
    return ops


@pytest.mark.parametrize("length", [1, 2, 8, 16, 64, 128, 1024, 8192])
@pytest.mark.parametrize("base", [0, 5000, (1 << 64) - 40000])
def test_engine_window_equals_oracle_random(length, base, R):
    rng = random.Random(length * 7919 + (base & 0xFFFF))
    o = R.Bits(length)
    e = LibWindow(length)
    for only_check, c in _random_ops(rng, length, 3000, base):
        assert e.check(c) == o.check(c), (length, c)
        if not only_check:
            assert e.update(c) == o.update(c), (length, c)
        assert e.current == o.current
    assert (e.lost, e.dupe, e.out_of_window) == (o.lost, o.dupe, o.out_of_window)
    assert [bool(x) for x in e.snapshot()] == o.snapshot()


def test_connection_state_seeds_window():
    """newConnectionStateFromResult (connection_state.go:52-75; test :123-160): IX leaves
    MessageIndex 2, counters 1 and 2 are marked seen, 3 is not, and MessageIndex >= ReplayWindow
    is refused."""
    from nebula_amd.connection_state import ConnectionState, ReplayWindow

    cs = ConnectionState(None, None, message_index=2)
    assert not cs.window.Check(1) and not cs.window.Check(2) and cs.window.Check(3)
    assert cs.NextMessageCounter() == (3, True)
    assert cs.window.lost == 0
    with pytest.raises(ValueError):
        ConnectionState(None, None, message_index=ReplayWindow)


def test_next_message_counter_pins_at_reject():
    """connection_state_test.go:84-104."""
    from nebula_amd.connection_state import ConnectionState
    from nebula_amd.noiseutil import RejectAfterMessages

    cs = ConnectionState(None, None)
    cs._ctr = RejectAfterMessages - 2
    assert cs.NextMessageCounter() == (RejectAfterMessages - 1, True)
    assert cs.NextMessageCounter() == (RejectAfterMessages, False)
    assert cs._ctr == RejectAfterMessages
    for _ in range(10):
        assert not cs.NextMessageCounter()[1]
    assert cs._ctr == RejectAfterMessages


def test_rx_sequential_oracle_semantics(R):
    """The oracle's receive loop: Check before decrypt, Update only after a good tag, a refused
    packet never decrypted; a genuine packet after a forged copy of it is still accepted."""
    w = {0: R.Bits(16)}
    keys = [0, 0, 0, 0, 0, 1]
    ctrs = [3, 3, 4, 4, 2, 1]
    auth = [True, True, False, True, True, True]
    st, dec = R.rx_sequential(w, keys, ctrs, auth)
    assert st == [R.OK, R.REPLAY, R.AUTH_FAILED, R.OK, R.OK, R.BAD_KEY]
    assert dec == [True, False, True, True, True, False]
