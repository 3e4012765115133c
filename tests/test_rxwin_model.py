"""CPU: the parallel form of the device batched receive (tools/rxwin_model.py, step for step as
nebula_amd/csrc/rxwin.hip) equals the sequential Check → Update of the reference's window
(oracle/replay_oracle.py, bits.go:134-262) on random receive streams whose tags all verify:
which packets are decrypted, and the window's current, bitmap and lost counter afterwards."""
import os
import random
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import rxwin_model as M  # noqa: E402


def _stream(rng, n, start, length):
    cur, out = start, []
    for _ in range(n):
        r = rng.random()
        if r < 0.55:
            cur += 1 + (rng.random() < 0.1) * rng.randrange(1, 3 * length + 2)
            out.append(cur)
        elif r < 0.8:
            out.append(max(0, cur - rng.randrange(0, 2 * length + 2)))
        elif r < 0.9:
            out.append(out[rng.randrange(len(out))] if out else cur)  # duplicate inside the batch
        else:
            out.append(cur + rng.randrange(1, length + 3))
    return out


@pytest.mark.parametrize("length", [1, 2, 8, 64, 128, 1024])
def test_parallel_form_matches_sequential(oracle_mod, length):
    import replay_oracle as R

    rng = random.Random(length)
    for trial in range(60):
        w = R.Bits(length)
        # a window state before the batch: warmup (small current) or steady state
        pre = _stream(rng, rng.randrange(0, 40), 0, length) if trial % 3 else []
        if trial % 4 == 1:
            pre = [length * rng.randrange(1, 5) + rng.randrange(0, length)] + pre
        for c in pre:
            if w.check(c):
                w.update(c)
        cur0, bits0, lost0 = w.current, list(w.bits), w.lost
        run = _stream(rng, rng.randrange(1, 120), cur0, length)
        adm = M.admit(run, cur0, bits0, length)
        exp_adm = []
        for c in run:  # the sequential receive, every tag verifying
            ok = w.check(c)
            exp_adm.append(ok)
            if ok:
                assert w.update(c)
        assert adm == exp_adm, (trial, run)
        for fin in (M.finish, M.finish_ranges):
            cur, bits, lost = fin(run, adm, cur0, bits0, lost0, length)
            assert cur == w.current, trial
            assert bits == w.bits, (trial, fin.__name__)
            assert lost == w.lost, (trial, fin.__name__, lost, w.lost)
