"""GPU: the submission queue (neb_queue_*) — many threads' Nebula-sized flushes gathered into
device batches (interface.go:381-487: 128-packet TX flushes, 64-packet RX flushes, from `routines`
goroutines at once). Every thread's arena bytes and statuses must equal the oracle's, whatever
batch its packets ended up in."""
import threading

import numpy as np
import pytest

from nebula_amd import _lib as L
from nebula_amd import workload as W

pytestmark = pytest.mark.gpu


def _flushes(b, per):
    """Split a batch into contiguous flushes of `per` packets, each with its own arena copy."""
    out = []
    for f0 in range(0, b.n, per):
        d = b.desc[f0:f0 + per].copy()
        lo = int(d["aad_off"].min())
        hi = int((d["src_off"] + d["len"].astype(np.uint64) + np.uint64(16)).max())
        for k in ("src_off", "dst_off", "aad_off"):
            d[k] -= np.uint64(lo)
        out.append((f0, d, b.arena[lo:hi].copy(), lo))
    return out


@pytest.mark.parametrize("alg,nkeys,threads,per,zc", [
    (L.ALG_AESGCM, 64, 16, 128, False),      # TX-sized flushes, many tunnels
    (L.ALG_AESGCM, 1, 32, 64, False),        # RX-sized flushes, one tunnel: single-key batches
    (L.ALG_CHACHAPOLY, 64, 8, 128, False),
    # every other flush's arena pinned and mapped (neb_host_alloc): submitted zero-copy, its
    # descriptors pointing at the caller's bytes, in the same device batches as staged flushes
    (L.ALG_AESGCM, 64, 16, 128, True),
    (L.ALG_CHACHAPOLY, 64, 8, 64, True),
])
def test_queue_many_threads_vs_oracle(engine, oracle_mod, alg, nkeys, threads, per, zc):
    from nebula_amd.batch import PinnedBuffer, SubmitQueue, install_keys, slot_desc

    b = W.make_batch(alg, 12000, nkeys, sizes=(90, 576, 1300), ratio=(7, 4, 1), seed=nkeys * 7 + per,
                     name="queue")
    ref, st_ref = b.arena.copy(), None
    st_ref = oracle_mod.batch(alg, 0, b.keys, b.desc, ref)
    assert (st_ref == 0).all()
    ciphers = install_keys(engine, b)
    seal_q = SubmitQueue(engine, alg, False, max_packets=4096, max_delay_us=200)
    open_q = SubmitQueue(engine, alg, True, max_packets=4096, max_delay_us=200)
    try:
        bd = W.Batch(alg, b.keys, b.remote_index, slot_desc(b, ciphers), b.arena, b.stride, "q")
        fl = _flushes(bd, per)
        pinned = []
        if zc:  # every other flush in pinned, mapped memory
            for j in range(1, len(fl), 2):
                f0, d, a, lo = fl[j]
                pb = PinnedBuffer(a.nbytes)
                pb.array[:] = a
                pinned.append(pb)
                fl[j] = (f0, d, pb.array, lo)
        results = {}
        errors = []

        def worker(t):
            try:
                for j in range(t, len(fl), threads):
                    f0, d, a, lo = fl[j]
                    st = seal_q.submit(d, a)
                    sealed = a.copy()
                    st2 = open_q.submit(d, a)
                    results[j] = (st, sealed, st2, a.copy())
            except Exception as ex:  # surfaced below
                errors.append(ex)

        ths = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        assert not errors, errors
        for j, (f0, d, a, lo) in enumerate(fl):
            st, sealed, st2, opened = results[j]
            assert (st == 0).all() and (st2 == 0).all()
            assert np.array_equal(sealed, ref[lo:lo + len(sealed)]), j
            # open restores the plaintext; the tags stay behind the payloads, as an in-place open
            exp = ref[lo:lo + len(sealed)].copy()
            oracle_mod.batch(alg, 1, b.keys, _rebase(b.desc[f0:f0 + len(d)], lo), exp)
            assert np.array_equal(opened, exp), j
        s1, s2 = seal_q.stats(), open_q.stats()
        assert s1["packets"] == b.n and s2["packets"] == b.n
        assert s1["submissions"] == len(fl)
        # the point of the queue: far fewer device batches than flushes
        assert s1["batches"] < len(fl), s1
        if zc:  # the pinned flushes staged nothing: only the others' bytes went through staging
            assert 0 < s1["bytes"] < sum(a.nbytes for _, _, a, _ in fl)
    finally:
        seal_q.close()
        open_q.close()
        if zc:
            for pb in pinned:
                pb.free()
        for c in ciphers:
            c.destroy()


def _rebase(d, lo):
    d = d.copy()
    for k in ("src_off", "dst_off", "aad_off"):
        d[k] -= np.uint64(lo)
    return d


def test_queue_failures_and_bad_descriptors(engine, oracle_mod):
    """Through the queue, a tampered packet fails only itself (its payload zeroed, as an in-place
    open does), an exhausted counter is refused with nothing written, an uninstalled key gets
    BAD_KEY, and a descriptor past the arena is refused before anything is staged."""
    from nebula_amd.batch import SubmitQueue, install_keys, slot_desc

    b = W.make_batch(L.ALG_AESGCM, 64, 4, name="qfail")
    ciphers = install_keys(engine, b)
    sq = SubmitQueue(engine, L.ALG_AESGCM, False)
    oq = SubmitQueue(engine, L.ALG_AESGCM, True)
    try:
        d = slot_desc(b, ciphers)
        a = b.arena.copy()
        d2 = d.copy()
        d2["counter"][5] = L.REJECT_AFTER_MESSAGES
        d2["key_id"][6] = engine.max_keys - 1
        st = sq.submit(d2, a)
        assert st[5] == L.STATUS_EXHAUSTED and st[6] == L.STATUS_BAD_KEY
        assert (np.delete(st, [5, 6]) == 0).all()
        s5 = int(d["src_off"][5])
        assert np.array_equal(a[s5:s5 + 1316], b.arena[s5:s5 + 1316])
        ref = b.arena.copy()
        oracle_mod.batch(L.ALG_AESGCM, 0, b.keys, b.desc, ref)
        ok = np.array([i not in (5, 6) for i in range(b.n)])
        for i in np.flatnonzero(ok):
            s, ln = int(d["src_off"][i]), int(d["len"][i])
            assert np.array_equal(a[s:s + ln + 16], ref[s:s + ln + 16])
        t = ref.copy()
        t[int(d["src_off"][9]) + 3] ^= 1
        st = oq.submit(d, t)
        assert st[9] == L.STATUS_AUTH_FAILED and (np.delete(st, 9) == 0).all()
        s9 = int(d["src_off"][9])
        assert not t[s9:s9 + 1300].any()
        bad = d.copy()
        bad["len"][-1] = b.stride * 4
        before = t.copy()
        with pytest.raises(Exception):
            oq.submit(bad, t)
        assert np.array_equal(t, before)
    finally:
        sq.close()
        oq.close()
        for c in ciphers:
            c.destroy()


def test_queue_first_batches_of_fresh_queues(engine, oracle_mod):
    """The first batch of a new queue runs on a freshly allocated scheduler workspace: its counters
    are cleared on the batch's own stream, before the binning (a null-stream clear raced the first
    mixed-key batches and left most of their statuses unwritten). Fresh queues, one full mixed-key
    batch each, seal then open, against the oracle."""
    from nebula_amd.batch import SubmitQueue, install_keys, slot_desc

    b = W.make_batch(L.ALG_AESGCM, 8192, 64, sizes=(90, 576, 1300), ratio=(7, 4, 1), seed=81, name="qfresh")
    ref = b.arena.copy()
    assert (oracle_mod.batch(L.ALG_AESGCM, 0, b.keys, b.desc, ref) == 0).all()
    ciphers = install_keys(engine, b)
    try:
        d = slot_desc(b, ciphers)
        for rep in range(6):
            sq = SubmitQueue(engine, L.ALG_AESGCM, False, max_packets=8192, max_delay_us=100000)
            oq = SubmitQueue(engine, L.ALG_AESGCM, True, max_packets=8192, max_delay_us=100000)
            try:
                a = b.arena.copy()
                st = sq.submit(d, a)
                assert (st == 0).all(), (rep, int((st != 0).sum()), int(st[st != 0][0]))
                assert np.array_equal(a, ref), rep
                st = oq.submit(d, a)
                assert (st == 0).all(), (rep, int((st != 0).sum()), int(st[st != 0][0]))
            finally:
                sq.close()
                oq.close()
    finally:
        for c in ciphers:
            c.destroy()
