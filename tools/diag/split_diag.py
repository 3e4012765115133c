"""Diagnostic: split host mode on a small batch vs the oracle; prints where bytes differ."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import oracle
from nebula_amd import _lib as L
from nebula_amd import workload as W
from nebula_amd.batch import PinnedBuffer, host_batch, install_keys, slot_desc
from nebula_amd.noiseutil import Engine
os.environ["NEB_HOST_MODE"] = sys.argv[1] if len(sys.argv) > 1 else "split"
for nkeys, n in ((1, 64), (4, 64), (1, 20000)):
    b = W.make_batch(L.ALG_AESGCM, n, nkeys, sizes=(90, 576, 1300), ratio=(7, 4, 1), name="diag")
    with Engine(0, 64) as eng:
        ciphers = install_keys(eng, b)
        buf = PinnedBuffer(b.arena.nbytes)
        buf.array[:] = b.arena
        d = slot_desc(b, ciphers)
        st = host_batch(eng, b.alg, False, d, buf.array, int(d["key_id"][0]) if nkeys == 1 else L.KEYS_MIXED)
        ref = b.arena.copy()
        oracle.batch(b.alg, 0, b.keys, b.desc, ref)
        got = buf.array.copy()
        diff = np.nonzero(got != ref)[0]
        print(f"keys={nkeys} n={n} status_ok={(st == 0).all()} differing_bytes={len(diff)}")
        if len(diff):
            bad_pk = sorted(set(int(np.searchsorted(b.desc['aad_off'], x, side='right') - 1) for x in diff[:2000]))
            print("  first diffs", diff[:8], "packets", bad_pk[:10], "of", n)
            i = bad_pk[0]
            dd = b.desc[i]
            print("  desc", dd)
            s0 = int(dd['src_off'])
            print("  got ", got[s0:s0 + 32].tobytes().hex())
            print("  ref ", ref[s0:s0 + 32].tobytes().hex())
            print("  orig", b.arena[s0:s0 + 32].tobytes().hex())
        buf.free()
        for c in ciphers:
            c.destroy()
