"""Generate the committed golden fixtures in tests/golden/ (run from the repo root:
`python tests/golden/make_golden.py`).

Sources, in order of authority:
  1. Vectors held by the reference's own tests (copied here as DATA, not code):
       noiseutil/fips140_test.go:18-31  AES-256-GCM KAT (the only AEAD known-answer test in the reference)
       header/header_test.go:17-29      header encode/parse KAT
  2. Published standards the reference's third-party dependencies implement:
       RFC 8439 §2.8.2 ChaCha20-Poly1305 AEAD vector (x/crypto v0.54.0 chacha20poly1305)
  3. Batch digests for the BASELINE.json configs, produced by the plain-C oracle
     (oracle/aead_oracle.c) and independently re-derived with OpenSSL EVP
     (oracle/evp_baseline.c); the script refuses to write if the two disagree. Scaled batches
     (tags committed) in batches.json, and the full C2-C5 batches (64 Ki x 1300 B; 1 Mi IMIX)
     as SHA-256 digests of the whole sealed and opened arenas in full_digests.json
     (`--no-full` skips them: about a minute on 8 cores).

The Go reference itself cannot run here (no Go toolchain), so (3) is pinned by (1)+(2) through
the oracle, not by Go output.
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402
from nebula_amd import workload as W  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))

KAT = {
    "aesgcm_fips140_test": {
        "source": "noiseutil/fips140_test.go:18-31",
        "key": "feffe9928665731c6d6a8f9467308308feffe9928665731c6d6a8f9467308308",
        "iv": "00000000facedbaddecaf888",
        "nebula_counter": "facedbaddecaf888",
        "plaintext": "d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a721c3c0c95956809532fcf0e2449a6b525b16aedf5aa0de657ba637b39",
        "aad": "feedfacedeadbeeffeedfacedeadbeefabaddad2",
        "expected": "6a65c2edd45bd63c7e29f40e3d2ed8ba2b99f4c83135383d5676652f255059ceb24863ff10afb1089db701245da87fb88d3acd5f9dd0770cac220c3c04145caf25e190aeb775e7080401c628",
    },
    "chachapoly_rfc8439_2_8_2": {
        "source": "RFC 8439 §2.8.2 (x/crypto chacha20poly1305 is pinned to it); tag cross-checked in SURVEY.md §8c",
        "key": "808182838485868788898a8b8c8d8e8f909192939495969798999a9b9c9d9e9f",
        "iv": "070000004041424344454647",
        "plaintext": b"Ladies and Gentlemen of the class of '99: If I could offer you only one tip for the future, sunscreen would be it.".hex(),
        "aad": "50515253c0c1c2c3c4c5c6c7",
        "expected_tag": "1ae10b594f09e26a7e902ecbd0600691",
        "expected_ct_prefix": "d31a8d34648e60db7b86afbc53ef7ec2",
    },
    "header_test": {
        "source": "header/header_test.go:17-29",
        "fields": {"Version": 5, "Type": 4, "Subtype": 0, "Reserved": 0, "RemoteIndex": 10, "MessageCounter": 9},
        "bytes": "540000000000000a0000000000000009",
    },
}

# small batches (sizes the oracle finishes in seconds)
BATCHES = {
    "c1_aesgcm_1key_1024x1300": lambda: W.config(0),
    "c3_aesgcm_4096keys_512x1300": lambda: W.make_batch(1, 512, 4096, name="C3 scaled"),
    "c4_chachapoly_4096keys_512x1300": lambda: W.make_batch(2, 512, 4096, name="C4 scaled"),
    "c5_aesgcm_imix_4096keys_2048": lambda: W.make_batch(1, 2048, 4096, sizes=(90, 576, 1300), ratio=(7, 4, 1),
                                                         name="C5 scaled"),
}


# the BASELINE.json configs at full size: only digests are committed. The script
# refuses to write unless the plain-C oracle (multithreaded over disjoint packet ranges) and the
# OpenSSL EVP port produce the same sealed arena byte for byte.
FULL = {
    "c2_full": lambda: W.config(1),
    "c3_full": lambda: W.config(2),
    "c4_full": lambda: W.config(3),
    "c5_full": lambda: W.config(4),
}


def oracle_threaded(alg, open_flag, keys, desc, arena, threads=8):
    """oracle.batch over `threads` disjoint descriptor ranges at once (ctypes drops the GIL)."""
    import threading

    st = np.zeros(len(desc), np.int32)
    bounds = [len(desc) * t // threads for t in range(threads + 1)]

    def run(t):
        st[bounds[t]:bounds[t + 1]] = oracle.batch(alg, open_flag, keys, desc[bounds[t]:bounds[t + 1]], arena)

    ths = [threading.Thread(target=run, args=(t,)) for t in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    return st


def full_digests(b):
    sealed = b.arena.copy()
    assert (oracle_threaded(b.alg, 0, b.keys, b.desc, sealed) == 0).all()
    evp = b.arena.copy()
    _, st = oracle.evp_batch(b.alg, 0, b.keys, b.desc, evp, threads=8)
    assert (st == 0).all()
    if not np.array_equal(sealed, evp):
        raise SystemExit("oracle and OpenSSL EVP disagree on a full batch — refusing to write fixtures")
    del evp
    opened = sealed.copy()
    assert (oracle_threaded(b.alg, 1, b.keys, b.desc, opened) == 0).all()
    return {
        "n": b.n, "nkeys": b.nkeys, "alg": b.alg, "stride": b.stride, "name": b.name,
        "plain_sha256": hashlib.sha256(b.arena.tobytes()).hexdigest(),
        "sealed_sha256": hashlib.sha256(sealed.tobytes()).hexdigest(),
        "opened_sha256": hashlib.sha256(opened.tobytes()).hexdigest(),
    }


def sealed_digest(b):
    arena = b.arena.copy()
    st = oracle.batch(b.alg, 0, b.keys, b.desc, arena)
    assert (st == 0).all()
    evp_arena = b.arena.copy()
    _, st2 = oracle.evp_batch(b.alg, 0, b.keys, b.desc, evp_arena, threads=4)
    assert (st2 == 0).all()
    if not np.array_equal(arena, evp_arena):
        raise SystemExit("oracle and OpenSSL EVP disagree — refusing to write fixtures")
    # round trip through the oracle's open
    rt = arena.copy()
    st3 = oracle.batch(b.alg, 1, b.keys, b.desc, rt)
    slots = arena.reshape(b.n, b.stride)
    tags = np.stack([slots[i, 16 + int(b.desc["len"][i]):32 + int(b.desc["len"][i])] for i in range(b.n)])
    rts = rt.reshape(b.n, b.stride)
    for i in range(b.n):  # the opened arena still carries the tags after the payload
        rts[i, 16 + int(b.desc["len"][i]):32 + int(b.desc["len"][i])] = 0
    assert (st3 == 0).all() and np.array_equal(rt, b.arena)
    return arena, tags


def main():
    oracle.build()
    with open(os.path.join(OUT, "kat.json"), "w") as f:
        json.dump(KAT, f, indent=1)
    meta = {}
    for name, mk in BATCHES.items():
        b = mk()
        arena, tags = sealed_digest(b)
        np.save(os.path.join(OUT, f"{name}_tags.npy"), tags)
        meta[name] = {
            "n": b.n, "nkeys": b.nkeys, "alg": b.alg, "stride": b.stride,
            "plain_sha256": hashlib.sha256(b.arena.tobytes()).hexdigest(),
            "sealed_sha256": hashlib.sha256(arena.tobytes()).hexdigest(),
            "tags_sha256": hashlib.sha256(tags.tobytes()).hexdigest(),
        }
        print(name, meta[name]["sealed_sha256"][:16])
    with open(os.path.join(OUT, "batches.json"), "w") as f:
        json.dump(meta, f, indent=1)
    if "--no-full" not in sys.argv:
        full = {}
        for name, mk in FULL.items():
            b = mk()
            full[name] = full_digests(b)
            print(name, full[name]["sealed_sha256"][:16])
            del b
        with open(os.path.join(OUT, "full_digests.json"), "w") as f:
            json.dump(full, f, indent=1)


if __name__ == "__main__":
    main()
