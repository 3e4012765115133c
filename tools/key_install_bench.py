"""Batched key install (neb_cipher_create_batch): 4096 AES-256-GCM (or ChaCha20-Poly1305) tunnel keys
in one call, against 4096 calls of neb_cipher_create. One JSON line: wall ms of each form; run
under `rocprofv3 --kernel-trace --stats` for the GPU time of gcm_key_setup_kernel."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from nebula_amd import _lib as L
    from nebula_amd.noiseutil import CipherAESGCM, CipherChaChaPoly, Engine

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    single = "--single" in sys.argv
    out = {}
    for name, cf in (("aesgcm", CipherAESGCM), ("chachapoly", CipherChaChaPoly)):
        keys = [os.urandom(32) for _ in range(n)]
        with Engine(0, n) as e:
            cf.CipherBatch(e, keys[:8])  # warm: module load, first launch
            for c in list(e.live.values()):
                c.destroy()
            t0 = time.perf_counter()
            cs = cf.CipherBatch(e, keys)
            out[f"{name}_batch_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
            for c in cs:
                c.destroy()
            if single:
                t0 = time.perf_counter()
                cs = [cf.Cipher(e, k) for k in keys]
                out[f"{name}_single_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
                for c in cs:
                    c.destroy()
    out["keys"] = n
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
