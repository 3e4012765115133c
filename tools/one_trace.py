"""Phase stamps of the per-packet AES-GCM kernel: run under NEB_LIB_PATH=build_var/onetrace (a
-DNEB_ONE_TRACE=1 build, tools/build_variant.sh), which prints fill / keys / packet times from lane 0
of each call's kernel (s_memrealtime, 10 ns units). 1300-B packets, seal then open, a few calls."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from nebula_amd import noiseutil as N  # noqa: E402
from nebula_amd.noiseutil import Engine  # noqa: E402

with Engine(0, 64) as e:
    enc = N.NewCipherState((e, bytes(range(32))), N.CipherAESGCM)
    dec = N.NewCipherState((e, bytes(range(32))), N.CipherAESGCM)
    pt, ad, nb = bytes(1300), bytes(16), bytearray(12)
    for i in range(6):
        ct = enc.EncryptDanger(None, ad, pt, i + 1, nb)
        assert dec.DecryptDanger(None, ad, ct, i + 1, nb).bytes() == pt
    enc.destroy(), dec.destroy()
print("one_trace done", flush=True)
