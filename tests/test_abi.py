"""CPU: the C-ABI library loads and exports every symbol include/nebula_aead.h declares; the
constants in the header, the Python binding and the oracle agree; host-only ABI calls (header
encode/parse, error paths that never reach a device) behave like the reference.
No compute call reaches a GPU here."""
import ctypes as C
import json
import os
import re

import pytest

from nebula_amd import _lib as L
from nebula_amd import header as Hd
from nebula_amd import noiseutil as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "nebula_aead.h")


def declared_symbols():
    text = open(HDR).read()
    return sorted(set(re.findall(r"NEB_API\s+[\w\s\*]+?\b(neb_\w+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = L.lib()
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(L.SIGNATURES), set(syms) ^ set(L.SIGNATURES)


def test_library_is_built_from_these_sources():
    """neb_build_id() is the SHA-256 of the sources the library was compiled from (nebula_amd/Makefile:
    SRC then HDR, concatenated): equal to the hash of the sources in this tree, so the .so a test
    run loads (here, or the prebuilt one shipped to a GPU box) is HEAD's code, not a stale build."""
    import hashlib

    nd = os.path.join(ROOT, "nebula_amd")
    mk = open(os.path.join(nd, "Makefile")).read()
    files = []
    for var in ("SRC", "HDR"):
        files += re.search(rf"^{var} := (.*)$", mk, re.M).group(1).split()
    h = hashlib.sha256(b"".join(open(os.path.join(nd, f), "rb").read() for f in files)).hexdigest()[:16]
    assert L.lib().neb_build_id().decode() == h


def test_library_has_no_unresolved_symbols():
    """Binding every symbol at load time (RTLD_NOW) fails on a reference the build left undefined,
    which a lazy load only reports at the first call into it."""
    C.CDLL(L.LIB_PATH, mode=os.RTLD_NOW | os.RTLD_LOCAL)


def test_header_constants_match_binding():
    text = open(HDR).read()

    def val(name):
        m = re.search(rf"#define {name} \(?(-?\w+)\)?", text)
        return int(m.group(1), 0)

    assert val("NEB_ALG_AESGCM") == L.ALG_AESGCM and val("NEB_ALG_CHACHAPOLY") == L.ALG_CHACHAPOLY
    assert val("NEB_OVERHEAD") == L.OVERHEAD == 16
    for n in ("INVALID", "AUTH", "EXHAUSTED", "NO_CIPHER", "SHORT_BUFFER", "HIP", "NO_DEVICE", "NO_KEY_SLOT"):
        assert val(f"NEB_ERR_{n}") == getattr(L, f"ERR_{n}")
    for n in ("OK", "AUTH_FAILED", "EXHAUSTED", "BAD_KEY"):
        assert val(f"NEB_STATUS_{n}") == getattr(L, f"STATUS_{n}")
    assert L.REJECT_AFTER_MESSAGES == 2**64 - 1 - 2**40  # cipher_state.go:11-15


def test_cipher_names():
    assert L.lib().neb_cipher_name(1) == b"AESGCM"
    assert L.lib().neb_cipher_name(2) == b"ChaChaPoly"
    assert L.lib().neb_cipher_name(3) is None


def test_header_kat_via_abi():  # header/header_test.go:17-53
    k = json.load(open(os.path.join(ROOT, "tests", "golden", "kat.json")))["header_test"]
    f = k["fields"]
    h = Hd.H(**f)
    assert h.Encode().hex() == k["bytes"]
    p = Hd.H()
    p.Parse(bytes.fromhex(k["bytes"]))
    assert p == h
    with pytest.raises(Hd.ErrHeaderTooShort):
        Hd.H().Parse(b"\0" * 15)


def test_header_encode_many_matches_encode():
    import numpy as np

    ri = np.array([0, 10, 0xDEADBEEF], np.uint32)
    c = np.array([9, 2**64 - 1, 3], np.uint64)
    many = Hd.encode_many(ri, c)
    for i in range(3):
        assert many[i].tobytes() == Hd.Encode(None, 1, 1, 0, int(ri[i]), int(c[i]))


def test_nil_cipher_paths_need_no_device():
    """Nil receiver semantics are resolved in the ABI before any device work (aesgcm.go:25-27,40-42,52-54)."""
    lib = L.lib()
    ret = C.c_size_t(7)
    assert lib.neb_encrypt_danger(None, None, 0, 0, None, 0, None, 0, 0, None, C.byref(ret)) == L.ERR_NO_CIPHER
    assert lib.neb_decrypt_danger(None, None, 0, 0, None, 0, None, 0, 0, None, C.byref(ret)) == L.OK
    assert ret.value == 0
    assert lib.neb_overhead(None) == 0
    nil = N.CipherStateAESGCM.nil()
    assert nil.Overhead() == 0 and len(nil.DecryptDanger(None, None, None, 0)) == 0


def test_engine_create_without_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(L.NebError) as ei:
        N.Engine(0, 16)
    assert ei.value.rc == L.ERR_NO_DEVICE


def test_batch_rejects_bad_args_without_gpu():
    lib = L.lib()
    assert lib.neb_seal_batch(None, 1, None, 0, None, None, L.KEYS_MIXED, None) == L.ERR_INVALID
    assert lib.neb_strerror(L.ERR_AUTH) == b"cipher: message authentication failed"


def test_knobs_set_get_and_defaults():
    """neb_set_knob / neb_get_knob: process-wide A/B and test knobs (no GPU involved). Defaults come
    from the environment once; an unknown knob is refused; a set value is read back and restored."""
    lib = L.lib()
    assert lib.neb_get_knob(-1) == -1 and lib.neb_get_knob(99) == -1
    assert lib.neb_set_knob(99, 1) == L.ERR_INVALID
    if "NEB_SUB_BINS_FROM" not in os.environ:
        assert lib.neb_get_knob(L.KNOB_SUB_BINS_FROM) == 1 << 18
    for k in (L.KNOB_HOST_MODE, L.KNOB_SUB_BINS_FROM, L.KNOB_SINGLE_MAX_GRID, L.KNOB_RX_STRICT, L.KNOB_TILE_BINS_FROM):
        old = lib.neb_get_knob(k)
        with L.knob(k, 12345):
            assert lib.neb_get_knob(k) == 12345
        assert lib.neb_get_knob(k) == old


def test_time_last_kernel_empty_before_any_batch():
    assert L.lib().neb_time_last_kernel() == b""
