"""ctypes front end for the CPU checkers in oracle/ — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
The product (nebula_amd/) never imports it and has no fallback to it.

liboracle.so is the plain-C restatement (aead_oracle.c; see its header for the reference
file:line each function follows). libevpbaseline.so is the OpenSSL-EVP port of the per-packet
loop used as the CPU baseline and as a second, independent checker.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
AES = 1
CHACHA = 2

DESC_DTYPE = np.dtype(
    [("src_off", "<u8"), ("dst_off", "<u8"), ("aad_off", "<u8"), ("counter", "<u8"),
     ("len", "<u4"), ("aad_len", "<u4"), ("key_id", "<u4"), ("flags", "<u4")]
)

_lib = None
_evp = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _load(name):
    path = os.path.join(HERE, name)
    if not os.path.exists(path):
        build()
    return C.CDLL(path)


def lib():
    global _lib
    if _lib is None:
        _lib = _load("liboracle.so")
        _lib.ora_encrypt_danger.restype = C.c_long
        _lib.ora_decrypt_danger.restype = C.c_long
        _lib.ora_reject_after_messages.restype = C.c_uint64
        _lib.ora_aes256gcm_open.restype = C.c_int
        _lib.ora_chacha20poly1305_open.restype = C.c_int
        _lib.ora_header_parse.restype = C.c_int
    return _lib


def evp():
    global _evp
    if _evp is None:
        _evp = _load("libevpbaseline.so")
        _evp.evb_run.restype = C.c_double
        _evp.evb_run.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t,
                                 C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                 C.POINTER(C.c_long)]
    return _evp


def _p(b):
    if isinstance(b, np.ndarray):
        return b.ctypes.data_as(C.c_void_p)
    return C.c_char_p(bytes(b))


def seal(alg: int, key: bytes, nonce: bytes, aad: bytes, pt: bytes) -> bytes:
    out = C.create_string_buffer(len(pt) + 16)
    f = lib().ora_aes256gcm_seal if alg == AES else lib().ora_chacha20poly1305_seal
    f(key, nonce, aad, C.c_size_t(len(aad)), pt, C.c_size_t(len(pt)), out)
    return out.raw


def open_(alg: int, key: bytes, nonce: bytes, aad: bytes, ct_tag: bytes):
    out = C.create_string_buffer(max(len(ct_tag) - 16, 1))
    f = lib().ora_aes256gcm_open if alg == AES else lib().ora_chacha20poly1305_open
    rc = f(key, nonce, aad, C.c_size_t(len(aad)), ct_tag, C.c_size_t(len(ct_tag)), out)
    return None if rc else out.raw[: len(ct_tag) - 16]


def nonce(alg: int, n: int) -> bytes:
    nb = C.create_string_buffer(12)
    lib().ora_nonce(alg, C.c_uint64(n), nb)
    return nb.raw


def header_encode(v: int, t: int, st: int, ri: int, c: int) -> bytes:
    b = C.create_string_buffer(16)
    lib().ora_header_encode(b, C.c_uint8(v), C.c_uint8(t), C.c_uint8(st), C.c_uint32(ri), C.c_uint64(c))
    return b.raw


def gf128_mul(x: bytes, y: bytes) -> bytes:
    z = C.create_string_buffer(16)
    lib().ora_gf128_mul(x, y, z)
    return z.raw


def aes_block(key: bytes, blk: bytes) -> bytes:
    out = C.create_string_buffer(16)
    lib().ora_aes256_encrypt_block(key, blk, out)
    return out.raw


def batch(alg: int, open_flag: int, keys: np.ndarray, desc: np.ndarray, arena: np.ndarray) -> np.ndarray:
    """Seal or open every descriptor in place on `arena` (uint8). Returns int32 status."""
    assert keys.dtype == np.uint8 and arena.dtype == np.uint8 and desc.dtype == DESC_DTYPE
    status = np.zeros(len(desc), np.int32)
    lib().ora_batch(C.c_int(alg), C.c_int(open_flag), _p(keys), _p(desc), C.c_size_t(len(desc)),
                    _p(arena), _p(status))
    return status


def evp_batch(alg: int, open_flag: int, keys: np.ndarray, desc: np.ndarray, arena: np.ndarray,
              threads: int = 1, iters: int = 1, pin: bool = True):
    """EVP port over the same descriptors. Returns (seconds, status)."""
    status = np.zeros(len(desc), np.int32)
    fails = C.c_long(0)
    t = evp().evb_run(alg, open_flag, _p(keys), len(keys) // 32, _p(desc), len(desc), _p(arena),
                      _p(status), threads, iters, 1 if pin else 0, C.byref(fails))
    return t, status
