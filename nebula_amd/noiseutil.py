"""Host-side mirror of Nebula's noiseutil data-plane surface, backed by the gfx950 engine.

Reference interface (slackhq/nebula):
  noiseutil/cipher_state.go:11-18   RejectHeadroom, RejectAfterMessages, ErrMessageCounterExhausted
  noiseutil/cipher_state.go:23-38   CipherState {EncryptDanger, DecryptDanger, Overhead}
  noiseutil/cipher_state.go:42-54   NewCipherState (plugin hook + dispatch by CipherName, panic on unknown)
  noiseutil/aesgcm.go:11-56         CipherStateAESGCM (nonce 00000000 || BE64(n))
  noiseutil/chachapoly.go:11-55     CipherStateChaChaPoly (nonce 00000000 || LE64(n))
  flynn/noise v1.1.0 CipherFunc     Cipher(k [32]byte), CipherName()  [ext; pattern: noiseutil/fips140.go:31-40]

Go slices are modelled by `Slice` (backing bytearray + offset + len + cap) so that the append,
aliasing and in-place rules of the reference (inside.go:131, connection_state.go:107,
cipher_state_test.go:194-237) are exercised for real: the engine receives raw pointers into the
same buffer Python holds.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Union

from . import _lib as L

RejectHeadroom = L.REJECT_HEADROOM
RejectAfterMessages = L.REJECT_AFTER_MESSAGES


class ErrMessageCounterExhausted(Exception):
    """noiseutil/cipher_state.go:18 — "message counter exhausted"."""


class ErrOpen(Exception):
    """crypto/cipher — "cipher: message authentication failed"."""


class ErrNoCipher(Exception):
    """aesgcm.go:26 — "no cipher state available to encrypt"."""


class Slice:
    """A Go []byte: a window [off, off+len) of `buf` with capacity `cap` (from off)."""

    __slots__ = ("buf", "off", "len", "cap")

    def __init__(self, buf: bytearray, off: int = 0, length: Optional[int] = None, cap: Optional[int] = None):
        self.buf = buf
        self.off = off
        self.cap = (len(buf) - off) if cap is None else cap
        self.len = self.cap if length is None else length
        assert 0 <= self.len <= self.cap and off + self.cap <= len(buf)

    @classmethod
    def make(cls, length: int, cap: Optional[int] = None) -> "Slice":
        cap = length if cap is None else cap
        return cls(bytearray(cap), 0, length, cap)

    @classmethod
    def of(cls, data: Union[bytes, bytearray, "Slice"]) -> "Slice":
        if isinstance(data, Slice):
            return data
        return cls(bytearray(data))

    def __getitem__(self, k: slice) -> "Slice":
        # Go reslicing s[a:b] (b may run up to cap)
        a = 0 if k.start is None else k.start
        b = self.len if k.stop is None else k.stop
        assert 0 <= a <= b <= self.cap
        return Slice(self.buf, self.off + a, b - a, self.cap - a)

    def __len__(self) -> int:
        return self.len

    def bytes(self) -> bytes:
        return bytes(self.buf[self.off:self.off + self.len])

    def __eq__(self, other) -> bool:
        if isinstance(other, Slice):
            other = other.bytes()
        return self.bytes() == bytes(other)

    def __repr__(self) -> str:
        return f"Slice(len={self.len}, cap={self.cap}, {self.bytes()[:32].hex()}...)"

    def ptr(self) -> int:
        # address of element 0 (valid even when len == 0, as long as cap > 0 or the buffer exists)
        if len(self.buf) == 0:
            return 0
        base = C.addressof((C.c_char * len(self.buf)).from_buffer(self.buf))
        return base + self.off

    def same_element(self, other: "Slice") -> bool:
        """&a[0] == &b[0] (cipher_state_test.go:236)."""
        return self.buf is other.buf and self.off == other.off


def _as_slice(x) -> Optional[Slice]:
    if x is None:
        return None
    return x if isinstance(x, Slice) else Slice(bytearray(x))


class Engine:
    """One engine per GPU (neb_engine_create): device stream + key table."""

    def __init__(self, device: int = 0, max_keys: int = 4096):
        h = C.c_void_p()
        L.check(L.lib().neb_engine_create(device, max_keys, C.byref(h)), "neb_engine_create")
        self.handle = h
        self.device = device
        self.max_keys = max_keys
        self.live = {}  # id -> CipherState: the keys installed and not yet destroyed

    def stats(self) -> dict:
        v = (C.c_uint64 * 4)()
        L.check(L.lib().neb_engine_stats(self.handle, v), "neb_engine_stats")
        c = (C.c_uint64 * 2)()
        L.check(L.lib().neb_engine_pkt_combined(self.handle, c), "neb_engine_pkt_combined")
        return {"pkt_slots": v[0], "pkt_calls": v[1], "pkt_waits": v[2], "installs": v[3],
                "pkt_combined_launches": c[0], "pkt_combined_calls": c[1]}

    def close(self) -> None:
        if self.handle:
            L.lib().neb_engine_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class CipherFunc:
    """flynn/noise CipherFunc: Cipher(k) installs the key on an engine; CipherName() is protocol."""

    def __init__(self, name: str, alg: int):
        self.name = name
        self.alg = alg

    def CipherName(self) -> str:
        return self.name

    def Cipher(self, engine: Engine, k: bytes) -> "CipherState":
        assert len(k) == 32
        h = C.c_void_p()
        L.check(L.lib().neb_cipher_create(engine.handle, self.alg, bytes(k), C.byref(h)), "neb_cipher_create")
        cls = CipherStateAESGCM if self.alg == L.ALG_AESGCM else CipherStateChaChaPoly
        cs = cls(h, engine)
        engine.live[id(cs)] = cs
        return cs


    def _wrap(self, h, engine: Engine) -> "CipherState":
        cls = CipherStateAESGCM if self.alg == L.ALG_AESGCM else CipherStateChaChaPoly
        cs = cls(C.c_void_p(h), engine)
        engine.live[id(cs)] = cs
        return cs

    def CipherBatch(self, engine: Engine, keys) -> "list[CipherState]":
        """Cipher(k) for many keys in one device launch (neb_cipher_create_batch): the tunnels a
        lighthouse or a rekey storm completes together (handshake_manager.go:752,877)."""
        keys = [bytes(k) for k in keys]
        assert all(len(k) == 32 for k in keys)
        if not keys:
            return []
        out = (C.c_void_p * len(keys))()
        L.check(L.lib().neb_cipher_create_batch(engine.handle, self.alg, b"".join(keys), len(keys), out),
                "neb_cipher_create_batch")
        return [self._wrap(h, engine) for h in out]

    def CipherMulti(self, engines, k: bytes) -> "list[CipherState]":
        """One tunnel key on every engine of a set, at one key_id (neb_cipher_create_multi): the
        install the multi-engine batch calls require (connection_state.go:37-49, one eKey/dKey)."""
        assert len(k) == 32
        hs = (C.c_void_p * len(engines))(*[e.handle.value for e in engines])
        out = (C.c_void_p * len(engines))()
        L.check(L.lib().neb_cipher_create_multi(hs, len(engines), self.alg, bytes(k), out), "neb_cipher_create_multi")
        return [self._wrap(h, e) for h, e in zip(out, engines)]


CipherAESGCM = CipherFunc("AESGCM", L.ALG_AESGCM)
CipherChaChaPoly = CipherFunc("ChaChaPoly", L.ALG_CHACHAPOLY)


class CipherState:
    """noiseutil.CipherState over one installed key. handle None models a nil receiver."""

    alg = 0

    def __init__(self, handle: Optional[C.c_void_p], engine: Optional[Engine] = None):
        self.handle = handle
        self.engine = engine

    @classmethod
    def nil(cls) -> "CipherState":
        return cls(None)

    @property
    def key_id(self) -> int:
        return int(L.lib().neb_cipher_key_id(self.handle))

    def destroy(self) -> None:
        if self.handle:
            L.lib().neb_cipher_destroy(self.handle)
            self.handle = None
            if self.engine is not None:
                self.engine.live.pop(id(self), None)

    def Overhead(self) -> int:
        return int(L.lib().neb_overhead(self.handle))

    def EncryptDanger(self, out, ad, plaintext, n: int, nb: Optional[bytearray] = None) -> Slice:
        out = _as_slice(out) if out is not None else Slice.make(0)
        ad = _as_slice(ad) if ad is not None else Slice.make(0)
        plaintext = _as_slice(plaintext) if plaintext is not None else Slice.make(0)
        if not self.handle:
            raise ErrNoCipher("no cipher state available to encrypt")
        need = out.len + plaintext.len + L.OVERHEAD
        if need > out.cap:
            # Go's append grows into a fresh backing array (the result no longer aliases `out`)
            grown = Slice.make(out.len, need)
            grown.buf[:out.len] = out.buf[out.off:out.off + out.len]
            out = grown
        ret = C.c_size_t(0)
        nbuf = (C.c_uint8 * 12)()
        rc = L.lib().neb_encrypt_danger(self.handle, out.ptr(), out.len, out.cap, ad.ptr(), ad.len,
                                        plaintext.ptr(), plaintext.len, C.c_uint64(n & (2**64 - 1)), nbuf,
                                        C.byref(ret))
        if rc == L.ERR_EXHAUSTED:
            raise ErrMessageCounterExhausted("message counter exhausted")
        L.check(rc, "EncryptDanger")
        if nb is not None:
            nb[:12] = bytes(nbuf)
        return Slice(out.buf, out.off, ret.value, out.cap)

    def DecryptDanger(self, out, ad, ciphertext, n: int, nb: Optional[bytearray] = None) -> Slice:
        if not self.handle:
            return Slice.make(0)  # aesgcm.go:40-42: []byte{}, nil
        out = _as_slice(out) if out is not None else Slice.make(0)
        ad = _as_slice(ad) if ad is not None else Slice.make(0)
        ciphertext = _as_slice(ciphertext) if ciphertext is not None else Slice.make(0)
        need = out.len + max(ciphertext.len - L.OVERHEAD, 0)
        if need > out.cap:
            grown = Slice.make(out.len, need)
            grown.buf[:out.len] = out.buf[out.off:out.off + out.len]
            out = grown
        ret = C.c_size_t(0)
        nbuf = (C.c_uint8 * 12)()
        rc = L.lib().neb_decrypt_danger(self.handle, out.ptr(), out.len, out.cap, ad.ptr(), ad.len,
                                        ciphertext.ptr(), ciphertext.len, C.c_uint64(n & (2**64 - 1)), nbuf,
                                        C.byref(ret))
        if nb is not None:
            nb[:12] = bytes(nbuf)
        if rc == L.ERR_AUTH:
            raise ErrOpen("cipher: message authentication failed")
        L.check(rc, "DecryptDanger")
        return Slice(out.buf, out.off, ret.value, out.cap)


class CipherStateAESGCM(CipherState):
    alg = L.ALG_AESGCM


class CipherStateChaChaPoly(CipherState):
    alg = L.ALG_CHACHAPOLY


def NewCipherState(s, cipher_func: CipherFunc) -> CipherState:
    """noiseutil/cipher_state.go:42-54. `s` is an already-installed CipherState (the plugin hook:
    returned as-is) or a (engine, key) pair from the handshake, installed under cipher_func."""
    if isinstance(s, CipherState):
        return s
    name = cipher_func.CipherName()
    if name not in (CipherAESGCM.CipherName(), CipherChaChaPoly.CipherName()):
        raise RuntimeError(f'noiseutil: unsupported cipher "{name}"')
    engine, key = s
    return cipher_func.Cipher(engine, key)
