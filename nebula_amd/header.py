"""Nebula v1 wire header (the AAD) — header/header.go:10-110,143-156, via the C ABI."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L

Version = 1
Len = 16

Handshake, Message, RecvError, LightHouse, Test, CloseTunnel, Control = range(7)
MessageNone, MessageRelay = 0, 1


class ErrHeaderTooShort(ValueError):
    pass


@dataclass
class H:
    Version: int = 0
    Type: int = 0
    Subtype: int = 0
    Reserved: int = 0
    RemoteIndex: int = 0
    MessageCounter: int = 0

    def Encode(self, b: bytearray = None) -> bytes:
        return Encode(b, self.Version, self.Type, self.Subtype, self.RemoteIndex, self.MessageCounter)

    def Parse(self, b: bytes) -> None:
        v, t, st, res, ri, c = C.c_uint8(), C.c_uint8(), C.c_uint8(), C.c_uint16(), C.c_uint32(), C.c_uint64()
        rc = L.lib().neb_header_parse(bytes(b), len(b), C.byref(v), C.byref(t), C.byref(st), C.byref(res),
                                      C.byref(ri), C.byref(c))
        if rc != L.OK:
            raise ErrHeaderTooShort("header is too short")
        self.Version, self.Type, self.Subtype = v.value, t.value, st.value
        self.Reserved, self.RemoteIndex, self.MessageCounter = res.value, ri.value, c.value


def Encode(b, v: int, t: int, st: int, ri: int, c: int) -> bytes:
    """header.Encode (header.go:102-110). Writes into b[:16] when b is a bytearray."""
    out = (C.c_uint8 * 16)()
    L.lib().neb_header_encode(out, v, t, st, ri, C.c_uint64(c))
    raw = bytes(out)
    if isinstance(b, bytearray):
        b[:16] = raw
    return raw


def encode_many(remote_index: np.ndarray, counter: np.ndarray, v: int = Version, t: int = Message,
                st: int = MessageNone) -> np.ndarray:
    """Vectorised header.Encode for batch construction: returns an (n, 16) uint8 array."""
    n = len(counter)
    h = np.zeros((n, 16), np.uint8)
    h[:, 0] = (v << 4) | (t & 0x0F)
    h[:, 1] = st
    ri = remote_index.astype(">u4").view(np.uint8).reshape(n, 4)
    h[:, 4:8] = ri
    h[:, 8:16] = counter.astype(">u8").view(np.uint8).reshape(n, 8)
    return h
