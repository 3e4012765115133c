"""Host-side mirror of Nebula's receive-side connection state, backed by the engine's C ABI.

Reference interface (slackhq/nebula):
  bits.go:15-262                  Bits (NewBits, Check, Update, lost/duplicate/out-of-window counters)
  connection_state.go:17          ReplayWindow = 8192
  connection_state.go:52-75       newConnectionStateFromResult (MessageIndex < ReplayWindow; counters
                                  1..MessageIndex pre-marked in the window)
  connection_state.go:85-93       NextMessageCounter (pinned at RejectAfterMessages)
  connection_state.go:99-119      Decrypt: window Check → DecryptDanger (in place) → window Update
  connection_state.go:121-148     VerifyRelay: the same with the whole body as AD (GMAC only)
  handshake_manager.go:415        ErrAlreadySeen

`ConnectionState.decrypt_batch` is the batched receive path: the whole
recvmmsg flush goes through `neb_rx_open_batch_host`, which gives the same statuses, window state
and counters as calling `Decrypt` on each packet in arrival order.
"""
from __future__ import annotations

import ctypes as C
import threading
from typing import Optional, Sequence

import numpy as np

from . import _lib as L
from .noiseutil import CipherState, ErrOpen, RejectAfterMessages, Slice

ReplayWindow = 8192


class ErrAlreadySeen(Exception):
    """handshake_manager.go:415 — "already seen"."""


class Bits:
    """nebula.Bits on the engine's C++ window (neb_window_*)."""

    def __init__(self, length: int):
        self._lib = L.lib()
        h = C.c_void_p()
        rc = self._lib.neb_window_create(length, C.byref(h))
        if rc != L.OK:
            raise ValueError(f"Bits length must be a power of two, got {length}")
        self._h = h
        self.length = length

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def Check(self, i: int) -> bool:
        return self._lib.neb_window_check(self._h, i) == 1

    def Update(self, i: int) -> bool:
        return self._lib.neb_window_update(self._h, i) == 1

    def _state(self):
        cur = C.c_uint64()
        ctr = (C.c_int64 * 3)()
        L.check(self._lib.neb_window_state(self._h, C.byref(cur), ctr), "neb_window_state")
        return cur.value, tuple(ctr)

    @property
    def current(self) -> int:
        return self._state()[0]

    @property
    def lost(self) -> int:
        return self._state()[1][0]

    @property
    def dupe(self) -> int:
        return self._state()[1][1]

    @property
    def out_of_window(self) -> int:
        return self._state()[1][2]

    def get(self, slot: int) -> bool:
        return self._lib.neb_window_slot(self._h, slot) == 1

    def snapshot(self):
        return [self.get(s) for s in range(self.length)]

    def reset_counters(self) -> None:
        self._lib.neb_window_reset_counters(self._h)

    def destroy(self) -> None:
        if self._h:
            self._lib.neb_window_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


def NewBits(length: int) -> Bits:
    return Bits(length)


class ConnectionState:
    """The data-plane half of nebula.ConnectionState: eKey/dKey, the message counter and the
    replay window."""

    def __init__(self, ekey: CipherState, dkey: CipherState, message_index: int = 0):
        if message_index >= ReplayWindow:  # connection_state.go:56-59
            raise ValueError(f"handshake message index {message_index} exceeds replay window")
        self.eKey, self.dKey = ekey, dkey
        self.window = NewBits(ReplayWindow)
        self._ctr = message_index
        self._ctr_lock = threading.Lock()
        for i in range(1, message_index + 1):
            self.window.Update(i)

    def NextMessageCounter(self):
        with self._ctr_lock:
            self._ctr += 1
            c = self._ctr
            if c >= RejectAfterMessages:
                self._ctr = RejectAfterMessages
                return c, False
            return c, True

    def Decrypt(self, message_counter: int, packet: Slice, nb: Optional[bytearray] = None) -> Slice:
        """connection_state.go:99-119: packet = header ‖ ct ‖ tag; plaintext written in place."""
        if not self.window.Check(message_counter):
            raise ErrAlreadySeen()
        h = L.HEADER_LEN
        out = Slice(packet.buf, packet.off + h, 0, packet.cap - h)
        ad = Slice(packet.buf, packet.off, h, packet.cap)
        ct = Slice(packet.buf, packet.off + h, packet.len - h, packet.cap - h)
        res = self.dKey.DecryptDanger(out, ad, ct, message_counter, nb)  # raises ErrOpen
        if not self.window.Update(message_counter):
            raise ErrAlreadySeen()
        return res

    def VerifyRelay(self, message_counter: int, packet: Slice, nb: Optional[bytearray] = None) -> None:
        """connection_state.go:121-148: the body minus the trailing tag is AD; nothing decrypted."""
        if not self.window.Check(message_counter):
            raise ErrAlreadySeen()
        ov = self.dKey.Overhead()
        n = max(packet.len - ov, 0)
        signed = Slice(packet.buf, packet.off, n, packet.cap)
        sig = Slice(packet.buf, packet.off + n, packet.len - n, packet.cap - n)
        self.dKey.DecryptDanger(Slice.make(0), signed, sig, message_counter, nb)
        if not self.window.Update(message_counter):
            raise ErrAlreadySeen()


def rx_open_batch(engine, alg: int, windows: Sequence[Optional[Bits]], desc: np.ndarray, arena: np.ndarray,
                  key_hint: int = L.KEYS_MIXED) -> np.ndarray:
    """Batched receive over a host arena: desc[i].key_id indexes `windows` (one per installed key,
    None where no tunnel). Returns the per-packet statuses (STATUS_OK / AUTH_FAILED / BAD_KEY /
    REPLAY). In place, arrival order = descriptor order."""
    lib = L.lib()
    n = len(desc)
    status = np.full(n, -1, dtype=np.int32)
    arr = (C.c_void_p * max(len(windows), 1))(*[(w.handle.value if w is not None else None) for w in windows])
    desc = np.ascontiguousarray(desc, dtype=L.DESC_DTYPE)
    rc = lib.neb_rx_open_batch_host(engine.handle, alg, arr, len(windows), desc.ctypes.data_as(C.c_void_p), n,
                                    arena.ctypes.data_as(C.c_void_p), arena.nbytes,
                                    status.ctypes.data_as(C.c_void_p), key_hint)
    L.check(rc, "neb_rx_open_batch_host")
    return status


def rx_open_wire_batch(engine, alg: int, windows: Sequence[Optional[Bits]], packets: np.ndarray,
                       arena: np.ndarray, key_hint: int = L.KEYS_MIXED) -> np.ndarray:
    """readOutsidePackets over a receive batch of wire packets (outside.go:30-133): the header
    parse, version / subtype / size checks and the counter from the header on the engine's side,
    then Decrypt or VerifyRelay through the windows. packets: RX_PACKET_DTYPE (off, len, key_id =
    the tunnel the caller's hostmap lookup resolved, KEYS_MIXED for none). Returns the statuses."""
    lib = L.lib()
    n = len(packets)
    status = np.full(n, -1, dtype=np.int32)
    arr = (C.c_void_p * max(len(windows), 1))(*[(w.handle.value if w is not None else None) for w in windows])
    pk = np.ascontiguousarray(packets, dtype=L.RX_PACKET_DTYPE)
    rc = lib.neb_rx_open_wire_batch_host(engine.handle, alg, arr, len(windows), pk.ctypes.data_as(C.c_void_p), n,
                                         arena.ctypes.data_as(C.c_void_p), arena.nbytes,
                                         status.ctypes.data_as(C.c_void_p), key_hint)
    L.check(rc, "neb_rx_open_wire_batch_host")
    return status


class DeviceWindows:
    """A set of replay windows in device memory (neb_dwindows_*), slot = the tunnel's key_id, for
    receive batches that stay on the device (rx_open_batch_device). load/store copy one window's
    whole state between a host Bits and a slot."""

    def __init__(self, engine, count: int, length: int = ReplayWindow):
        self._lib = L.lib()
        h = C.c_void_p()
        L.check(self._lib.neb_dwindows_create(engine.handle, count, length, C.byref(h)), "neb_dwindows_create")
        self._h = h
        self.count, self.length = count, length

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def load(self, idx: int, w: Optional[Bits]) -> None:
        L.check(self._lib.neb_dwindows_load(self._h, idx, w.handle if w is not None else None), "neb_dwindows_load")

    def store(self, idx: int, w: Bits) -> None:
        L.check(self._lib.neb_dwindows_store(self._h, idx, w.handle), "neb_dwindows_store")

    def set_spin_limit(self, limit: int) -> None:
        """Fault injection (tests): neb_dwindows_set_spin_limit; 0 fails every scan that waits."""
        L.check(self._lib.neb_dwindows_set_spin_limit(self._h, limit), "neb_dwindows_set_spin_limit")

    def destroy(self) -> None:
        if self._h:
            self._lib.neb_dwindows_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


def rx_open_batch_device(engine, alg: int, windows: DeviceWindows, d_desc, d_arena, d_status,
                         key_hint: int = L.KEYS_MIXED, stream=None) -> None:
    """Batched receive over a device-resident batch (torch tensors: descriptors as uint8 bytes,
    arena, int32 statuses): neb_rx_open_batch. Returns when the batch is done."""
    n = d_desc.numel() // L.DESC_DTYPE.itemsize
    rc = L.lib().neb_rx_open_batch(engine.handle, alg, windows.handle, d_desc.data_ptr(), n, d_arena.data_ptr(),
                                   d_status.data_ptr(), key_hint, stream)
    L.check(rc, "neb_rx_open_batch")


__all__ = ["Bits", "NewBits", "ConnectionState", "ReplayWindow", "ErrAlreadySeen", "ErrOpen", "rx_open_batch",
           "DeviceWindows", "rx_open_batch_device"]


def rx_open_wire_batch_device(engine, alg: int, windows: DeviceWindows, d_packets, d_arena, d_status,
                              key_hint: int = L.KEYS_MIXED, stream=None) -> None:
    """rx_open_wire_batch with the wire packets, the arena, the statuses and the windows in device
    memory (torch tensors: d_packets uint8 of RX_PACKET_DTYPE records)."""
    import torch

    s = torch.cuda.current_stream().cuda_stream if stream is None else stream
    n = d_packets.numel() // L.RX_PACKET_DTYPE.itemsize
    rc = L.lib().neb_rx_open_wire_batch(engine.handle, alg, windows.handle, C.c_void_p(d_packets.data_ptr()), n,
                                        C.c_void_p(d_arena.data_ptr()), C.c_void_p(d_status.data_ptr()), key_hint,
                                        C.c_void_p(s))
    L.check(rc, "neb_rx_open_wire_batch")
