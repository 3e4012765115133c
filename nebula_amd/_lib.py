"""ctypes binding of libnebula_aead.so (the C ABI in include/nebula_aead.h).

The product path has exactly one implementation: the gfx950 kernels behind this library. If the
library is missing or does not load, every entry point raises — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# NEB_LIB_PATH selects an alternative build of the same library (e.g. an ablation build in tools/).
LIB_PATH = os.environ.get("NEB_LIB_PATH") or os.path.join(PKG_DIR, "libnebula_aead.so")

ALG_AESGCM = 1
ALG_CHACHAPOLY = 2

OK = 0
ERR_INVALID = -1
ERR_AUTH = -2
ERR_EXHAUSTED = -3
ERR_NO_CIPHER = -4
ERR_SHORT_BUFFER = -5
ERR_HIP = -6
ERR_NO_DEVICE = -7
ERR_NO_KEY_SLOT = -8

STATUS_OK = 0
STATUS_AUTH_FAILED = 1
STATUS_EXHAUSTED = 2
STATUS_BAD_KEY = 3
STATUS_REPLAY = 4
STATUS_INVALID = 5
STATUS_NO_SPACE = 6
STATUS_NOT_MESSAGE = 7

OVERHEAD = 16
HEADER_LEN = 16
REJECT_HEADROOM = 1 << 40
REJECT_AFTER_MESSAGES = (1 << 64) - 1 - REJECT_HEADROOM
KEYS_MIXED = 0xFFFFFFFF
# neb_set_knob (include/nebula_aead.h)
KNOB_HOST_MODE, KNOB_SUB_BINS_FROM, KNOB_SINGLE_MAX_GRID, KNOB_RX_STRICT, KNOB_TILE_BINS_FROM = 0, 1, 2, 3, 4
KNOB_SMALL_BATCH, KNOB_FRONT_GROUPS = 5, 6
RX_OWN_SOURCE = 0x80000000  # or-ed into neb_rx_packet.len: outside.go:66-74 refused the datagram

# neb_desc (include/nebula_aead.h)
DESC_DTYPE = np.dtype(
    [("src_off", "<u8"), ("dst_off", "<u8"), ("aad_off", "<u8"), ("counter", "<u8"),
     ("len", "<u4"), ("aad_len", "<u4"), ("key_id", "<u4"), ("flags", "<u4")]
)
assert DESC_DTYPE.itemsize == 48
# neb_rx_packet (include/nebula_aead.h): one received wire packet and its tunnel
RX_PACKET_DTYPE = np.dtype([("off", "<u8"), ("len", "<u4"), ("key_id", "<u4")])
assert RX_PACKET_DTYPE.itemsize == 16

# Every symbol include/nebula_aead.h declares, with (restype, argtypes).
_vp, _u8p, _sz, _u32, _u64, _i = C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint64, C.c_int
SIGNATURES = {
    "neb_engine_create": (_i, [_i, _u32, C.POINTER(_vp)]),
    "neb_engine_destroy": (_i, [_vp]),
    "neb_engine_info": (_i, [_vp, C.POINTER(_i), C.POINTER(_u32), C.POINTER(_u32)]),
    "neb_strerror": (C.c_char_p, [_i]),
    "neb_last_error": (C.c_char_p, []),
    "neb_build_id": (C.c_char_p, []),
    "neb_time_next_kernel": (_i, [_vp, _vp]),
    "neb_time_last_kernel": (C.c_char_p, []),
    "neb_set_knob": (_i, [_i, C.c_int64]),
    "neb_get_knob": (C.c_int64, [_i]),
    "neb_cipher_create": (_i, [_vp, _i, _u8p, C.POINTER(_vp)]),
    "neb_cipher_create_batch": (_i, [_vp, _i, _u8p, _u32, _vp]),
    "neb_cipher_create_multi": (_i, [_vp, _u32, _i, _u8p, _vp]),
    "neb_engine_stats": (_i, [_vp, _vp]),
    "neb_engine_pkt_combined": (_i, [_vp, _vp]),
    "neb_cipher_destroy": (_i, [_vp]),
    "neb_cipher_key_id": (_u32, [_vp]),
    "neb_cipher_alg": (_i, [_vp]),
    "neb_cipher_name": (C.c_char_p, [_i]),
    "neb_overhead": (_i, [_vp]),
    "neb_encrypt_danger": (_i, [_vp, _u8p, _sz, _sz, _u8p, _sz, _u8p, _sz, _u64, _u8p, C.POINTER(_sz)]),
    "neb_decrypt_danger": (_i, [_vp, _u8p, _sz, _sz, _u8p, _sz, _u8p, _sz, _u64, _u8p, C.POINTER(_sz)]),
    "neb_seal_batch": (_i, [_vp, _i, _vp, _u32, _vp, _vp, _u32, _vp]),
    "neb_open_batch": (_i, [_vp, _i, _vp, _u32, _vp, _vp, _u32, _vp]),
    "neb_seal_batch_host": (_i, [_vp, _i, _vp, _u32, _vp, _sz, _vp, _u32]),
    "neb_open_batch_host": (_i, [_vp, _i, _vp, _u32, _vp, _sz, _vp, _u32]),
    "neb_host_alloc": (_i, [_sz, C.POINTER(_vp)]),
    "neb_host_free": (_i, [_vp]),
    "neb_header_encode": (None, [_u8p, C.c_uint8, C.c_uint8, C.c_uint8, _u32, _u64]),
    "neb_header_parse": (_i, [_u8p, _sz, _u8p, _u8p, _u8p, C.POINTER(C.c_uint16), C.POINTER(_u32),
                              C.POINTER(_u64)]),
    "neb_window_create": (_i, [_u64, C.POINTER(_vp)]),
    "neb_window_destroy": (_i, [_vp]),
    "neb_window_check": (_i, [_vp, _u64]),
    "neb_window_update": (_i, [_vp, _u64]),
    "neb_window_state": (_i, [_vp, C.POINTER(_u64), C.POINTER(C.c_int64)]),
    "neb_window_slot": (_i, [_vp, _u64]),
    "neb_window_reset_counters": (_i, [_vp]),
    "neb_rx_open_batch_host": (_i, [_vp, _i, _vp, _u32, _vp, _u32, _vp, _sz, _vp, _u32]),
    "neb_dwindows_create": (_i, [_vp, _u32, _u64, _vp]),
    "neb_dwindows_destroy": (_i, [_vp]),
    "neb_dwindows_load": (_i, [_vp, _u32, _vp]),
    "neb_dwindows_store": (_i, [_vp, _u32, _vp]),
    "neb_dwindows_set_spin_limit": (_i, [_vp, _u32]),
    "neb_rx_open_batch": (_i, [_vp, _i, _vp, _vp, _u32, _vp, _vp, _u32, _vp]),
    "neb_tx_seal_batch": (_i, [_vp, _i, _vp, _u32, _vp, _u32, _vp, _vp, _sz, _vp, _vp, _u32, _vp, _vp, _u32, _vp]),
    "neb_tx_seal_batch_host": (_i, [_vp, _i, _vp, _u32, _vp, _u32, _vp, _sz, _vp, _sz, _vp, _vp, _u32, _vp, _vp,
                                    _u32]),
    "neb_rx_open_wire_batch_host": (_i, [_vp, _i, _vp, _u32, _vp, _u32, _vp, _sz, _vp, _u32]),
    "neb_rx_open_wire_batch": (_i, [_vp, _i, _vp, _vp, _u32, _vp, _vp, _u32, _vp]),
    "neb_seal_batch_host_multi": (_i, [_vp, _u32, _i, _vp, _u32, _vp, _sz, _vp, _u32]),
    "neb_open_batch_host_multi": (_i, [_vp, _u32, _i, _vp, _u32, _vp, _sz, _vp, _u32]),
    "neb_seal_batch_sharded": (_i, [_i, _vp, _u32, _u32]),
    "neb_open_batch_sharded": (_i, [_i, _vp, _u32, _u32]),
    "neb_queue_create": (_i, [_vp, _i, _i, _vp, C.POINTER(_vp)]),
    "neb_queue_destroy": (_i, [_vp]),
    "neb_queue_submit": (_i, [_vp, _vp, _u32, _vp, _sz, _vp]),
    "neb_queue_flush": (_i, [_vp]),
    "neb_queue_stats": (_i, [_vp, _vp]),
    "neb_queue_phases": (_i, [_vp, _vp]),
}


class Shard(C.Structure):
    """neb_shard (include/nebula_aead.h): one engine's device-resident part of a sharded batch."""
    _fields_ = [("e", C.c_void_p), ("d_desc", C.c_void_p), ("n", C.c_uint32), ("d_arena", C.c_void_p),
                ("d_status", C.c_void_p), ("stream", C.c_void_p)]


class QueueConfig(C.Structure):
    """neb_queue_config (include/nebula_aead.h)."""
    _fields_ = [("max_packets", C.c_uint32), ("max_delay_us", C.c_uint32), ("arena_bytes", C.c_uint64),
                ("depth", C.c_uint32), ("reserved", C.c_uint32)]

_lib = None


class NebError(RuntimeError):
    def __init__(self, rc: int, what: str = ""):
        self.rc = rc
        msg = strerror(rc) if _lib is not None else str(rc)
        if _lib is not None and rc in (ERR_HIP, ERR_NO_DEVICE):
            detail = _lib.neb_last_error().decode()
            if detail:
                msg += f" [{detail}]"
        super().__init__(f"{what}: {msg} ({rc})" if what else f"{msg} ({rc})")


def build() -> None:
    """Compile libnebula_aead.so in-tree (hipcc --offload-arch=gfx950)."""
    subprocess.run(["make", "-s", "-C", PKG_DIR], check=True)


def _pin_hip_runtime() -> None:
    """Load PyTorch's HIP runtime before ours when torch is installed.

    torch-ROCm ships its own libamdhip64.so.7 (same SONAME as /opt/rocm's). Whichever is loaded
    first serves the whole process, and torch cannot initialise the GPU on a runtime it did not
    bring. Importing torch first makes every HIP call in the process, ours included, go through
    one runtime, so torch tensors, streams and events interoperate with the engine.
    """
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def lib():
    global _lib
    if _lib is None:
        _pin_hip_runtime()
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C {PKG_DIR}` "
                               "(nebula_amd has no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("NEB_LIB_PATH") and not hasattr(L, name):
                continue  # an older A/B build (tools/ab.sh) may predate some entry points
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def strerror(rc: int) -> str:
    return lib().neb_strerror(rc).decode()


def check(rc: int, what: str = "") -> None:
    if rc != OK:
        raise NebError(rc, what)


class knob:
    """`with knob(KNOB_X, v):` sets a process-wide knob (neb_set_knob) and restores it after."""

    def __init__(self, k: int, value: int):
        self.k, self.value = k, value

    def __enter__(self):
        self.old = lib().neb_get_knob(self.k)
        check(lib().neb_set_knob(self.k, self.value), "neb_set_knob")
        return self

    def __exit__(self, *exc):
        lib().neb_set_knob(self.k, self.old)
