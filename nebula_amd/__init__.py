"""nebula_amd — MI355X-native (gfx950) engine for Nebula's per-packet AEAD data plane.

Product path: include/nebula_aead.h (C ABI) -> libnebula_aead.so (hand-written HIP kernels for
AES-256-GCM and ChaCha20-Poly1305). The Python modules mirror the reference's noiseutil /
header surface on top of that ABI; they never compute a byte of ciphertext themselves.
"""
from . import _lib
from ._lib import (ALG_AESGCM, ALG_CHACHAPOLY, DESC_DTYPE, KEYS_MIXED, OVERHEAD, REJECT_AFTER_MESSAGES,
                   NebError, build)
from .noiseutil import (CipherAESGCM, CipherChaChaPoly, CipherState, CipherStateAESGCM, CipherStateChaChaPoly,
                        Engine, ErrMessageCounterExhausted, ErrNoCipher, ErrOpen, NewCipherState,
                        RejectAfterMessages, RejectHeadroom, Slice)

__all__ = [
    "ALG_AESGCM", "ALG_CHACHAPOLY", "DESC_DTYPE", "KEYS_MIXED", "OVERHEAD", "REJECT_AFTER_MESSAGES",
    "NebError", "build", "CipherAESGCM", "CipherChaChaPoly", "CipherState", "CipherStateAESGCM",
    "CipherStateChaChaPoly", "Engine", "ErrMessageCounterExhausted", "ErrNoCipher", "ErrOpen",
    "NewCipherState", "RejectAfterMessages", "RejectHeadroom", "Slice", "_lib",
]
