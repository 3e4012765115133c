"""Host-side mirror of Nebula's transmit path for a batch of TUN reads, on the engine's device
TX batch (neb_tx_seal_batch[_host], nebula_amd/csrc/tx.hip).

Reference (slackhq/nebula):
  inside.go:154-240         sendInsideMessage: SegmentSuperpacket, one Reserve(16+len+16) slot per segment
  inside.go:123-146         sendInsideEncrypt: messageCounter.Add(1), header.Encode, EncryptDanger; a refused
                            segment is dropped (its counter stays used)
  overlay/tio/tio_gso_linux.go:231-280   decodeRead (virtio_net_hdr checks, FinishChecksum)
  overlay/tio/virtio/segment_linux.go    CheckValid, CorrectHdrLen, SegmentTCP, SegmentUDP, FinishChecksum
  overlay/batch/tx_batch.go:15-59        SendBatch / Arena slots handed to WriteBatch
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L

TX_PACKET_DTYPE = np.dtype({
    "names": ["in_off", "len", "tunnel", "vnet_flags", "gso_type", "hdr_len", "gso_size", "csum_start",
              "csum_offset", "reserved"],
    "formats": ["<u8", "<u4", "<u4", "u1", "u1", "<u2", "<u2", "<u2", "<u2", "<u2"],
    "offsets": [0, 8, 12, 16, 17, 18, 20, 22, 24, 26],
    "itemsize": 32,
})
TX_TUNNEL_DTYPE = np.dtype([("message_counter", "<u8"), ("key_id", "<u4"), ("remote_index", "<u4")])
TX_WIRE_DTYPE = np.dtype([("out_off", "<u8"), ("counter", "<u8"), ("len", "<u4"), ("packet", "<u4"),
                          ("segment", "<u4"), ("reserved", "<u4")])
assert TX_TUNNEL_DTYPE.itemsize == 16 and TX_WIRE_DTYPE.itemsize == 32

# virtio_net_hdr values
VNET_F_NEEDS_CSUM = 1
VNET_F_RSC_INFO = 4
GSO_NONE, GSO_TCPV4, GSO_TCPV6, GSO_UDP_L4, GSO_ECN = 0, 1, 4, 5, 0x80


def slot_bytes(seg_len: int) -> int:
    """Output bytes of one wire packet (header ‖ ct ‖ tag), 16-byte aligned."""
    return (seg_len + 32 + 15) & ~15


@dataclass
class TxResult:
    out: np.ndarray          # output arena
    wires: np.ndarray        # TX_WIRE_DTYPE, one per segment of the batch
    wire_status: np.ndarray  # seal status per wire (OK / EXHAUSTED)
    packet_status: np.ndarray
    tunnels: np.ndarray      # message counters advanced

    def wire_bytes(self, i: int) -> bytes:
        w = self.wires[i]
        return self.out[int(w["out_off"]):int(w["out_off"]) + int(w["len"])].tobytes()


def tx_seal_batch_host(engine, alg: int, tunnels: np.ndarray, packets: np.ndarray, in_arena: np.ndarray,
                       out_cap: int, max_wires: int, key_hint: int = L.KEYS_MIXED) -> TxResult:
    """sendInsideMessage over a whole batch of TUN reads held in host memory."""
    lib = L.lib()
    tunnels = np.ascontiguousarray(tunnels, dtype=TX_TUNNEL_DTYPE).copy()
    packets = np.ascontiguousarray(packets, dtype=TX_PACKET_DTYPE)
    in_arena = np.ascontiguousarray(in_arena, dtype=np.uint8)
    out = np.zeros(out_cap, np.uint8)
    wires = np.zeros(max_wires, TX_WIRE_DTYPE)
    wst = np.zeros(max_wires, np.int32)
    pst = np.zeros(len(packets), np.int32)
    nw = C.c_uint32(0)
    vp = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    rc = lib.neb_tx_seal_batch_host(engine.handle, alg, vp(tunnels), len(tunnels), vp(packets), len(packets),
                                    vp(in_arena), in_arena.nbytes, vp(out), out_cap, vp(wires), vp(wst), max_wires,
                                    C.byref(nw), vp(pst), key_hint)
    L.check(rc, "neb_tx_seal_batch_host")
    n = nw.value
    return TxResult(out, wires[:n].copy(), wst[:n].copy(), pst, tunnels)


class DeviceTxBatch:
    """A TX batch resident in device memory (torch tensors as plain allocations): the input arena
    of TUN reads, the tunnel table and the output arena; `seal()` runs neb_tx_seal_batch on torch's
    current stream."""

    def __init__(self, engine, alg: int, tunnels: np.ndarray, packets: np.ndarray, in_arena: np.ndarray,
                 out_cap: int, max_wires: int, key_hint: int = L.KEYS_MIXED):
        import torch

        dev = torch.device("cuda", engine.device)
        self.engine, self.alg, self.key_hint = engine, alg, key_hint
        self.tunnels0 = np.ascontiguousarray(tunnels, dtype=TX_TUNNEL_DTYPE).copy()
        self.tunnels = torch.from_numpy(self.tunnels0.view(np.uint8).copy()).to(dev)
        self.packets = torch.from_numpy(np.ascontiguousarray(packets, dtype=TX_PACKET_DTYPE).view(np.uint8).copy()).to(dev)
        self.npk = len(packets)
        self.ntun = len(tunnels)
        self.inp = torch.from_numpy(np.ascontiguousarray(in_arena, dtype=np.uint8).copy()).to(dev)
        self.out = torch.zeros(out_cap, dtype=torch.uint8, device=dev)
        self.wires = torch.zeros(max_wires * TX_WIRE_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        self.wire_status = torch.zeros(max_wires, dtype=torch.int32, device=dev)
        self.pk_status = torch.zeros(self.npk, dtype=torch.int32, device=dev)
        self.nwires = torch.zeros(1, dtype=torch.int32, device=dev)
        self.max_wires = max_wires

    def reset_counters(self) -> None:
        import torch

        self.tunnels.copy_(torch.from_numpy(self.tunnels0.view(np.uint8).copy()))

    def seal(self) -> None:
        import torch

        lib = L.lib()
        p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
        rc = lib.neb_tx_seal_batch(self.engine.handle, self.alg, p(self.tunnels), self.ntun, p(self.packets),
                                   self.npk, p(self.inp), p(self.out), self.out.numel(), p(self.wires),
                                   p(self.wire_status), self.max_wires, p(self.nwires), p(self.pk_status),
                                   self.key_hint, C.c_void_p(torch.cuda.current_stream().cuda_stream))
        L.check(rc, "neb_tx_seal_batch")

    def result(self) -> TxResult:
        n = int(self.nwires.cpu()[0])
        wires = self.wires.cpu().numpy().view(TX_WIRE_DTYPE)[:n].copy()
        return TxResult(self.out.cpu().numpy(), wires, self.wire_status.cpu().numpy()[:n].copy(),
                        self.pk_status.cpu().numpy(), self.tunnels.cpu().numpy().view(TX_TUNNEL_DTYPE).copy())


__all__ = ["TX_PACKET_DTYPE", "TX_TUNNEL_DTYPE", "TX_WIRE_DTYPE", "tx_seal_batch_host", "DeviceTxBatch", "TxResult",
           "slot_bytes"]
