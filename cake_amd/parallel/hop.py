"""Device-side pipeline hops over xGMI (hop.hip), for graph-resident decode.

The reference moves the hidden state master -> worker -> master over TCP once
per contiguous remote run and token (cake-core/src/cake/client.rs:50-59,
116-124; worker.rs:236-252).  Here every receive point of a rank owns an
*inbox* in uncached device memory; its IPC handle is exchanged once over the
process group, and the sender's kernel stores the message straight into the
peer's HBM as tagged 8-byte granules (see csrc/kernels/hop.hip).  Both kernels
are ordinary launches on the compute stream, so a rank's receive -> layers ->
send sequence is captured in its decode hipGraph and the host only enqueues
replays.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from ..ops._lib import check, kernels

_SIGS = {
    "cake_hop_alloc": [C.c_size_t, C.POINTER(C.c_void_p)],
    "cake_hop_free": [C.c_void_p],
    "cake_ipc_handle": [C.c_void_p, C.c_void_p],
    "cake_ipc_handle_size": [],
    "cake_ipc_open": [C.c_void_p, C.POINTER(C.c_void_p)],
    "cake_ipc_close": [C.c_void_p],
    "cake_hop_words": [C.c_int, C.c_int, C.c_int],
    "cake_hop_send": [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p],
    "cake_hop_recv": [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                      C.c_double, C.c_void_p],
    "cake_bulk_send": [C.POINTER(C.c_void_p), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                       C.c_int, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p],
    "cake_bulk_recv": [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_double,
                       C.c_void_p],
}
_bound = False


def _lib():
    global _bound
    lib = kernels()
    if not _bound:
        for name, argtypes in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = C.c_int
        _bound = True
    return lib


def hop_timeout_s() -> float:
    """Bound on a receive's wait before it flags an error instead of hanging."""
    return float(os.environ.get("CAKE_HOP_TIMEOUT", "60"))


class Inbox:
    """A receive buffer on this rank's GPU: `words` tagged 8-byte granules."""

    def __init__(self, words: int):
        self.words = int(words)
        p = C.c_void_p()
        check(_lib().cake_hop_alloc(self.words * 8, C.byref(p)), "hop_alloc")
        self.ptr = int(p.value)

    def handle(self) -> bytes:
        lib = _lib()
        n = lib.cake_ipc_handle_size()
        buf = C.create_string_buffer(64)
        check(lib.cake_ipc_handle(C.c_void_p(self.ptr), buf), "ipc_handle")
        return buf.raw[:n]

    def close(self) -> None:
        if self.ptr:
            _lib().cake_hop_free(C.c_void_p(self.ptr))
            self.ptr = 0


class PeerInbox:
    """Another rank's inbox, mapped into this process (IPC)."""

    def __init__(self, handle: bytes):
        buf = C.create_string_buffer(bytes(handle).ljust(64, b"\0"), 64)
        p = C.c_void_p()
        check(_lib().cake_ipc_open(buf, C.byref(p)), "ipc_open")
        self.ptr = int(p.value)

    def close(self) -> None:
        if self.ptr:
            _lib().cake_ipc_close(C.c_void_p(self.ptr))
            self.ptr = 0


def hop_words(H: int, nhdr: int, bf16: bool) -> int:
    return int(_lib().cake_hop_words(int(H), int(nhdr), int(bool(bf16))))


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _msg_ok(msg: torch.Tensor, H: int, nhdr: int) -> None:
    if not (msg.is_cuda and msg.dtype == torch.float32 and msg.is_contiguous()
            and msg.numel() == H + nhdr):
        raise ValueError(f"hop message must be a contiguous f32 [H + {nhdr}] device tensor")


def send(msg: torch.Tensor, H: int, nhdr: int, bf16: bool, peer: PeerInbox,
         seq: torch.Tensor) -> None:
    """Store msg ([H hidden f32 | nhdr int32 words]) into the peer's inbox (async)."""
    _msg_ok(msg, H, nhdr)
    if seq.dtype != torch.int32 or not seq.is_cuda:
        raise ValueError("seq must be an int32 device scalar")
    check(_lib().cake_hop_send(C.c_void_p(msg.data_ptr()), H, nhdr, int(bool(bf16)),
                               C.c_void_p(peer.ptr), C.c_void_p(seq.data_ptr()),
                               C.c_void_p(_stream())), "hop_send")


def recv(inbox: Inbox, msg: torch.Tensor, H: int, nhdr: int, bf16: bool, seq: torch.Tensor,
         err: torch.Tensor, timeout_s: float | None = None) -> None:
    """Wait (on the device) for the next message in `inbox` and unpack it into msg."""
    _msg_ok(msg, H, nhdr)
    if seq.dtype != torch.int32 or err.dtype != torch.int32:
        raise ValueError("seq / err must be int32 device scalars")
    if inbox.words < hop_words(H, nhdr, bf16):
        raise ValueError("inbox too small for this message")
    check(_lib().cake_hop_recv(C.c_void_p(inbox.ptr), H, nhdr, int(bool(bf16)),
                               C.c_void_p(msg.data_ptr()), C.c_void_p(seq.data_ptr()),
                               C.c_void_p(err.data_ptr()),
                               float(timeout_s or hop_timeout_s()), C.c_void_p(_stream())),
          "hop_recv")


# ---------------------------------------------------------------------------
# bulk hops: multi-megabyte messages (hop.hip bulk_send_kernel / bulk_recv_kernel)

BULK_MAX_SEGMENTS = 32


def _align16(n: int) -> int:
    return (int(n) + 15) // 16 * 16


class BulkInbox:
    """Receiving end of a bulk channel on this rank's GPU: `nbytes` of message in
    uncached device memory (+ one flag line), exported to the sender by IPC, and the
    receive-side sequence / error words."""

    def __init__(self, nbytes: int, device):
        self.nbytes = _align16(nbytes)
        self.box = Inbox((self.nbytes + 64) // 8)
        z = lambda: torch.zeros(1, dtype=torch.int32, device=device)  # noqa: E731
        self.seq, self.err = z(), z()

    def handle(self) -> bytes:
        return self.box.handle()

    def recv(self, dst: torch.Tensor, timeout_s: float | None = None) -> None:
        """Wait (on the device) for the next message and copy it into dst (a contiguous
        device buffer of at least nbytes)."""
        if not dst.is_cuda or not dst.is_contiguous() or \
                dst.numel() * dst.element_size() < self.nbytes or dst.data_ptr() % 16:
            raise ValueError("bulk recv: dst must be a 16-byte aligned contiguous device "
                             f"buffer of >= {self.nbytes} bytes")
        check(_lib().cake_bulk_recv(C.c_void_p(self.box.ptr), self.nbytes,
                                    C.c_void_p(dst.data_ptr()), C.c_void_p(self.seq.data_ptr()),
                                    C.c_void_p(self.err.data_ptr()),
                                    float(timeout_s or hop_timeout_s()), C.c_void_p(_stream())),
              "bulk_recv")

    def error(self) -> bool:
        return bool(int(self.err.item()))

    def close(self) -> None:
        self.box.close()


class BulkPeer:
    """Sending end of a bulk channel: the receiver's inbox mapped here, and the
    send-side sequence / arrival counter words."""

    def __init__(self, handle: bytes, nbytes: int, device):
        self.nbytes = _align16(nbytes)
        self.peer = PeerInbox(handle)
        z = lambda: torch.zeros(1, dtype=torch.int32, device=device)  # noqa: E731
        self.seq, self.count = z(), z()

    def send(self, tensors: list, offsets: list[int]) -> None:
        """Store each tensor's bytes (dense, 16-byte multiples) at its offset of the
        peer's inbox, then raise the message flag (async, graph-capturable)."""
        n = len(tensors)
        if not 1 <= n <= BULK_MAX_SEGMENTS or len(offsets) != n:
            raise ValueError(f"bulk send: 1..{BULK_MAX_SEGMENTS} segments")
        ptrs = (C.c_void_p * n)(*[t.data_ptr() for t in tensors])
        sizes = (C.c_uint64 * n)(*[t.numel() * t.element_size() for t in tensors])
        offs = (C.c_uint64 * n)(*[int(o) for o in offsets])
        check(_lib().cake_bulk_send(ptrs, sizes, offs, n, C.c_void_p(self.peer.ptr), self.nbytes,
                                    C.c_void_p(self.seq.data_ptr()),
                                    C.c_void_p(self.count.data_ptr()), C.c_void_p(_stream())),
              "bulk_send")

    def close(self) -> None:
        self.peer.close()
