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
