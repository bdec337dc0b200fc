"""Python face of the native wire codec (csrc/runtime/proto.cpp).

Message kinds mirror cake-core/src/cake/proto/message.rs:60-81 (tags 0-4) plus
our extensions 5-8 (Reset, Error, Ping, Pong).  ``RawTensor`` payloads are the
tensor's raw little-endian bytes with candle dtype names (message.rs:9-39).
"""
from __future__ import annotations

import torch

from ..utils.native import runtime

HELLO, WORKER_INFO, SINGLE_OP, BATCH, TENSOR, RESET, ERROR, PING, PONG = range(9)
PROTO_VERSION = "0.1.0"   # worker.rs:35 reports the crate version

CANDLE_DTYPES = {torch.float16: "f16", torch.bfloat16: "bf16", torch.float32: "f32",
                 torch.float64: "f64", torch.uint8: "u8", torch.int64: "i64"}
FROM_CANDLE = {v: k for k, v in CANDLE_DTYPES.items()}
FROM_CANDLE["u32"] = torch.int32  # ids travel as u32; int32 holds any vocab id


def tensor_payload(t: torch.Tensor):
    """(dtype name, shape, bytes buffer) of a tensor (copied to host if needed)."""
    t = t.detach()
    if t.dtype == torch.int32:
        name = "u32"
    else:
        name = CANDLE_DTYPES[t.dtype]
    host = t.to("cpu").contiguous()
    return name, list(host.shape), host.view(torch.uint8).numpy().reshape(-1)


def tensor_from_payload(msg: dict, body: bytes, device=None) -> torch.Tensor:
    dt = FROM_CANDLE[msg["dtype"]]
    off, n = msg["offset"], msg["nbytes"]
    raw = torch.frombuffer(bytearray(body[off:off + n]), dtype=torch.uint8)
    t = raw.view(dt).reshape(msg["shape"])
    return t.to(device) if device is not None else t


def encode(msg: dict, data=None) -> bytes:
    return runtime().encode_message(msg, data)


def decode(body: bytes) -> dict:
    return runtime().decode_message(body)


def frame(msg: dict, data=None) -> bytes:
    body = encode(msg, data)
    return runtime().encode_header(len(body)) + body


class Connection:
    """One framed TCP connection (native sockets; GIL released while blocked)."""

    def __init__(self, fd: int, peer: str = ""):
        self.fd = fd
        self.peer = peer
        self.bytes_in = 0
        self.bytes_out = 0

    @classmethod
    def connect(cls, addr: str, timeout: float = 10.0) -> "Connection":
        host, _, port = addr.rpartition(":")
        return cls(runtime().tcp_connect(host, int(port), timeout), addr)

    def send(self, msg: dict, tensor: torch.Tensor | None = None) -> int:
        if tensor is not None:
            name, shape, buf = tensor_payload(tensor)
            msg = dict(msg, dtype=name, shape=shape)
            n = runtime().send_message(self.fd, msg, buf)
        else:
            n = runtime().send_message(self.fd, msg, None)
        self.bytes_out += n
        return n

    def recv(self) -> tuple[dict, bytes]:
        msg, body, n = runtime().recv_message(self.fd)
        self.bytes_in += n
        return msg, body

    def set_timeout(self, seconds: float) -> None:
        runtime().tcp_set_timeout(self.fd, float(seconds))

    def close(self) -> None:
        if self.fd >= 0:
            runtime().tcp_close(self.fd)
            self.fd = -1
