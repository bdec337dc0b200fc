"""Device hop payload round trip (hop.hip) in one process: the sender's kernel stores into
this GPU's own inbox, the receiver's kernel unpacks it.  Pins the payload encodings the
multi-rank pipeline uses: f32 words bit-exact, bf16 pairs equal to round-to-nearest-even
of the f32 hidden, header words raw, sequence tags advancing across messages."""
import pytest
import torch

pytestmark = pytest.mark.gpu


class _Self:
    """A 'peer inbox' that is this process's own inbox (no IPC mapping needed)."""

    def __init__(self, inbox):
        self.ptr = inbox.ptr


@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("H", [64, 4096, 8192])
def test_hop_roundtrip_payload(cuda, bf16, H):
    from cake_amd.parallel import hop
    nhdr = 16
    inbox = hop.Inbox(hop.hop_words(H, nhdr, bf16))
    try:
        sseq = torch.zeros(1, dtype=torch.int32, device=cuda)
        rseq = torch.zeros(1, dtype=torch.int32, device=cuda)
        err = torch.zeros(1, dtype=torch.int32, device=cuda)
        g = torch.Generator(device=cuda).manual_seed(H + bf16)
        for it in range(3):  # tags advance: every message must be taken, none twice
            msg = torch.empty(H + nhdr, device=cuda)
            msg[:H] = torch.randn(H, device=cuda, generator=g) * (10.0 ** (it - 1))
            hdr = torch.arange(nhdr, dtype=torch.int32, device=cuda) * 7919 + it
            msg[H:] = hdr.view(torch.float32)
            out = torch.full_like(msg, float("nan"))
            hop.send(msg, H, nhdr, bf16, _Self(inbox), sseq)
            hop.recv(inbox, out, H, nhdr, bf16, rseq, err, timeout_s=5.0)
            torch.cuda.synchronize()
            assert int(err.item()) == 0
            want = msg[:H].to(torch.bfloat16).float() if bf16 else msg[:H]
            assert torch.equal(out[:H], want), (it, (out[:H] - want).abs().max())
            assert torch.equal(out[H:].view(torch.int32), hdr)
            assert int(sseq.item()) == int(rseq.item()) == it + 1
    finally:
        inbox.close()


def test_hop_recv_times_out_with_error_word(cuda):
    """No sender: the receive gives up after its bound and raises the error word."""
    from cake_amd.parallel import hop
    H, nhdr = 128, 4
    inbox = hop.Inbox(hop.hop_words(H, nhdr, False))
    try:
        rseq = torch.zeros(1, dtype=torch.int32, device=cuda)
        err = torch.zeros(1, dtype=torch.int32, device=cuda)
        out = torch.zeros(H + nhdr, device=cuda)
        hop.recv(inbox, out, H, nhdr, False, rseq, err, timeout_s=0.05)
        torch.cuda.synchronize()
        assert int(err.item()) == 1
    finally:
        inbox.close()
