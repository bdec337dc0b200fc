"""CPU tests: Llama torch path (KV cache, chunked prefill, sessions), sampling rules,
the conv planner, and the SD channels-last layout plumbing (fallback ops)."""
import math

import pytest
import torch

from cake_amd.models.llama3.config import preset
from cake_amd.models.llama3.factory import random_model
from cake_amd.models.sampling import LogitsProcessor, SamplingConfig
from cake_amd.ops import reference as R


@pytest.fixture(scope="module")
def tiny():
    torch.manual_seed(0)
    return random_model(preset("tiny"), "cpu", torch.float32, max_seq=64,
                        backend="torch")


def test_decode_matches_full_forward(tiny):
    toks = [1, 17, 42, 99, 5, 300, 7]
    tiny.reset()
    full = tiny.forward(toks, 0)
    tiny.reset()
    tiny.forward(toks[:-1], 0)
    step = tiny.forward(toks[-1:], len(toks) - 1)
    torch.testing.assert_close(step, full, atol=1e-4, rtol=1e-4)


def test_chunked_prefill_matches_single(tiny):
    toks = list(range(3, 40))
    tiny.reset()
    one = tiny.forward(toks, 0)
    tiny.reset()
    tiny.forward(toks[:13], 0)
    tiny.forward(toks[13:29], 13)
    two = tiny.forward(toks[29:], 29)
    torch.testing.assert_close(two, one, atol=1e-4, rtol=1e-4)


def test_sessions_have_independent_caches(tiny):
    a, b = [5, 6, 7, 8], [9, 10, 11]
    tiny.reset()
    ref_a = tiny.forward(a, 0)
    tiny.reset()
    ref_b = tiny.forward(b, 0)
    tiny.stack.reset()
    tiny.session = 1
    try:
        tiny.forward(a[:2], 0)
        tiny.session = 2
        tiny.forward(b[:2], 0)
        tiny.session = 1
        got_a = tiny.forward(a[2:], 2)
        tiny.session = 2
        got_b = tiny.forward(b[2:], 2)
    finally:
        tiny.session = 0
    torch.testing.assert_close(got_a, ref_a, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(got_b, ref_b, atol=1e-4, rtol=1e-4)


def test_repeat_penalty_unique_tokens():
    logits = torch.tensor([2.0, -2.0, 1.0, 0.5])
    out = R.apply_repeat_penalty(logits.clone(), 2.0, [0, 1, 0, 0])  # duplicates count once
    torch.testing.assert_close(out, torch.tensor([1.0, -4.0, 1.0, 0.5]))


def test_sampling_rules():
    logits = torch.tensor([0.1, 3.0, 0.2, 2.9, -1.0])
    assert LogitsProcessor(SamplingConfig(temperature=0.0)).sample(logits) == 1
    assert LogitsProcessor(SamplingConfig(temperature=None)).sample(logits) == 1
    lp = LogitsProcessor(SamplingConfig(temperature=1.0, top_k=2, seed=3))
    assert {lp.sample(logits) for _ in range(50)} <= {1, 3}
    lp = LogitsProcessor(SamplingConfig(temperature=1.0, top_p=0.4, seed=3))
    assert {lp.sample(logits) for _ in range(50)} == {1}  # first token alone reaches p
    # top-k then top-p: p applies to full-vocabulary probabilities (no renormalisation
    # inside top-k): the top-2 mass here is ~0.93 < 0.95, so both stay in the set
    lp = LogitsProcessor(SamplingConfig(temperature=1.0, top_k=2, top_p=0.95, seed=5))
    assert {lp.sample(logits) for _ in range(200)} == {1, 3}
    # fixture where the two top-p readings give DIFFERENT sets: probabilities
    # (0.30, 0.25, 0.20, 0.15, 0.10), top-k 3, top-p 0.6.  candle's sample_topk_topp
    # (full-vocabulary probabilities of the top k, cutoff while the running sum is below
    # p): 0 -> 0.30, 1 -> 0.55 < 0.6, so token 2 stays: {0, 1, 2}.  Renormalised inside
    # top-k (0.40, 0.33, 0.27): 0.73 >= 0.6 after token 1: {0, 1}.
    fx = torch.log(torch.tensor([0.30, 0.25, 0.20, 0.15, 0.10]))
    lp = LogitsProcessor(SamplingConfig(temperature=1.0, top_k=3, top_p=0.6, seed=9))
    assert {lp.sample(fx) for _ in range(400)} == {0, 1, 2}
    a = LogitsProcessor(SamplingConfig(temperature=0.8, seed=7))
    b = LogitsProcessor(SamplingConfig(temperature=0.8, seed=7))
    assert [a.sample(logits) for _ in range(20)] == [b.sample(logits) for _ in range(20)]


@pytest.mark.parametrize("P,OC,ks", [(8192, 320, 45), (128, 1280, 180), (32768, 128, 18),
                                     (2048, 4, 45)])
def test_conv_plan_is_valid(P, OC, ks):
    from cake_amd.ops import hip as K
    cfg, splits = K.conv_plan(P, OC, ks)
    assert 0 <= cfg < 4 and splits in (1, 2, 4, 8)
    assert splits == 1 or ks // splits >= 4


@pytest.mark.parametrize("OH,OW,bn", [(64, 64, 128), (8, 8, 64), (21, 19, 128), (128, 128, 256),
                                      (5, 40, 64)])
def test_halo_tile_fits(OH, OW, bn):
    from cake_amd.ops import hip as K
    th, tw = K.halo_tile(OH, OW, bn)
    assert th * tw <= bn
    hrows = {256: 384, 128: 192, 64: 128}[bn]
    assert (th + 2) * (tw + 2) <= hrows


def test_conv_supported_rules():
    from cake_amd.ops import hip as K
    assert K.conv_supported(320, 320) and K.conv_supported(64, 4)
    assert K.conv_supported(4, 320) and K.conv_supported(3, 128)  # conv_in: direct kernel
    assert not K.conv_supported(4, 320, k=1) and not K.conv_supported(4, 4)  # 3x3, OC % 8
    assert not K.conv_supported(4, 1024)      # filter exceeds the kernel's LDS copy
    assert not K.conv_supported(8, 320)       # IC neither 3/4 nor a multiple of 64
    assert not K.conv_supported(320, 3)       # OC not a multiple of 4
    assert not K.conv_supported(64, 64, stride=2, up=True)
    assert K.group_norm_nhwc_supported(320, 32) and K.group_norm_nhwc_supported(128, 32)
    assert not K.group_norm_nhwc_supported(160, 32)  # Cg = 5 spans 3 groups per vector


def test_sd_layout_ops_nhwc_matches_nchw():
    """The channels-last plumbing (fallback ops on CPU) equals the NCHW path:
    conv with fused upsample / per-sample bias / residual, GroupNorm, tokens."""
    from cake_amd.models.sd import ops
    torch.manual_seed(1)
    W = {"c.weight": torch.randn(8, 6, 3, 3) / 7, "c.bias": torch.randn(8)}
    x = torch.randn(2, 6, 5, 7)
    b2 = torch.randn(2, 8)
    r = torch.randn(2, 8, 10, 14)
    ref = ops.conv(W, "c", x, up=True, bias2=b2, resid=r)
    with ops.layout_nhwc(True):
        got = ops.conv(W, "c", ops.to_internal(x), up=True, bias2=b2, resid=ops.to_internal(r))
        got = ops.to_external(got)
    torch.testing.assert_close(got, ref, atol=1e-5, rtol=1e-5)
    g, b = torch.randn(6), torch.randn(6)
    ref = ops.group_norm(x, g, b, 3, 1e-5, silu=True)
    with ops.layout_nhwc(True):
        got = ops.to_external(ops.group_norm(ops.to_internal(x), g, b, 3, 1e-5, silu=True))
        t = ops.tokens(ops.to_internal(x))
        assert t.shape == (2, 35, 6)
        back = ops.to_external(ops.untokens(t, ops.to_internal(x)))
    torch.testing.assert_close(got, ref, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(back, x)
    torch.testing.assert_close(ops.untokens(ops.tokens(x), x), x)
    padded = ops.pad_hw_end(x)
    with ops.layout_nhwc(True):
        padded2 = ops.to_external(ops.pad_hw_end(ops.to_internal(x)))
    torch.testing.assert_close(padded2, padded)
    assert math.isclose(float(padded[..., -1, :].abs().sum()), 0.0)


@pytest.mark.parametrize("impl", [1, 2])
def test_attention_split_policy_and_buckets(impl):
    """Host mirror of the decode-attention split policy (ops.hip.attn_splits, used to pick
    a position-bucket graph) for both cores: at most 64 splits, never more than a max_seq
    grid holds, and the 8/16/32/64 buckets cover the live lengths the policy maps to them.
    Core 1 is not monotone: past 1024 keys a split takes two chunks, so 1025 keys use 9
    splits where 1024 use 16.  Core 2 splits in 16-key blocks, >= 64 keys per split."""
    from cake_amd.ops import hip as K
    saved = K._ATTN_IMPL[0]
    K._ATTN_IMPL[0] = impl
    try:
        for tk in range(1, 20000, 7):
            n = K.attn_splits(tk)
            assert 1 <= n <= 64
            assert n <= K.attn_max_split(tk)
        assert max(K.attn_splits(t) for t in range(1, 513)) <= 8
        if impl == 1:
            assert K.attn_splits(1024) == 16 and K.attn_splits(1025) == 9
            assert max(K.attn_splits(t) for t in range(1, 2049)) <= 16
            assert max(K.attn_splits(t) for t in range(1, 4097)) <= 32
        else:
            # default split target 16: never more than 16 splits
            assert K.attn_splits(320) == 1 and K.attn_splits(321) == 6
            assert K.attn_splits(1024) == 16 and K.attn_splits(4096) == 16
            assert max(K.attn_splits(t) for t in range(1, 20000, 3)) <= 16
            saved_t = K._ATTN_TARGET[0]
            K._ATTN_TARGET[0] = 64
            try:
                assert K.attn_splits(4096) == 64
                assert max(K.attn_splits(t) for t in range(1, 2049)) <= 32
            finally:
                K._ATTN_TARGET[0] = saved_t
        assert K.attn_split_caps(4096) == ([8, 16, 32] if impl == 1 else [8, 16])
        assert K.attn_split_caps(100) == [2]
    finally:
        K._ATTN_IMPL[0] = saved
    assert K.attn_max_split(4096) == 64 and K.attn_max_split(100) == 2
