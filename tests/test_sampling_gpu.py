"""Device sampling (sampling.hip): top-k / top-p sets, Gumbel-max draw distribution (chi^2
against softmax(l / T) restricted to the set), seed determinism, and sampled decoding
inside the DeviceDecoder graph."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _expected_set(logits, T, k, p):
    """Token set of the host LogitsProcessor (models/sampling.py, candle's
    TopKThenTopP): top-k, then the top-p cutoff on the top-k tokens' FULL-vocabulary
    probabilities (not renormalised: a top-k mass below p keeps all k)."""
    probs = torch.softmax(logits.double() / T, 0)
    keep = torch.ones_like(probs, dtype=torch.bool)
    if k:
        idx = torch.topk(logits, k).indices
        keep = torch.zeros_like(keep)
        keep[idx] = True
    if p is not None and 0 < p < 1:
        pr = torch.where(keep, probs, torch.zeros_like(probs))
        order = torch.argsort(pr, descending=True, stable=True)
        before = torch.cumsum(pr[order], 0) - pr[order]
        kp = torch.zeros_like(keep)
        kp[order[before < p]] = True
        keep &= kp
    return keep


@pytest.mark.parametrize("V,k,p", [(128256, 40, None), (128256, None, 0.9), (128256, 50, 0.8),
                                   (1000, 7, None), (1000, None, 0.5), (300, 300, 0.999),
                                   (128256, 5, 0.9), (1000, 20, 0.3)])
def test_threshold_set(cuda, V, k, p):
    from cake_amd.ops import hip as K
    torch.manual_seed(V + (k or 0))
    logits = torch.randn(V, device=cuda) * 3
    thr = torch.zeros(1, dtype=torch.int32, device=cuda)
    K.sample_threshold(logits, 0.8, k, p, thr)
    u = logits.view(torch.int32).cpu().numpy().view("uint32").astype("int64")
    key = torch.tensor(((u ^ 0x80000000) * ((u >> 31) == 0) + (0xFFFFFFFF - u) * ((u >> 31) == 1)))
    t = int(thr.item()) & 0xFFFFFFFF
    got = key >= t
    exp = _expected_set(logits.cpu(), 0.8, k, p)
    assert torch.equal(got, exp), (int(got.sum()), int(exp.sum()))


def test_topk_topp_full_mass_fixture(cuda):
    """Renormalised and full-mass top-p cutoffs differ on this fixture (see
    test_model_cpu.test_sampling_rules): the device threshold keeps {0, 1, 2} as candle's
    sample_topk_topp does, not the renormalised {0, 1}."""
    from cake_amd.ops import hip as K
    logits = torch.log(torch.tensor([0.30, 0.25, 0.20, 0.15, 0.10])).to(cuda)
    thr = torch.zeros(1, dtype=torch.int32, device=cuda)
    K.sample_threshold(logits, 1.0, 3, 0.6, thr)
    u = logits.view(torch.int32).cpu().numpy().view("uint32").astype("int64")
    key = torch.tensor(((u ^ 0x80000000) * ((u >> 31) == 0) + (0xFFFFFFFF - u) * ((u >> 31) == 1)))
    got = (key >= (int(thr.item()) & 0xFFFFFFFF)).nonzero().flatten().tolist()
    assert got == [0, 1, 2]


@pytest.mark.parametrize("T,k,p", [(1.0, None, None), (0.7, 5, None), (1.3, None, 0.8)])
def test_gumbel_draw_distribution(cuda, T, k, p):
    """chi^2 of 40k device draws against the renormalised softmax over the kept set."""
    from cake_amd.models.sampling import SamplingConfig
    from cake_amd.ops import hip as K
    torch.manual_seed(11)
    V = 24
    logits = torch.randn(V, device=cuda) * 1.5
    keep = _expected_set(logits.cpu(), T, k, p)
    probs = torch.softmax(logits.double().cpu() / T, 0) * keep
    probs = probs / probs.sum()
    cfg = SamplingConfig(temperature=T, top_k=k, top_p=p, seed=1234)
    slot = torch.zeros(1, dtype=torch.int64, device=cuda)
    thr = torch.zeros(1, dtype=torch.int32, device=cuda)
    tok = torch.zeros(1, dtype=torch.int32, device=cuda)
    pos = torch.zeros(1, dtype=torch.int32, device=cuda)
    n = 40000
    hist = torch.zeros(n + 1, dtype=torch.int32, device=cuda)
    hist_len = torch.zeros(1, dtype=torch.int32, device=cuda)
    g = torch.cuda.CUDAGraph()
    K.select_token(logits, slot, hist, hist_len, tok, pos, cfg, thr)  # warm
    hist_len.zero_()
    with torch.cuda.graph(g):
        K.select_token(logits, slot, hist, hist_len, tok, pos, cfg, thr)
    for _ in range(n):  # the step counter (history length) advances every draw
        g.replay()
    torch.cuda.synchronize()
    draws = hist[:n].cpu().long()
    counts = torch.bincount(draws, minlength=V).double()
    assert counts[~keep].sum() == 0
    e = probs * n
    m = e > 0
    chi2 = float(((counts[m] - e[m]) ** 2 / e[m]).sum())
    dof = int(m.sum()) - 1
    # mean dof, sd sqrt(2 dof): 6 sigma is a loose, flake-free bound
    assert chi2 < dof + 6 * math.sqrt(2 * dof) + 10, (chi2, dof)


def test_seed_determinism_and_decoder(cuda):
    from cake_amd.models.llama3.config import preset
    from cake_amd.models.llama3.decode_loop import run_decode
    from cake_amd.models.llama3.factory import random_model
    from cake_amd.models.llama3.model import DeviceDecoder
    from cake_amd.models.sampling import SamplingConfig
    cfg = preset("llama3-8b", num_hidden_layers=2, vocab_size=4096, intermediate_size=1024,
                 hidden_size=512, num_attention_heads=4, num_key_value_heads=1)
    model = random_model(cfg, "cuda:0", torch.bfloat16, max_seq=256, seed=5)
    prompt = [5, 6, 7, 8, 9]

    def gen(seed, T=1.0, k=None, p=None, n=24):
        s = SamplingConfig(temperature=T, top_k=k, top_p=p, seed=seed)
        dec = DeviceDecoder(model, repeat_penalty=1.1, repeat_last_n=16, sampling=s)
        first = dec.start(prompt)
        dec.capture()
        return [first] + run_decode(dec, n).tokens
    a, b, c = gen(7), gen(7), gen(8)
    assert a == b and a != c
    assert len(set(a)) > 3  # a real draw, not argmax repeated
    d = gen(7, T=0.5, k=5, p=0.9)
    assert len(d) == 25


def test_device_params_match_static_and_switch_without_recapture(cuda):
    """set_sampling (API per-request config): the decode graph reads the sampling
    parameters from device memory — same tokens as the launch-argument path, greedy
    (temperature 0) equals argmax, and later switches reuse the captured graph."""
    from cake_amd.models.llama3.config import preset
    from cake_amd.models.llama3.decode_loop import run_decode
    from cake_amd.models.llama3.factory import random_model
    from cake_amd.models.llama3.model import DeviceDecoder
    from cake_amd.models.sampling import SamplingConfig
    cfg = preset("llama3-8b", num_hidden_layers=2, vocab_size=4096, intermediate_size=1024,
                 hidden_size=512, num_attention_heads=4, num_key_value_heads=1)
    model = random_model(cfg, "cuda:0", torch.bfloat16, max_seq=256, seed=5)
    prompt = [5, 6, 7, 8, 9]

    def run(dec, n=20):
        first = dec.start(prompt)
        dec.capture()
        return [first] + run_decode(dec, n).tokens

    s1 = SamplingConfig(temperature=0.8, top_k=40, top_p=0.9, seed=3)
    g0 = SamplingConfig(temperature=0.0)
    static_s = run(DeviceDecoder(model, repeat_penalty=1.1, repeat_last_n=16, sampling=s1))
    static_g = run(DeviceDecoder(model, repeat_penalty=1.1, repeat_last_n=16))
    dyn = DeviceDecoder(model, repeat_penalty=1.1, repeat_last_n=16)
    dyn.set_sampling(s1)
    assert run(dyn) == static_s
    graph = dyn.graph
    dyn.set_sampling(g0)
    assert run(dyn) == static_g
    dyn.set_sampling(s1)
    assert run(dyn) == static_s
    assert dyn.graph is graph  # captured once
