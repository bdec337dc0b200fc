"""MFMA GEMM (gemm.hip) vs a plain-PyTorch f32 reference, every epilogue and tile config,
split-K, ragged M/N edges, strided inputs, and the Llama-3 8B/70B + SDXL shapes."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DTYPES = [torch.bfloat16, torch.float16]


def _r(*shape, dt, std=1.0):
    return (torch.randn(*shape, device="cuda") * std).to(dt)


def _ref(x, w, b=None):
    y = x.float() @ w.float().t()
    return y if b is None else y + b.float()


def _close(got, ref, K):
    # bf16/f16 output rounding + f32 accumulation-order differences
    tol = 2e-2 * max(1.0, float(ref.abs().max()))
    torch.testing.assert_close(got.float(), ref, atol=tol, rtol=2e-2)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5, 6, 7, 8, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27])
@pytest.mark.parametrize("M,N,K,splits", [(128, 256, 256, 1), (77, 200, 320, 1),
                                          (300, 520, 1024, 3), (1, 64, 64, 1),
                                          (513, 136, 648, 2)])
def test_gemm_store_configs(cuda, dt, cfg, M, N, K, splits):
    from cake_amd.ops import gemm as G
    torch.manual_seed(M + N + K)
    x, w, b = _r(M, K, dt=dt), _r(N, K, dt=dt, std=K ** -0.5), _r(N, dt=dt)
    if cfg in G.K64_ONLY and K % 64:  # refused, not wrong
        from cake_amd.ops._lib import KernelError
        with pytest.raises(KernelError):
            G.linear(x, w, b, cfg=cfg, splits=splits)
        return
    y = G.linear(x, w, b, cfg=cfg, splits=splits)
    _close(y, _ref(x, w, b), K)
    y2 = G.linear(x, w, cfg=cfg, splits=splits)
    _close(y2, _ref(x, w), K)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("splits", [1, 4])
def test_gemm_resid32_and_add16(cuda, dt, splits):
    from cake_amd.ops import gemm as G
    torch.manual_seed(1)
    M, N, K = 200, 4096, 1024
    x, w = _r(M, K, dt=dt), _r(N, K, dt=dt, std=K ** -0.5)
    r = torch.randn(M, N, device="cuda")
    ref = r + _ref(x, w)
    G.linear(x, w, epi="resid32", resid=r, splits=splits)
    torch.testing.assert_close(r, ref, atol=3e-2, rtol=1e-2)
    b, r16 = _r(N, dt=dt), _r(M, N, dt=dt)
    y = G.linear(x, w, b, epi="add16", resid=r16, splits=splits)
    _close(y, _ref(x, w, b) + r16.float(), K)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("epi", ["silu", "quick_gelu", "gelu"])
@pytest.mark.parametrize("cfg,splits", [(None, 1), (0, 1), (4, 2)])
def test_gemm_activation_epilogues(cuda, dt, epi, cfg, splits):
    """Activation epilogue (time-embedding SiLU, CLIP quick_gelu / erf GELU) with bias,
    direct and through the split-K finalize."""
    from cake_amd.ops import gemm as G
    torch.manual_seed(4)
    M, N, K = 154, 3072, 768  # CLIP fc1 at batch 2 x 77 tokens
    x, w, b = _r(M, K, dt=dt), _r(N, K, dt=dt, std=K ** -0.5), _r(N, dt=dt)
    y = _ref(x, w, b)
    ref = {"silu": F.silu(y), "quick_gelu": y * torch.sigmoid(1.702 * y), "gelu": F.gelu(y)}[epi]
    _close(G.linear(x, w, b, epi=epi, cfg=cfg, splits=splits), ref, K)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("M,Fh,K,splits", [(37, 512, 512, 1), (130, 1024, 1024, 2),
                                          (257, 48, 320, 1)])
def test_gemm_gated(cuda, dt, M, Fh, K, splits):
    from cake_amd.ops import gemm as G
    torch.manual_seed(2)
    x, w = _r(M, K, dt=dt), _r(2 * Fh, K, dt=dt, std=K ** -0.5)
    y = _ref(x, w)
    g = G.linear(x, w, epi="swiglu", splits=splits)
    _close(g, F.silu(y[:, :Fh]) * y[:, Fh:], K)
    b = _r(2 * Fh, dt=dt)
    yb = _ref(x, w, b)
    h = G.linear(x, w, b, epi="geglu", splits=splits)
    _close(h, yb[:, :Fh] * F.gelu(yb[:, Fh:], approximate="tanh"), K)


def test_gemm_strided_views(cuda):
    """q|k|v column slices as inputs, 3-D token tensors, an output written into a view."""
    from cake_amd.ops import gemm as G
    dt = torch.bfloat16
    torch.manual_seed(3)
    qkv = _r(2, 50, 3 * 320, dt=dt)
    q = qkv[..., :320]
    w = _r(640, 320, dt=dt, std=320 ** -0.5)
    _close(G.linear(q, w), _ref(q.reshape(-1, 320), w).view(2, 50, 640), 320)
    out = torch.zeros(100, 2 * 640, device="cuda", dtype=dt)
    G.linear(q.reshape(100, 320), w, out=out[:, 640:])
    assert out[:, :640].abs().sum() == 0
    _close(out[:, 640:], _ref(q.reshape(100, 320), w), 320)


@pytest.mark.parametrize("name,M,N,K,epi", [
    ("8b_qkv", 512, 6144, 4096, "store"), ("8b_o", 512, 4096, 4096, "resid32"),
    ("8b_gateup", 512, 14336, 4096, "swiglu"), ("8b_down", 512, 4096, 14336, "resid32"),
    ("8b_qkv_t32", 32, 6144, 4096, "store"), ("70b_qkv", 256, 10240, 8192, "store"),
    ("70b_down", 128, 8192, 28672, "resid32"),
    ("sdxl_ff_in", 2048, 5120, 640, "geglu"), ("sdxl_ff_out", 2048, 640, 2560, "add16"),
    ("sdxl_qkv_1280", 2048, 3840, 1280, "store"), ("clip_fc1", 77, 3072, 768, "store")])
def test_gemm_model_shapes(cuda, name, M, N, K, epi):
    from cake_amd.ops import gemm as G
    dt = torch.bfloat16
    torch.manual_seed(4)
    x = _r(M, K, dt=dt)
    if epi in ("swiglu", "geglu"):
        w = _r(2 * N, K, dt=dt, std=K ** -0.5)
        y = _ref(x, w)
        ref = (F.silu(y[:, :N]) * y[:, N:]) if epi == "swiglu" else \
            y[:, :N] * F.gelu(y[:, N:], approximate="tanh")
        _close(G.linear(x, w, epi=epi), ref, K)
        return
    w = _r(N, K, dt=dt, std=K ** -0.5)
    if epi == "resid32":
        r = torch.randn(M, N, device="cuda")
        ref = r + _ref(x, w)
        G.linear(x, w, epi=epi, resid=r)
        torch.testing.assert_close(r, ref, atol=3e-2, rtol=1e-2)
    elif epi == "add16":
        r16 = _r(M, N, dt=dt)
        _close(G.linear(x, w, epi=epi, resid=r16), _ref(x, w) + r16.float(), K)
    else:
        _close(G.linear(x, w), _ref(x, w), K)



@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("cfg", [5, 0, 13, 14, 15, 16, 17, 20, 21, 22, 23, 24, 25, 26, 27])
@pytest.mark.parametrize("M,N,K", [(300, 700, 640), (257, 272, 2112), (520, 776, 200)])
def test_gemm_interleaved_all_epilogues(cuda, dt, cfg, M, N, K):
    """Interleaved-schedule tiles with ragged M/N and every epilogue."""
    from cake_amd.ops import gemm as G
    torch.manual_seed(M + N + K + cfg)
    x, w, b = _r(M, K, dt=dt), _r(N, K, dt=dt, std=K ** -0.5), _r(N, dt=dt)
    if cfg in G.K64_ONLY and K % 64:
        from cake_amd.ops._lib import KernelError
        with pytest.raises(KernelError):
            G.linear(x, w, b, cfg=cfg, splits=1)
        return
    _close(G.linear(x, w, b, cfg=cfg, splits=1), _ref(x, w, b), K)
    r = torch.randn(M, N, device="cuda")
    ref = r + _ref(x, w)
    G.linear(x, w, epi="resid32", resid=r, cfg=cfg, splits=1)
    torch.testing.assert_close(r, ref, atol=3e-2, rtol=1e-2)
    r16 = _r(M, N, dt=dt)
    _close(G.linear(x, w, b, epi="add16", resid=r16, cfg=cfg, splits=1),
           _ref(x, w, b) + r16.float(), K)
    Fh = N // 32 * 16
    w2 = _r(2 * Fh, K, dt=dt, std=K ** -0.5)
    if cfg in G.NO_GATED:  # 80-column wave tiles: the gated epilogue is refused, not wrong
        from cake_amd.ops._lib import KernelError
        with pytest.raises(KernelError):
            G.linear(x, w2, epi="swiglu", cfg=cfg, splits=1)
        return
    y = _ref(x, w2)
    _close(G.linear(x, w2, epi="swiglu", cfg=cfg, splits=1), F.silu(y[:, :Fh]) * y[:, Fh:], K)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("epi", ["store", "store32", "resid32", "swiglu"])
@pytest.mark.parametrize("M,N,K", [(513, 1024, 4096), (64, 640, 1280), (2048, 4096, 4096)])
def test_library_gemm_path(cuda, dt, epi, M, N, K):
    """The plan cfg LIB (hipBLASLt, csrc/driver/blaslt.cpp): every epilogue it carries,
    against the f32 reference; strided input rows and a strided f32 output."""
    from cake_amd.ops import _lib
    from cake_amd.ops import gemm as G
    torch.manual_seed(M + N)
    lib = _lib.kernels()
    assert hasattr(lib, "cake_blaslt_gemm"), "library GEMM entry point missing"
    xs = _r(M, K + 64, dt=dt)
    x = xs[:, 16:16 + K]                     # row stride K + 64
    Nv = 2 * N if epi == "swiglu" else N
    w = _r(Nv, K, dt=dt, std=K ** -0.5)
    y = _ref(x, w)
    if epi == "store":
        _close(G.linear(x, w, cfg=G.LIB), y, K)
    elif epi == "swiglu":
        ref = F.silu(y[:, :N]) * y[:, N:]
        _close(G.linear(x, w, epi="swiglu", cfg=G.LIB), ref, K)
    else:
        big = torch.randn(M, N + 8, device="cuda")
        r = big[:, :N]                       # f32 output with row stride N + 8
        ref = (r + y) if epi == "resid32" else y
        pad = big[:, N:].clone()
        G.linear(x, w, epi=epi, resid=r, cfg=G.LIB)
        torch.testing.assert_close(r, ref, atol=3e-2, rtol=1e-2)
        assert torch.equal(big[:, N:], pad)  # the row padding is not written


_NO_TORCH_LIB_GEMM = r"""
import ctypes as C, sys
import numpy as np
hip = C.CDLL("libamdhip64.so")
lib = C.CDLL(sys.argv[1])
assert "torch" not in sys.modules
M, N, K = 300, 512, 1024
rng = np.random.default_rng(0)
def bf16(a):  # round-to-nearest-even f32 -> bf16 bits
    u = a.astype(np.float32).view(np.uint32)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
x, w = rng.standard_normal((M, K)), rng.standard_normal((N, K)) / 32
xb, wb = bf16(x), bf16(w)
c0 = rng.standard_normal((M, N)).astype(np.float32)
ptr = lambda: C.c_void_p()
dx, dw, dc, ws = ptr(), ptr(), ptr(), ptr()
for p, n in ((dx, xb.nbytes), (dw, wb.nbytes), (dc, c0.nbytes), (ws, 32 << 20)):
    assert hip.hipMalloc(C.byref(p), C.c_size_t(n)) == 0
H2D, D2H = 1, 2
for p, a in ((dx, xb), (dw, wb), (dc, c0)):
    assert hip.hipMemcpy(p, a.ctypes.data_as(C.c_void_p), C.c_size_t(a.nbytes), H2D) == 0
L = C.c_longlong
rc = lib.cake_blaslt_gemm(0, 2, dx, L(K), dw, L(K), dc, L(N), M, N, K, ws,
                          C.c_size_t(32 << 20), C.c_void_p(0))
assert rc == 0, rc
assert hip.hipDeviceSynchronize() == 0
out = np.empty_like(c0)
assert hip.hipMemcpy(out.ctypes.data_as(C.c_void_p), dc, C.c_size_t(out.nbytes), D2H) == 0
f = lambda b: (b.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
ref = c0 + f(xb) @ f(wb).T
err = np.abs(out - ref).max()
assert err < 1e-2 * np.abs(ref).max(), err
maps = open("/proc/self/maps").read()
print("ok", err, "libhipblaslt from", sorted({l.split()[-1] for l in maps.splitlines() if "libhipblaslt" in l}))
"""


def test_library_gemm_without_torch(cuda):
    """The native engine / cake-cli / native worker processes load no torch: the kernel
    library's hipBLASLt dependency resolves on its own (RUNPATH) and the f32-accumulate
    GEMM is right there too."""
    import subprocess
    import sys
    from cake_amd.ops import _lib
    r = subprocess.run([sys.executable, "-c", _NO_TORCH_LIB_GEMM, str(_lib.lib_path())],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr[-3000:]


def test_library_gemm_plan_cache_eviction(cuda):
    """More distinct shapes than the library plan cache holds (4096): the cache empties and
    rebuilds, and results stay right before and after (a server sees every prompt length)."""
    from cake_amd.ops import gemm as G
    torch.manual_seed(3)
    w = _r(64, 64, dt=torch.bfloat16, std=0.125)
    xs = _r(4200, 64, dt=torch.bfloat16)
    out = torch.empty(4200, 64, device="cuda", dtype=torch.bfloat16)
    for M in range(1, 4200, 1):
        G.linear(xs[:M], w, cfg=G.LIB, out=out[:M])
    torch.cuda.synchronize()
    _close(out[:4199], _ref(xs[:4199], w), 64)
    y = G.linear(xs[:5], w, cfg=G.LIB)  # an evicted shape, rebuilt
    _close(y, _ref(xs[:5], w), 64)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("M,N,K,splits", [(2048, 6144, 4096, 1), (1000, 4096, 14336, 2),
                                          (2048, 2 * 14336, 4096, 1), (2048, 2 * 14336, 4096, 2)])
@pytest.mark.parametrize("cfg", [20, 21, 22, 23, 24, 25, 26, 27])
def test_big_tile_gemm_llama_shapes(cuda, dt, M, N, K, splits, cfg):
    """The ping-pong (cfg 20) and register-staged (cfg 21) 256x256 kernels on Llama
    prefill shapes: plain store, f32 residual accumulate (split-K included) and the fused
    SwiGLU, random operands."""
    from cake_amd.ops import gemm as G
    torch.manual_seed(M + N + K)
    x, w = _r(M, K, dt=dt), _r(N, K, dt=dt, std=K ** -0.5)
    if N > 16384:  # the fused gate|up weight
        Fh = N // 2
        y = _ref(x, w)
        _close(G.linear(x, w, epi="swiglu", cfg=cfg, splits=splits),
               F.silu(y[:, :Fh]) * y[:, Fh:], K)
        return
    _close(G.linear(x, w, cfg=cfg, splits=splits), _ref(x, w), K)
    r = torch.randn(M, N, device="cuda")
    ref = r + _ref(x, w)
    G.linear(x, w, epi="resid32", resid=r, cfg=cfg, splits=splits)
    torch.testing.assert_close(r, ref, atol=3e-2, rtol=1e-2)


@pytest.mark.parametrize("epi", ["store", "resid32", "swiglu"])
@pytest.mark.parametrize("cfg", [22, 23, 24, 25, 26, 27])
def test_four_wave_split_pair(cuda, epi, cfg):
    """cfg 22 with split-K 2 runs the in-kernel pair (the first split of a tile parks its
    accumulators, the second adds them and runs the epilogue; gemm_4w.h): equal to the
    f32 reference, bitwise repeatable whichever split arrives first, and the tile counters
    left clean for the next launch (a third call still matches)."""
    from cake_amd.ops import gemm as G
    torch.manual_seed(3)
    M, K = 2048, 4096
    N = 4096 if epi != "swiglu" else 2 * 2048
    x, w = _r(M, K, dt=torch.bfloat16), _r(N, K, dt=torch.bfloat16, std=K ** -0.5)
    y = _ref(x, w)
    outs = []
    for _ in range(3):
        if epi == "resid32":
            r = torch.zeros(M, N, device="cuda")
            G.linear(x, w, epi="resid32", resid=r, cfg=cfg, splits=2)
            outs.append(r)
        elif epi == "swiglu":
            outs.append(G.linear(x, w, epi="swiglu", cfg=cfg, splits=2))
        else:
            outs.append(G.linear(x, w, cfg=cfg, splits=2))
    ref = F.silu(y[:, :N // 2]) * y[:, N // 2:] if epi == "swiglu" else y
    _close(outs[0], ref, K)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


@pytest.mark.parametrize("cfg,N,epi", [(22, 2 * 14336, "swiglu"), (22, 9216, "store"),
                                       (25, 9216, "resid32"), (27, 4608, "store")])
def test_four_wave_remainder_pair(cuda, cfg, N, epi):
    """Split-K 2 on a grid of more than one wave: the tiles past the last whole wave run as
    in-kernel k-half pairs, the rest whole (8B gate|up at 2048 tokens: 896 tiles = 3 waves
    + 128 paired) -- equal to the f32 reference and repeatable."""
    from cake_amd.ops import gemm as G
    torch.manual_seed(5)
    M, K = 2048, 4096
    x, w = _r(M, K, dt=torch.bfloat16), _r(N, K, dt=torch.bfloat16, std=K ** -0.5)
    y = _ref(x, w)
    outs = []
    for _ in range(2):
        if epi == "resid32":
            r = torch.zeros(M, N, device="cuda")
            G.linear(x, w, epi="resid32", resid=r, cfg=cfg, splits=2)
            outs.append(r)
        else:
            outs.append(G.linear(x, w, epi=epi, cfg=cfg, splits=2))
    ref = F.silu(y[:, :N // 2]) * y[:, N // 2:] if epi == "swiglu" else y
    _close(outs[0], ref, K)
    assert torch.equal(outs[0], outs[1])
