"""SD component files: resolution, loading, random init and synthetic checkpoints.

Resolution mirrors ``ModelFile::get`` (cake-core/src/models/sd/sd.rs:19-102):
an explicit ``--sd-{unet,vae,clip,clip2,tokenizer,tokenizer-2}`` path wins;
otherwise the file is looked up under ``--model`` either in a diffusers
directory layout (``unet/diffusion_pytorch_model[.fp16].safetensors`` …) or in
an HF hub cache (``hub/models--org--name/snapshots/*/…``) for the repo the
reference would download (no network here: nothing is fetched).
"""
from __future__ import annotations

import glob
import json
import math
from pathlib import Path

import torch

from ...utils.safetensors_io import SafeTensors, save_file
from . import clip as clip_mod
from .config import SDConfig
from .unet import UNet2DConditionModel
from .vae import AutoencoderKL, normalize_vae_weights

REPOS = {"v1-5": "runwayml/stable-diffusion-v1-5", "v2-1": "stabilityai/stable-diffusion-2-1",
         "xl": "stabilityai/stable-diffusion-xl-base-1.0", "turbo": "stabilityai/sdxl-turbo"}
TOKENIZER_REPOS = {"v1-5": "openai/clip-vit-base-patch32", "v2-1": "openai/clip-vit-base-patch32",
                   "xl": "openai/clip-vit-large-patch14", "turbo": "openai/clip-vit-large-patch14"}
TOKENIZER2_REPO = "laion/CLIP-ViT-bigG-14-laion2B-39B-b160k"
VAE_FP16_FIX_REPO = "madebyollin/sdxl-vae-fp16-fix"

COMPONENT_FILES = {
    "unet": ("unet/diffusion_pytorch_model{f}.safetensors",),
    "vae": ("vae/diffusion_pytorch_model{f}.safetensors",),
    "clip": ("text_encoder/model{f}.safetensors",),
    "clip2": ("text_encoder_2/model{f}.safetensors",),
    "tokenizer": ("tokenizer/tokenizer.json", "tokenizer.json"),
    "tokenizer_2": ("tokenizer_2/tokenizer.json",),
}


def _hub_lookup(root: Path, repo: str, rel: str) -> Path | None:
    pat = root / "hub" / ("models--" + repo.replace("/", "--")) / "snapshots" / "*" / rel
    hits = sorted(glob.glob(str(pat)))
    return Path(hits[-1]) if hits else None


def resolve(component: str, override: str | None, version: str, use_f16: bool, model_dir) -> Path:
    if override:
        return Path(override)
    root = Path(model_dir)
    cands = []
    for pattern in COMPONENT_FILES[component]:
        for f in ((".fp16", "") if use_f16 else ("",)):
            cands.append(pattern.format(f=f))
    for rel in cands:
        if (root / rel).exists():
            return root / rel
    if component == "tokenizer":
        repo, rels = TOKENIZER_REPOS[version], ["tokenizer.json"]
    elif component == "tokenizer_2":
        repo, rels = TOKENIZER2_REPO, ["tokenizer.json"]
    elif component == "vae" and version in ("xl", "turbo") and use_f16:
        repo, rels = VAE_FP16_FIX_REPO, ["diffusion_pytorch_model.safetensors"]
    else:
        repo, rels = REPOS[version], cands
    for rel in rels:
        hit = _hub_lookup(root, repo, rel)
        if hit is not None:
            return hit
    raise FileNotFoundError(f"{component}: none of {cands} under {root} (and no HF-cache copy of "
                            f"{repo}); pass --sd-{component.replace('_', '-')} or write a synthetic "
                            "model with `python -m cake_amd.models.sd.weights --out DIR`")


def component_shapes(name: str, cfg: SDConfig) -> dict[str, tuple]:
    if name == "unet":
        return UNet2DConditionModel(cfg.unet).params()
    if name == "vae":
        return AutoencoderKL(cfg.vae).params()
    if name == "clip":
        return clip_mod.param_shapes(cfg.clip)
    if name == "clip2":
        return clip_mod.param_shapes(cfg.clip2)
    raise ValueError(name)


def load_component(name: str, path: Path, cfg: SDConfig, device, dtype) -> dict[str, torch.Tensor]:
    st = SafeTensors(path)
    raw = {k: st.get(k) for k in st.keys()}
    if name == "vae":
        raw = normalize_vae_weights(raw)
    shapes = component_shapes(name, cfg)
    out = {}
    for k, shp in shapes.items():
        if k not in raw:
            raise KeyError(f"{path}: missing tensor {k}")
        t = raw[k]
        if tuple(t.shape) != tuple(shp):
            raise ValueError(f"{path}: {k} has shape {tuple(t.shape)}, expected {shp}")
        out[k] = t.to(device=device, dtype=dtype).clone() if t.device.type == "cpu" and \
            torch.device(device).type == "cpu" else t.to(device=device, dtype=dtype)
    return out


def random_component(name: str, cfg: SDConfig, device, dtype, seed: int = 0) -> dict[str, torch.Tensor]:
    g = torch.Generator(device="cpu")
    g.manual_seed(seed * 131 + sum(map(ord, name)))
    out = {}
    for k, shp in component_shapes(name, cfg).items():
        if k.endswith(".bias"):
            t = torch.zeros(shp)
        elif len(shp) == 1:  # norm weights
            t = torch.ones(shp)
        elif "embedding" in k:
            t = torch.randn(shp, generator=g) * (0.02 if "token" in k else 0.01)
        else:
            fan_in = math.prod(shp[1:])
            t = torch.randn(shp, generator=g) * (0.7 / math.sqrt(fan_in))
        out[k] = t.to(device=device, dtype=dtype)
    return out


def unet_stage_keep(stages: list[str], n_stages: int):
    """Predicate over UNet parameter names: the weights the block-group stages `stages`
    run (UNet2DConditionModel.run_stage), plus what every stage needs (the time
    embedding and every resnet's time projection: time_biases is one stacked GEMM)."""
    pre = []
    for s in stages:
        kind, _, i = s.partition(".")
        if kind == "down":
            pre.append(f"down_blocks.{i}.")
            if i == "0":
                pre.append("conv_in.")
        elif kind == "mid":
            pre.append("mid_block.")
        else:
            pre.append(f"up_blocks.{i}.")
            if int(i) == (n_stages - 1) // 2 - 1:
                pre += ["conv_norm_out.", "conv_out."]

    def keep(k: str) -> bool:
        return (k.startswith("time_embedding.") or "time_emb_proj" in k
                or any(k.startswith(p) for p in pre))
    return keep


def random_component_on_device(name: str, cfg: SDConfig, device, dtype, seed: int = 0,
                               keep=None) -> dict[str, torch.Tensor]:
    """random_component's distributions drawn on the device (seconds instead of minutes
    for a full SDXL UNet on a busy host), restricted to the names `keep` accepts.  The
    same seed gives the same tensors on every rank of one device type."""
    import zlib
    g = torch.Generator(device=device)
    out = {}
    for k, shp in component_shapes(name, cfg).items():
        if keep is not None and not keep(k):
            continue
        # one seed per tensor: a rank keeping a subset draws the same values for it
        g.manual_seed(seed * 1000003 + zlib.crc32(f"{name}/{k}".encode()))
        if k.endswith(".bias"):
            t = torch.zeros(shp, device=device, dtype=dtype)
        elif len(shp) == 1:
            t = torch.ones(shp, device=device, dtype=dtype)
        else:
            std = (0.02 if "token" in k else 0.01) if "embedding" in k else \
                0.7 / math.sqrt(math.prod(shp[1:]))
            t = torch.empty(shp, device=device, dtype=dtype).normal_(0.0, std, generator=g)
        out[k] = t
    return out


# --------------------------------------------------------------------- synthetic files
def write_clip_tokenizer(path: Path, vocab_size: int) -> None:
    """Byte-level BPE tokenizer with CLIP's <|startoftext|>/<|endoftext|> wrapping."""
    from tokenizers import AddedToken, Tokenizer, decoders, models, pre_tokenizers, processors

    from ...utils.synth import _bytes_to_unicode
    b2u = _bytes_to_unicode()
    vocab = {b2u[b]: b for b in range(256)}
    specials = {"<|startoftext|>": vocab_size - 2, "<|endoftext|>": vocab_size - 1}
    by_id = {i: s for s, i in specials.items()}
    for i in range(256, vocab_size):
        vocab[by_id.get(i, f"<unused_{i}>")] = i
    tok = Tokenizer(models.BPE(vocab=vocab, merges=[]))
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    tok.add_special_tokens([AddedToken(s, special=True) for s in specials])
    tok.post_processor = processors.TemplateProcessing(
        single="<|startoftext|> $A <|endoftext|>",
        special_tokens=[(s, i) for s, i in specials.items()])
    path.parent.mkdir(parents=True, exist_ok=True)
    tok.save(str(path))


def write_sd_checkpoint(out_dir, cfg: SDConfig, dtype=torch.float16, seed: int = 0,
                        tiny: bool = False, mini: bool = False) -> Path:
    out = Path(out_dir)
    suffix = ".fp16" if dtype == torch.float16 else ""
    names = ["unet", "vae", "clip"] + (["clip2"] if cfg.clip2 else [])
    for n in names:
        rel = COMPONENT_FILES[n][0].format(f=suffix)
        p = out / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        save_file(random_component(n, cfg, "cpu", dtype, seed), p, {"format": "pt"})
    write_clip_tokenizer(out / "tokenizer" / "tokenizer.json", cfg.clip.vocab_size)
    if cfg.clip2:
        write_clip_tokenizer(out / "tokenizer_2" / "tokenizer.json", cfg.clip2.vocab_size)
    (out / "cake_sd.json").write_text(json.dumps({"version": cfg.version, "synthetic": True,
                                                     "tiny": tiny, "mini": mini}))
    return out


def main(argv=None) -> int:
    import argparse

    from .config import get_config, mini_config, tiny_config
    ap = argparse.ArgumentParser(description="write a random-init SD checkpoint (diffusers layout)")
    ap.add_argument("--version", default="v1-5", choices=["v1-5", "v2-1", "xl", "turbo"])
    ap.add_argument("--tiny", action="store_true")
    ap.add_argument("--mini", action="store_true", help="the small all-HIP-shapes architecture")
    ap.add_argument("--out", required=True)
    ap.add_argument("--f32", action="store_true")
    a = ap.parse_args(argv)
    cfg = (mini_config(a.version) if a.mini else tiny_config(a.version) if a.tiny
           else get_config(a.version))
    write_sd_checkpoint(a.out, cfg, torch.float32 if a.f32 else torch.float16, tiny=a.tiny,
                        mini=a.mini)
    print(a.out)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
