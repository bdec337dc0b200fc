"""Synthetic model directories (no network): random-init weights in HF layout.

Produces what the reference expects under ``--model``:
``config.json``, ``model.safetensors.index.json`` + shards (or one
``model.safetensors``), and a byte-level BPE ``tokenizer.json`` carrying the
Llama-3 special tokens (``<|begin_of_text|>``, ``<|start_header_id|>``,
``<|end_header_id|>``, ``<|eot_id|>``, ``<|end_of_text|>``) at the ids the
config names.  Ids not covered by bytes or specials decode to placeholder
strings, so any id a random model emits is decodable.

CLI: ``python -m cake_amd.utils.synth --preset tiny --out DIR``
"""
from __future__ import annotations

import argparse
import json
from pathlib import Path

import torch

from ..models.llama3.config import LlamaConfig, preset
from ..models.llama3.weights import BlockWeights, HeadWeights, layer_name
from .safetensors_io import save_file

SPECIALS = ["<|begin_of_text|>", "<|end_of_text|>", "<|start_header_id|>", "<|end_header_id|>",
            "<|eot_id|>"]


def special_ids(cfg: LlamaConfig) -> dict[str, int]:
    """Llama-3 layout when the vocab is large enough, else right after the 256 bytes."""
    if cfg.vocab_size >= 128256:
        return {"<|begin_of_text|>": 128000, "<|end_of_text|>": 128001,
                "<|start_header_id|>": 128006, "<|end_header_id|>": 128007, "<|eot_id|>": 128009}
    base = 256
    return {s: base + i for i, s in enumerate(SPECIALS)}


def tiny_config(**kw) -> LlamaConfig:
    """Tiny test architecture whose bos/eos match the synthetic tokenizer."""
    d = dict(bos_token_id=256, eos_token_id=260)
    d.update(kw)
    return preset("tiny", **d)


def _bytes_to_unicode() -> dict[int, str]:
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {b: chr(c) for b, c in zip(bs, cs)}


def write_tokenizer(out_dir: Path, cfg: LlamaConfig) -> Path:
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers
    from tokenizers import AddedToken

    specials = special_ids(cfg)
    b2u = _bytes_to_unicode()
    vocab: dict[str, int] = {}
    for b in range(256):
        vocab[b2u[b]] = b
    by_id = {i: s for s, i in specials.items()}
    for i in range(256, cfg.vocab_size):
        vocab[by_id.get(i, f"<unused_{i}>")] = i  # specials live in the vocab at their ids
    tok = Tokenizer(models.BPE(vocab=vocab, merges=[], fuse_unk=False))
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=True)
    tok.decoder = decoders.ByteLevel()
    # added tokens must land on their fixed ids: add them in id order
    tok.add_special_tokens([AddedToken(s, special=True, normalized=False)
                            for s, _ in sorted(specials.items(), key=lambda kv: kv[1])])
    path = out_dir / "tokenizer.json"
    tok.save(str(path))
    check = Tokenizer.from_file(str(path))
    for s, i in specials.items():
        assert check.token_to_id(s) == i, (s, check.token_to_id(s), i)
    return path


def write_checkpoint(out_dir: str | Path, cfg: LlamaConfig, dtype: torch.dtype = torch.bfloat16,
                     seed: int = 0, shard_bytes: int = 2 << 30, single_file: bool = False) -> Path:
    """Random-init Llama weights (same values as factory.random_model(seed) on CPU)."""
    out = Path(out_dir)
    out.mkdir(parents=True, exist_ok=True)
    sp = special_ids(cfg)
    cfgd = cfg.to_hf_dict()
    cfgd["torch_dtype"] = {torch.bfloat16: "bfloat16", torch.float16: "float16",
                           torch.float32: "float32"}[dtype]
    (out / "config.json").write_text(json.dumps(cfgd, indent=2))
    write_tokenizer(out, cfg)
    del sp
    gen = torch.Generator(device="cpu")
    shards: list[dict[str, torch.Tensor]] = [{}]
    size = 0

    def add(name: str, t: torch.Tensor):
        nonlocal size
        nb = t.numel() * t.element_size()
        if not single_file and size + nb > shard_bytes and shards[-1]:
            shards.append({})
            size = 0
        shards[-1][name] = t
        size += nb

    gen.manual_seed(seed * 7919 + 17)
    head = HeadWeights.random(cfg, "cpu", dtype, gen)
    for li in range(cfg.num_hidden_layers):
        gen.manual_seed(seed * 1000003 + li)
        bw = BlockWeights.random(cfg, "cpu", dtype, gen)
        for k, v in bw.state_dict(layer_name(li)).items():
            add(k, v)
    for k, v in head.state_dict().items():
        add(k, v)
    if single_file or len(shards) == 1:
        save_file(shards[0], out / "model.safetensors", {"format": "pt"})
        return out
    weight_map = {}
    n = len(shards)
    for i, sh in enumerate(shards):
        fname = f"model-{i + 1:05d}-of-{n:05d}.safetensors"
        save_file(sh, out / fname, {"format": "pt"})
        weight_map.update({k: fname for k in sh})
    total = sum(t.numel() * t.element_size() for sh in shards for t in sh.values())
    (out / "model.safetensors.index.json").write_text(json.dumps(
        {"metadata": {"total_size": total}, "weight_map": weight_map}, indent=2))
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="write a random-init Llama-3 checkpoint")
    ap.add_argument("--preset", default="tiny")
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--out", required=True)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--shard-mb", type=int, default=2048)
    a = ap.parse_args(argv)
    from ..models.llama3.factory import parse_dtype
    kw = {} if a.layers is None else {"num_hidden_layers": a.layers}
    cfg = tiny_config(**kw) if a.preset == "tiny" else preset(a.preset, **kw)
    write_checkpoint(a.out, cfg, parse_dtype(a.dtype), a.seed, a.shard_mb << 20)
    print(a.out)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
