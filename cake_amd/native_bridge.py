"""Tokenizer side of the native text path.

cake-cli generates text with the native engine (libcake_engine.so: checkpoint load,
prefill, graph-replayed decode, device token selection — no PyTorch); the one piece it
leaves to the interpreter it embeds is the HF tokenizer (tokenizers' Rust core behind
its Python binding), reached through these JSON-in / JSON-out functions
(csrc/runtime/embed.cpp call_python).  Prompt rendering and token text follow the
Python generator exactly (models/llama3/generator.py: the Llama-3 dialog template of
models/chat.py, per-token decode with special tokens kept).
"""
from __future__ import annotations

import json
from pathlib import Path

_cache: dict = {}


def _tokenizer(model_dir: str):
    t = _cache.get(model_dir)
    if t is None:
        from .models.llama3.config import LlamaConfig
        from .models.llama3.generator import load_tokenizer
        cfg = LlamaConfig.from_path(Path(model_dir))
        t = _cache[model_dir] = load_tokenizer(model_dir, cfg.eos_token_id)
    return t


def encode_chat(req: str) -> str:
    """{"model", "system", "prompt"} -> {"ids": [...], "eos": [...]}"""
    from .models.chat import History, Message
    r = json.loads(req)
    tok, eos = _tokenizer(r["model"])
    h = History()
    h.append(Message.system(r.get("system", "")))
    h.append(Message.user(r["prompt"]))
    ids = tok.encode(h.encode_dialog_to_prompt(), add_special_tokens=False).ids
    return json.dumps({"ids": list(ids), "eos": sorted(eos)})


def decode_token(req: str) -> str:
    """{"model", "id"} -> the token's text ("" when undecodable)."""
    r = json.loads(req)
    tok, _ = _tokenizer(r["model"])
    try:
        return tok.decode([int(r["id"])], skip_special_tokens=False) or ""
    except Exception:  # noqa: BLE001  (the generator streams nothing for such ids)
        return ""
