"""cake-cli: one entry point, master or worker mode (cake-cli/src/main.rs:8-63).

Flag names and defaults follow cake-core/src/lib.rs:21-200;
the image-generation flags double as the JSON keys of the image API.
MI355X additions: ``--max-seq-len``, ``--no-graph``, ``--trace FILE``,
``--log-level``.

    cake_amd/lib/cake-cli --model DIR --topology topology.yml --prompt "..."
    cake_amd/lib/cake-cli --mode worker --name w1 --model DIR --topology t.yml --address 0.0.0.0:10128
    cake_amd/lib/cake-cli --model DIR --api 0.0.0.0:8080

``cake-cli`` is the native executable (csrc/tools/cake_cli.cpp): it parses and
validates these flags and resolves the topology natively, then runs the role
with the compute runtime embedded in-process (:func:`run_parsed`).  ``python -m
cake_amd.cli`` takes the same flags (development entry).
"""
from __future__ import annotations

import argparse
import logging
import os
import sys

SD_VERSIONS = ["v1-5", "v2-1", "xl", "turbo"]


def _bool(s: str) -> bool:
    return str(s).lower() in ("1", "true", "yes", "on")


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="cake-cli", description="MI355X-native distributed inference")
    a = ap.add_argument
    a("--device", type=int, default=0, help="GPU ordinal")
    a("--mode", choices=["master", "worker"], default="master")
    a("--name", default=None, help="worker name (must be in the topology)")
    a("--address", default="127.0.0.1:10128", help="worker bind address")
    a("--api", default=None, help="serve the REST API on this address instead of one CLI generation")
    a("--model", default="./cake-data/Meta-Llama-3-8B/")
    a("--topology", default="./cake-data/topology.yml")
    a("--prompt", default="The sky is blue because ")
    a("--system-prompt", default="You are a helpful AI assistant.")
    a("--seed", type=int, default=299792458)
    a("-n", "--sample-len", type=int, default=100)
    a("--temperature", type=float, default=1.0)
    a("--top-p", type=float, default=None)
    a("--top-k", type=int, default=None)
    a("--repeat-penalty", type=float, default=1.1)
    a("--repeat-last-n", type=int, default=128)
    a("--dtype", default=None, help="f16 (default), bf16 or f32")
    a("--cpu", action="store_true")
    a("--model-type", choices=["text-model", "image-model"], default="text-model")
    # SD args (lib.rs:90-127)
    a("--sd-tokenizer", default=None)
    a("--sd-tokenizer-2", default=None)
    a("--sd-version", choices=SD_VERSIONS, default="v1-5")
    a("--sd-use-f16", type=_bool, default=True)
    a("--sd-width", type=int, default=None)
    a("--sd-height", type=int, default=None)
    a("--sd-sliced-attention-size", type=int, default=None)
    a("--sd-clip", default=None)
    a("--sd-clip2", default=None)
    a("--sd-vae", default=None)
    a("--sd-unet", default=None)
    a("--sd-use-flash-attention", action="store_true")
    # image generation args (lib.rs:129-200)
    a("--sd-image-prompt", default="A very realistic photo of a rusty robot walking on a sandy beach")
    a("--sd-uncond-prompt", default="")
    a("--sd-tracing", action="store_true")
    a("--sd-n-steps", type=int, default=None)
    a("--sd-num-samples", type=int, default=1)
    a("--sd-bsize", type=int, default=1)
    a("--sd-intermediary-images", type=int, default=0)
    a("--sd-guidance-scale", type=float, default=None)
    a("--sd-img2img", default=None)
    a("--sd-img2img-strength", type=float, default=0.8)
    a("--sd-seed", type=int, default=None)
    # MI355X-native extras
    a("--transport", choices=["tcp", "rccl", "loopback"], default="tcp",
      help="rccl: torchrun one rank per GPU, rank 0 master, rank i serves topology node i; "
           "loopback: every topology node served in-process (wire protocol over 127.0.0.1)")
    a("--parallel", choices=["pp", "tp"], default="pp",
      help="with --transport rccl: pp = the topology's layer sharding (reference), "
           "tp = tensor parallel (every rank 1/N of every layer; topology layers ignored)")
    a("--hop", choices=["ipc", "dist"], default="ipc",
      help="--transport rccl pp: ipc = device-side hops captured in each rank's decode graph, "
           "dist = host-issued RCCL p2p per hop")
    a("--hop-dtype", choices=["f32", "bf16"], default="f32",
      help="hidden-state payload of an ipc hop (bf16 = the reference's 16-bit transport)")
    a("--max-seq-len", type=int, default=4096)
    a("--no-graph", action="store_true", help="disable hipGraph capture of the decode step")
    a("--trace", default=None, help="write a chrome-trace JSON of each text generation")
    a("--metrics", default=None, help="append one JSON line of stats per generation")
    a("--log-level", default=os.environ.get("CAKE_LOG", "info"))
    return ap


def setup_logging(level: str) -> None:
    # RUST_LOG default "info,tokenizers=error,actix_server=warn" (cake-cli/src/main.rs:14-22)
    logging.basicConfig(level=getattr(logging, level.upper(), logging.INFO),
                        format="[%(asctime)s %(levelname)s] %(message)s", datefmt="%H:%M:%S")
    logging.getLogger("uvicorn.access").setLevel(logging.WARNING)


def run_parsed(opts: dict) -> int:
    """Entry point of the native cake-cli / cake_start_worker (csrc/tools/cake_cli.cpp,
    csrc/runtime/capi.cpp): the flags were parsed and validated natively; ``opts``
    maps argparse dests to typed values.  Unknown keys are rejected."""
    ap = build_parser()
    args = ap.parse_args([])
    for k, v in opts.items():
        if not hasattr(args, k):
            raise ValueError(f"unknown option {k!r}")
        setattr(args, k, v)
    return _run(args)


def main(argv: list[str] | None = None) -> int:
    return _run(build_parser().parse_args(argv))


def _run(args) -> int:
    setup_logging(args.log_level)
    from .context import Context
    ctx = Context.from_args(args)
    if args.transport == "rccl":
        from .parallel.rccl_roles import run_rccl
        run_rccl(ctx)
        return 0
    if args.mode == "worker":
        from .parallel.worker import Worker
        Worker(ctx).run()
        return 0
    workers = []
    if args.transport == "loopback":
        from .parallel.loopback import start_loopback_workers
        workers = start_loopback_workers(ctx)
    from .master import Master
    try:
        Master(ctx).run()
    finally:
        if workers:
            from .parallel.loopback import stop_loopback_workers
            stop_loopback_workers(workers)
    return 0


if __name__ == "__main__":
    sys.exit(main())
