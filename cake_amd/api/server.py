"""REST API (cake-core/src/cake/api/{mod,text,image}.rs).

* ``POST /api/v1/chat/completions`` — OpenAI-shaped, one JSON response
  ``{id (uuid4), object: "chat.completion", created, model: "llama3",
  choices: [{index: 0, message: {role, content}}]}`` (text.rs:16-52,54-96).
  One request at a time (the reference's global write lock, text.rs:67):
  reset → add messages → generate.  Superset (Appendix E Q4/Q5): honours
  ``max_tokens``, ``stream`` (server-sent events) and per-request
  ``temperature`` / ``top_p`` / ``top_k`` / ``seed`` (the server's CLI values
  when absent; on the device path they are read by the decode graph from device
  memory, no recapture), adds a ``usage`` block
  and lowercase ``role`` (``CAKE_API_REFERENCE_ROLES=1`` restores the
  capitalised reference serialisation).
* ``POST /api/v1/image`` — body ``{"image_args": {...sd-* keys...}}``,
  returns ``{"images": [base64 PNG, ...]}`` (image.rs:15-68).
* anything else → 404 with body ``nope`` (mod.rs:19-21,40).
"""


import base64
import io
import json
import logging
import os
import threading
import time
import uuid

log = logging.getLogger("cake.api")


def _reference_roles() -> bool:
    return os.environ.get("CAKE_API_REFERENCE_ROLES", "0") == "1"


def request_sampling(body: dict, default):
    """SamplingConfig of one chat request: the server default with the request's
    temperature / top_p / top_k / seed.  ValueError on an invalid value."""
    import dataclasses
    over = {}
    if body.get("temperature") is not None:
        t = float(body["temperature"])
        if not t >= 0.0:
            raise ValueError("temperature must be >= 0")
        over["temperature"] = t
    if body.get("top_p") is not None:
        p = float(body["top_p"])
        if not 0.0 < p <= 1.0:
            raise ValueError("top_p must be in (0, 1]")
        over["top_p"] = None if p >= 1.0 else p
    if body.get("top_k") is not None:
        k = body["top_k"]
        if isinstance(k, bool) or not isinstance(k, int) or k < 0:
            raise ValueError("top_k must be a non-negative integer")
        over["top_k"] = k or None
    if body.get("seed") is not None:
        sd = body["seed"]
        if isinstance(sd, bool) or not isinstance(sd, int):
            raise ValueError("seed must be an integer")
        over["seed"] = sd & 0xFFFFFFFFFFFFFFFF
    return dataclasses.replace(default, **over)


def create_app(master):
    from fastapi import FastAPI, Request
    from fastapi.responses import JSONResponse, PlainTextResponse, StreamingResponse

    from ..models.chat import Message

    app = FastAPI(title="cake_amd", docs_url=None, redoc_url=None, openapi_url=None)
    lock = threading.Lock()  # one generation at a time (text.rs:67)

    @app.post("/api/v1/chat/completions")
    async def chat(request: Request):
        body = await request.json()
        client = request.client.host if request.client else "?"
        log.info("starting chat for %s ...", client)
        if master.llm is None:
            return JSONResponse({"error": "LLM model not found"}, status_code=400)
        try:
            messages = [Message.from_dict(m) for m in body["messages"]]
        except (KeyError, TypeError, ValueError) as e:
            return JSONResponse({"error": f"bad request: {e}"}, status_code=400)
        max_tokens = body.get("max_tokens")
        default = getattr(master.ctx, "sampling", None)
        sampling = None
        if default is not None and hasattr(master.llm, "set_sampling"):
            try:
                sampling = request_sampling(body, default)
                check = getattr(master.llm, "check_sampling", None)
                if check is not None:
                    check(sampling)  # a generator may support only part of the space
            except (TypeError, ValueError) as e:
                return JSONResponse({"error": f"bad request: {e}"}, status_code=400)
        model_name = master.llm.MODEL_NAME
        rid, created = str(uuid.uuid4()), int(time.time())
        role = "Assistant" if _reference_roles() else "assistant"

        def run(sink):
            with lock:
                master.reset()
                # a new configuration, or an explicit seed (restart its stream)
                if sampling is not None and (body.get("seed") is not None or
                                             sampling != getattr(master.llm, "sampling", None)):
                    master.llm.set_sampling(sampling)
                for m in messages:
                    master.llm.add_message(m)
                return master.generate_text(sink, max_tokens=max_tokens)

        if body.get("stream"):
            import queue
            q: queue.Queue = queue.Queue()

            def worker():
                try:
                    run(lambda s: q.put(s))
                finally:
                    q.put(None)
            threading.Thread(target=worker, daemon=True).start()

            def events():
                while True:
                    s = q.get()
                    if s is None:
                        break
                    chunk = {"id": rid, "object": "chat.completion.chunk", "created": created,
                             "model": model_name,
                             "choices": [{"index": 0, "delta": {"content": s}, "finish_reason": None}]}
                    yield f"data: {json.dumps(chunk)}\n\n"
                yield "data: [DONE]\n\n"
            return StreamingResponse(events(), media_type="text/event-stream")

        import anyio
        parts: list[str] = []
        stats = await anyio.to_thread.run_sync(lambda: run(parts.append))
        text = "".join(parts)
        return JSONResponse({
            "id": rid, "object": "chat.completion", "created": created, "model": model_name,
            "choices": [{"index": 0, "message": {"role": role, "content": text},
                         "finish_reason": "stop"}],
            "usage": {"completion_tokens": stats.get("generated", 0)},
        })

    @app.post("/api/v1/image")
    async def image(request: Request):
        body = await request.json()
        if master.sd is None:
            return JSONResponse({"error": "image model not found"}, status_code=400)
        from ..models.sd.args import ImageGenerationArgs
        args = ImageGenerationArgs.from_json(body.get("image_args", {}))
        out: list[str] = []

        def cb(images):
            for img in images:
                buf = io.BytesIO()
                img.save(buf, format="PNG")
                out.append(base64.b64encode(buf.getvalue()).decode())

        import anyio

        def run():
            with lock:
                master.generate_image(args, cb)
        await anyio.to_thread.run_sync(run)
        return JSONResponse({"images": out})

    @app.api_route("/{path:path}", methods=["GET", "POST", "PUT", "DELETE", "PATCH"])
    async def nope(path: str):
        return PlainTextResponse("nope", status_code=404)

    return app


def start(master, address: str) -> None:
    import uvicorn
    host, _, port = address.rpartition(":")
    log.info("starting api on http://%s:%s ...", host, port)
    uvicorn.run(create_app(master), host=host or "0.0.0.0", port=int(port), log_level="warning")
