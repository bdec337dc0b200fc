"""Model plug-in contract (cake-core/src/models/mod.rs:14-71).

``Generator`` (load from a Context), ``TextGenerator`` (add_message / reset /
next_token(index) / generated_tokens) and ``ImageGenerator``
(generate_image(args, callback)).  ``Token`` carries the id, its decoded text
and the end-of-stream flag; ``str(token)`` is the text (mod.rs:27-36).
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from dataclasses import dataclass
from typing import Callable


@dataclass
class Token:
    id: int
    text: str | None
    is_end_of_stream: bool

    def __str__(self) -> str:
        return self.text or ""


class Generator(ABC):
    MODEL_NAME: str = ""

    @classmethod
    @abstractmethod
    def load(cls, ctx) -> "Generator | None":
        ...


class TextGenerator(Generator):
    @abstractmethod
    def add_message(self, message) -> None: ...

    @abstractmethod
    def reset(self) -> None: ...

    @abstractmethod
    def next_token(self, index: int) -> Token: ...

    @abstractmethod
    def generated_tokens(self) -> int: ...


class ImageGenerator(Generator):
    @abstractmethod
    def generate_image(self, args, callback: Callable[[list], None]) -> None: ...
