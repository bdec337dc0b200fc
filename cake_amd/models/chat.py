"""Chat message types and the Llama-3 dialog template.

* ``MessageRole`` / ``Message``: cake-core/src/models/chat.rs:3-64 — roles
  deserialize from lower- or capitalised names; the reference serializes the
  *capitalised* variant name ("Assistant").  We emit
  lowercase by default (OpenAI clients expect it) and keep the reference form
  available via ``role_str(reference=True)``.
* ``History``: cake-core/src/models/llama3/history.rs:4-34 —
  ``<|begin_of_text|>`` + per message
  ``<|start_header_id|>{role}<|end_header_id|>\\n\\n{content.trim()}<|eot_id|>``
  + the assistant header.
"""
from __future__ import annotations

from dataclasses import dataclass
from enum import Enum


class MessageRole(str, Enum):
    SYSTEM = "system"
    USER = "user"
    ASSISTANT = "assistant"

    @classmethod
    def parse(cls, s: str) -> "MessageRole":
        try:
            return cls(s.lower())
        except ValueError:
            raise ValueError(f"unknown role {s!r}") from None

    def role_str(self, reference: bool = False) -> str:
        return self.value.capitalize() if reference else self.value

    def __str__(self) -> str:
        return self.value


@dataclass
class Message:
    role: MessageRole
    content: str

    @classmethod
    def system(cls, c: str) -> "Message":
        return cls(MessageRole.SYSTEM, c)

    @classmethod
    def user(cls, c: str) -> "Message":
        return cls(MessageRole.USER, c)

    @classmethod
    def assistant(cls, c: str) -> "Message":
        return cls(MessageRole.ASSISTANT, c)

    @classmethod
    def from_dict(cls, d: dict) -> "Message":
        return cls(MessageRole.parse(d["role"]), str(d.get("content", "")))

    def to_dict(self, reference: bool = False) -> dict:
        return {"role": self.role.role_str(reference), "content": self.content}


class History(list):
    @staticmethod
    def encode_header(role: MessageRole) -> str:
        return f"<|start_header_id|>{role}<|end_header_id|>\n\n"

    @classmethod
    def encode_message(cls, m: Message) -> str:
        return cls.encode_header(m.role) + m.content.strip() + "<|eot_id|>"

    def encode_dialog_to_prompt(self) -> str:
        out = "<|begin_of_text|>"
        for m in self:
            out += self.encode_message(m)
        return out + self.encode_header(MessageRole.ASSISTANT)
