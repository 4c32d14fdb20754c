"""Tokenizers.

Llama-3 weights/tokenizers are gated and there is no network here, so the default is a
deterministic synthetic tokenizer with the Llama-3 vocabulary *layout*: 128,000 ordinary
pieces followed by 256 special tokens (``<|begin_of_text|>`` = 128000,
``<|eot_id|>`` = 128009, header tokens 128006/128007).  Ordinary pieces are the 256 raw
bytes, then letter n-grams with optional leading space / capital, digit groups and
punctuation runs, so English text costs roughly 1 token per 3 characters (close to the
real tokenizer's ~4) and ``decode(encode(s)) == s`` for any string.

If ``tokenizer.json`` exists in a local model directory, the HF ``tokenizers`` library is
used instead (real Llama-3 vocabulary).

The reference applies the Llama-3 chat template by hand when the vLLM tokenizer has none
(llm/serve_llm.py:637-678); ``apply_chat_template`` reproduces that format.
"""
from __future__ import annotations

import itertools
import os
import re
import string
from functools import lru_cache
from pathlib import Path

import numpy as np

SPECIAL_NAMES = {
    0: "<|begin_of_text|>", 1: "<|end_of_text|>", 2: "<|reserved_special_token_0|>",
    3: "<|reserved_special_token_1|>", 4: "<|finetune_right_pad_id|>",
    5: "<|reserved_special_token_2|>", 6: "<|start_header_id|>", 7: "<|end_header_id|>",
    8: "<|eom_id|>", 9: "<|eot_id|>", 10: "<|python_tag|>",
}

_SPLIT = re.compile(r" ?[A-Za-z]+| ?[0-9]+| ?[^\sA-Za-z0-9]+|\s+")


class SyntheticTokenizer:
    """Deterministic, invertible tokenizer with a Llama-3-shaped vocabulary."""

    def __init__(self, vocab_size: int = 128256, num_special: int = 256):
        self.vocab_size = vocab_size
        self.num_special = num_special
        self.num_ordinary = vocab_size - num_special
        self.bos_token_id = self.num_ordinary + 0
        self.eos_token_id = self.num_ordinary + 9  # <|eot_id|>
        self.eot_token_id = self.eos_token_id
        self.start_header_id = self.num_ordinary + 6
        self.end_header_id = self.num_ordinary + 7
        pieces = _build_pieces(self.num_ordinary)
        self._id_to_piece: list[bytes] = pieces
        self._piece_to_id: dict[bytes, int] = {}
        for i, p in enumerate(pieces):
            self._piece_to_id.setdefault(p, i)
        self._special_text = {self.num_ordinary + k: v for k, v in SPECIAL_NAMES.items()}
        for k in range(num_special):
            self._special_text.setdefault(self.num_ordinary + k,
                                          f"<|reserved_special_token_{k}|>")
        self._special_ids = {v: k for k, v in self._special_text.items()}
        self._special_re = re.compile("(" + "|".join(
            re.escape(s) for s in sorted(self._special_ids, key=len, reverse=True)) + ")")

    # -- encode ----------------------------------------------------------------------------
    def _encode_chunk(self, chunk: str, out: list[int]):
        b = chunk.encode("utf-8")
        p2i = self._piece_to_id
        i = 0
        n = len(b)
        while i < n:
            # greedy longest match, pieces are at most 5 bytes long
            for L in (5, 4, 3, 2, 1):
                if i + L <= n:
                    t = p2i.get(b[i:i + L])
                    if t is not None:
                        out.append(t)
                        i += L
                        break
            else:  # pragma: no cover - every single byte is a piece
                out.append(b[i])
                i += 1

    def encode(self, text: str, add_special_tokens: bool = False,
               allow_special: bool = True) -> list[int]:
        ids: list[int] = []
        if add_special_tokens:
            ids.append(self.bos_token_id)
        parts = self._special_re.split(text) if allow_special else [text]
        for part in parts:
            if not part:
                continue
            sid = self._special_ids.get(part) if allow_special else None
            if sid is not None:
                ids.append(sid)
                continue
            for m in _SPLIT.finditer(part):
                self._encode_chunk(m.group(0), ids)
        return ids

    def __call__(self, text, add_special_tokens=False):
        return {"input_ids": self.encode(text, add_special_tokens=add_special_tokens)}

    # -- decode ----------------------------------------------------------------------------
    def decode(self, ids, skip_special_tokens: bool = True) -> str:
        buf = bytearray()
        out = []
        for t in ids:
            t = int(t)
            if t >= self.num_ordinary:
                if not skip_special_tokens:
                    out.append(buf.decode("utf-8", errors="replace"))
                    buf = bytearray()
                    out.append(self._special_text.get(t, ""))
                continue
            if 0 <= t < len(self._id_to_piece):
                buf += self._id_to_piece[t]
        out.append(buf.decode("utf-8", errors="replace"))
        return "".join(out)

    def count(self, text: str) -> int:
        return len(self.encode(text))

    def random_ids(self, n: int, rng: np.random.Generator) -> list[int]:
        """n ordinary (word-like) token ids, for synthetic prompts of exact length."""
        lo = 256
        return rng.integers(lo, self.num_ordinary, size=n).tolist()


@lru_cache(maxsize=4)
def _build_pieces(num_ordinary: int) -> list[bytes]:
    pieces: list[bytes] = [bytes([i]) for i in range(256)]
    seen = set(pieces)

    def add(p: str):
        b = p.encode()
        if b not in seen and len(pieces) < num_ordinary:
            seen.add(b)
            pieces.append(b)

    lower = string.ascii_lowercase
    # frequent short words / affixes first so small vocabularies still tokenise well
    common = ("the of and to in is it you that he was for on are with as his they be at one "
              "have this from or had by not word but what some we can out other were all "
              "there when up use your how said an each she which do their time if will way "
              "about many then them write would like so these her long make thing see him two "
              "has look more day could go come did number sound no most people my over know "
              "water than call first who may down side been now find any new work part take "
              "get place made live where after back little only round man year came show "
              "every good me give our under name very through just form sentence great think "
              "say help low line differ turn cause much mean before move right boy old too "
              "same tell does set three want air well also play small end put home read hand "
              "port large spell add even land here must big high such follow act why ask men "
              "change went light kind off need house picture try us again animal point mother "
              "world near build self earth father agent task tool plan step result answer "
              "ing ed er est ly tion ment ness able ous ive al").split()
    for w in common:
        for v in (w, " " + w, w.capitalize(), " " + w.capitalize()):
            add(v)
    for ch in string.punctuation:
        add(ch)
        add(" " + ch)
    for d in range(1000):
        add(str(d))
        add(" " + str(d))
    for a in lower:
        for v in (a, " " + a, a.upper(), " " + a.upper()):
            add(v)
    for a, b in itertools.product(lower, repeat=2):
        w = a + b
        for v in (w, " " + w, w.capitalize(), " " + w.capitalize()):
            add(v)
    for a, b, c in itertools.product(lower, repeat=3):
        w = a + b + c
        for v in (w, " " + w, w.capitalize(), " " + w.capitalize()):
            add(v)
    for s in ("\n", "\n\n", "  ", "    ", "\t", "**", "##", "###", "```", "->", "=>", "...",
              "\": \"", "\", \"", "{\"", "\"}", "\":"):
        add(s)
    # fill to size with deterministic 4-letter pieces
    rng = np.random.default_rng(1234)
    while len(pieces) < num_ordinary:
        w = "".join(rng.choice(list(lower), size=4))
        add(" " + w if rng.random() < 0.5 else w)
    return pieces[:num_ordinary]


class HFTokenizer:
    """Wrapper over a local ``tokenizer.json`` (HF tokenizers library)."""

    def __init__(self, path: str):
        from tokenizers import Tokenizer

        self._tok = Tokenizer.from_file(str(Path(path) / "tokenizer.json"))
        self.vocab_size = self._tok.get_vocab_size()
        self.bos_token_id = self._tok.token_to_id("<|begin_of_text|>") or 128000
        self.eos_token_id = self._tok.token_to_id("<|eot_id|>") or 128009
        self.eot_token_id = self.eos_token_id
        self.num_ordinary = self.vocab_size

    def encode(self, text, add_special_tokens=False, allow_special=True):
        return self._tok.encode(text, add_special_tokens=add_special_tokens).ids

    def decode(self, ids, skip_special_tokens=True):
        return self._tok.decode(list(map(int, ids)), skip_special_tokens=skip_special_tokens)

    def count(self, text):
        return len(self.encode(text))

    def random_ids(self, n, rng):
        return rng.integers(1000, min(self.vocab_size, 128000), size=n).tolist()


def get_tokenizer(model: str | None = None, vocab_size: int = 128256):
    if model:
        p = Path(model)
        if p.is_dir() and (p / "tokenizer.json").exists():
            try:
                return HFTokenizer(str(p))
            except Exception:
                pass
    return _synthetic(vocab_size)


@lru_cache(maxsize=4)
def _synthetic(vocab_size: int) -> SyntheticTokenizer:
    return SyntheticTokenizer(vocab_size=vocab_size)


DEFAULT_SYSTEM_PROMPT = os.environ.get(
    "LLM_DEFAULT_SYSTEM_PROMPT",
    "You are a helpful AI assistant. Provide clear, concise, and accurate responses.")


def apply_chat_template(prompt: str, system_prompt: str | None = None) -> str:
    """Llama-3 instruct chat format, built exactly as the reference's manual fallback
    (llm/serve_llm.py:655-678): optional system turn, user turn, open assistant header."""
    sys_p = system_prompt or DEFAULT_SYSTEM_PROMPT
    parts = ["<|begin_of_text|>"]
    if sys_p:
        parts.append(f"<|start_header_id|>system<|end_header_id|>\n\n{sys_p}<|eot_id|>")
    parts.append(f"<|start_header_id|>user<|end_header_id|>\n\n{prompt}<|eot_id|>")
    parts.append("<|start_header_id|>assistant<|end_header_id|>\n\n")
    return "".join(parts)
