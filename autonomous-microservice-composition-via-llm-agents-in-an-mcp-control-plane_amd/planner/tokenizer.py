"""Byte-level BPE tokenizer for the planner.

No network means no Meta tokenizer files, so the framework ships its own
byte-level BPE (HF ``tokenizers`` runtime), trained once, deterministically,
on a synthetic control-plane corpus (registries, prompts, DAG JSON, intents)
and stored as ``planner/tokenizer.json``.  Token ids live inside Llama-3's
128,256-entry vocabulary (the learned merges use the low ids; ``BOS`` is
128000 as in Llama-3), so the model shapes are exactly Llama-3's.  At ~3.5-4
characters per token on prompt text it produces prompt lengths comparable to
the real Llama-3 tokenizer (chars/4).
"""
from __future__ import annotations

import functools
import json
import os
import random
from typing import List, Optional

LLAMA3_VOCAB = 128256
BOS_ID = 128000
EOS_ID = 128001
_HERE = os.path.dirname(os.path.abspath(__file__))
TOKENIZER_PATH = os.path.join(_HERE, "tokenizer.json")
TRAIN_VOCAB = 32000


def _corpus(seed: int = 0) -> List[str]:
    from ..registry.records import synthetic_registry
    from .prompt import HEADER, SYNTHETIC_INTENTS, build_prompt, service_line
    rng = random.Random(seed)
    docs = [HEADER] * 50
    for n, sd in [(10, 1), (50, 2), (200, 3), (1000, 4)]:
        reg = synthetic_registry(n, seed=sd)
        docs += [service_line(s) for s in reg]
        for i in range(60):
            chosen = rng.sample(reg, min(len(reg), rng.randint(1, 5)))
            nodes, edges = [], []
            for j, s in enumerate(chosen):
                keys = list((s["input_schema"].get("properties") or {}).keys())
                srcs = [x["name"] for x in chosen[:j]] or keys
                nodes.append({"name": s["name"], "endpoint": s["endpoint"],
                              "inputs": {k: rng.choice(srcs + [k]) for k in keys},
                              "retries": rng.randint(0, 3)})
                if j:
                    edges.append({"from": chosen[j - 1]["name"], "to": s["name"],
                                  "fallback": s["fallback"]})
            docs.append(json.dumps({"nodes": nodes, "edges": edges}, separators=(",", ":")))
        docs.append(build_prompt(reg[:10], SYNTHETIC_INTENTS[sd % len(SYNTHETIC_INTENTS)]))
    for i in range(400):
        docs.append("User intent: “" + SYNTHETIC_INTENTS[i % len(SYNTHETIC_INTENTS)].format(i=i) + "”")
    english = ("the quick brown fox jumps over the lazy dog while the service mesh routes "
               "requests between microservices with retries timeouts and fallbacks so that "
               "every order payment and shipment is processed exactly once for each customer ")
    docs += [english] * 200
    return docs


def train(path: str = TOKENIZER_PATH, vocab_size: int = TRAIN_VOCAB) -> str:
    from tokenizers import Tokenizer as HFTok, decoders, models, pre_tokenizers, trainers
    tok = HFTok(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=True)
    tok.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(vocab_size=vocab_size, min_frequency=2, show_progress=False,
                                  initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tok.train_from_iterator(_corpus(), trainer=trainer)
    tok.save(path)
    return path


class Tokenizer:
    """``tokenizer.json`` (HF ``tokenizers`` runtime) plus the ids the planner
    needs: BOS (prepended to every prompt), EOS and the model vocabulary size.

    The default is the shipped synthetic BPE (ids inside Llama-3's 128,256,
    BOS 128000 / EOS 128001 as in Llama-3).  A real checkpoint brings its own
    vocabulary: ``Tokenizer.from_pretrained(<checkpoint dir>)`` reads its
    ``tokenizer.json``, takes BOS / EOS from ``tokenizer_config.json`` (token
    strings, resolved to ids) or ``config.json`` (ids), and the vocabulary size
    from ``config.json`` - the grammar tries and the native decoder tables are
    then built from that vocabulary, since every id they hold comes from
    ``encode``.  Parity against Meta's own Llama-3 tokenizer is unpinned (no
    tokenizer files offline); any byte-level BPE ``tokenizer.json`` loads."""

    def __init__(self, path: str = TOKENIZER_PATH, bos_id: Optional[int] = BOS_ID,
                 eos_id: Optional[int] = EOS_ID, vocab_size: int = LLAMA3_VOCAB,
                 synthetic: bool = True):
        from tokenizers import Tokenizer as HFTok
        if synthetic and not os.path.exists(path):
            train(path)
        self.path = path
        self._tok = HFTok.from_file(path)
        self.synthetic = synthetic
        # ids below learned_vocab are ordinary tokens; the synthetic BPE keeps
        # its learned ids below Llama-3's BOS, a real tokenizer's added
        # (special) tokens are dropped by decode instead
        self.learned_vocab = self._tok.get_vocab_size(with_added_tokens=not synthetic)
        self.vocab_size = vocab_size
        self.bos_id = bos_id
        self.eos_id = eos_id
        if synthetic:
            assert self.learned_vocab < BOS_ID
        elif self.learned_vocab > vocab_size:
            raise ValueError(f"tokenizer has {self.learned_vocab} tokens but the model "
                             f"vocabulary is {vocab_size}")

    @classmethod
    def from_pretrained(cls, model_dir: str) -> "Tokenizer":
        """The tokenizer of an HF checkpoint directory (``tokenizer.json``)."""
        from tokenizers import Tokenizer as HFTok
        d = os.path.abspath(model_dir)
        path = os.path.join(d, "tokenizer.json")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{model_dir}: no tokenizer.json")
        hf = HFTok.from_file(path)

        def load(name):
            f = os.path.join(d, name)
            if os.path.exists(f):
                with open(f) as fh:
                    return json.load(fh)
            return {}

        tcfg, mcfg = load("tokenizer_config.json"), load("config.json")

        def special(name):
            tok = tcfg.get(name)
            if isinstance(tok, dict):             # {"content": "<|begin_of_text|>", ...}
                tok = tok.get("content")
            if isinstance(tok, str):
                i = hf.token_to_id(tok)
                if i is None:
                    raise ValueError(f"{name} {tok!r} is not in {path}")
                return i
            i = mcfg.get(name + "_id")
            if isinstance(i, list):               # e.g. eos_token_id: [128001, 128009]
                i = i[0] if i else None
            return None if i is None else int(i)

        vocab = int(mcfg.get("vocab_size") or hf.get_vocab_size(with_added_tokens=True))
        return cls(path, bos_id=special("bos_token"), eos_id=special("eos_token"),
                   vocab_size=vocab, synthetic=False)

    # repeated texts only (registry prefixes, repeated intents): every unique
    # intent's suffix also passes through here, so a large cache is ~700 B per
    # request of dead entries (65,536 entries held ~50 MB in a serving
    # replica: the RSS growth of the round-6 950 s soak)
    @functools.lru_cache(maxsize=2048)
    def _encode_cached(self, text: str) -> tuple:
        return tuple(self._tok.encode(text, add_special_tokens=False).ids)

    def encode(self, text: str) -> List[int]:
        return list(self._encode_cached(text))

    def encode_batch(self, texts: List[str]) -> List[List[int]]:
        return [e.ids for e in self._tok.encode_batch(texts, add_special_tokens=False)]

    def decode(self, ids) -> str:
        if self.synthetic:
            ids = [i for i in ids if i < self.learned_vocab]
            return self._tok.decode(ids, skip_special_tokens=False)
        return self._tok.decode(list(ids), skip_special_tokens=True)

    def token_str(self, i: int) -> str:
        return self.decode([i])

    def prompt_ids(self, text: str) -> List[int]:
        """BOS (when the vocabulary has one) + the encoded text."""
        ids = self.encode(text)
        return ([self.bos_id] if self.bos_id is not None else []) + ids


@functools.lru_cache(maxsize=1)
def get_tokenizer() -> Tokenizer:
    return Tokenizer()


@functools.lru_cache(maxsize=8)
def tokenizer_for(model: Optional[str]) -> Tokenizer:
    """The checkpoint's own tokenizer when ``model`` is a directory holding a
    ``tokenizer.json`` (``MCP_MODEL=<dir>``); the synthetic BPE for a named
    random-init architecture (or a checkpoint without tokenizer files)."""
    if model and os.path.isdir(model) and os.path.exists(os.path.join(model, "tokenizer.json")):
        return Tokenizer.from_pretrained(model)
    return get_tokenizer()
