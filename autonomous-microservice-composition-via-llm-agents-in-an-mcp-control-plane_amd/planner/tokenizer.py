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
from typing import List

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
    def __init__(self, path: str = TOKENIZER_PATH):
        from tokenizers import Tokenizer as HFTok
        if not os.path.exists(path):
            train(path)
        self._tok = HFTok.from_file(path)
        self.learned_vocab = self._tok.get_vocab_size()
        self.vocab_size = LLAMA3_VOCAB
        self.bos_id = BOS_ID
        self.eos_id = EOS_ID
        assert self.learned_vocab < BOS_ID

    @functools.lru_cache(maxsize=65536)
    def _encode_cached(self, text: str) -> tuple:
        return tuple(self._tok.encode(text, add_special_tokens=False).ids)

    def encode(self, text: str) -> List[int]:
        return list(self._encode_cached(text))

    def encode_batch(self, texts: List[str]) -> List[List[int]]:
        return [e.ids for e in self._tok.encode_batch(texts, add_special_tokens=False)]

    def decode(self, ids) -> str:
        ids = [i for i in ids if i < self.learned_vocab]
        return self._tok.decode(ids, skip_special_tokens=False)

    def token_str(self, i: int) -> str:
        return self.decode([i])


@functools.lru_cache(maxsize=1)
def get_tokenizer() -> Tokenizer:
    return Tokenizer()
