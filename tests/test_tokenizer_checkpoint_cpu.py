"""A real checkpoint is served with its own tokenizer (MCP_MODEL=<dir>).

The checkpoint directory written here holds a tiny Llama (vocabulary 4096),
its ``config.json`` and a ``tokenizer.json`` trained on a different corpus than
the shipped synthetic BPE, so every token id differs from the synthetic ones.
``LocalPlanner.from_settings`` must pick that tokenizer up (BOS from
``tokenizer_config.json``), build the grammar from its vocabulary and emit
valid T2 plans.  Parity against Meta's own Llama-3 tokenizer stays unpinned:
no tokenizer files are available offline.
"""
import dataclasses
import json

import pytest

from mcp_amd.config import Settings
from mcp_amd.models.llama import get_config, random_weights
from mcp_amd.models.weights import save_llama_safetensors
from mcp_amd.orchestrator import validate_dag
from mcp_amd.planner.grammar import GrammarSpec
from mcp_amd.planner.local import LocalPlanner
from mcp_amd.planner.prompt import synthetic_intent
from mcp_amd.planner.tokenizer import Tokenizer, get_tokenizer, tokenizer_for
from mcp_amd.registry import MemoryRegistry, synthetic_registry

VOCAB = 4096


def _train_tokenizer(path):
    from tokenizers import Tokenizer as HFTok, decoders, models, pre_tokenizers, trainers
    tok = HFTok(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=True)
    tok.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(vocab_size=1500, min_frequency=1, show_progress=False,
                                  special_tokens=["<|begin_of_text|>", "<|end_of_text|>"],
                                  initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    corpus = ["a completely different corpus about invoices, parcels and weather reports " * 4,
              '{"nodes": [], "edges": []} service endpoint inputs outputs fallback retries'] * 50
    tok.train_from_iterator(corpus, trainer=trainer)
    tok.save(str(path))


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    d = tmp_path_factory.mktemp("ckpt")
    cfg = dataclasses.replace(get_config("tiny"), vocab_size=VOCAB)
    save_llama_safetensors(cfg, random_weights(cfg, "cpu", seed=4), d)
    _train_tokenizer(d / "tokenizer.json")
    (d / "tokenizer_config.json").write_text(json.dumps(
        {"bos_token": "<|begin_of_text|>", "eos_token": {"content": "<|end_of_text|>"}}))
    return d


def test_from_pretrained_reads_specials(ckpt):
    tok = tokenizer_for(str(ckpt))
    assert isinstance(tok, Tokenizer) and not tok.synthetic
    assert tok.bos_id == tok._tok.token_to_id("<|begin_of_text|>")
    assert tok.eos_id == tok._tok.token_to_id("<|end_of_text|>")
    assert tok.vocab_size == VOCAB
    text = 'Compose: {"nodes": [{"name": "svc-1"}], "edges": []} “quoted” ü'
    ids = tok.encode(text)
    assert max(ids) < VOCAB and tok.decode(ids) == text
    assert ids != get_tokenizer().encode(text)            # a different vocabulary
    assert tok.prompt_ids("x")[0] == tok.bos_id
    # named architectures keep the synthetic BPE
    assert tokenizer_for("llama3-8b") is get_tokenizer()


def test_planner_serves_checkpoint_tokenizer(ckpt):
    reg = MemoryRegistry(synthetic_registry(4, seed=2))
    s = Settings(model=str(ckpt), max_batch=4, max_step_tokens=512, kv_blocks=128,
                 temperature=0.0, max_nodes=3, embed_dim=64)
    planner = LocalPlanner.from_settings(s, reg)
    tok = planner.tok
    assert not tok.synthetic and tok.vocab_size == VOCAB
    names = [x.name for x in reg.list_services()]
    intents = [synthetic_intent(i) for i in range(3)]
    dags = planner.plan_many(intents)
    for d in dags:
        validate_dag(d, names)
    # the prompt starts with the checkpoint's BOS and every grammar token is
    # an id of its vocabulary
    services = reg.list_services()
    _, ptoks, stoks = planner.prepare(intents[0])
    assert ptoks[0] == tok.bos_id and max(ptoks + stoks) < VOCAB
    spec = GrammarSpec(services, tok, max_nodes=2)
    for alt in spec.jnames:
        ids = spec.encode(alt)
        assert max(ids) < VOCAB and tok.decode(ids) == alt      # decoded text round-trips


def test_vocab_larger_than_model_is_refused(tmp_path, ckpt):
    import shutil
    d = tmp_path / "bad"
    shutil.copytree(ckpt, d)
    cfg = json.loads((d / "config.json").read_text())
    cfg["vocab_size"] = 64                                   # smaller than the tokenizer
    (d / "config.json").write_text(json.dumps(cfg))
    with pytest.raises(ValueError):
        Tokenizer.from_pretrained(str(d))


def test_encode_cache_stays_small():
    """Every unique intent's suffix passes through the tokenizer's encode
    cache: a large bound held ~700 B per request of dead entries (~50 MB in a
    serving replica at 65,536 entries, the RSS growth of the round-6 soak)."""
    from mcp_amd.planner.tokenizer import get_tokenizer
    tok = get_tokenizer()
    for i in range(3000):
        tok.encode(f"\nUser intent: “book trip {i}”\n\nJSON DAG:")
    info = type(tok)._encode_cached.cache_info()
    assert info.maxsize <= 4096 and info.currsize <= 4096
