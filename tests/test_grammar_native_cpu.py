"""The native grammar decoder (csrc/runtime/grammar.cpp) against the Python
DagDecoder (planner/grammar.py): both are driven in lock-step with the same
random choices and must produce identical forced-token spans, allowed sets (in
the same order: the sampling kernel keys its draw by list position), done
flags and final text."""
import json
import random

import pytest

from mcp_amd.engine import native
from mcp_amd.orchestrator import validate_dag
from mcp_amd.planner.grammar import DagDecoder, GrammarSpec
from mcp_amd.planner.tokenizer import get_tokenizer
from mcp_amd.registry import make_service, synthetic_registry

pytestmark = pytest.mark.skipif(not native.available() or not hasattr(native._RT, "grammar_spec"),
                                reason="native runtime not built")


def lockstep(spec, rng):
    py_dec, c_dec = DagDecoder(spec), native._RT.DagDecoder(spec._native_for_test)
    a, b = py_dec.advance(), c_dec.advance()
    assert a == b
    n = 0
    while not py_dec.done:
        assert not c_dec.done
        al_py, al_c = py_dec.allowed(), c_dec.allowed()
        assert al_py == al_c and len(al_py) >= 2
        t = rng.choice(al_py)
        py_dec.feed(t)
        c_dec.feed(t)
        a, b = py_dec.advance(), c_dec.advance()
        assert a == b
        n += 1
    assert c_dec.done and c_dec.allowed() == []
    assert c_dec.text == py_dec.text
    assert c_dec.result() == py_dec.result()
    return py_dec.result(), n


def _spec(reg, **kw):
    spec = GrammarSpec(reg, get_tokenizer(), **kw)
    spec._native_for_test = native._RT.grammar_spec(spec.native_payload())
    return spec


@pytest.mark.parametrize("compact", [True, False])
@pytest.mark.parametrize("nsvc,max_nodes,min_nodes,retries",
                         [(1, 3, 1, True), (3, 6, 1, True), (10, 5, 5, True), (10, 6, 2, False),
                          (50, 8, 1, True), (200, 4, 4, True)])
def test_native_matches_python(nsvc, max_nodes, min_nodes, retries, compact):
    reg = synthetic_registry(nsvc, seed=nsvc)
    spec = _spec(reg, max_nodes=max_nodes, min_nodes=min_nodes, allow_retries=retries,
                 compact=compact)
    rng = random.Random(nsvc)
    names = [s["name"] for s in reg]
    for _ in range(30):
        dag, _ = lockstep(spec, rng)
        validate_dag(dag, names)


def test_native_payload_key_named_like_a_service():
    """An input key equal to a service name: the payload source of that key is
    also a node name (an edge when that service was chosen earlier), exactly as
    the Python program's string comparison has it."""
    reg = [make_service("alpha", {"q": "string"}, {"alpha_out": "string"}, fallback=""),
           make_service("beta", {"alpha": "string", "q": "string"}, {"r": "string"},
                        fallback="http://beta-b/api"),
           make_service("gamma", {"beta": "string", "alpha": "string"}, {"s": "string"}, fallback="")]
    spec = _spec(reg, max_nodes=3, min_nodes=3)
    rng = random.Random(3)
    for _ in range(50):
        lockstep(spec, rng)


def test_native_rejects_disallowed_token():
    spec = _spec(synthetic_registry(5, seed=2), max_nodes=3)
    dec = native._RT.DagDecoder(spec._native_for_test)
    dec.advance()
    bad = max(dec.allowed()) + 1
    while bad in dec.allowed():
        bad += 1
    with pytest.raises(ValueError):
        dec.feed(bad)


def test_spec_decoder_factory(monkeypatch):
    reg = synthetic_registry(4, seed=1)
    spec = GrammarSpec(reg, get_tokenizer(), max_nodes=2)
    d = spec.decoder()
    assert type(d).__name__ == "DagDecoder" and not isinstance(d, DagDecoder)   # native
    monkeypatch.setenv("MCP_NATIVE_GRAMMAR", "0")
    spec2 = GrammarSpec(reg, get_tokenizer(), max_nodes=2)
    assert isinstance(spec2.decoder(), DagDecoder)
    json.dumps(spec.native_payload()["chunks"])        # the payload is plain data (+ encode)


@pytest.mark.parametrize("corrupt", [
    lambda p: p["keys"][0]["pos"].append(0),                       # pos row longer than S
    lambda p: p["keys"][0]["pos"].__setitem__(0, 10 ** 4),         # pos entry past the trie
    lambda p: p["keys"][0]["alt_name"].pop(),                      # alt_name shorter than the trie
    lambda p: p["keys"][0]["alt_name"].__setitem__(0, 10 ** 4),    # alt_name names no service
    lambda p: p.__setitem__("cont_trie", (["a"], [[1]])),          # continue needs 2 alternatives
    lambda p: p["services"].pop(),                                 # fewer services than S
    lambda p: p.__setitem__("jnames", p["jnames"][:-1]),
    lambda p: p.__setitem__("min_nodes", 0),
    lambda p: p["services"][0].__setitem__("fallback", (["x"], [[5]])),  # 1-alternative fallback
])
def test_native_spec_rejects_malformed_payload(corrupt):
    """Malformed payloads raise ValueError at spec build time instead of
    indexing out of range later inside the decoder."""
    reg = [dict(s) for s in synthetic_registry(5, seed=2)]
    reg[1]["input_schema"] = {"type": "object", "properties": {"q": {"type": "string"}}}
    spec = GrammarSpec(reg, get_tokenizer(), max_nodes=3)
    p = spec.native_payload()
    assert p["keys"], "the registry must give at least one input key"
    native._RT.grammar_spec(p)                                     # the intact payload builds
    corrupt(p)
    with pytest.raises(ValueError):
        native._RT.grammar_spec(p)


def _take(dec, idx, toks):
    """Feed the tokens of alternative ``idx`` of the decoder's current choice."""
    ch = dec._choice
    while dec._choice is ch and not dec.done:
        dec.feed(next(t for t, c in dec._node.children.items() if (c.mask >> idx) & 1))
        toks += dec.advance()


def test_compact_view_emits_the_same_dag_in_fewer_tokens():
    """The compact model view (endpoints and fallback URLs filled from the
    registry, never fed to the model) and the full view emit identical DAGs
    for the same decisions; the compact token stream is shorter."""
    reg = synthetic_registry(10, seed=4)
    full = GrammarSpec(reg, get_tokenizer(), max_nodes=5, min_nodes=5, compact=False)
    comp = GrammarSpec(reg, get_tokenizer(), max_nodes=5, min_nodes=5, compact=True)
    rng = random.Random(5)
    saved = []
    for _ in range(30):
        decs = [DagDecoder(full), DagDecoder(comp)]
        toks = [d.advance() for d in decs]
        while not decs[0].done:
            assert not decs[1].done
            live = decs[0]._choice[2]
            assert live == decs[1]._choice[2]
            idx = rng.choice([i for i in range(live.bit_length()) if (live >> i) & 1])
            for d, tk in zip(decs, toks):
                _take(d, idx, tk)
        assert decs[1].done
        assert decs[0].result() == decs[1].result()
        saved.append(len(toks[0]) - len(toks[1]))
    assert min(saved) > 0


def test_native_spec_does_not_keep_its_grammar_spec_alive():
    """The native spec holds the tokenizer's encode, not a bound method of the
    Python spec: a reference back would be a cycle through C++ that the
    collector cannot see, leaking every retrieved candidate set's spec."""
    import gc
    import weakref
    spec = GrammarSpec(synthetic_registry(6, seed=3), get_tokenizer(), max_nodes=3)
    dec = spec.decoder()
    assert type(dec).__module__ != DagDecoder.__module__      # the native decoder
    ref = weakref.ref(spec)
    del spec, dec
    gc.collect()
    assert ref() is None
