"""Fuzz script run inside the ASan/UBSan-instrumented runtime harness
(sanitize_main.cc).  Usage: harness sanitize_fuzz.py <engine/batch.py> [iters]

Drives every entry point of the native runtime through valid and invalid
inputs and checks the step packer against the Python reference
(``engine/batch.py:pack_step_py``).  torch is replaced by an empty module: the
packing code only needs numpy, and an uninstrumented torch inside an ASan
process adds minutes of start-up for no coverage.
"""
import importlib.util
import random
import sys
import types

import numpy as np

import _runtime_san as rt

sys.modules.setdefault("torch", types.ModuleType("torch"))
spec = importlib.util.spec_from_file_location("mcp_batch_ref", sys.argv[1])
batch = importlib.util.module_from_spec(spec)
sys.modules[spec.name] = batch          # dataclasses look the module up
spec.loader.exec_module(batch)
ITERS = int(sys.argv[2]) if len(sys.argv) > 2 else 200
BS = batch.BLOCK_SIZE
rng = random.Random(1234)


def expect(exc, fn, *a):
    try:
        fn(*a)
    except exc:
        return
    raise AssertionError(f"{fn.__name__}{a!r} did not raise {exc.__name__}")


# ---- block allocator: random traces, every error path
for trial in range(ITERS // 4 + 1):
    n = rng.randint(1, 96)
    a = rt.BlockAllocator(n)
    ref = [0] * n
    live = []
    for _ in range(300):
        op = rng.random()
        if op < 0.4:
            k = rng.randint(0, n + 2)
            if k > a.num_free:
                expect(RuntimeError, a.alloc, k)
                continue
            b = a.alloc(k)
            for x in b:
                assert ref[x] == 0
                ref[x] = 1
            live.append(b)
        elif op < 0.55 and live:
            b = rng.choice(live)
            a.incref(b)
            for x in b:
                ref[x] += 1
            live.append(list(b))
        elif op < 0.9 and live:
            b = live.pop(rng.randrange(len(live)))
            a.free(b)
            for x in b:
                ref[x] -= 1
        else:
            bad = rng.choice([-1, n, n + 7, -(1 << 30)])
            expect(IndexError, a.free, [bad])
            expect(IndexError, a.incref, [bad])
            expect(IndexError, a.refcount, bad)
        assert a.num_free == sum(1 for r in ref if r == 0)
    for b in live:
        a.free(b)
    assert a.num_free == n
    free_blk = rng.randrange(n)
    expect(RuntimeError, a.free, [free_blk])
    expect(RuntimeError, a.incref, [free_blk])
expect(ValueError, rt.BlockAllocator, 0)
expect(ValueError, rt.BlockAllocator(4).alloc, -1)


# ---- step packer vs the Python reference, including edge shapes
def random_step(cascade):
    entries, allowed, ctr, nblk = [], [], [], 0
    for s in range(rng.randint(1, 64)):
        start = rng.randint(0, 400)
        take = rng.choice([1, 1, 2, 3, 15, 16, 17, 63, 64, 65, 200])
        blocks = [nblk + i for i in range((start + take + BS - 1) // BS + rng.randint(0, 2))]
        nblk += len(blocks)
        toks = [rng.randrange(128256) for _ in range(take + rng.randint(0, 3))]
        sample = rng.random() < 0.6
        entries.append((toks, take, start, blocks, 128 if cascade and s < 5 else 0, sample))
        if sample:
            allowed.append([rng.randrange(128256) for _ in range(rng.randint(1, 40))])
            ctr.append(rng.randrange(1 << 31))
    copies = [(rng.randrange(4096), rng.randrange(4096)) for _ in range(rng.randint(0, 5))]
    pre = list(range(rng.randint(1, 4))) if cascade else None
    pre_tokens = sum(e[1] for e in entries[:5]) if cascade else 0
    return entries, copies, pre, pre_tokens, (allowed or None), (ctr or None)


for it in range(ITERS):
    for group in (1, 2, 4, 8):
        args = random_step(cascade=it % 2 == 1)
        h_n, l_n = rt.pack_step(args[0], BS, group, *args[1:])
        h_p, l_p = batch.pack_step_py(args[0], BS, group, *args[1:])
        assert list(l_n) == list(l_p), (l_n, l_p)
        np.testing.assert_array_equal(h_n, h_p)

h, l = rt.pack_step([], BS, 4, [(1, 2)])            # copy-only step
assert int(sum(l)) == h.size
expect(ValueError, rt.pack_step, [([1, 2], 3, 0, [0], 0, False)], BS, 4)          # take > len(tokens)
expect(ValueError, rt.pack_step, [([1, 2], 0, 0, [0], 0, False)], BS, 4)          # empty span
expect(ValueError, rt.pack_step, [([1] * 70, 70, 0, [0], 0, False)], BS, 4)       # too few blocks
expect(ValueError, rt.pack_step, [([1], 1, 0, [0], 0, True)], BS, 4, None, None, 0, [], [])
expect(ValueError, rt.pack_step, [([1], 1, 0, [0], 0, True)], BS, 4, None, None, 0, [[1]], [])

# ---- topological generations: random DAGs vs a plain Kahn, cycles, bad ids
for _ in range(ITERS):
    n = rng.randint(0, 40)
    perm = list(range(n))
    rng.shuffle(perm)
    edges = [(perm[i], perm[j]) for i in range(n) for j in range(i + 1, n) if rng.random() < 0.15]
    rng.shuffle(edges)
    gens = rt.topo_generations(n, edges)
    indeg = [0] * n
    succ = [[] for _ in range(n)]
    for u, v in edges:
        succ[u].append(v)
        indeg[v] += 1
    cur, want = [v for v in range(n) if indeg[v] == 0], []
    while cur:
        want.append(cur)
        nxt = []
        for u in cur:
            for v in succ[u]:
                indeg[v] -= 1
                if indeg[v] == 0:
                    nxt.append(v)
        cur = nxt
    assert [list(g) for g in gens] == want
    if n >= 2 and edges:
        u, v = edges[0]
        expect(RuntimeError, rt.topo_generations, n, edges + [(v, u)])
    expect(IndexError, rt.topo_generations, max(n, 1), [(0, max(n, 1))])
    expect(IndexError, rt.topo_generations, max(n, 1), [(-1, 0)])

# ---- native grammar decoder (grammar.cpp) in lock-step with planner/grammar.py,
# char-level token ids (JSON-quoted alternatives stay prefix-free)
import json  # noqa: E402
import os  # noqa: E402

gspec = importlib.util.spec_from_file_location(
    "mcp_grammar_ref", os.path.join(os.path.dirname(sys.argv[1]), "..", "planner", "grammar.py"))
grammar = importlib.util.module_from_spec(gspec)
gspec.loader.exec_module(grammar)


class CharTok:
    @staticmethod
    def encode(text):
        return [ord(c) for c in text]


for it in range(max(1, ITERS // 4)):
    S = rng.randint(1, 12)
    keys_pool = [f"k{i}" for i in range(6)] + ["svc0", "svc1"]
    services = []
    for i in range(S):
        ks = rng.sample(keys_pool, rng.randint(0, 4))
        services.append({"name": f"svc{i}", "endpoint": f"http://svc{i}/api",
                         "input_schema": {"type": "object", "properties": {k: {"type": "string"} for k in ks}},
                         "fallback": f"http://fb{i}/api" if rng.random() < 0.5 else None})
    mx = rng.randint(1, 6)
    spec = grammar.GrammarSpec(services, CharTok(), max_nodes=mx, min_nodes=rng.randint(1, mx),
                               allow_retries=rng.random() < 0.7)
    nspec = rt.grammar_spec(spec.native_payload())
    for _ in range(4):
        a, b = grammar.DagDecoder(spec), rt.DagDecoder(nspec)
        assert a.advance() == b.advance()
        while not a.done:
            al = a.allowed()
            assert al == b.allowed()
            if rng.random() < 0.1:
                expect(ValueError, b.feed, max(al) + 1000)
            t = rng.choice(al)
            a.feed(t)
            b.feed(t)
            assert a.advance() == b.advance()
        assert b.done and b.text == a.text
        json.loads(b.text)
        expect(ValueError, b.feed, 34)
bad = spec.native_payload()
bad["name_trie"] = (["a", "ab"], [[1], [1, 2]])                 # not prefix-free
expect(ValueError, rt.grammar_spec, bad)
bad = spec.native_payload()
bad["services"][0]["keys"] = [10 ** 6]                           # key id out of range
expect(ValueError, rt.grammar_spec, bad)
bad = spec.native_payload()
bad["keys"] and bad["keys"][0]["pos"].append(0)                # pos row longer than S
bad["keys"] and expect(ValueError, rt.grammar_spec, bad)
bad = spec.native_payload()
bad["cont_trie"] = (["a"], [[1]])                              # cont needs 2 alternatives
expect(ValueError, rt.grammar_spec, bad)

# ---- feature-hashing embedder (embed.cpp): random ASCII, empty texts, odd dims
alphabet = "abcXYZ019 _-#.,{}\"\t"
for _ in range(ITERS):
    texts = ["".join(rng.choice(alphabet) for _ in range(rng.randint(0, 80)))
             for _ in range(rng.randint(0, 6))]
    dim = rng.randint(1, 70)
    out = rt.hash_embed_sums(texts, dim)
    assert out.shape == (len(texts), dim) and np.isfinite(out).all()
    for t, row in zip(texts, out):
        if not any(c.isalnum() for c in t):
            assert not row.any()
expect(ValueError, rt.hash_embed_sums, ["x"], 0)

print(f"sanitize_fuzz OK ({ITERS} iterations)")
