"""DAG-JSON grammar -> token constraints.

A random-init (or any) model's unconstrained output would rarely parse (the
reference returns HTTP 500 on non-JSON, control_plane.py:74).  The
planner therefore decodes under a grammar that can only produce a T2 DAG over
registry services:

    {"nodes":[{"name":"<svc>","endpoint":"<its endpoint>",
               "inputs":{"<key>":"<payload field | earlier node>",...},
               "retries":<0-3>}, ...],
     "edges":[{"from":"<src>","to":"<dst>"[,"fallback":"<registry fallback>"]}, ...]}

The model decides: which service comes next (or stop), the source of every
input field, the retry count and whether each edge carries a fallback.  Every
other character is forced.  Edges are derived from the chosen input sources
(producer -> consumer), so the graph is acyclic and names are unique by
construction.

Compact model view (``MCP_PLAN_COMPACT=1``, the default): fields that are a
function of earlier choices - a node's endpoint (its name's registry record)
and an edge's fallback URL (the target's registry fallback) - are written to
the output text by the decoder but never enter the model's token stream; the
model sees ``{"name":"svc","inputs":{...`` and ``"fallback":true``.  Edges follow
from the chosen input sources, so the model sees only those it decides on
(``{"to":"<dst>"`` before a fallback choice).  The DAG is the same T2 JSON;
the model's context holds the same information (names determine the URLs,
inputs determine the edges) in fewer tokens, each of which would otherwise
run through every layer.  The reference's own prompt never asks its LLM for
endpoints either (control_plane.py:61-62: service_name, input_keys,
next_steps, fallback) although its executor reads them (:107).

Decoding mechanics: a *choice* is a prefix-free set of alternative strings;
each alternative is tokenised standalone and the choice becomes a token trie.
At a trie node with one child the token is forced (no sampling); with several
children the engine samples from exactly those children (``allowed``).  Forced
text after a decision is appended as a jump-forward span: its tokens still run
through the model (their KV is needed) but in a single batched forward.
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional, Sequence, Tuple

RETRY_CHOICES = ["0", "1", "2", "3"]
COMPACT = os.environ.get("MCP_PLAN_COMPACT", "1") == "1"
INPUTS_OPEN = ',"inputs":{'
FALLBACK_MARK = ',"fallback":true}'


class Trie:
    __slots__ = ("children", "leaf", "mask")

    def __init__(self):
        self.children: Dict[int, "Trie"] = {}
        self.leaf: int = -1        # alternative index ending here
        self.mask: int = 0         # bitmask of alternatives below


def build_trie(token_seqs: Sequence[Sequence[int]]) -> Trie:
    """Prefix-freeness is checked on insertion: an earlier alternative that is
    a prefix of this one is a leaf on its path, one that this one prefixes
    gives its end node children."""
    root = Trie()
    for i, seq in enumerate(token_seqs):
        if not seq:
            raise ValueError("empty alternative")
        node = root
        bit = 1 << i
        node.mask |= bit
        for t in seq:
            if node.leaf >= 0:
                raise ValueError("alternatives are not prefix-free")
            nxt = node.children.get(t)
            if nxt is None:
                nxt = node.children[t] = Trie()
            node = nxt
            node.mask |= bit
        if node.leaf >= 0 or node.children:
            raise ValueError("alternatives are not prefix-free")
        node.leaf = i
    return root


class GrammarSpec:
    """Per-plan constants: candidate services, their token tries, caches."""

    def __init__(self, services: Sequence[dict], tokenizer, max_nodes: int = 6,
                 allow_retries: bool = True, min_nodes: int = 1, compact: Optional[bool] = None):
        self.services = list(services)
        self.tok = tokenizer
        # compact model view: endpoints / fallback URLs written to the output only
        self.compact = COMPACT if compact is None else bool(compact)
        self.max_nodes = max(1, max_nodes)
        # the model decides when to stop only between min_nodes and max_nodes
        # (a fixed-size plan gives the benchmark a model-independent token count)
        self.min_nodes = max(1, min(min_nodes, self.max_nodes, len(self.services)))
        self.allow_retries = allow_retries
        self.names = [s["name"] for s in self.services]
        self.keys = [self._input_keys(s) for s in self.services]
        self._trie_cache: Dict[Tuple[str, ...], Trie] = {}
        self._enc_cache: Dict[str, List[int]] = {}      # forced spans repeat across requests
        self._chain_cache: Dict[tuple, tuple] = {}       # (trie node, live mask) -> forced walk
        self._kids_cache: Dict[tuple, List[int]] = {}    # (trie node, live mask) -> allowed tokens
        self.jnames = tuple(json.dumps(n) for n in self.names)
        # input sources of key k: the payload key itself, then any earlier node.
        # ONE trie per key over every candidate; the live mask selects the key
        # plus the nodes chosen so far (a trie restricted by a mask is the trie
        # of the live alternatives, so the allowed tokens are the same)
        self._src_cache: Dict[str, tuple] = {}

    @staticmethod
    def _input_keys(s) -> List[str]:
        sch = s.get("input_schema") or {}
        if isinstance(sch.get("properties"), dict):
            return list(sch["properties"].keys())
        return [k for k in sch.keys() if k not in ("type", "required", "$schema", "title")]

    def encode(self, text: str) -> List[int]:
        t = self._enc_cache.get(text)
        if t is None:
            t = self.tok.encode(text)
            if len(self._enc_cache) < 65536:
                self._enc_cache[text] = t
        return list(t)

    def live_children(self, node: Trie, live: int) -> List[int]:
        """Allowed next tokens at ``node`` under the live mask (memoised)."""
        key = (id(node), live)
        r = self._kids_cache.get(key)
        if r is None:
            r = [t for t, c in node.children.items() if c.mask & live]
            if len(self._kids_cache) < (1 << 18):
                self._kids_cache[key] = r
        return r

    def forced_chain(self, node: Trie, live: int):
        """Tokens forced from ``node`` under the live-alternative mask: the walk
        while exactly one live child remains, stopping at a leaf (a resolved
        choice).  Memoised per (node, mask) - the same walks repeat across
        requests, and the per-token Python walk was most of the engine's
        per-step host update."""
        key = (id(node), live)
        r = self._chain_cache.get(key)
        if r is None:
            toks, n = [], node
            while n.leaf < 0:
                kids = [t for t, c in n.children.items() if c.mask & live]
                if len(kids) != 1:
                    break
                toks.append(kids[0])
                n = n.children[kids[0]]
            r = (tuple(toks), n)
            if len(self._chain_cache) < (1 << 18):
                self._chain_cache[key] = r
        return r

    @property
    def name_trie(self) -> Trie:
        return self.trie(self.jnames)

    def sources(self, key: str):
        """(source names, their JSON alternatives, name -> position) for input
        ``key``; the Python decoder's trie of the alternatives is
        ``trie(alts)`` (built on first use: the native decoder never needs
        it, and the tries were most of a retrieved request's host time)."""
        r = self._src_cache.get(key)
        if r is None:
            srcs = (key,) + tuple(n for n in self.names if n != key)
            alts = (json.dumps(key),) + tuple(j for n, j in zip(self.names, self.jnames) if n != key)
            r = (srcs, alts, {x: i for i, x in enumerate(srcs)})
            self._src_cache[key] = r
        return r

    def endpoint_chunk(self, svc) -> Tuple[str, str]:
        """(output text, model text) of the forced span after a node's name."""
        text = ',"endpoint":' + json.dumps(svc["endpoint"]) + INPUTS_OPEN
        return text, (INPUTS_OPEN if self.compact else text)

    def edge_chunk(self, first: bool, src: str, dst_idx: int) -> Tuple[str, str]:
        """(output text, model text) of an edge's opening.  Edges follow from
        the input sources already chosen; in the compact view the model sees
        only the edges it decides on (a target with a registry fallback), as
        ``{"to":"<dst>"`` before the fallback choice, and nothing otherwise."""
        dst = self.names[dst_idx]
        out = ("" if first else ",") + '{"from":' + json.dumps(src) + ',"to":' + json.dumps(dst)
        if not self.compact:
            return out, out
        return out, ('{"to":' + json.dumps(dst) if self.services[dst_idx].get("fallback") else "")

    def fallback_alts(self, fb: str) -> Tuple[Tuple[str, ...], Tuple[str, ...]]:
        """(output alternatives, model alternatives) of an edge's fallback choice."""
        out = (',"fallback":' + json.dumps(fb) + "}", "}")
        return out, ((FALLBACK_MARK, "}") if self.compact else out)

    def trie(self, alts: Tuple[str, ...]) -> Trie:
        t = self._trie_cache.get(alts)
        if t is None:
            t = build_trie([self.tok.encode(a) for a in alts])
            self._trie_cache[alts] = t
        return t

    # ------------------------------------------------------------ native
    _native = None          # engine._runtime GrammarSpec, False when unavailable

    def decoder(self):
        """A fresh per-request decoder: the C++ state machine
        (csrc/runtime/grammar.cpp, same tokens / allowed sets / text) when the
        native runtime is built, else ``DagDecoder``.  MCP_NATIVE_GRAMMAR=0
        forces the Python one."""
        if self._native is None:
            self._native = False
            if os.environ.get("MCP_NATIVE_GRAMMAR", "1") != "0":
                from ..engine import native
                if native.available() and hasattr(native._RT, "grammar_spec") \
                        and len(self.names) < 256:
                    self._native = native._RT.grammar_spec(self.native_payload())
        if self._native is not False:
            from ..engine import native
            return native._RT.DagDecoder(self._native)
        return DagDecoder(self)

    def native_payload(self) -> dict:
        """Every forced chunk and choice of the program, tokenised here (the
        Python tokenizer stays the single source of token ids)."""
        def chunk(text):
            return (text, self.encode(text))

        def alts(a):
            return (list(a), [self.tok.encode(x) for x in a])

        names = self.names
        name_idx = {}
        for i, n in enumerate(names):
            name_idx.setdefault(n, i)
        key_ids: Dict[str, int] = {}
        keys = []
        for ks in self.keys:
            for k in ks:
                if k not in key_ids:
                    key_ids[k] = len(keys)
                    srcs, a_s, pos = self.sources(k)
                    keys.append({
                        "first": chunk(json.dumps(k) + ":"),
                        "rest": chunk("," + json.dumps(k) + ":"),
                        "alt0": chunk(a_s[0]),
                        "trie": alts(a_s),
                        "pos": [-1 if n == k else pos[n] for n in names],
                        "alt_name": [name_idx.get(x, -1) for x in srcs],
                    })
        services = []
        for svc, ks in zip(self.services, self.keys):
            fb = svc.get("fallback")
            ep_out, ep_model = self.endpoint_chunk(svc)
            if fb:
                fb_out, fb_model = self.fallback_alts(fb)
                fallback = (list(fb_out), [list(self.tok.encode(x)) for x in fb_model])
            else:
                fallback = None
            services.append({
                "endpoint": (ep_out, self.encode(ep_model)),    # text out, tokens in
                "keys": [key_ids[k] for k in ks],
                "fallback": fallback,
            })
        return {
            "S": len(names), "max_nodes": self.max_nodes, "min_nodes": self.min_nodes,
            "allow_retries": bool(self.allow_retries), "jnames": list(self.jnames),
            "name_trie": alts(self.jnames), "retry_trie": alts(tuple(RETRY_CHOICES)),
            "cont_trie": alts((',{"name":', '],"edges":[')),
            "chunks": {"start": chunk('{"nodes":[{"name":'), "retries": chunk('},"retries":'),
                       "close1": chunk("}"), "close2": chunk("}}"), "next": chunk(',{"name":'),
                       "edges": chunk('],"edges":['), "end": chunk("]}"),
                       # closes an edge without a fallback choice: silent in the compact view
                       "close_edge": ("}", [] if self.compact else self.encode("}"))},
            # the tokenizer's own encode, not a bound method of this spec: the
            # native spec keeps it, and a reference back to the spec would be a
            # cycle through C++ that the garbage collector cannot see (a leak per
            # retrieved candidate set)
            "services": services, "keys": keys, "encode": self.tok.encode,
            "compact": self.compact,
        }


class DagDecoder:
    """Per-request grammar state machine.

    Protocol with the engine::

        toks = dec.advance()      # forced tokens to append (may be empty)
        if dec.done: ...
        allowed = dec.allowed()   # >=2 token ids: sample one
        dec.feed(token)           # then advance() again
    """

    def __init__(self, spec: GrammarSpec):
        self.spec = spec
        self.text_parts: List[str] = []
        self.done = False
        self._gen = self._program()
        self._choice: Optional[Tuple[Tuple[str, ...], Trie, int]] = None   # (alts, node, live mask)
        self._node: Optional[Trie] = None
        self._pending_tokens: List[int] = []
        self._result_index: Optional[int] = None
        self._step_gen(None)

    # ------------------------------------------------------------- program
    def _program(self):
        sp = self.spec
        yield ('{"nodes":[{"name":', None)
        used_mask = 0
        chosen: List[int] = []
        node_inputs: List[Dict[str, str]] = []
        while True:
            live = ((1 << len(sp.names)) - 1) & ~used_mask
            idx = yield (None, (sp.jnames, sp.name_trie, live))
            used_mask |= 1 << idx
            yield (sp.endpoint_chunk(sp.services[idx]), None)
            inputs = {}
            prev_names = [sp.names[j] for j in chosen]
            for ki, key in enumerate(sp.keys[idx]):
                yield (("," if ki else "") + json.dumps(key) + ":", None)
                srcs, alts_s, pos = sp.sources(key)
                live_s = 1
                for n in prev_names:
                    if n != key:
                        live_s |= 1 << pos[n]
                if live_s == 1:
                    yield (alts_s[0], None)
                    inputs[key] = srcs[0]
                else:
                    si = yield (None, (alts_s, sp.trie(alts_s), live_s))
                    inputs[key] = srcs[si]
            if sp.allow_retries:
                yield ('},"retries":', None)
                alts_r = tuple(RETRY_CHOICES)
                yield (None, (alts_r, sp.trie(alts_r), (1 << len(alts_r)) - 1))
                yield ("}", None)
            else:
                yield ("}}", None)
            chosen.append(idx)
            node_inputs.append(inputs)
            can_more = len(chosen) < sp.max_nodes and used_mask != (1 << len(sp.names)) - 1
            if not can_more:
                break
            if len(chosen) < sp.min_nodes:
                yield (',{"name":', None)
                continue
            alts_c = (',{"name":', '],"edges":[')
            ci = yield (None, (alts_c, sp.trie(alts_c), 3))
            if ci == 1:
                break
        if not (len(chosen) < sp.max_nodes and used_mask != (1 << len(sp.names)) - 1):
            yield ('],"edges":[', None)
        # edges: producer -> consumer for every node-valued input source
        first = True
        for j, idx in enumerate(chosen):
            dst = sp.names[idx]
            srcs = []
            for v in node_inputs[j].values():
                if v in sp.names and v != dst and v not in srcs and \
                        sp.names.index(v) in chosen[:j]:
                    srcs.append(v)
            for src in srcs:
                yield (sp.edge_chunk(first, src, idx), None)
                first = False
                fb = sp.services[idx].get("fallback")
                if fb:
                    alts_f, model_f = sp.fallback_alts(fb)
                    yield (None, (alts_f, sp.trie(model_f), 3))
                else:
                    yield (("}", "" if sp.compact else "}"), None)
        yield ("]}", None)

    def _step_gen(self, send):
        """Run the program until the next choice (or the end), collecting forced text."""
        try:
            item = self._gen.send(send) if send is not None or self._gen.gi_frame.f_lasti >= 0 \
                else next(self._gen)
        except StopIteration:
            self.done = True
            self._choice = None
            return
        while True:
            text, choice = item
            if text is not None:
                # (output text, model text) when they differ (compact view)
                out, model = text if isinstance(text, tuple) else (text, text)
                self.text_parts.append(out)
                if model:
                    self._pending_tokens += self.spec.encode(model)
                try:
                    item = next(self._gen)
                except StopIteration:
                    self.done = True
                    self._choice = None
                    return
                continue
            alts, trie, live = choice
            self._choice = (alts, trie, live)
            self._node = trie
            return

    # ------------------------------------------------------------ protocol
    def _live_children(self):
        return self.spec.live_children(self._node, self._choice[2])

    def advance(self) -> List[int]:
        """Return forced tokens (jump-forward), resolving single-child trie steps."""
        while not self.done and self._choice is not None:
            toks, end = self.spec.forced_chain(self._node, self._choice[2])
            if not toks:
                break
            self._pending_tokens += toks
            self._node = end
            if end.leaf >= 0:
                self._resolve()
        out, self._pending_tokens = self._pending_tokens, []
        return out

    def allowed(self) -> List[int]:
        return self._live_children()

    def feed(self, token: int) -> None:
        if token not in self._node.children or not (self._node.children[token].mask & self._choice[2]):
            raise ValueError(f"token {token} not allowed by the grammar")
        self._take(token)

    def _take(self, token: int):
        self._pending_tokens.append(token)
        self._node = self._node.children[token]
        if self._node.leaf >= 0:
            self._resolve()

    def _resolve(self):
        """The walk reached a leaf: the choice is made, run the program on."""
        idx = self._node.leaf
        self.text_parts.append(self._choice[0][idx])
        self._choice = None
        self._step_gen(idx)

    # -------------------------------------------------------------- result
    @property
    def text(self) -> str:
        return "".join(self.text_parts)

    def result(self) -> dict:
        return json.loads(self.text)
