// Native DAG-JSON grammar decoder: the per-request state machine of
// planner/grammar.py (DagDecoder) in C++, for the engine's per-step host path
// (feed the sampled token, jump-forward the forced chain, list the allowed
// tokens of the next choice for ~256 requests between two GPU steps).
//
// The Python GrammarSpec stays the source of truth: it tokenises every forced
// text chunk and every choice alternative and hands them over once per spec
// (NativeSpec).  Edge chunks ('{"from":"a","to":"b"') depend on a (src, dst)
// pair, so they are encoded lazily through the spec's Python encode callback
// and cached here.  Tries are flattened; children keep insertion order, so
// allowed() lists tokens in the same order as the Python decoder (the sampling
// kernel's Gumbel draw is keyed by position in that list).  The program is the
// generator DagDecoder._program written as an explicit program counter; the
// emitted token stream, allowed sets and text are identical
// (tests/test_grammar_native_cpu.py runs both in lock-step).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <array>
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

namespace py = pybind11;

namespace {

constexpr int MAXA = 256;                     // alternatives per choice (bitset width)

struct Mask {
  std::array<uint64_t, MAXA / 64> w{};
  void set(int i) { w[i >> 6] |= 1ull << (i & 63); }
  bool test(int i) const { return (w[i >> 6] >> (i & 63)) & 1; }
  bool any_and(const Mask& o) const {
    for (size_t k = 0; k < w.size(); ++k)
      if (w[k] & o.w[k]) return true;
    return false;
  }
  bool operator==(const Mask& o) const { return w == o.w; }
};

struct Trie {
  struct Node {
    int leaf = -1;
    Mask mask;
    std::vector<std::pair<int, int>> kids;    // (token, child), insertion order
  };
  std::vector<Node> nodes;
  std::vector<std::string> alts;              // alternative texts

  Trie(const std::vector<std::vector<int>>& seqs, std::vector<std::string> texts)
      : alts(std::move(texts)) {
    if ((int)seqs.size() > MAXA) throw std::invalid_argument("too many alternatives");
    nodes.emplace_back();
    for (int i = 0; i < (int)seqs.size(); ++i) {
      if (seqs[i].empty()) throw std::invalid_argument("empty alternative");
      int n = 0;
      nodes[0].mask.set(i);
      for (int t : seqs[i]) {
        int c = -1;
        for (auto& kv : nodes[n].kids)
          if (kv.first == t) c = kv.second;
        if (c < 0) {
          c = (int)nodes.size();
          nodes[n].kids.emplace_back(t, c);
          nodes.emplace_back();
        }
        n = c;
        nodes[n].mask.set(i);
      }
      if (nodes[n].leaf >= 0 || !nodes[n].kids.empty())
        throw std::invalid_argument("alternatives are not prefix-free");
      nodes[n].leaf = i;
    }
    for (auto& nd : nodes)
      if (nd.leaf >= 0 && !nd.kids.empty()) throw std::invalid_argument("alternatives are not prefix-free");
  }
};

struct Chunk {
  std::string text;
  std::vector<int> toks;
};

Chunk chunk_of(const py::tuple& t) { return {t[0].cast<std::string>(), t[1].cast<std::vector<int>>()}; }

Trie trie_of(const py::tuple& t) {
  return Trie(t[1].cast<std::vector<std::vector<int>>>(), t[0].cast<std::vector<std::string>>());
}

// Per-plan constants (planner/grammar.py GrammarSpec), built once per spec.
struct NativeSpec {
  int S = 0, max_nodes = 1, min_nodes = 1;
  bool allow_retries = true;
  std::vector<std::string> jnames;
  std::unique_ptr<Trie> name_trie, retry_trie, cont_trie;
  Chunk c_start, c_retries, c_close1, c_close2, c_next, c_edges, c_close_edge, c_end;
  std::vector<Chunk> endpoint;                // per service
  std::vector<std::vector<int>> keys;         // per service: key ids
  std::vector<std::unique_ptr<Trie>> fb_trie; // per service (null: no fallback)
  // per key
  std::vector<Chunk> key_first, key_rest, src_alt0;
  std::vector<std::unique_ptr<Trie>> src_trie;
  std::vector<std::vector<int>> pos;          // [key][service] -> alternative or -1
  std::vector<std::vector<int>> alt_name;     // [key][alt] -> service index of that source or -1
  py::object encode;                          // str -> list[int] (edge chunks)
  bool compact = false;                       // compact model view (planner/grammar.py)
  std::map<std::tuple<int, int, int>, Chunk> edge_cache;

  // an edge's opening: the output text, and the model's tokens - in the
  // compact view only edges to a service with a fallback choice, as
  // {"to":"<dst>" (GrammarSpec.edge_chunk)
  const Chunk& edge(bool first, int src, int dst) {
    auto key = std::make_tuple((int)first, src, dst);
    auto it = edge_cache.find(key);
    if (it != edge_cache.end()) return it->second;
    Chunk c;
    c.text = std::string(first ? "" : ",") + "{\"from\":" + jnames[src] + ",\"to\":" + jnames[dst];
    const std::string model = !compact ? c.text : fb_trie[dst] ? "{\"to\":" + jnames[dst] : "";
    if (!model.empty()) c.toks = encode(model).cast<std::vector<int>>();
    return edge_cache.emplace(key, std::move(c)).first->second;
  }
};

enum Pc {
  PC_START, PC_NAME, PC_AFTER_NAME, PC_KEY, PC_AFTER_SRC, PC_NODE_TAIL, PC_AFTER_RETRY,
  PC_NODE_END, PC_AFTER_CONT, PC_BREAK, PC_EDGE_NODE, PC_EDGE_SRC, PC_AFTER_FB, PC_END, PC_DONE
};

class NativeDecoder {
 public:
  explicit NativeDecoder(std::shared_ptr<NativeSpec> sp) : sp_(std::move(sp)) {
    used_.assign(sp_->S, 0);
    run(-1);
  }

  bool done() const { return done_; }
  const std::string& text() const { return text_; }

  // jump-forward: walk while exactly one live child remains (a forced token),
  // resolving choices whose walk reaches a leaf (GrammarSpec.forced_chain)
  std::vector<int> advance() {
    while (!done_ && trie_) {
      int n = node_;
      bool moved = false;
      while (trie_->nodes[n].leaf < 0) {
        int cnt = 0, tok = -1, child = -1;
        for (auto& kv : trie_->nodes[n].kids)
          if (trie_->nodes[kv.second].mask.any_and(live_)) {
            if (++cnt > 1) break;
            tok = kv.first;
            child = kv.second;
          }
        if (cnt != 1) break;
        pending_.push_back(tok);
        n = child;
        moved = true;
      }
      if (!moved) break;
      node_ = n;
      if (trie_->nodes[n].leaf >= 0) resolve();
    }
    std::vector<int> out;
    out.swap(pending_);
    return out;
  }

  std::vector<int> allowed() const {
    std::vector<int> r;
    if (!trie_) return r;
    for (auto& kv : trie_->nodes[node_].kids)
      if (trie_->nodes[kv.second].mask.any_and(live_)) r.push_back(kv.first);
    return r;
  }

  void feed(int token) {
    if (!trie_) throw py::value_error("token " + std::to_string(token) + " not allowed by the grammar");
    for (auto& kv : trie_->nodes[node_].kids)
      if (kv.first == token && trie_->nodes[kv.second].mask.any_and(live_)) {
        pending_.push_back(token);
        node_ = kv.second;
        if (trie_->nodes[node_].leaf >= 0) resolve();
        return;
      }
    throw py::value_error("token " + std::to_string(token) + " not allowed by the grammar");
  }

 private:
  std::shared_ptr<NativeSpec> sp_;
  std::vector<int> pending_;
  std::string text_;
  bool done_ = false;
  // current choice
  const Trie* trie_ = nullptr;
  int node_ = 0;
  Mask live_;
  // program state
  Pc pc_ = PC_START;
  std::vector<char> used_;
  int n_used_ = 0;
  std::vector<int> chosen_;
  std::vector<std::vector<int>> node_inputs_;   // per chosen node: source service per key (-1 payload)
  std::vector<int> inputs_;
  int cur_ = 0, ki_ = 0, key_ = 0, j_ = 0, si_ = 0;
  bool first_ = true;
  std::vector<int> srcs_;

  void emit(const Chunk& c) {
    text_ += c.text;
    pending_.insert(pending_.end(), c.toks.begin(), c.toks.end());
  }

  void choose(const Trie* t, const Mask& live, Pc next) {
    trie_ = t;
    live_ = live;
    node_ = 0;
    pc_ = next;
  }

  void resolve() {
    const int idx = trie_->nodes[node_].leaf;
    text_ += trie_->alts[idx];
    trie_ = nullptr;
    run(idx);
  }

  bool can_more() const { return (int)chosen_.size() < sp_->max_nodes && n_used_ != sp_->S; }

  void run(int choice) {
    NativeSpec& sp = *sp_;
    while (true) {
      switch (pc_) {
        case PC_START:
          emit(sp.c_start);
          pc_ = PC_NAME;
          break;
        case PC_NAME: {
          Mask live;
          for (int i = 0; i < sp.S; ++i)
            if (!used_[i]) live.set(i);
          choose(sp.name_trie.get(), live, PC_AFTER_NAME);
          return;
        }
        case PC_AFTER_NAME:
          cur_ = choice;
          used_[cur_] = 1;
          ++n_used_;
          emit(sp.endpoint[cur_]);
          ki_ = 0;
          inputs_.clear();
          pc_ = PC_KEY;
          break;
        case PC_KEY: {
          if (ki_ == (int)sp.keys[cur_].size()) {
            pc_ = PC_NODE_TAIL;
            break;
          }
          key_ = sp.keys[cur_][ki_];
          emit(ki_ ? sp.key_rest[key_] : sp.key_first[key_]);
          Mask live, only0;
          live.set(0);
          only0.set(0);
          for (int n : chosen_)
            if (sp.pos[key_][n] >= 0) live.set(sp.pos[key_][n]);
          if (live == only0) {
            emit(sp.src_alt0[key_]);
            inputs_.push_back(sp.alt_name[key_][0]);
            ++ki_;
            break;
          }
          choose(sp.src_trie[key_].get(), live, PC_AFTER_SRC);
          return;
        }
        case PC_AFTER_SRC:
          inputs_.push_back(sp.alt_name[key_][choice]);
          ++ki_;
          pc_ = PC_KEY;
          break;
        case PC_NODE_TAIL:
          if (sp.allow_retries) {
            emit(sp.c_retries);
            Mask live;
            for (int i = 0; i < (int)sp.retry_trie->alts.size(); ++i) live.set(i);
            choose(sp.retry_trie.get(), live, PC_AFTER_RETRY);
            return;
          }
          emit(sp.c_close2);
          pc_ = PC_NODE_END;
          break;
        case PC_AFTER_RETRY:
          emit(sp.c_close1);
          pc_ = PC_NODE_END;
          break;
        case PC_NODE_END: {
          chosen_.push_back(cur_);
          node_inputs_.push_back(inputs_);
          if (!can_more()) {
            pc_ = PC_BREAK;
            break;
          }
          if ((int)chosen_.size() < sp.min_nodes) {
            emit(sp.c_next);
            pc_ = PC_NAME;
            break;
          }
          Mask live;
          live.set(0);
          live.set(1);
          choose(sp.cont_trie.get(), live, PC_AFTER_CONT);
          return;
        }
        case PC_AFTER_CONT:
          pc_ = choice == 1 ? PC_BREAK : PC_NAME;
          break;
        case PC_BREAK:
          if (!can_more()) emit(sp.c_edges);
          j_ = 0;
          first_ = true;
          pc_ = PC_EDGE_NODE;
          break;
        case PC_EDGE_NODE: {
          if (j_ == (int)chosen_.size()) {
            pc_ = PC_END;
            break;
          }
          // producer -> consumer for every node-valued input source of node j
          // that was chosen before it (first occurrence order)
          const int dst = chosen_[j_];
          srcs_.clear();
          for (int v : node_inputs_[j_]) {
            if (v < 0 || v == dst) continue;
            bool dup = false, earlier = false;
            for (int s : srcs_) dup |= s == v;
            for (int q = 0; q < j_; ++q) earlier |= chosen_[q] == v;
            if (!dup && earlier) srcs_.push_back(v);
          }
          si_ = 0;
          pc_ = PC_EDGE_SRC;
          break;
        }
        case PC_EDGE_SRC: {
          if (si_ == (int)srcs_.size()) {
            ++j_;
            pc_ = PC_EDGE_NODE;
            break;
          }
          const int dst = chosen_[j_];
          emit(sp.edge(first_, srcs_[si_], dst));
          first_ = false;
          if (sp.fb_trie[dst]) {
            Mask live;
            live.set(0);
            live.set(1);
            choose(sp.fb_trie[dst].get(), live, PC_AFTER_FB);
            return;
          }
          emit(sp.c_close_edge);
          ++si_;
          break;
        }
        case PC_AFTER_FB:
          ++si_;
          pc_ = PC_EDGE_SRC;
          break;
        case PC_END:
          emit(sp.c_end);
          done_ = true;
          pc_ = PC_DONE;
          return;
        case PC_DONE:
          return;
      }
    }
  }
};

// Every index the decoder later uses without a bound check (used_[], pos[][],
// alt_name[][], the live-mask bits, fb_trie[]) is checked once here, so a
// malformed payload raises ValueError instead of reading out of range.
void validate(const NativeSpec& sp) {
  auto need = [](bool ok, const char* what) {
    if (!ok) throw std::invalid_argument(std::string("grammar spec: ") + what);
  };
  const int S = sp.S;
  need(S >= 1, "S must be >= 1");
  need(sp.min_nodes >= 1 && sp.max_nodes >= sp.min_nodes, "need 1 <= min_nodes <= max_nodes");
  need((int)sp.jnames.size() == S, "jnames must hold S names");
  need((int)sp.name_trie->alts.size() == S, "name_trie must hold S alternatives");
  need(!sp.retry_trie->alts.empty(), "retry_trie is empty");
  need(sp.cont_trie->alts.size() == 2, "cont_trie must hold 2 alternatives");
  need((int)sp.endpoint.size() == S && (int)sp.keys.size() == S && (int)sp.fb_trie.size() == S,
       "services must hold S entries");
  for (auto& f : sp.fb_trie) need(!f || f->alts.size() == 2, "a fallback trie must hold 2 alternatives");
  const int nk = (int)sp.key_first.size();
  for (auto& k : sp.keys)
    for (int id : k) need(id >= 0 && id < nk, "key id out of range");
  for (int k = 0; k < nk; ++k) {
    const int na = (int)sp.src_trie[k]->alts.size();
    need(na >= 1, "a source trie is empty");
    need((int)sp.pos[k].size() == S, "pos[key] must hold S entries");
    for (int p : sp.pos[k]) need(p >= -1 && p < na, "pos entry out of range");
    need((int)sp.alt_name[k].size() == na, "alt_name[key] must match the source trie");
    for (int a : sp.alt_name[k]) need(a >= -1 && a < S, "alt_name entry out of range");
  }
}

// spec dict (planner/grammar.py GrammarSpec.native_payload) -> NativeSpec
std::shared_ptr<NativeSpec> make_spec(const py::dict& d) {
  auto sp = std::make_shared<NativeSpec>();
  sp->S = d["S"].cast<int>();
  // a source choice has up to S + 1 alternatives (the payload key + every service)
  if (sp->S >= MAXA) throw std::invalid_argument("too many services for the native grammar");
  sp->max_nodes = d["max_nodes"].cast<int>();
  sp->min_nodes = d["min_nodes"].cast<int>();
  sp->allow_retries = d["allow_retries"].cast<bool>();
  sp->jnames = d["jnames"].cast<std::vector<std::string>>();
  sp->name_trie = std::make_unique<Trie>(trie_of(d["name_trie"]));
  sp->retry_trie = std::make_unique<Trie>(trie_of(d["retry_trie"]));
  sp->cont_trie = std::make_unique<Trie>(trie_of(d["cont_trie"]));
  py::dict c = d["chunks"];
  sp->c_start = chunk_of(c["start"]);
  sp->c_retries = chunk_of(c["retries"]);
  sp->c_close1 = chunk_of(c["close1"]);
  sp->c_close2 = chunk_of(c["close2"]);
  sp->c_next = chunk_of(c["next"]);
  sp->c_edges = chunk_of(c["edges"]);
  sp->c_close_edge = chunk_of(c["close_edge"]);
  sp->c_end = chunk_of(c["end"]);
  for (auto h : d["services"]) {
    py::dict s = h.cast<py::dict>();
    sp->endpoint.push_back(chunk_of(s["endpoint"]));
    sp->keys.push_back(s["keys"].cast<std::vector<int>>());
    sp->fb_trie.push_back(s["fallback"].is_none() ? nullptr
                                                  : std::make_unique<Trie>(trie_of(s["fallback"])));
  }
  for (auto h : d["keys"]) {
    py::dict k = h.cast<py::dict>();
    sp->key_first.push_back(chunk_of(k["first"]));
    sp->key_rest.push_back(chunk_of(k["rest"]));
    sp->src_alt0.push_back(chunk_of(k["alt0"]));
    sp->src_trie.push_back(std::make_unique<Trie>(trie_of(k["trie"])));
    sp->pos.push_back(k["pos"].cast<std::vector<int>>());
    sp->alt_name.push_back(k["alt_name"].cast<std::vector<int>>());
  }
  validate(*sp);
  sp->encode = d["encode"];
  sp->compact = d.contains("compact") && d["compact"].cast<bool>();
  return sp;
}

}  // namespace

void register_grammar(py::module_& m) {
  py::class_<NativeSpec, std::shared_ptr<NativeSpec>>(m, "GrammarSpec");
  m.def("grammar_spec", &make_spec, "native grammar constants from GrammarSpec.native_payload()");
  py::class_<NativeDecoder>(m, "DagDecoder")
      .def(py::init<std::shared_ptr<NativeSpec>>())
      .def("advance", &NativeDecoder::advance)
      .def("allowed", &NativeDecoder::allowed)
      .def("feed", &NativeDecoder::feed)
      .def_property_readonly("done", &NativeDecoder::done)
      .def_property_readonly("text", &NativeDecoder::text)
      .def("result", [](const NativeDecoder& d) {
        return py::module_::import("json").attr("loads")(d.text());
      });
  // one engine step's sampled tokens: feed + advance for every decoder in one
  // call (the per-sequence Python loop was most of the host update per step)
  m.def("allowed_many", [](const py::list& decs) {
    py::list out(py::len(decs));
    for (size_t i = 0; i < (size_t)py::len(decs); ++i)
      out[i] = py::cast(decs[i].cast<const NativeDecoder&>().allowed());
    return out;
  });
  // decision lookahead (engine MCP_LOOKAHEAD): every outcome of a decoder's
  // pending choice, each as (token, the tokens it appends - the token itself
  // then its jump-forward span -, done, the next choice's allowed tokens, the
  // decoder state after it).  The engine launches the next forward for all
  // outcomes at once and the device picks the sampled one.
  m.def("branches", [](const NativeDecoder& d) {
    py::list out;
    for (int tok : d.allowed()) {
      NativeDecoder c(d);
      c.feed(tok);
      std::vector<int> toks = c.advance();
      const bool fin = c.done();
      std::vector<int> nxt = fin ? std::vector<int>{} : c.allowed();
      out.append(py::make_tuple(tok, std::move(toks), fin, std::move(nxt), std::move(c)));
    }
    return out;
  });
  m.def("feed_advance_many", [](const py::list& decs, const std::vector<int>& toks) {
    if ((size_t)py::len(decs) != toks.size()) throw py::value_error("decoders / tokens length");
    py::list out(toks.size());
    for (size_t i = 0; i < toks.size(); ++i) {
      NativeDecoder& d = decs[i].cast<NativeDecoder&>();
      d.feed(toks[i]);
      out[i] = py::cast(d.advance());
    }
    return out;
  });
}
