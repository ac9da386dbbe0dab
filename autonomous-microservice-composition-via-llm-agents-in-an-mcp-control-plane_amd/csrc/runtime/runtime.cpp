// Native CPU runtime of the planner engine (engine/_runtime*.so, pybind11).
//
// The engine's scheduler thread runs once per forward step (~40 ms of GPU work
// at 256 concurrent intents) and, in the large-batch mode, the GPU idles while
// it runs: everything here is on that critical path.
//
//  * BlockAllocator - paged-KV block free list with reference counts (prefix
//    blocks are shared by every request of a registry prompt).
//  * pack_step      - builds the whole int32 step descriptor of one ragged
//    forward in ONE host buffer (the single H2D copy of the step): token ids,
//    positions, physical KV slots, per-sequence query/context spans, the block
//    table, the attention work lists (1-wave items for short spans, 4-wave for
//    long ones, csrc/attention.hip), copy-on-write block pairs, cascade
//    metadata and the grammar-allowed token sets (CSR) with their RNG
//    counters.  Same part order as engine/batch.py pack_host/views.
//  * topo_generations - generational Kahn order of a DAG given as index edge
//    lists (the orchestrator's trace order), with the
//    reference's semantics: generation 0 in node order, children in the order
//    they are reached; cycle -> error.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

struct OutOfBlocks : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class BlockAllocator {
 public:
  explicit BlockAllocator(int num_blocks) : num_blocks_(num_blocks), ref_(num_blocks, 0) {
    if (num_blocks <= 0) throw std::invalid_argument("num_blocks must be positive");
    free_.reserve(num_blocks);
    for (int b = num_blocks - 1; b >= 0; --b) free_.push_back(b);   // pop_back hands out 0, 1, ...
  }

  std::vector<int> alloc(int n) {
    if (n < 0) throw std::invalid_argument("negative block count");
    if ((size_t)n > free_.size())
      throw OutOfBlocks("need " + std::to_string(n) + " KV blocks, " +
                        std::to_string(free_.size()) + " free");
    std::vector<int> out(n);
    for (int i = 0; i < n; ++i) {
      const int b = free_.back();
      free_.pop_back();
      ref_[b] = 1;
      out[i] = b;
    }
    return out;
  }

  void incref(const std::vector<int>& blocks) {
    for (int b : blocks) {
      check(b);
      if (ref_[b] <= 0) throw std::runtime_error("incref of free block " + std::to_string(b));
      ++ref_[b];
    }
  }

  void free(const std::vector<int>& blocks) {
    for (int b : blocks) {
      check(b);
      if (ref_[b] <= 0) throw std::runtime_error("double free of block " + std::to_string(b));
      if (--ref_[b] == 0) free_.push_back(b);
    }
  }

  int num_free() const { return (int)free_.size(); }
  int num_blocks() const { return num_blocks_; }
  int refcount(int b) const {
    check(b);
    return ref_[b];
  }
  double utilization() const { return 1.0 - (double)free_.size() / (double)num_blocks_; }

 private:
  void check(int b) const {
    if (b < 0 || b >= num_blocks_) throw std::out_of_range("block id " + std::to_string(b));
  }
  int num_blocks_;
  std::vector<int> ref_;
  std::vector<int> free_;
};

// Python int sequence -> appended ints (lists and tuples without per-item
// pybind casts)
void append_ints(std::vector<int32_t>& dst, const py::handle& seq, Py_ssize_t limit = -1) {
  PyObject* fast = PySequence_Fast(seq.ptr(), "expected a sequence of ints");
  if (!fast) throw py::error_already_set();
  const Py_ssize_t n0 = PySequence_Fast_GET_SIZE(fast);
  const Py_ssize_t n = limit >= 0 && limit < n0 ? limit : n0;
  PyObject** items = PySequence_Fast_ITEMS(fast);
  for (Py_ssize_t i = 0; i < n; ++i) {
    const long v = PyLong_AsLong(items[i]);
    if (v == -1 && PyErr_Occurred()) {
      Py_DECREF(fast);
      throw py::error_already_set();
    }
    dst.push_back((int32_t)v);
  }
  Py_DECREF(fast);
}

// One ragged step.  seqs: list of (tokens, take, start, blocks, kv_begin,
// sample) - the first `take` of `tokens` enter at positions
// [start, start + take) of a sequence whose KV blocks are `blocks`; `sample`
// marks that its last token's hidden state is sampled.  Returns
// (host int32 array, layout) exactly like engine.batch.pack_host.
py::tuple pack_step(const py::list& seqs, int block_size, int group, const py::object& copies,
                    const py::object& pre_bt, int pre_tokens, const py::object& allowed,
                    const py::object& ctr) {
  const int S = (int)py::len(seqs);
  std::vector<int32_t> ids, pos, slots, rows, q_start(S), q_len(S), ctx_len(S), kv_begin(S);
  std::vector<std::vector<int32_t>> tables(S);
  size_t maxb = 1;
  int T = 0;
  for (int s = 0; s < S; ++s) {
    const py::tuple it = seqs[s].cast<py::tuple>();
    const int take = it[1].cast<int>();
    const int start = it[2].cast<int>();
    auto& tab = tables[s];
    append_ints(tab, it[3]);
    if (take <= 0) throw std::invalid_argument("pack_step: empty span");
    const size_t before = ids.size();
    append_ints(ids, it[0], take);
    if ((int)(ids.size() - before) != take) throw std::invalid_argument("pack_step: take > len(tokens)");
    if ((int64_t)(start + take) > (int64_t)tab.size() * block_size)
      throw std::invalid_argument("pack_step: sequence has too few KV blocks");
    for (int p = start; p < start + take; ++p) {
      pos.push_back(p);
      slots.push_back(tab[p / block_size] * block_size + p % block_size);
    }
    q_start[s] = T;
    q_len[s] = take;
    ctx_len[s] = start + take;
    kv_begin[s] = it[4].cast<int>();
    T += take;
    if (it[5].cast<bool>()) rows.push_back(T - 1);
    maxb = std::max(maxb, tab.size());
  }
  // attention work lists (engine.batch.build_work)
  const int t1 = 16 / group, t4 = 4 * (16 / group);
  static const char* cut_env = getenv("MCP_ATTN_NW1_CUTOFF");
  static const char* xcd_env = getenv("MCP_ATTN_XCD_ORDER");
  const int cutoff = cut_env ? atoi(cut_env) : 2 * t1;
  const bool xcd_order = !xcd_env || atoi(xcd_env) == 1;
  std::vector<int32_t> w1s, w1q, w4s, w4q;
  std::vector<int> depth1(S, 0);
  for (int s = 0; s < S; ++s) {
    const int ql = q_len[s];
    const bool small = ql <= cutoff;
    const int qt = small ? t1 : t4;
    for (int q0 = 0; q0 < ql; q0 += qt) {
      (small ? w1s : w4s).push_back(s);
      (small ? w1q : w4q).push_back(q0);
      if (small) ++depth1[s];
    }
  }
  if (xcd_order && !w1s.empty()) {
    // 1-wave items of one sequence read the same K/V: sequences bucketed by
    // item count (deepest first), blocks of 8, item d of the block's i-th
    // sequence at 8 d + i - one XCD (block id % 8) and its L2 per sequence
    int maxd = 0;
    for (int s = 0; s < S; ++s) maxd = std::max(maxd, depth1[s]);
    std::vector<int32_t> rs, rq;
    rs.reserve(w1s.size());
    rq.reserve(w1q.size());
    for (int d = maxd; d >= 1; --d) {
      std::vector<int> order;
      for (int s = 0; s < S; ++s)
        if (depth1[s] == d) order.push_back(s);
      for (size_t b = 0; b < order.size(); b += 8) {
        const size_t e = std::min(order.size(), b + 8);
        for (int k = 0; k < d; ++k)
          for (size_t i = b; i < e; ++i) {
            rs.push_back(order[i]);
            rq.push_back(k * t1);
          }
      }
    }
    w1s.swap(rs);
    w1q.swap(rq);
  }
  std::vector<int32_t> csrc, cdst;
  if (!copies.is_none())
    for (const auto& pr : copies.cast<py::list>()) {
      const py::tuple t = pr.cast<py::tuple>();
      csrc.push_back(t[0].cast<int>());
      cdst.push_back(t[1].cast<int>());
    }
  std::vector<int32_t> prebt;
  if (!pre_bt.is_none()) append_ints(prebt, pre_bt);
  const bool cascade = pre_tokens > 0 && !prebt.empty();
  std::vector<int32_t> aptr, aids, actr;
  if (!allowed.is_none()) {
    const py::list al = allowed.cast<py::list>();
    aptr.push_back(0);
    for (const auto& a : al) {
      append_ints(aids, a);
      aptr.push_back((int32_t)aids.size());
    }
    append_ints(actr, ctr);
    if (actr.size() != rows.size() || aptr.size() != rows.size() + 1)
      throw std::invalid_argument("pack_step: allowed sets / counters do not match sampled rows");
  }

  const size_t bt_n = (size_t)S * maxb;
  std::vector<size_t> sizes = {ids.size(), pos.size(), slots.size(), rows.size(), (size_t)S,
                               (size_t)S, (size_t)S, bt_n, w1s.size(), w1q.size(), w4s.size(),
                               w4q.size(), csrc.size(), cdst.size(),
                               cascade ? (size_t)S : 0, cascade ? prebt.size() : 0,
                               aptr.size(), aids.size(), actr.size()};
  size_t total = 0;
  for (size_t n : sizes) total += n;
  py::array_t<int32_t> host(total);
  int32_t* o = host.mutable_data();
  auto put = [&](const std::vector<int32_t>& v) {
    std::copy(v.begin(), v.end(), o);
    o += v.size();
  };
  put(ids); put(pos); put(slots); put(rows); put(q_start); put(q_len); put(ctx_len);
  for (int s = 0; s < S; ++s) {
    std::copy(tables[s].begin(), tables[s].end(), o);
    std::fill(o + tables[s].size(), o + maxb, 0);
    o += maxb;
  }
  put(w1s); put(w1q); put(w4s); put(w4q); put(csrc); put(cdst);
  if (cascade) {
    put(kv_begin);
    put(prebt);
  }
  put(aptr); put(aids); put(actr);
  py::list layout;
  for (size_t n : sizes) layout.append((int)n);
  layout.append(S);
  layout.append(cascade ? pre_tokens : 0);
  return py::make_tuple(host, layout);
}

// Generational Kahn order (networkx.topological_sort semantics).
std::vector<std::vector<int>> topo_generations(int n, const std::vector<std::pair<int, int>>& edges) {
  std::vector<std::vector<int>> succ(n);
  std::vector<int> indeg(n, 0);
  for (const auto& e : edges) {
    if (e.first < 0 || e.first >= n || e.second < 0 || e.second >= n)
      throw std::out_of_range("edge endpoint out of range");
    succ[e.first].push_back(e.second);
    ++indeg[e.second];
  }
  std::vector<std::vector<int>> gens;
  std::vector<int> cur;
  for (int v = 0; v < n; ++v)
    if (indeg[v] == 0) cur.push_back(v);
  int seen = 0;
  while (!cur.empty()) {
    seen += (int)cur.size();
    std::vector<int> nxt;
    for (int v : cur)
      for (int w : succ[v])
        if (--indeg[w] == 0) nxt.push_back(w);
    gens.push_back(std::move(cur));
    cur = std::move(nxt);
  }
  if (seen != n) throw std::runtime_error("Graph contains a cycle or graph changed during iteration");
  return gens;
}

}  // namespace

void register_grammar(py::module_& m);     // grammar.cpp

void register_embed(py::module_& m);   // embed.cpp

PYBIND11_MODULE(MODULE_NAME, m) {
  register_embed(m);
  m.doc() = "native CPU runtime of the MI355X planner engine";
  py::register_exception<OutOfBlocks>(m, "OutOfBlocks", PyExc_RuntimeError);
  py::class_<BlockAllocator>(m, "BlockAllocator")
      .def(py::init<int>())
      .def("alloc", &BlockAllocator::alloc)
      .def("incref", &BlockAllocator::incref)
      .def("free", &BlockAllocator::free)
      .def("refcount", &BlockAllocator::refcount)
      .def("utilization", &BlockAllocator::utilization)
      .def_property_readonly("num_free", &BlockAllocator::num_free)
      .def_property_readonly("num_blocks", &BlockAllocator::num_blocks);
  m.def("pack_step", &pack_step, py::arg("seqs"), py::arg("block_size"), py::arg("group"),
        py::arg("copies") = py::none(), py::arg("pre_bt") = py::none(), py::arg("pre_tokens") = 0,
        py::arg("allowed") = py::none(), py::arg("ctr") = py::none());
  m.def("topo_generations", &topo_generations);
  register_grammar(m);
}
