"""Python entry points of the gfx950 kernel library.

GPU tensors always run the hand-written HIP kernels from the in-tree
``_kernels*.so`` (built by ``csrc/build.py``); if that library is missing on a
GPU box the first GPU op raises — there is no silent eager fallback.  CPU
tensors run the fp32 references in ``ops.reference`` (CPU test tier only).
"""
from __future__ import annotations

import glob
import importlib.machinery
import importlib.util
import os
from typing import Optional

import torch

from . import reference as ref

_LIB = None
_HERE = os.path.dirname(os.path.abspath(__file__))


class KernelLibraryMissing(RuntimeError):
    pass


def lib():
    """Load (once) and return the HIP kernel extension module."""
    global _LIB
    if _LIB is None:
        cands = sorted(glob.glob(os.path.join(_HERE, "_kernels*.so")))
        if os.environ.get("MCP_KERNELS_SO"):           # A/B of two builds (tools/gpu_run.sh ab)
            cands = [os.environ["MCP_KERNELS_SO"]]
        if not cands:
            raise KernelLibraryMissing(
                "HIP kernel library not built: run `python csrc/build.py` "
                "(or __graft_entry__.build()) before using GPU tensors")
        loader = importlib.machinery.ExtensionFileLoader("_kernels", cands[0])
        spec = importlib.util.spec_from_file_location("_kernels", cands[0], loader=loader)
        mod = importlib.util.module_from_spec(spec)
        loader.exec_module(mod)
        _load_gemm_plan(mod)
        if torch.cuda.is_available() and hasattr(mod, "gemm_splitk_init"):
            # fp32 split-K partials of small-M projections (gemm.hip); allocated
            # here, never inside a hipGraph capture
            mod.gemm_splitk_init(int(os.environ.get("MCP_GEMM_SPLITK_MB", "256")) << 20)
        if torch.cuda.is_available() and hasattr(mod, "attn_split_init"):
            mod.attn_split_init()          # fused split-KV tickets (outside any capture)
        _LIB = mod
    return _LIB


GEMM_PLAN_FILE = os.path.join(_HERE, "gemm_plan_gfx950.json")


def _load_gemm_plan(mod, path: Optional[str] = None) -> int:
    """Install the measured GEMM tile plans (tools/tune_gemm_plan.py) into the
    kernel library's selector.  MCP_GEMM_PLAN=<path> picks another file, "0"
    disables (the analytic wave-quantisation model then decides alone).
    Returns the number of (N, K) shapes installed."""
    import json

    path = path or os.environ.get("MCP_GEMM_PLAN", GEMM_PLAN_FILE)
    if path == "0" or not os.path.exists(path) or not hasattr(mod, "gemm_plan_set"):
        return 0
    with open(path) as f:
        plan = json.load(f)
    mod.gemm_plan_clear()
    for sh in plan["shapes"]:
        mod.gemm_plan_set(int(sh["N"]), int(sh["K"]), [int(c) for c in sh["codes"]])
        if "splits" in sh and hasattr(mod, "gemm_plan_set_splits"):
            mod.gemm_plan_set_splits(int(sh["N"]), int(sh["K"]), [int(c) for c in sh["splits"]])
        if "flex" in sh and hasattr(mod, "gemm_plan_set_flex"):
            mod.gemm_plan_set_flex(int(sh["N"]), int(sh["K"]), [int(c) for c in sh["flex"]])
        if "fsplit" in sh and hasattr(mod, "gemm_plan_set_fsplit"):
            mod.gemm_plan_set_fsplit(int(sh["N"]), int(sh["K"]), [int(c) for c in sh["fsplit"]])
        if "group" in sh and hasattr(mod, "gemm_plan_set_group"):
            mod.gemm_plan_set_group(int(sh["N"]), int(sh["K"]), [int(c) for c in sh["group"]])
        if "persist" in sh and hasattr(mod, "gemm_plan_set_persist"):
            mod.gemm_plan_set_persist(int(sh["N"]), int(sh["K"]), [int(c) for c in sh["persist"]])
        if "silu" in sh and hasattr(mod, "gemm_plan_set_silu"):
            mod.gemm_plan_set_silu(int(sh["N"]), int(sh["K"]), [int(c) for c in sh["silu"]])
        if "rope" in sh and hasattr(mod, "gemm_plan_set_rope"):
            mod.gemm_plan_set_rope(int(sh["N"]), int(sh["K"]), [int(c) for c in sh["rope"]])
    return len(plan["shapes"])


def library_path() -> Optional[str]:
    if os.environ.get("MCP_KERNELS_SO"):
        return os.environ["MCP_KERNELS_SO"]
    c = sorted(glob.glob(os.path.join(_HERE, "_kernels*.so")))
    return c[0] if c else None


def available() -> bool:
    try:
        lib()
        return True
    except (KernelLibraryMissing, ImportError, OSError):
        return False


# GEMM shape histogram for tile-selection tuning: MCP_GEMM_TRACE=<path> counts
# eager (M, N, K, kind) calls and writes them as JSON lines at exit (calls made
# while a HIP graph is being captured are counted under kind "+graph")
_TRACE = None
if os.environ.get("MCP_GEMM_TRACE"):
    import atexit
    import collections
    import json

    _TRACE = collections.Counter()

    def _dump_trace(path=os.environ["MCP_GEMM_TRACE"]):
        with open(path, "w") as f:
            for (M, N, K, kind), c in sorted(_TRACE.items()):
                f.write(json.dumps({"M": M, "N": N, "K": K, "kind": kind, "calls": c}) + "\n")

    atexit.register(_dump_trace)


def _trace(X, W, kind):
    cap = torch.cuda.is_current_stream_capturing()
    _TRACE[(X.numel() // X.shape[-1], W.shape[0], W.shape[1], kind + ("+graph" if cap else ""))] += 1


# --------------------------------------------------------------------- ops
def rmsnorm(x, w, eps, out=None):
    if x.is_cuda:
        out = torch.empty_like(x) if out is None else out
        lib().rmsnorm(x, w, out, eps)
        return out
    r = ref.rmsnorm(x, w, eps)
    return r if out is None else out.copy_(r)


def add_rmsnorm(x, residual, w, eps, out=None):
    """residual += x (in place, bf16); returns rmsnorm(residual) * w."""
    if x.is_cuda:
        out = torch.empty_like(x) if out is None else out
        lib().add_rmsnorm(x, residual, w, out, eps)
        return out
    r = ref.add_rmsnorm(x, residual, w, eps)
    return r if out is None else out.copy_(r)


def silu_mul(x, out=None):
    F = x.shape[-1] // 2
    if x.is_cuda:
        out = x.new_empty(*x.shape[:-1], F) if out is None else out
        lib().silu_mul(x, out)
        return out
    r = ref.silu_mul(x)
    return r if out is None else out.copy_(r)


def embedding(ids, table, out=None):
    if table.is_cuda:
        out = table.new_empty(ids.numel(), table.shape[1]) if out is None else out
        lib().embedding(ids, table, out)
        return out
    r = table[ids.long()]
    return r if out is None else out.copy_(r)


def gemm(X, W, R=None, out=None, algo: int = -1, ss_out=None):
    """Y = X @ W^T (+ R).  X [M, K], W [N, K].  algo: -1 auto (the measured
    plan), 0 = 128^2, 1 = 256^2 path, 9..13 = AGPR kernel at plan code algo - 8.
    ``ss_out`` (int64 [M], residual GEMMs only): += each output row's sum of
    squares, fixed point - the fused RMSNorm statistic of the next layer input."""
    if X.is_cuda:
        if _TRACE is not None:
            _trace(X, W, "gemm" if R is None else "gemm+res")
        out = X.new_empty(*X.shape[:-1], W.shape[0]) if out is None else out
        lib().gemm(X, W, out, R, algo, ss_out)
        return out
    r = ref.gemm(X, W, R)
    if ss_out is not None:
        ss_out[:r.shape[0]] += ref.row_sumsq(r)
    return r if out is None else out.copy_(r)


_PF_SINK = {}


def weight_prefetch(W, nbytes: int = -1, wgs: int = 256):
    """Read up to ``nbytes`` of ``W`` once on the current stream, so a GEMM that
    streams it next finds it in the Infinity Cache (csrc/prefetch.hip).  No-op
    on CPU."""
    if not W.is_cuda:
        return
    lib().weight_prefetch(W, int(nbytes), int(wgs), weight_prefetch_init(W.device))


def weight_prefetch_init(device):
    """The prefetch kernel's sink buffer for ``device`` (allocate it outside
    hipGraph capture: the model does at construction)."""
    device = torch.device(device)
    if device.index is None:
        device = torch.device(device.type, torch.cuda.current_device())
    sink = _PF_SINK.get(device)
    if sink is None:
        sink = _PF_SINK[device] = torch.zeros(256, dtype=torch.int32, device=device)
    return sink


def gemm_silu(X, W, out=None, ss_in=None, eps: float = 0.0):
    """SwiGLU projection: silu(X Wg^T) * (X Wu^T) with W = interleave_gate_up(Wg, Wu)
    ([2F, K], 16-row groups); the activation is fused into the MFMA GEMM epilogue.
    ``ss_in`` (int64 [M]): fused RMSNorm - the accumulators of row m are scaled
    by rsqrt(ss_in[m] / K + eps) first (the norm weight folded into W)."""
    if X.is_cuda:
        if _TRACE is not None:
            _trace(X, W, "swiglu")
        out = X.new_empty(*X.shape[:-1], W.shape[0] // 2) if out is None else out
        lib().gemm_silu(X, W, out, ss_in, eps)
        return out
    r = ref.gemm_silu(X, W, ss_in, eps)
    return r if out is None else out.copy_(r)


def row_sumsq(x, ss):
    """ss[t] = sum of x[t]^2 (int64 fixed point): the fused-norm statistic of a
    row no GEMM epilogue produced (the embedding output)."""
    if x.is_cuda:
        lib().row_sumsq(x, ss)
    else:
        ss[:x.shape[0]] = ref.row_sumsq(x)
    return ss


def qkv_rope(h, wqkv, pos, slots, cos_sin, q_out, k_cache, v_cache, Hq, Hkv, D, qkv=None,
             ss_in=None, eps: float = 0.0):
    """q_out, K/V cache <- rope(h wqkv^T).  On the GPU the rotation and the
    paged K/V write run in the QKV GEMM's epilogue when the AGPR kernel serves
    the shape (``qkv`` is then untouched scratch); otherwise GEMM + rope_kv.
    ``ss_in``: fused RMSNorm of the rows of ``h`` (see ``gemm_silu``)."""
    if h.is_cuda:
        if _TRACE is not None:
            _trace(h, wqkv, "qkv_rope")
        T = h.numel() // h.shape[-1]
        qkv = h.new_empty(T, wqkv.shape[0]) if qkv is None else qkv
        lib().qkv_rope(h, wqkv, qkv, pos, slots, cos_sin, q_out, k_cache, v_cache, Hq, Hkv, D,
                       ss_in, eps)
        return q_out
    if ss_in is not None:
        qkv = ((h.float() @ wqkv.float().t())
               * ref.norm_row_scale(ss_in[:h.shape[0]], h.shape[-1], eps)).to(h.dtype)
    else:
        qkv = ref.gemm(h, wqkv)
    ref.rope_kv(qkv, pos, slots, cos_sin, q_out, k_cache, v_cache, Hq, Hkv, D)
    return q_out


def rope_kv(qkv, pos, slots, cos_sin, q_out, k_cache, v_cache, Hq, Hkv, D):
    if qkv.is_cuda:
        lib().rope_kv(qkv, pos, slots, cos_sin, q_out, k_cache, v_cache, Hq, Hkv, D)
    else:
        ref.rope_kv(qkv, pos, slots, cos_sin, q_out, k_cache, v_cache, Hq, Hkv, D)
    return q_out


_SIDE = {}
# split-KV steps as one launch with the combine fused (attention.hip MIXED);
# MCP_ATTN_MIXED=0 keeps a launch + combine per work list
_MIXED_SPLIT = os.environ.get("MCP_ATTN_MIXED", "1") == "1"
# split-KV steps on the decode kernel (csrc/attention_decode.hip: key tiles
# fixed by the grid position, every tile of a block in flight at once, the
# waves merged in LDS); MCP_ATTN_DECODE=0 keeps the work-list split launch
_DECODE_SPLIT = os.environ.get("MCP_ATTN_DECODE", "1") == "1"
_DECODE_BLOCKS_PER_CU = 2
_DECODE_FORCE = os.environ.get("MCP_ATTN_DECODE_FORCE", "0") == "1"
# unsplit steps' items on the decode kernel in own-span mode (attention_decode.hip
# rel): 0 off, 1 the 1-wave items, 2 both work lists
_DECODE_OWN = int(os.environ.get("MCP_ATTN_DECODE_OWN", "0"))


_CUS = {}


def _num_cus(device) -> int:
    key = torch.device(device).index
    n = _CUS.get(key)
    if n is None:
        n = _CUS[key] = torch.cuda.get_device_properties(device).multi_processor_count
    return n


def _side_stream(device):
    """One persistent side stream per device (concurrent cascade attention)."""
    key = torch.device(device).index
    st = _SIDE.get(key)
    if st is None:
        st = torch.cuda.Stream(device=device)
        _SIDE[key] = st
    return st


def prefix_splits(pre_tokens: int, pre_keys: int, hkv: int, num_cus: int = 256) -> int:
    """Key-split factor of the cascade prefix pass (csrc/attention.hip): a
    step with few query tokens launches ceil(tokens / 32) x Hkv workgroups that
    each walk every prefix tile; split the tiles so the grid reaches ~2
    workgroups per CU, >= 2 tiles per split.  ``pre_tokens`` / ``pre_keys``
    are the grid capacities under a hipGraph.  Only for small grids (<= a
    quarter of the CUs): the unsplit pass walks the ~11 prefix tiles with one
    tile of DMA lookahead, ~25 us even for 16 query tokens; split, 4-16
    requests take 25-37 us instead of 34-45 for the whole attention, while at
    256 requests the merge costs more than it saves
    (tools/bench_attention.py, profiles/attention_tuning.md).
    ``MCP_PREFIX_SPLIT``: -1 auto (default), 0 off, N forces N."""
    forced = int(os.environ.get("MCP_PREFIX_SPLIT", "-1"))
    if forced == 0:
        return 1
    tiles = pre_keys // 64
    grid = -(-pre_tokens // 32) * hkv
    if forced > 1:
        return max(1, min(forced, tiles))
    if grid > num_cus // 4:
        return 1
    ns = min(-(-2 * num_cus // max(grid, 1)), tiles // 2, 8)
    return ns if ns >= 2 else 1


# decode attention + o-projection in one launch (csrc/attention_decode.hip
# attn_oproj_kernel; MCP_ATTN_OPROJ=1 enables).  Measured and off: config 2
# p50 86.2 ms unfused vs 88.8-89.0 fused (weights preloaded) and 91.2 (loaded
# after the wait): the in-launch hand-off (writer count, poll, acquire, the
# attention rows re-read) costs more than the launch boundary it removes, and
# the preloaded weight stream slows the attention's round trips
# (profiles/config2_attn_oproj_fused_ab_r6.md)
_ATTN_OPROJ = os.environ.get("MCP_ATTN_OPROJ", "0") == "1"


def _decode_lists(q, k_cache, meta):
    """The decode kernel's work lists and grid z when a step takes it (the
    use_dec rule of paged_attention), else None."""
    L = lib()
    ns = int(getattr(meta, "kv_splits", 1))
    if not (ns > 1 and _DECODE_SPLIT and hasattr(L, "paged_attention_decode")):
        return None
    lists = {nw: (ws, wq) for nw, ws, wq in meta.work_lists()}
    e = torch.empty(0, dtype=torch.int32, device=q.device)
    ws4, wq4 = lists.get(4, (e, e))
    ws1, wq1 = lists.get(1, (e, e))
    nz = L.attn_decode_blocks(int(meta.block_table.shape[1]))
    use = _DECODE_FORCE or getattr(meta, "padded", False) or (
        (4 * ws4.numel() + ws1.numel()) * k_cache.shape[1] * nz
        <= _DECODE_BLOCKS_PER_CU * _num_cus(q.device))
    return (ws4, wq4, ws1, wq1, nz) if use else None


def attention_oproj(q, k_cache, v_cache, meta, scale, wo, x, ss_out=None, out=None) -> bool:
    """Decode-sized step, TP = 1: paged attention into ``out`` and
    ``x += out.view(T, -1) @ wo.T`` (in place, the rows' fused-norm statistic
    added to ``ss_out``) in ONE launch, the o-projection's weights streamed
    while the attention runs.  True when done; False when the step is outside
    the fused form (cascade prefix, no split-KV decode path, > 16 tokens,
    K != 4096) - nothing was launched and the caller runs both ops apart.
    Reference semantics: ``paged_attention`` then ``gemm(a, wo, R=x, out=x,
    ss_out=ss_out)``."""
    if not (q.is_cuda and _ATTN_OPROJ) or meta.pre_tokens > 0 or q.shape[0] > 16:
        return False
    L = lib()
    if not hasattr(L, "paged_attention_decode_oproj"):
        return False
    dl = _decode_lists(q, k_cache, meta)
    if dl is None:
        return False
    ws4, wq4, ws1, wq1, nz = dl
    global ATTN_OPROJ_LAUNCHES
    out = torch.empty_like(q) if out is None else out
    so = torch.empty(nz if nz > 1 else 0, *q.shape, device=q.device, dtype=torch.float32)
    sl = torch.empty(nz if nz > 1 else 0, q.shape[0], q.shape[1], device=q.device,
                     dtype=torch.float32)
    done = bool(L.paged_attention_decode_oproj(q, k_cache, v_cache, out, meta.q_start, meta.q_len,
                                               meta.ctx_len, meta.block_table, ws4, wq4, ws1, wq1,
                                               scale, nz, so, sl, wo, x, ss_out))
    ATTN_OPROJ_LAUNCHES += done
    return done


ATTN_OPROJ_LAUNCHES = 0          # host-side count of fused launches (captures count once)


def paged_attention(q, k_cache, v_cache, meta, scale, out=None):
    """``meta`` is an ``AttnMeta`` (engine.batch) holding the per-sequence and
    work-list int32 tensors."""
    if q.is_cuda:
        out = torch.empty_like(q) if out is None else out
        L = lib()
        kw = {}
        pre_dims = getattr(meta, "pre_dims", None)
        concurrent = meta.pre_tokens > 0 and os.environ.get("MCP_ATTN_CONCURRENT", "0") == "1"
        main = torch.cuda.current_stream(q.device)
        if concurrent:
            # the prefix pass and the own-key pass are independent: run the
            # prefix pass on a side stream (fork / join events, hipGraph-safe),
            # then merge the two partials (attn_cascade_merge)
            side = _side_stream(q.device)
            side.wait_stream(main)
        if meta.pre_tokens > 0:
            # cascade: all requests' query tokens vs the shared prefix K/V in full
            # MFMA tiles, then each request's own keys + LSE merge (csrc/attention.hip);
            # with device pre_dims (hipGraph) the sizes are read on the device
            pre_o = torch.empty_like(q)
            pre_lse = torch.empty(q.shape[0], q.shape[1], device=q.device, dtype=torch.float32)
            ps = prefix_splits(meta.pre_tokens, meta.pre_keys, k_cache.shape[1])
            kw_split = {}
            if ps > 1:
                kw_split = {"nsplit": ps,
                            "split_o": torch.empty(ps * meta.pre_tokens * q.shape[1] * q.shape[2],
                                                   device=q.device, dtype=torch.float32),
                            "split_lse": torch.empty(ps * meta.pre_tokens * q.shape[1],
                                                     device=q.device, dtype=torch.float32)}
            if concurrent:
                with torch.cuda.stream(side):
                    L.prefix_attention(q, k_cache, v_cache, pre_o, pre_lse, meta.pre_bt,
                                       meta.pre_keys, meta.pre_tokens, scale, pre_dims=pre_dims,
                                       **kw_split)
                own_lse = torch.empty(q.shape[0], q.shape[1], device=q.device, dtype=torch.float32)
                kw = {"kv_begin": meta.kv_begin, "own_lse": own_lse}
            else:
                L.prefix_attention(q, k_cache, v_cache, pre_o, pre_lse, meta.pre_bt, meta.pre_keys,
                                   meta.pre_tokens, scale, pre_dims=pre_dims, **kw_split)
                kw = {"kv_begin": meta.kv_begin, "pre_o": pre_o, "pre_lse": pre_lse}
        ns = int(getattr(meta, "kv_splits", 1))
        if ns > 1 and _DECODE_SPLIT and not concurrent and hasattr(L, "paged_attention_decode"):
            lists = {nw: (ws, wq) for nw, ws, wq in meta.work_lists()}
            e = torch.empty(0, dtype=torch.int32, device=q.device)
            ws4, wq4 = lists.get(4, (e, e))
            ws1, wq1 = lists.get(1, (e, e))
            nz = L.attn_decode_blocks(int(meta.block_table.shape[1]))
            # a grid past two blocks per CU (several sequences with long spans
            # and contexts) runs the work-list split launch below instead
            # (profiles/attention_decode_r3.jsonl).  A hipGraph step's lists are
            # padded to the key's capacity (52 items at the smallest key), so
            # the rule would always reject it there; a split key is chosen only
            # while the real items stay under 2 x CUs of work
            # (batch.choose_kv_splits, work factor 2) and the padding items
            # exit at once: graph steps take the decode kernel (config 2 p50
            # 99.1 -> 94.3 ms, config 5 at 20 / 40 intents/s equal,
            # profiles/attention_decode_graph_ab.jsonl); its cascade folds are
            # checked against fp32 (test_decode_kernel_cascade_fold)
            use_dec = _DECODE_FORCE or getattr(meta, "padded", False) or (
                (4 * ws4.numel() + ws1.numel()) * k_cache.shape[1] * nz
                <= _DECODE_BLOCKS_PER_CU * _num_cus(q.device))
        else:
            use_dec = False
        if use_dec:
            so = torch.empty(nz if nz > 1 else 0, *q.shape, device=q.device, dtype=torch.float32)
            sl = torch.empty(nz if nz > 1 else 0, q.shape[0], q.shape[1], device=q.device,
                             dtype=torch.float32)
            if L.paged_attention_decode(q, k_cache, v_cache, out, meta.q_start, meta.q_len,
                                        meta.ctx_len, meta.block_table, ws4, wq4, ws1, wq1, scale,
                                        nz, so, sl, **kw):
                return out
        if ns > 1 and _MIXED_SPLIT and hasattr(L, "paged_attention_mixed"):
            # split-KV step (few sequences, long own contexts: config 2 / low
            # QPS) in ONE launch: both work lists, the combine fused in
            lists = {nw: (ws, wq) for nw, ws, wq in meta.work_lists()}
            e = torch.empty(0, dtype=torch.int32, device=q.device)
            ws4, wq4 = lists.get(4, (e, e))
            ws1, wq1 = lists.get(1, (e, e))
            so = torch.empty(ns, *q.shape, device=q.device, dtype=torch.float32)
            sl = torch.empty(ns, q.shape[0], q.shape[1], device=q.device, dtype=torch.float32)
            if L.paged_attention_mixed(q, k_cache, v_cache, out, meta.q_start, meta.q_len,
                                       meta.ctx_len, meta.block_table, ws4, wq4, ws1, wq1, scale,
                                       ns, so, sl, **kw):
                if concurrent:
                    main.wait_stream(side)
                    L.cascade_merge(out, kw["own_lse"], pre_o, pre_lse, meta.pre_tokens,
                                    pre_dims=pre_dims)
                return out
        done_nw = ()
        own = int(getattr(meta, "own_tiles", 0))
        if (ns == 1 and _DECODE_OWN and not concurrent and not getattr(meta, "padded", False)
                and own > 0 and hasattr(L, "attn_decode_rel_blocks")):
            # unsplit step on the decode kernel in own-span mode: every item's
            # own key tiles in flight at once (4 waves x 4 tiles per block)
            # instead of one wave walking them (MCP_ATTN_DECODE_OWN: 1 = the
            # 1-wave items, 2 = both lists)
            lists = {nw: (ws, wq) for nw, ws, wq in meta.work_lists()}
            e = torch.empty(0, dtype=torch.int32, device=q.device)
            ws1, wq1 = lists.get(1, (e, e))
            ws4, wq4 = lists.get(4, (e, e)) if _DECODE_OWN == 2 else (e, e)
            if ws1.numel() or ws4.numel():
                nz = L.attn_decode_rel_blocks(own)
                so = torch.empty(nz if nz > 1 else 0, *q.shape, device=q.device, dtype=torch.float32)
                sl = torch.empty(nz if nz > 1 else 0, q.shape[0], q.shape[1], device=q.device,
                                 dtype=torch.float32)
                if L.paged_attention_decode(q, k_cache, v_cache, out, meta.q_start, meta.q_len,
                                            meta.ctx_len, meta.block_table, ws4, wq4, ws1, wq1,
                                            scale, nz, so, sl, own_tiles=own, **kw):
                    done_nw = (1, 4) if _DECODE_OWN == 2 else (1,)
        for nw, ws, wq in meta.work_lists():
            if nw in done_nw:
                continue
            if ns > 1:
                # split-KV (K6): fp32 partials + LSE per split, merged by a second kernel
                so = torch.empty(ns, *q.shape, device=q.device, dtype=torch.float32)
                sl = torch.empty(ns, q.shape[0], q.shape[1], device=q.device, dtype=torch.float32)
                L.paged_attention(q, k_cache, v_cache, out, meta.q_start, meta.q_len,
                                  meta.ctx_len, meta.block_table, ws, wq, nw, scale, nsplit=ns,
                                  split_o=so, split_lse=sl, **kw)
                continue
            L.paged_attention(q, k_cache, v_cache, out, meta.q_start, meta.q_len, meta.ctx_len,
                              meta.block_table, ws, wq, nw, scale, **kw)
        if concurrent:
            main.wait_stream(side)
            L.cascade_merge(out, kw["own_lse"], pre_o, pre_lse, meta.pre_tokens, pre_dims=pre_dims)
        return out
    r = ref.paged_attention(q, k_cache, v_cache, meta.q_start, meta.q_len, meta.ctx_len,
                            meta.block_table, scale)
    return r if out is None else out.copy_(r)


def sample_allowed(hidden, W, allow_ptr, allow_ids, ctr, temperature, seed, out_tok=None,
                   out_logit=None):
    if hidden.is_cuda:
        out_tok = torch.empty(hidden.shape[0], dtype=torch.int32, device=hidden.device) \
            if out_tok is None else out_tok
        lib().sample_allowed(hidden, W, allow_ptr, allow_ids, ctr, temperature, seed, out_tok,
                             out_logit)
        return out_tok
    # CPU: same Gumbel-max semantics with torch's RNG, one stream per (seed, counter)
    toks = []
    for i, (ids, logits) in enumerate(ref.sample_allowed_logits(hidden, W, allow_ptr, allow_ids)):
        if len(ids) == 0:
            toks.append(-1)
            continue
        if temperature > 0:
            g = torch.Generator().manual_seed(int(seed) * 1_000_003 + int(ctr[i]))
            u = torch.rand(logits.shape, generator=g).clamp_(1e-7, 1 - 1e-7)
            sc = logits / temperature - torch.log(-torch.log(u))
        else:
            sc = logits
        toks.append(int(ids[int(torch.argmax(sc))]))
    t = torch.tensor(toks, dtype=torch.int32)
    return t if out_tok is None else out_tok.copy_(t)


def branch_select(prev_tok, tab, n: int, dstep, err):
    """Decision lookahead: write the sampled outcome of each sequence's
    pending choice into ``dstep``'s views (tokens, q_len, ctx_len, logit row,
    allowed set; the rows past the outcome's span lose their KV slot) -
    csrc/sampling.hip ``branch_select_kernel``; ``tab`` is the
    int32 table of engine._launch_branch, already bounded on the host."""
    a = dstep.attn
    if prev_tok.is_cuda:
        lib().branch_select(prev_tok, tab, int(n), dstep.token_ids, dstep.slots, a.q_len, a.ctx_len,
                            dstep.logit_rows, dstep.allow_ptr, dstep.allow_ids, err)
        return
    t = tab.tolist()
    off, chosen = 0, []
    for i in range(n):
        prev, qs, start, L, nb, rec = t[2 + 6 * i: 8 + 6 * i]
        tok = int(prev_tok[prev])
        b = next((b for b in range(nb) if t[rec + b * (4 + L)] == tok), None)
        if b is None:
            err[0] = 1 + i
            b = 0
        r = rec + b * (4 + L)
        ql, aoff, alen = t[r + 1], t[r + 2], t[r + 3]
        a.q_len[i], a.ctx_len[i], dstep.logit_rows[i] = ql, start + ql, qs + ql - 1
        dstep.token_ids[qs:qs + L] = torch.tensor(t[r + 4:r + 4 + L], dtype=torch.int32)
        dstep.slots[qs + ql:qs + L] = -1
        dstep.allow_ptr[i] = off
        dstep.allow_ids[off:off + alen] = torch.tensor(t[aoff:aoff + alen], dtype=torch.int32)
        off += alen
    tail = t[1]
    if not tail:
        dstep.allow_ptr[n:] = off
        return
    nt = t[tail]
    rel = t[tail + 1: tail + 2 + nt]
    for i in range(n, dstep.allow_ptr.numel()):
        dstep.allow_ptr[i] = off + rel[min(i - n, nt)]
    dstep.allow_ids[off:off + rel[nt]] = torch.tensor(t[tail + 2 + nt: tail + 2 + nt + rel[nt]],
                                                      dtype=torch.int32)


def add_inplace(y, x):
    if y.is_cuda:
        lib().add_inplace(y, x)
    else:
        y.add_(x)
    return y


def l2norm_rows(x):
    """In-place row L2 normalisation of a [N, D] bf16 matrix."""
    if x.is_cuda:
        lib().l2norm_rows(x)
    else:
        x.copy_(torch.nn.functional.normalize(x.float(), dim=-1).to(x.dtype))
    return x


FUSED_TOPK_MIN_SCORES = 1 << 27


def topk_cosine(queries, corpus, k: int, seg_len: int = 4096, n_valid: Optional[int] = None,
                fused: Optional[bool] = None):
    """Top-k cosine similarity of unit-norm ``queries`` [B, D] against unit-norm
    ``corpus`` [N, D] (both bf16).  Returns (scores [B, k] f32, index [B, k] int32),
    best first (ties: lower row first).

    GPU, B <= 64, k <= 64, D in {512, 1024}: the fused kernel (csrc/topk.hip
    ``topk_fused``) scores 4096-row segments with MFMA and keeps each
    segment's k best per query in LDS - no [B, N] score matrix, no padding of
    the corpus - then the hierarchical segmented top-k merges the
    ``N / 4096 x k`` candidates.  Other shapes: fp32-output scoring GEMM +
    segmented top-k (the scoring GEMM needs N % 4: such corpora are padded at
    index build, ``retrieval.store``; ``n_valid`` = the real rows, the rest
    are never returned).

    ``fused=None`` picks by size: the fused kernel once the [B, N] fp32 score
    matrix would pass 2^27 entries (512 MB), the GEMM path below that - measured
    on MI355X (profiles/config3_topk.md): 1M x 64 queries 1.56 vs 2.26 ms, 10k
    rows 0.12 vs 0.45-2.1 ms, but 10M x 16 / x 64 4.2 / 5.3 ms fused vs 7.0 /
    14.7 through the score matrix.  True / False force a path."""
    eligible = queries.shape[0] <= 64 and k <= 64 and queries.shape[1] in (512, 1024)
    n_rows = n_valid if n_valid is not None else corpus.shape[0]
    if fused is None:
        # (the GEMM path needs rows % 4: an unpadded corpus stays on the fused kernel)
        fused = queries.shape[0] * n_rows >= FUSED_TOPK_MIN_SCORES or corpus.shape[0] % 4 != 0
    use_fused = fused and eligible
    if n_valid is not None and n_valid < corpus.shape[0] and (not queries.is_cuda or use_fused):
        corpus = corpus[:n_valid]                  # a row prefix: contiguous, no copy
        n_valid = None
    B, N = queries.shape[0], corpus.shape[0]
    k = min(k, N)
    if not queries.is_cuda:
        v, i = torch.topk(queries.float() @ corpus.float().t(), k=k, dim=-1)
        return v, i.int()
    L_ = lib()
    D = queries.shape[1]
    if use_fused:
        nseg = L_.topk_fused_segments(N, queries.shape[0])
        vals = torch.empty(B, nseg * k, device=queries.device, dtype=torch.float32)
        idx = torch.empty(B, nseg * k, device=queries.device, dtype=torch.int32)
        L_.topk_fused(queries.contiguous(), corpus, k, vals, idx)
        L = nseg * k
        if nseg == 1:
            return vals, idx
    else:
        if N % 4:
            # the scoring GEMM writes 16-B column groups: pad a copy (slow path;
            # the indexes pad once at build, retrieval.store / retrieval.sharded)
            corpus = torch.cat([corpus, corpus.new_zeros(4 - N % 4, corpus.shape[1])])
            n_valid = N if n_valid is None else n_valid
            N = corpus.shape[0]
        vals = torch.empty(B, N, device=queries.device, dtype=torch.float32)
        L_.gemm_f32out(queries, corpus, vals)
        if n_valid is not None and n_valid < N:
            vals[:, n_valid:] = float("-inf")
        idx, L = None, N
    while True:
        sl = min(seg_len, max(L, k))
        nseg = (L + sl - 1) // sl
        ov = torch.empty(B, nseg * k, device=queries.device, dtype=torch.float32)
        oi = torch.empty(B, nseg * k, device=queries.device, dtype=torch.int32)
        L_.segment_topk(vals, idx, sl, k, ov, oi)
        vals, idx, L = ov, oi, nseg * k
        if nseg == 1:
            return vals, idx


def copy_blocks(kv_data, src, dst):
    """kv_data [L, 2, nb, Hkv, BS, D]: copy block src[i] -> dst[i] (all layers, K and V)."""
    if kv_data.is_cuda:
        lib().copy_blocks(kv_data, src, dst)
    else:
        keep = (src >= 0) & (dst >= 0)          # negative pairs are padding
        kv_data[:, :, dst[keep].long()] = kv_data[:, :, src[keep].long()]
    return kv_data
