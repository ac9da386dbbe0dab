"""Numerics of every gfx950 HIP kernel against the plain-PyTorch fp32 reference
(SURVEY §4.3.2).  Runs only on a real MI355X (``-m gpu``)."""
import math

import numpy as np
import pytest
import torch

import mcp_amd.ops as ops
from mcp_amd.engine.batch import StepInputs, pack
from mcp_amd.ops import reference as ref

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")]

DEV = "cuda"


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def test_native_library_loaded():
    assert ops.library_path() is not None
    ops.lib()   # raises if the .so cannot be loaded


@pytest.mark.parametrize("T,H", [(1, 4096), (37, 4096), (5, 8192), (3, 256)])
def test_rmsnorm(T, H):
    x = torch.randn(T, H, device=DEV).bfloat16()
    w = (torch.rand(H, device=DEV) + 0.5).bfloat16()
    out = ops.rmsnorm(x, w, 1e-5)
    assert rel_err(out, ref.rmsnorm(x, w, 1e-5)) < 1e-2
    r = torch.randn(T, H, device=DEV).bfloat16()
    r_ref = r.clone()
    out2 = ops.add_rmsnorm(x, r, w, 1e-5)
    exp = ref.add_rmsnorm(x, r_ref, w, 1e-5)
    assert rel_err(r, r_ref) < 1e-2 and rel_err(out2, exp) < 1e-2


def test_silu_mul_embedding_add():
    x = torch.randn(19, 2 * 1024, device=DEV).bfloat16()
    assert rel_err(ops.silu_mul(x), ref.silu_mul(x)) < 1e-2
    table = torch.randn(1000, 512, device=DEV).bfloat16()
    ids = torch.randint(0, 1000, (33,), device=DEV, dtype=torch.int32)
    assert torch.equal(ops.embedding(ids, table), table[ids.long()])
    y = torch.randn(64, 64, device=DEV).bfloat16()
    y0 = y.clone()
    z = torch.randn(64, 64, device=DEV).bfloat16()
    ops.add_inplace(y, z)
    assert rel_err(y, y0.float() + z.float()) < 1e-2


@pytest.mark.parametrize("M,N,K", [(1, 128, 64), (17, 384, 256), (128, 128, 4096), (300, 1024, 512),
                                   (1000, 6144, 4096), (64, 1284, 128), (4096, 4096, 4096)])
def test_gemm(M, N, K):
    torch.manual_seed(0)
    X = torch.randn(M, K, device=DEV).bfloat16()
    W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    Y = ops.gemm(X, W)
    assert rel_err(Y, ref.gemm(X, W)) < 1e-2
    R = torch.randn(M, N, device=DEV).bfloat16()
    Y2 = ops.gemm(X, W, R=R)
    assert rel_err(Y2, ref.gemm(X, W, R)) < 1e-2


@pytest.mark.parametrize("M,N,K", [(1, 384, 256), (77, 1028, 512), (300, 6144, 4096), (1000, 4096, 1024),
                                   (513, 640, 14336)])
def test_gemm_flex_tiles(M, N, K):
    """Every flex tile (gemm_flex.hip), 2- and 4-stage forms, plain and
    + residual, against fp32 - ragged M / N edges included."""
    torch.manual_seed(11)
    L = ops.lib()
    X = torch.randn(M, K, device=DEV).bfloat16()
    W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    R = torch.randn(M, N, device=DEV).bfloat16()
    exp = ref.gemm(X, W)
    exp_r = ref.gemm(X, W, R)
    for c in list(range(L.gemm_flex_count())) + [32 + c for c in range(L.gemm_flex_count())]:
        Y = torch.full((M, N), float("nan"), device=DEV).bfloat16()
        L.gemm(X, W, Y, None, 16 + c)
        assert rel_err(Y, exp) < 1e-2, c
        L.gemm(X, W, Y, R, 16 + c)
        assert rel_err(Y, exp_r) < 1e-2, c


def test_gemm_plan_flex_dispatch():
    """A plan that names a flex tile for a bucket routes ops.gemm there."""
    L = ops.lib()
    M, N, K = 320, 640, 512
    X = torch.randn(M, K, device=DEV).bfloat16()
    W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    try:
        L.gemm_plan_set(N, K, [0] * 8)
        L.gemm_plan_set_flex(N, K, [-1] * 4 + [32 + 4] * 4)
        assert L.gemm_plan_flex(M, N, K) == 36 and L.gemm_plan_flex(200, N, K) == -1
        assert rel_err(ops.gemm(X, W), ref.gemm(X, W)) < 1e-2
    finally:
        L.gemm_plan_clear()
        ops._load_gemm_plan(L)


@pytest.mark.parametrize("M,K", [(100, 512), (320, 1792)])
def test_gemm_plan_fsplit_dispatch(M, K):
    """A plan "fsplit" entry (flex tile x split-K: fp32 partials + the reduce)
    routes ops.gemm there; every tile and split, plain and residual + the
    fused-norm statistic, against fp32 (ragged M tiles included)."""
    torch.manual_seed(29)
    L = ops.lib()
    N = 768
    X = torch.randn(M, K, device=DEV).bfloat16()
    W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    R = torch.randn(M, N, device=DEV).bfloat16()
    try:
        for c in range(14):
            for S in (2, 4, 7):
                if (K // 64) % S:
                    continue
                fs = 16 * c + S
                L.gemm_plan_set(N, K, [0] * 8)
                L.gemm_plan_set_fsplit(N, K, [fs] * 8)
                assert L.gemm_plan_fsplit(M, N, K) == fs
                assert rel_err(ops.gemm(X, W), ref.gemm(X, W)) < 1e-2, fs
                y = R.clone()
                ss = torch.zeros(M, dtype=torch.int64, device=DEV)
                ops.gemm(X, W, R=y, out=y, ss_out=ss)
                assert rel_err(y, ref.gemm(X, W, R)) < 1e-2, fs
                exp = y.float().pow(2).sum(-1) * ref.SS_FIX
                assert ((ss.double() - exp.double()).abs() / exp.double()).max().item() < 1e-5, fs
    finally:
        L.gemm_plan_clear()
        ops._load_gemm_plan(L)


def test_gemm_orientation_exact():
    # A = I, asymmetric B: catches a transposed C-write (cdna_hip_programming.md §3)
    K = 128
    X = torch.eye(K, device=DEV).bfloat16()
    W = torch.arange(K * K, device=DEV).reshape(K, K).remainder(97).bfloat16()
    Y = ops.gemm(X, W)
    assert torch.equal(Y.float(), W.t().float())


def _cache(nb, Hkv, D=128, BS=64):
    k = torch.randn(nb, Hkv, BS, D, device=DEV).bfloat16()
    v = torch.randn(nb, Hkv, BS, D, device=DEV).bfloat16()
    return k, v


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1), (8, 8), (16, 8)])
def test_rope_kv(Hq, Hkv):
    D, T = 128, 45
    cs = ref.rope_cos_sin(4096, D, 500000.0, DEV)
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=DEV).bfloat16()
    pos = torch.randint(0, 4000, (T,), device=DEV, dtype=torch.int32)
    slots = torch.randperm(8 * 64, device=DEV)[:T].int()
    slots[3] = -1
    kc, vc = _cache(8, Hkv)
    kc2, vc2 = kc.clone(), vc.clone()
    q1 = torch.empty(T, Hq, D, device=DEV).bfloat16()
    q2 = q1.clone()
    ops.rope_kv(qkv, pos, slots, cs, q1, kc, vc, Hq, Hkv, D)
    ref.rope_kv(qkv.cpu(), pos.cpu(), slots.cpu(), cs.cpu(), q2_cpu := q2.cpu(), kc2_cpu := kc2.cpu(),
                vc2_cpu := vc2.cpu(), Hq, Hkv, D)
    assert rel_err(q1.cpu(), q2_cpu) < 1e-2
    assert rel_err(kc.cpu(), kc2_cpu) < 1e-2
    assert torch.equal(vc.cpu(), vc2_cpu)


def _attn_case(q_lens, ctx_lens, Hq, Hkv, seed=0, kv_splits=1):
    torch.manual_seed(seed)
    D, BS = 128, 64
    S = len(q_lens)
    nblk = [(c + BS - 1) // BS for c in ctx_lens]
    nb = sum(nblk) + 3
    kc, vc = _cache(nb, Hkv)
    perm = torch.randperm(nb).tolist()
    maxb = max(nblk)
    bt = np.zeros((S, maxb), np.int32)
    o = 0
    for s in range(S):
        bt[s, :nblk[s]] = perm[o:o + nblk[s]]
        o += nblk[s]
    T = sum(q_lens)
    q = torch.randn(T, Hq, D, device=DEV).bfloat16()
    qs = np.concatenate([[0], np.cumsum(q_lens)[:-1]]).astype(np.int32)
    step = StepInputs(token_ids=np.zeros(T, np.int32), positions=np.zeros(T, np.int32),
                      slots=np.zeros(T, np.int32), q_start=qs,
                      q_len=np.asarray(q_lens, np.int32), ctx_len=np.asarray(ctx_lens, np.int32),
                      block_table=bt, logit_rows=np.zeros(0, np.int32))
    dev = pack(step, Hq // Hkv, DEV)
    dev.attn.kv_splits = kv_splits
    out = ops.paged_attention(q, kc, vc, dev.attn, 1 / math.sqrt(D))
    exp = ref.paged_attention(q.cpu(), kc.cpu(), vc.cpu(), torch.from_numpy(qs),
                              torch.tensor(q_lens), torch.tensor(ctx_lens), torch.from_numpy(bt),
                              1 / math.sqrt(D))
    return out.cpu(), exp


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1), (8, 8)])
def test_paged_attention_mixed(Hq, Hkv):
    q_lens = [1, 1, 7, 130, 64, 3, 1]
    ctx_lens = [1, 900, 200, 130, 700, 64, 65]
    out, exp = _attn_case(q_lens, ctx_lens, Hq, Hkv)
    assert rel_err(out, exp) < 2e-2
    assert torch.isfinite(out.float()).all()


@pytest.mark.parametrize("ctx", [8192, 32768, 131072])
@pytest.mark.parametrize("batch", [1, 4])
def test_paged_attention_split_kv_long_context(ctx, batch):
    """Split-KV decode (K6): 1-wave items whose key range is split over
    workgroups (fp32 partials + LSE, merged by attn_split_combine), at 8k-128k
    contexts, batch 1 and 4 (one decode token each, plus a 3-token
    jump-forward span), against fp32; the engine's split rule too."""
    from mcp_amd.engine.batch import choose_kv_splits
    q_lens = [1] * batch
    q_lens[-1] = 3
    ctx_lens = [ctx - 37 * i for i in range(batch)]
    ns = choose_kv_splits(q_lens, ctx_lens, 4, 8, hq=32)
    assert ns > 1
    out, exp = _attn_case(q_lens, ctx_lens, 32, 8, seed=6, kv_splits=ns)
    assert rel_err(out, exp) < 2e-2
    assert torch.isfinite(out.float()).all()


def test_paged_attention_split_kv_uneven():
    """Split counts that do not divide the tiles, splits with no tiles (short
    contexts), 4-wave items (jump-forward spans, 70 tokens) split too."""
    for ns in (3, 7, 32):
        out, exp = _attn_case([1, 1, 1, 70, 2], [5000, 65, 900, 700, 64], 32, 8, seed=7, kv_splits=ns)
        assert rel_err(out, exp) < 2e-2
    for ns in (2, 5):                     # only 4-wave items, one sequence, 1k-4k keys
        out, exp = _attn_case([12, 30], [1000, 4100], 32, 8, seed=8, kv_splits=ns)
        assert rel_err(out, exp) < 2e-2


@pytest.mark.parametrize("mixed", [True, False])
def test_paged_attention_split_fused_vs_per_list(mixed, monkeypatch):
    """Split-KV step as ONE launch (both work lists, last-arriver combine fused,
    ops._MIXED_SPLIT) and as per-list launches + attn_split_combine: both match
    fp32, and repeated launches re-arm the arrival tickets (same output)."""
    monkeypatch.setattr(ops, "_MIXED_SPLIT", mixed)
    monkeypatch.setattr(ops, "_DECODE_SPLIT", False)
    q_lens, ctx_lens = [1, 3, 9, 70, 2], [5000, 65, 900, 700, 1200]
    outs = []
    for _ in range(3):
        out, exp = _attn_case(q_lens, ctx_lens, 32, 8, seed=9, kv_splits=6)
        assert rel_err(out, exp) < 2e-2
        outs.append(out)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])
    for Hq, Hkv in ((8, 1), (64, 8)):             # GQA groups 8 (70B TP=8 / TP=1)
        out, exp = _attn_case([1, 5], [3000, 800], Hq, Hkv, seed=10, kv_splits=4)
        assert rel_err(out, exp) < 2e-2


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1), (64, 8), (8, 8), (16, 8)])
def test_paged_attention_decode_kernel(Hq, Hkv, monkeypatch):
    """Split-KV steps on the decode kernel (csrc/attention_decode.hip: key
    tiles fixed by the grid position, 4 waves on 4 tiles, LDS merge of the
    waves, last-arriver merge of the blocks) against fp32: single sequences
    with 1-16 new tokens over 64-4100 keys (one block / several blocks / one
    tile past a block edge), narrow and wide items in one launch, a 70-token
    span (5 wide items), tables wider than 256 blocks (several tiles per
    wave), and bitwise-equal repeats (the arrival tickets re-arm)."""
    monkeypatch.setattr(ops, "_DECODE_SPLIT", True)
    monkeypatch.setattr(ops, "_DECODE_BLOCKS_PER_CU", 1 << 20)   # no fallback by grid size
    cases = [([1], [64]), ([1], [700]), ([4], [1100]), ([16], [1025]), ([3], [4100]),
             ([1, 3, 9, 70, 2], [5000, 65, 900, 700, 1200]), ([12, 1], [257, 16500])]
    for i, (q_lens, ctx_lens) in enumerate(cases):
        outs = []
        for _ in range(2):
            out, exp = _attn_case(q_lens, ctx_lens, Hq, Hkv, seed=20 + i, kv_splits=2)
            assert rel_err(out, exp) < 2e-2, (q_lens, ctx_lens)
            assert torch.isfinite(out.float()).all()
            outs.append(out)
        assert torch.equal(outs[0], outs[1]), (q_lens, ctx_lens)


def test_paged_attention_spike():
    # a single large score forces the online-softmax rescale path (rule 26)
    out, exp = _attn_case([40], [300], 32, 8, seed=3)
    assert rel_err(out, exp) < 2e-2


def test_sample_allowed_greedy_and_distribution():
    torch.manual_seed(0)
    S, H, V = 6, 4096, 2000
    hidden = torch.randn(S, H, device=DEV).bfloat16()
    W = (torch.randn(V, H, device=DEV) * 0.02).bfloat16()
    allowed = [torch.randperm(V)[:n].tolist() for n in (1, 2, 5, 17, 64, 300)]
    ptr = np.cumsum([0] + [len(a) for a in allowed]).astype(np.int32)
    ids = torch.tensor(sum(allowed, []), dtype=torch.int32, device=DEV)
    ptr_t = torch.from_numpy(ptr).to(DEV)
    ctr = torch.arange(S, dtype=torch.int32, device=DEV)
    tok = ops.sample_allowed(hidden, W, ptr_t, ids, ctr, 0.0, 1234)
    for s, (aid, logits) in enumerate(ref.sample_allowed_logits(hidden.cpu(), W.cpu(), ptr, ids.cpu())):
        assert int(tok[s]) == int(aid[int(torch.argmax(logits))])
    # temperature sampling follows softmax(logits / T) over the allowed set
    s = 3
    T = 0.5
    aid, logits = ref.sample_allowed_logits(hidden.cpu(), W.cpu(), ptr, ids.cpu())[s]
    p = torch.softmax(logits / T, dim=0)
    counts = torch.zeros(len(aid))
    pos = {int(t): i for i, t in enumerate(aid)}
    h1 = hidden[s:s + 1].contiguous()
    p1 = torch.tensor([0, len(aid)], dtype=torch.int32, device=DEV)
    ids1 = aid.int().to(DEV)
    N = 4000
    for i in range(N // 200):
        hh = h1.expand(200, H).contiguous()
        pp = torch.arange(0, 201, dtype=torch.int32, device=DEV) * 0
        ptr_b = torch.tensor(np.arange(201) * len(aid), dtype=torch.int32, device=DEV)
        ids_b = ids1.repeat(200)
        c = torch.arange(i * 200, (i + 1) * 200, dtype=torch.int32, device=DEV)
        t = ops.sample_allowed(hh, W, ptr_b, ids_b, c, T, 99)
        for x in t.cpu().tolist():
            counts[pos[x]] += 1
    freq = counts / counts.sum()
    assert (freq - p).abs().max().item() < 0.05


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (300, 512, 192), (1000, 6144, 4096), (513, 1028, 256)])
def test_gemm_256_tile(M, N, K):
    torch.manual_seed(1)
    X = torch.randn(M, K, device=DEV).bfloat16()
    W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    assert rel_err(ops.gemm(X, W, algo=1), ref.gemm(X, W)) < 1e-2
    R = torch.randn(M, N, device=DEV).bfloat16()
    assert rel_err(ops.gemm(X, W, R=R, algo=1), ref.gemm(X, W, R)) < 1e-2
    # in-place residual (out aliases R), as the model's Wo / Wdown use it
    R2 = R.clone()
    ops.gemm(X, W, R=R2, out=R2, algo=1)
    assert rel_err(R2, ref.gemm(X, W, R)) < 1e-2


def test_copy_blocks():
    data = torch.randn(3, 2, 10, 2, 64, 128, device=DEV).bfloat16()
    exp = data.clone()
    src = torch.tensor([1, 4], dtype=torch.int32, device=DEV)
    dst = torch.tensor([7, 2], dtype=torch.int32, device=DEV)
    ops.copy_blocks(data, src, dst)
    exp[:, :, [7, 2]] = exp[:, :, [1, 4]]
    assert torch.equal(data, exp)


@pytest.mark.parametrize("B,N,D,k", [(1, 10000, 1024, 32), (4, 70000, 256, 64), (3, 50, 128, 8),
                                     (64, 1_000_003, 1024, 32), (16, 300001, 512, 64),
                                     (5, 4095, 1024, 10), (64, 4097, 1024, 64), (17, 9000, 1024, 1),
                                     (33, 20000, 512, 64)])
@pytest.mark.parametrize("fused", [True, None])
def test_topk_cosine(B, N, D, k, fused):
    """Fused scoring + per-segment top-k (B <= 64, D in {512, 1024}) and the
    unfused GEMM path (other D; corpus padded to a multiple of 4 once, the pad
    rows never returned): values equal torch's top-k, indices point at rows
    with those scores (ties may pick another row), best first."""
    torch.manual_seed(2)
    Np = (N + 3) // 4 * 4 if D not in (512, 1024) else N
    corpus = torch.randn(Np, D, device=DEV).bfloat16()
    corpus[N:] = 0
    ops.l2norm_rows(corpus)
    q = torch.randn(B, D, device=DEV).bfloat16()
    ops.l2norm_rows(q)
    vals, idx = ops.topk_cosine(q, corpus, k, n_valid=N, fused=fused)
    corpus = corpus[:N]
    assert int(idx.max()) < N and int(idx.min()) >= 0
    ref_s = q.float() @ corpus.float().t()
    rv, ri = torch.topk(ref_s, k=min(k, N), dim=-1)
    assert torch.allclose(vals, rv, atol=1e-4)
    # indices may differ only where scores tie
    got = ref_s.gather(1, idx.long())
    assert torch.allclose(got, rv, atol=1e-4)
    assert (vals[:, :-1] >= vals[:, 1:]).all()


@pytest.mark.parametrize("B,N,D", [(70, 1001, 1024), (3, 4099, 256)])
def test_topk_cosine_unpadded_corpus_unfused(B, N, D):
    """The unfused scoring path (B > 64, or D outside {512, 1024}) on a corpus
    whose row count is not a multiple of 4 pads a copy instead of raising."""
    torch.manual_seed(3)
    corpus = torch.randn(N, D, device=DEV).bfloat16()
    ops.l2norm_rows(corpus)
    q = torch.randn(B, D, device=DEV).bfloat16()
    ops.l2norm_rows(q)
    vals, idx = ops.topk_cosine(q, corpus, 16, fused=False)
    assert int(idx.max()) < N and int(idx.min()) >= 0
    ref_s = q.float() @ corpus.float().t()
    rv, _ = torch.topk(ref_s, k=16, dim=-1)
    assert torch.allclose(vals, rv, atol=1e-4)
    assert torch.allclose(ref_s.gather(1, idx.long()), rv, atol=1e-4)


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1)])
@pytest.mark.parametrize("kv_splits", [1, 4])
@pytest.mark.parametrize("prefix_split", ["0", "-1", "3"])
@pytest.mark.parametrize("concurrent", ["0", "1"])
def test_cascade_prefix_attention(Hq, Hkv, kv_splits, prefix_split, concurrent, monkeypatch):
    """Shared-prefix pass + per-sequence pass with LSE merge == full attention
    (also with split-KV: split 0 folds the prefix partial in; with the prefix
    pass itself split over its key tiles + merged: off / auto / 3; and with
    the prefix pass on a side stream concurrent with the own-key pass, the
    two partials merged afterwards)."""
    monkeypatch.setenv("MCP_PREFIX_SPLIT", prefix_split)
    monkeypatch.setenv("MCP_ATTN_CONCURRENT", concurrent)
    torch.manual_seed(5)
    D, BS = 128, 64
    P_full = 640                                   # 10 shared blocks
    q_lens = [1, 5, 17, 2, 40]
    own_keys = [70, 5, 130, 64, 300]               # keys after the shared prefix
    ctx = [P_full + k for k in own_keys]
    n_pre = P_full // BS
    own_blocks = [(k + BS - 1) // BS for k in own_keys]
    nb = n_pre + sum(own_blocks) + 2
    kc, vc = _cache(nb, Hkv)
    pre = list(range(n_pre))
    o = n_pre
    tables = []
    for nbk in own_blocks:
        tables.append(pre + list(range(o, o + nbk)))
        o += nbk
    maxb = max(len(t) for t in tables)
    bt = np.zeros((len(q_lens), maxb), np.int32)
    for i, t in enumerate(tables):
        bt[i, :len(t)] = t
    T = sum(q_lens)
    q = torch.randn(T, Hq, D, device=DEV).bfloat16()
    qs = np.concatenate([[0], np.cumsum(q_lens)[:-1]]).astype(np.int32)
    step = StepInputs(token_ids=np.zeros(T, np.int32), positions=np.zeros(T, np.int32),
                      slots=np.zeros(T, np.int32), q_start=qs,
                      q_len=np.asarray(q_lens, np.int32), ctx_len=np.asarray(ctx, np.int32),
                      block_table=bt, logit_rows=np.zeros(0, np.int32),
                      kv_begin=np.full(len(q_lens), P_full, np.int32),
                      pre_bt=np.asarray(pre, np.int32), pre_tokens=T)
    dev = pack(step, Hq // Hkv, DEV)
    dev.attn.kv_splits = kv_splits
    assert dev.attn.pre_tokens == T and dev.attn.pre_keys == P_full
    out = ops.paged_attention(q, kc, vc, dev.attn, 1 / math.sqrt(D)).cpu()
    exp = ref.paged_attention(q.cpu(), kc.cpu(), vc.cpu(), torch.from_numpy(qs),
                              torch.tensor(q_lens), torch.tensor(ctx), torch.from_numpy(bt),
                              1 / math.sqrt(D))
    assert rel_err(out, exp) < 2e-2


@pytest.mark.parametrize("own_keys,q_lens", [([5], [1]), ([40, 60], [3, 1]),
                                              ([70], [4]), ([300, 130, 64], [1, 9, 2])])
def test_decode_kernel_cascade_fold(own_keys, q_lens, monkeypatch):
    """the decode kernel (attention_decode.hip, forced, as
    graph-replayed split steps take it) with cascade inputs - every sequence
    after a 640-key shared prefix (kv_begin), the prefix partial (pre_o /
    pre_lse) folded in - against fp32 full attention: own key spans of one
    block (the single-block fold, nact == 1) and of several blocks (the
    last-arriver fold)."""
    monkeypatch.setattr(ops, "_DECODE_SPLIT", True)
    monkeypatch.setattr(ops, "_DECODE_FORCE", True)
    monkeypatch.setenv("MCP_ATTN_CONCURRENT", "0")
    torch.manual_seed(31)
    Hq, Hkv, D, BS, P_full = 32, 8, 128, 64, 640
    ctx = [P_full + k for k in own_keys]
    n_pre = P_full // BS
    own_blocks = [(k + BS - 1) // BS for k in own_keys]
    nb = n_pre + sum(own_blocks) + 2
    kc, vc = _cache(nb, Hkv)
    pre = list(range(n_pre))
    o = n_pre
    tables = []
    for nbk in own_blocks:
        tables.append(pre + list(range(o, o + nbk)))
        o += nbk
    bt = np.zeros((len(q_lens), max(len(t) for t in tables)), np.int32)
    for i, t in enumerate(tables):
        bt[i, :len(t)] = t
    T = sum(q_lens)
    q = torch.randn(T, Hq, D, device=DEV).bfloat16()
    qs = np.concatenate([[0], np.cumsum(q_lens)[:-1]]).astype(np.int32)
    step = StepInputs(token_ids=np.zeros(T, np.int32), positions=np.zeros(T, np.int32),
                      slots=np.zeros(T, np.int32), q_start=qs,
                      q_len=np.asarray(q_lens, np.int32), ctx_len=np.asarray(ctx, np.int32),
                      block_table=bt, logit_rows=np.zeros(0, np.int32),
                      kv_begin=np.full(len(q_lens), P_full, np.int32),
                      pre_bt=np.asarray(pre, np.int32), pre_tokens=T)
    dev = pack(step, Hq // Hkv, DEV)
    dev.attn.kv_splits = 2
    exp = ref.paged_attention(q.cpu(), kc.cpu(), vc.cpu(), torch.from_numpy(qs),
                              torch.tensor(q_lens), torch.tensor(ctx), torch.from_numpy(bt),
                              1 / math.sqrt(D))
    outs = []
    for _ in range(2):                                  # the arrival tickets re-arm
        out = ops.paged_attention(q, kc, vc, dev.attn, 1 / math.sqrt(D)).cpu()
        assert rel_err(out, exp) < 2e-2, (own_keys, q_lens)
        outs.append(out)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1), (16, 8)])
@pytest.mark.parametrize("T", [1, 77, 300, 2100])
@pytest.mark.parametrize("rt", ["1", "2", "4"])
def test_prefix_pass_row_tile_forms(Hq, Hkv, T, rt, monkeypatch):
    """The shared-prefix pass alone (normalised O and its log2-sum-exp over
    the prefix keys) in every row-tile form (1 = MODE 1 of attn_kernel, 2 / 4
    = attn_prefix_kernel: each LDS fragment feeds 2 / 4 row tiles) against
    fp32 softmax attention; T covers partial row tiles and blocks, and 2100
    tokens over 8 kv heads the 8-wave grid (the 4-wave one below a block per CU)."""
    monkeypatch.setenv("MCP_ATTN_PREFIX_RT", rt)
    torch.manual_seed(11)
    D, P = 128, 640
    n_pre = P // 64
    kc, vc = _cache(n_pre + 3, Hkv)
    pre_bt = torch.tensor([2, 0, 5, 1, 3, 4, 6, 8, 7, 9][:n_pre], dtype=torch.int32, device=DEV)
    q = torch.randn(T, Hq, D, device=DEV).bfloat16()
    out = torch.empty_like(q)
    lse = torch.empty(T, Hq, device=DEV, dtype=torch.float32)
    scale = 1 / math.sqrt(D)
    ops.lib().prefix_attention(q, kc, vc, out, lse, pre_bt, P, T, scale)
    G = Hq // Hkv
    k = kc[pre_bt.long()].float().permute(1, 0, 2, 3).reshape(Hkv, P, D)      # [Hkv, P, D]
    v = vc[pre_bt.long()].float().permute(1, 0, 2, 3).reshape(Hkv, P, D)
    qf = q.float().view(T, Hkv, G, D)
    s = torch.einsum("thgd,hpd->thgp", qf, k) * scale
    exp_o = torch.einsum("thgp,hpd->thgd", torch.softmax(s, -1), v).reshape(T, Hq, D)
    exp_lse = (torch.logsumexp(s, -1) / math.log(2)).reshape(T, Hq)
    assert rel_err(out, exp_o) < 2e-2
    assert torch.allclose(lse, exp_lse, atol=2e-2, rtol=1e-3)


@pytest.mark.parametrize("T,P", [(2100, 640), (4096, 704), (2500, 64)])
def test_prefix_pass_ping_pong_form(T, P, monkeypatch):
    """MCP_ATTN_PREFIX_PP=1: the 8-wave prefix pass with its two wave groups
    half a phase apart (3-slot K|V ring) gives the same bits as the lock-step
    form - every lane runs the same operations in the same order - and
    matches fp32 softmax attention.  T >= 2048 tokens over 8 kv heads takes
    the 8-wave grid; P = 64 is a one-tile prefix (group B only in its tail)."""
    monkeypatch.setenv("MCP_ATTN_PREFIX_RT", "2")
    torch.manual_seed(13)
    Hq, Hkv, D = 32, 8, 128
    n_pre = P // 64
    kc, vc = _cache(n_pre + 2, Hkv)
    pre_bt = torch.randperm(n_pre + 2, device=DEV)[:n_pre].to(torch.int32)
    q = torch.randn(T, Hq, D, device=DEV).bfloat16()
    scale = 1 / math.sqrt(D)
    outs = []
    for pp in ("0", "1"):
        monkeypatch.setenv("MCP_ATTN_PREFIX_PP", pp)
        out = torch.empty_like(q)
        lse = torch.empty(T, Hq, device=DEV, dtype=torch.float32)
        ops.lib().prefix_attention(q, kc, vc, out, lse, pre_bt, P, T, scale)
        torch.cuda.synchronize()
        outs.append((out, lse))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    G = Hq // Hkv
    k = kc[pre_bt.long()].float().permute(1, 0, 2, 3).reshape(Hkv, P, D)
    v = vc[pre_bt.long()].float().permute(1, 0, 2, 3).reshape(Hkv, P, D)
    s = torch.einsum("thgd,hpd->thgp", q.float().view(T, Hkv, G, D), k) * scale
    exp_o = torch.einsum("thgp,hpd->thgd", torch.softmax(s, -1), v).reshape(T, Hq, D)
    assert rel_err(outs[1][0], exp_o) < 2e-2


@pytest.mark.parametrize("T,P", [(300, 704), (2100, 640), (4096, 704)])
def test_prefix_pass_conflict_free_image(T, P, monkeypatch):
    """MCP_ATTN_PREFIX_SWZ=1: the prefix pass's K|V image swizzled chunk ^
    ((row & 7) << 1) (conflict-free transposed V reads) gives the same bits as
    the chunk ^ (row & 15) image - only addresses change - in the 4- and
    8-wave lock-step forms, and matches fp32 attention."""
    monkeypatch.setenv("MCP_ATTN_PREFIX_RT", "2")
    torch.manual_seed(17)
    Hq, Hkv, D = 32, 8, 128
    n_pre = P // 64
    kc, vc = _cache(n_pre + 2, Hkv)
    pre_bt = torch.randperm(n_pre + 2, device=DEV)[:n_pre].to(torch.int32)
    q = torch.randn(T, Hq, D, device=DEV).bfloat16()
    scale = 1 / math.sqrt(D)
    outs = []
    for sw in ("0", "1"):
        monkeypatch.setenv("MCP_ATTN_PREFIX_SWZ", sw)
        out = torch.empty_like(q)
        lse = torch.empty(T, Hq, device=DEV, dtype=torch.float32)
        ops.lib().prefix_attention(q, kc, vc, out, lse, pre_bt, P, T, scale)
        torch.cuda.synchronize()
        outs.append((out, lse))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    G = Hq // Hkv
    k = kc[pre_bt.long()].float().permute(1, 0, 2, 3).reshape(Hkv, P, D)
    v = vc[pre_bt.long()].float().permute(1, 0, 2, 3).reshape(Hkv, P, D)
    s_ = torch.einsum("thgd,hpd->thgp", q.float().view(T, Hkv, G, D), k) * scale
    exp_o = torch.einsum("thgp,hpd->thgd", torch.softmax(s_, -1), v).reshape(T, Hq, D)
    assert rel_err(outs[1][0], exp_o) < 2e-2


@pytest.fixture
def lazy_rescale():
    """Switch the prefix pass's lazy max rescaling; restored afterwards."""
    def set_(on):
        ops.lib().attn_lazy_rescale(int(on))
    yield set_
    ops.lib().attn_lazy_rescale(-1)


@pytest.mark.parametrize("lazy", [0, 1])
@pytest.mark.parametrize("rt", ["1", "2", "4"])
def test_prefix_pass_growing_max(rt, lazy, monkeypatch, lazy_rescale):
    """Keys whose scale grows tile by tile (the online-softmax max jumps by
    large and small amounts between tiles): O and LSE still match fp32
    softmax attention - also with lazy rescaling (the max and the O / sum
    rescale held back while it grows by <= 2^8; rt 2 / 4 = attn_prefix_kernel)."""
    monkeypatch.setenv("MCP_ATTN_PREFIX_RT", rt)
    lazy_rescale(lazy)
    torch.manual_seed(12)
    Hq, Hkv, D, P, T = 32, 8, 128, 768, 200
    n_pre = P // 64
    kc, vc = _cache(n_pre, Hkv)
    ramp = torch.tensor([0.5, 4.0, 1.0, 8.0, 8.5, 2.0, 16.0, 3.0, 16.5, 30.0, 1.0, 31.0],
                        device=DEV)[:n_pre]
    kc = (kc.float() * ramp.view(-1, 1, 1, 1)).bfloat16()
    pre_bt = torch.arange(n_pre, dtype=torch.int32, device=DEV)
    q = torch.randn(T, Hq, D, device=DEV).bfloat16()
    out = torch.empty_like(q)
    lse = torch.empty(T, Hq, device=DEV, dtype=torch.float32)
    scale = 1 / math.sqrt(D)
    ops.lib().prefix_attention(q, kc, vc, out, lse, pre_bt, P, T, scale)
    G = Hq // Hkv
    k = kc.float().permute(1, 0, 2, 3).reshape(Hkv, P, D)
    v = vc.float().permute(1, 0, 2, 3).reshape(Hkv, P, D)
    s = torch.einsum("thgd,hpd->thgp", q.float().view(T, Hkv, G, D), k) * scale
    exp_o = torch.einsum("thgp,hpd->thgd", torch.softmax(s, -1), v).reshape(T, Hq, D)
    exp_lse = (torch.logsumexp(s, -1) / math.log(2)).reshape(T, Hq)
    assert rel_err(out, exp_o) < 2e-2
    assert torch.allclose(lse, exp_lse, atol=5e-2, rtol=1e-3)


@pytest.mark.parametrize("M,F,K", [(7, 512, 256), (300, 1792, 4096), (3000, 14336, 4096), (520, 3584, 1024)])
def test_gemm_silu_fused(M, F, K):
    torch.manual_seed(3)
    X = torch.randn(M, K, device=DEV).bfloat16()
    g = (torch.randn(F, K, device=DEV) / math.sqrt(K)).bfloat16()
    u = (torch.randn(F, K, device=DEV) / math.sqrt(K)).bfloat16()
    W = ref.interleave_gate_up(g, u).contiguous()
    y = ops.gemm_silu(X, W)
    exp = (torch.nn.functional.silu(X.float() @ g.float().t()) * (X.float() @ u.float().t()))
    assert rel_err(y, exp) < 2e-2


@pytest.mark.parametrize("M", [100, 200, 330])
def test_gemm_silu_every_path(M):
    """Every SwiGLU path the "silu" plan can name (launch_gemm_silu_algo: AGPR
    heights, 128^2 x split-K, stream, flex tiles, flex x split-K) against fp32,
    with the fused-norm statistic applied (rows scaled by rsqrt(mean x^2 + eps))."""
    torch.manual_seed(5)
    L = ops.lib()
    F, K = 1792, 4096
    X = torch.randn(M, K, device=DEV).bfloat16()
    g = (torch.randn(F, K, device=DEV) / math.sqrt(K)).bfloat16()
    u = (torch.randn(F, K, device=DEV) / math.sqrt(K)).bfloat16()
    W = ref.interleave_gate_up(g, u).contiguous()
    eps = 1e-5
    ss = (X.float().pow(2).sum(-1) * (1 << 20)).round().to(torch.int64)
    rs = torch.rsqrt(ss.double() / (1 << 20) / K + eps).float()[:, None]
    exp = torch.nn.functional.silu((X.float() @ g.float().t()) * rs) * ((X.float() @ u.float().t()) * rs)
    algos = [1, 2, 3, 4, 5, 101, 102, 104, 200, 400, 401, 402, 403, 404, 405]
    algos += [300 + f for f in range(L.gemm_flex_count()) if L.gemm_flex_silu_ok(f)]
    algos += [1000 + 16 * c + S for c in (0, 6, 10) for S in (2, 4)]
    ran = 0
    for a in algos:
        Y = torch.full((M, F), float("nan"), device=DEV, dtype=torch.bfloat16)
        if L.gemm_silu_algo(X, W, Y, a, ss, eps):
            continue                                   # path does not take this shape
        torch.cuda.synchronize()
        assert rel_err(Y, exp) < 2e-2, a
        ran += 1
    assert ran >= 10


@pytest.mark.parametrize("M,N,K", [(3584, 6144, 4096), (3584, 4096, 14336), (1000, 1024, 4096),
                                   (700, 520, 320)])
def test_gemm_stream_k(M, N, K):
    """Stream-K hybrid (partial tiles reduced by the last-arriving workgroup)
    against fp32, forced and auto-selected, plain / ping-pong / residual / SwiGLU."""
    torch.manual_seed(4)
    L = ops.lib()
    X = torch.randn(M, K, device=DEV).bfloat16()
    W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    exp = ref.gemm(X, W)
    for v in (31, 33, 32, 30):
        Y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        L.gemm_variant(X, W, Y, v)
        assert rel_err(Y, exp) < 1e-2, v
    Y1 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    Y2 = torch.empty_like(Y1)
    L.gemm_variant(X, W, Y1, 31)
    L.gemm_variant(X, W, Y2, 31)
    assert torch.equal(Y1, Y2)          # fixed reduction order: deterministic
    R = torch.randn(M, N, device=DEV).bfloat16()
    R2 = R.clone()
    ops.gemm(X, W, R=R2, out=R2, algo=1)
    assert rel_err(R2, ref.gemm(X, W, R)) < 1e-2
    if N % 64 == 0:
        g, u = W[: N // 2], W[N // 2:]
        Wi = ref.interleave_gate_up(g, u).contiguous()
        y = ops.gemm_silu(X, Wi)
        e = torch.nn.functional.silu(X.float() @ g.float().t()) * (X.float() @ u.float().t())
        assert rel_err(y, e) < 2e-2


@pytest.mark.parametrize("M", [1, 7, 16, 33, 64, 100, 128])
@pytest.mark.parametrize("N,K", [(4096, 4096), (1280, 8192), (512, 384)])
def test_gemm_skinny(M, N, K):
    """K2 weight-streaming GEMM (decode-sized M) against fp32: plain, in-place
    residual and fused SwiGLU."""
    torch.manual_seed(5)
    X = torch.randn(M, K, device=DEV).bfloat16()
    W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    assert rel_err(ops.gemm(X, W, algo=2), ref.gemm(X, W)) < 1e-2
    assert rel_err(ops.gemm(X, W), ref.gemm(X, W)) < 1e-2
    R = torch.randn(M, N, device=DEV).bfloat16()
    R2 = R.clone()
    ops.gemm(X, W, R=R2, out=R2, algo=2)
    assert rel_err(R2, ref.gemm(X, W, R)) < 1e-2
    g, u = W[: N // 2], W[N // 2:]
    Wi = ref.interleave_gate_up(g, u).contiguous()
    e = torch.nn.functional.silu(X.float() @ g.float().t()) * (X.float() @ u.float().t())
    assert rel_err(ops.gemm_silu(X, Wi), e) < 2e-2


@pytest.mark.parametrize("M", [1, 3, 8])
@pytest.mark.parametrize("half", [2, 0])
def test_gemm_skinny_swiglu_forms(M, half):
    """Both SwiGLU forms of the skinny kernel (8 gate + 8 up rows per block,
    default; 32-row blocks) at decode M on a wide gate|up (N >= 16384 goes to
    the skinny kernel up to M = 8), with and without the fused RMSNorm row
    scale, against fp32."""
    torch.manual_seed(23)
    L = ops.lib()
    H, F, eps = 512, 8192, 1e-5
    x = (torch.randn(M, H, device=DEV) * 2).bfloat16()
    Wg = (torch.randn(2 * F, H, device=DEV) / math.sqrt(H)).bfloat16()
    g, u = ref.deinterleave_gate_up(Wg.float())
    e_plain = torch.nn.functional.silu(x.float() @ g.t()) * (x.float() @ u.t())
    ss = ref.row_sumsq(x.cpu()).to(DEV)
    xn = x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + eps)
    e_norm = torch.nn.functional.silu(xn @ g.t()) * (xn @ u.t())
    try:
        L.gemm_skinny_half(half)
        assert rel_err(ops.gemm_silu(x, Wg), e_plain) < 2e-2
        assert rel_err(ops.gemm_silu(x, Wg, ss_in=ss, eps=eps), e_norm) < 2e-2
    finally:
        L.gemm_skinny_half(1)


@pytest.mark.parametrize("M,N,K", [(2600, 4096, 4096), (100, 512, 256), (513, 1024, 384),
                                   (4096, 6144, 4096)])
def test_gemm_256d_agpr(M, N, K):
    """One-wave-per-SIMD AGPR kernel (gemm256d.hip, variant 49 / production 256 path):
    partial last M-tile (clamped rows), plain / residual in place / SwiGLU."""
    torch.manual_seed(6)
    L = ops.lib()
    X = torch.randn(M, K, device=DEV).bfloat16()
    W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    Y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    # data-parallel 256-row tiles, stream-K (last-arriver slab sums), 192-,
    # 160-, 224- and 128-row tiles
    for v in (49, 50, 51, 53, 54, 55):
        Y.zero_()
        L.gemm_variant(X, W, Y, v)
        assert rel_err(Y, ref.gemm(X, W)) < 1e-2, v
    R = torch.randn(M, N, device=DEV).bfloat16()
    R2 = R.clone()
    ops.gemm(X, W, R=R2, out=R2, algo=1)
    assert rel_err(R2, ref.gemm(X, W, R)) < 1e-2
    g, u = W[: N // 2], W[N // 2:]
    Wi = ref.interleave_gate_up(g, u).contiguous()
    y = ops.gemm_silu(X, Wi)
    e = torch.nn.functional.silu(X.float() @ g.float().t()) * (X.float() @ u.float().t())
    assert rel_err(y, e) < 2e-2


@pytest.mark.parametrize("code", [0, 1, 2, 3, 4, 5])
def test_gemm_plan_codes(code):
    """Every kernel a measured tile plan can name (0 = 128^2, 1..5 = AGPR
    256-, 192-, 160-, 224-, 128-row tiles) through the production entry points: plain, residual
    in place, SwiGLU; M not a multiple of any tile height."""
    torch.manual_seed(7)
    L = ops.lib()
    N, K = 1024, 512
    try:
        L.gemm_plan_set(N, K, [code] * 64)
        for M in (300, 700):
            assert L.gemm_select(M, N, K) == (0 if code == 0 else 1)
            X = torch.randn(M, K, device=DEV).bfloat16()
            W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
            assert rel_err(ops.gemm(X, W), ref.gemm(X, W)) < 1e-2
            R = torch.randn(M, N, device=DEV).bfloat16()
            R2 = R.clone()
            ops.gemm(X, W, R=R2, out=R2)
            assert rel_err(R2, ref.gemm(X, W, R)) < 1e-2
            g, u = W[: N // 2], W[N // 2:]
            y = ops.gemm_silu(X, ref.interleave_gate_up(g, u).contiguous())
            e = torch.nn.functional.silu(X.float() @ g.float().t()) * (X.float() @ u.float().t())
            assert rel_err(y, e) < 2e-2
    finally:
        L.gemm_plan_clear()
        ops._load_gemm_plan(L)


@pytest.mark.parametrize("M,N,K", [(32, 4096, 4096), (100, 1024, 14336), (256, 6144, 4096),
                                   (300, 4096, 4096), (64, 2048, 1024)])
def test_gemm_splitk128(M, N, K):
    """Split-K over the 128^2 kernel (fp32 partials in the load-time workspace +
    reduce with the epilogue): plain, residual in place, SwiGLU; small M."""
    torch.manual_seed(8)
    L = ops.lib()
    S = L.gemm128_splits(M, N, K)
    assert S > 1, (M, N, K)
    X = torch.randn(M, K, device=DEV).bfloat16()
    W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    assert rel_err(ops.gemm(X, W), ref.gemm(X, W)) < 1e-2
    assert rel_err(ops.gemm(X, W, algo=0), ref.gemm(X, W)) < 1e-2
    R = torch.randn(M, N, device=DEV).bfloat16()
    R2 = R.clone()
    ops.gemm(X, W, R=R2, out=R2)
    assert rel_err(R2, ref.gemm(X, W, R)) < 1e-2
    g, u = W[: N // 2], W[N // 2:]
    y = ops.gemm_silu(X, ref.interleave_gate_up(g, u).contiguous())
    e = torch.nn.functional.silu(X.float() @ g.float().t()) * (X.float() @ u.float().t())
    assert rel_err(y, e) < 2e-2


@pytest.mark.parametrize("S", [0, 1, 2, 3, 8])
@pytest.mark.parametrize("M", [1, 9, 16, 33, 64, 100, 128])
def test_gemm_stream(M, S):
    """K2 weight-streaming kernel (gemm_stream.hip, algo 3): register-ring
    prefetch, 4-wave LDS reduction, fused split-K (S forced; 0 = auto) -
    plain, residual in place, SwiGLU, against fp32; repeated launches reuse
    the split tickets."""
    torch.manual_seed(12)
    L = ops.lib()
    try:
        L.gemm_stream_force_splits(S)
        for (N, K) in [(1024, 4096), (2048, 1536)]:
            X = torch.randn(M, K, device=DEV).bfloat16()
            W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
            e = ref.gemm(X, W)
            for _ in range(2):
                assert rel_err(ops.gemm(X, W, algo=3), e) < 1e-2
            assert rel_err(ops.gemm(X, W), e) < 1e-2       # production path picks it too
            R = torch.randn(M, N, device=DEV).bfloat16()
            R2 = R.clone()
            ops.gemm(X, W, R=R2, out=R2, algo=3)
            assert rel_err(R2, ref.gemm(X, W, R)) < 1e-2
            g, u = W[: N // 2], W[N // 2:]
            Wi = ref.interleave_gate_up(g, u).contiguous()
            es = torch.nn.functional.silu(X.float() @ g.float().t()) * (X.float() @ u.float().t())
            assert rel_err(ops.gemm_silu(X, Wi), es) < 2e-2
    finally:
        L.gemm_stream_force_splits(0)


@pytest.mark.parametrize("S", [2, 3, 4, 8, 16])
def test_gemm_splitk_forced(S):
    """Split-K of the 128^2 kernel at forced split counts: back-to-back
    launches sharing the load-time workspace and replay of a captured
    hipGraph, against fp32."""
    torch.manual_seed(11)
    L = ops.lib()
    try:
        L.gemm_splitk_force(S)
        ran = 0
        for (M, N, K) in [(48, 4096, 4096), (200, 6144, 4096), (130, 2048, 3072)]:
            if (K // 64) % S or (K // 64) // S < 4:
                continue
            assert L.gemm128_splits(M, N, K) == S
            ran += 1
            X = torch.randn(M, K, device=DEV).bfloat16()
            W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
            e = ref.gemm(X, W)
            for _ in range(3):
                assert rel_err(ops.gemm(X, W, algo=0), e) < 1e-2
            R = torch.randn(M, N, device=DEV).bfloat16()
            R2 = R.clone()
            ops.gemm(X, W, R=R2, out=R2, algo=0)
            assert rel_err(R2, ref.gemm(X, W, R)) < 1e-2
            g, u = W[: N // 2], W[N // 2:]
            Wi = ref.interleave_gate_up(g, u).contiguous()
            es = torch.nn.functional.silu(X.float() @ g.float().t()) * (X.float() @ u.float().t())
            assert rel_err(ops.gemm_silu(X, Wi), es) < 2e-2
            out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            ops.gemm(X, W, out=out, algo=0)
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                ops.gemm(X, W, out=out, algo=0)
            out.zero_()
            for _ in range(2):
                graph.replay()
            torch.cuda.synchronize()
            assert rel_err(out, e) < 1e-2
        assert ran > 0
    finally:
        L.gemm_splitk_force(-1)


@pytest.mark.parametrize("M,long_ctx", [(1500, False), (3000, False), (200, False),
                                         (1500, True), (200, True), (64, False), (5, True),
                                         (128, False), (77, True)])
def test_qkv_rope_fused(M, long_ctx):
    """QKV GEMM with RoPE + paged K/V write in its epilogue (AGPR path; M = 200
    takes the GEMM + rope_kv fallback) against fp32 GEMM + reference rope_kv,
    including rows without a cache slot (-1).  ``long_ctx``: Llama-3.1's
    scaled 128k-position table with positions past 8k."""
    torch.manual_seed(9)
    Hq, Hkv, D, H, BS = 32, 8, 128, 4096, 64
    L = ops.lib()
    X = torch.randn(M, H, device=DEV).bfloat16()
    W = (torch.randn((Hq + 2 * Hkv) * D, H, device=DEV) / math.sqrt(H)).bfloat16()
    nb = (M + BS - 1) // BS + 2
    P = 131072 if long_ctx else 8192
    pos = torch.randint(0, P - 192, (M,), device=DEV, dtype=torch.int32)
    perm = torch.randperm(nb * BS, device=DEV)[:M].to(torch.int32)
    slots = torch.where(torch.rand(M, device=DEV) < 0.1, torch.full_like(perm, -1), perm)
    cs = ref.rope_cos_sin(P, D, 500000.0, DEV, (8.0, 1.0, 4.0, 8192) if long_ctx else None)
    q = torch.zeros(M, Hq, D, device=DEV, dtype=torch.bfloat16)
    kc = torch.zeros(nb, Hkv, BS, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    ops.qkv_rope(X, W, pos, slots, cs, q, kc, vc, Hq, Hkv, D)
    qkv = ref.gemm(X, W).cpu()
    qr_c, kr_c, vr_c = torch.zeros_like(q.cpu()), torch.zeros_like(kc.cpu()), torch.zeros_like(vc.cpu())
    ref.rope_kv(qkv, pos.cpu(), slots.cpu(), cs.cpu(), qr_c, kr_c, vr_c, Hq, Hkv, D)
    assert rel_err(q.cpu(), qr_c) < 1e-2
    assert rel_err(kc.cpu(), kr_c) < 1e-2 and rel_err(vc.cpu(), vr_c) < 1e-2
    # untouched slots stay zero (rows with slot -1 wrote nothing)
    used = torch.zeros(nb * BS, dtype=torch.bool)
    used[slots.cpu()[slots.cpu() >= 0].long()] = True
    assert kc.cpu().permute(0, 2, 1, 3).reshape(nb * BS, -1)[~used].abs().sum() == 0


@pytest.mark.parametrize("M", [100, 200, 330])
def test_qkv_rope_every_path(M):
    """Every QKV + RoPE + K/V-write path the "rope" plan can name
    (launch_qkv_rope_algo: AGPR heights, stream, unfused GEMM + rope_kv, flex x
    split-K with the RoPE reduce) gives the fp32 reference's q / K / V rows."""
    torch.manual_seed(14)
    L = ops.lib()
    Hq, Hkv, D, H, BS = 32, 8, 128, 4096, 64
    N = (Hq + 2 * Hkv) * D
    X = torch.randn(M, H, device=DEV).bfloat16()
    W = (torch.randn(N, H, device=DEV) / math.sqrt(H)).bfloat16()
    nb = (M + BS - 1) // BS + 1
    pos = torch.randint(0, 8000, (M,), device=DEV, dtype=torch.int32)
    slots = torch.randperm(nb * BS, device=DEV)[:M].to(torch.int32)
    cs = ref.rope_cos_sin(8192, D, 500000.0, DEV)
    qkv_ref = ref.gemm(X, W).cpu()
    qr, kr, vr = (torch.zeros(M, Hq, D), torch.zeros(nb, Hkv, BS, D), torch.zeros(nb, Hkv, BS, D))
    ref.rope_kv(qkv_ref, pos.cpu(), slots.cpu(), cs.cpu(), qr, kr, vr, Hq, Hkv, D)
    ran = 0
    for a in [1, 2, 3, 4, 5, 200, 500] + [1000 + 16 * c + S for c in (0, 6, 10) for S in (2, 4)]:
        q = torch.zeros(M, Hq, D, device=DEV, dtype=torch.bfloat16)
        kc = torch.zeros(nb, Hkv, BS, D, device=DEV, dtype=torch.bfloat16)
        vc = torch.zeros_like(kc)
        qkv = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        if L.qkv_rope_algo(X, W, qkv, pos, slots, cs, q, kc, vc, Hq, Hkv, D, a):
            continue
        torch.cuda.synchronize()
        assert rel_err(q.cpu(), qr) < 1e-2, a
        assert rel_err(kc.cpu(), kr) < 1e-2 and rel_err(vc.cpu(), vr) < 1e-2, a
        ran += 1
    assert ran >= 8


@pytest.mark.parametrize("M,N,K", [(4352, 4096, 4096), (3000, 28672, 4096), (2304, 6144, 4096)])
def test_gemm_hybrid_streamk_tail(M, N, K):
    """Hybrid launch (gemm256d.hip full waves + gemm256sk.hip stream-K tail when
    the last wave of 256-row tiles is at most half full): plain, residual in
    place and SwiGLU against fp32."""
    torch.manual_seed(10)
    L = ops.lib()
    X = torch.randn(M, K, device=DEV).bfloat16()
    W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    Y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    L.gemm_variant(X, W, Y, 49)                     # 256-row tiles: hybrid when the tail is short
    assert rel_err(Y, ref.gemm(X, W)) < 1e-2
    R = torch.randn(M, N, device=DEV).bfloat16()
    R2 = R.clone()
    ops.gemm(X, W, R=R2, out=R2, algo=1)
    assert rel_err(R2, ref.gemm(X, W, R)) < 1e-2
    g, u = W[: N // 2], W[N // 2:]
    y = ops.gemm_silu(X, ref.interleave_gate_up(g, u).contiguous())
    e = torch.nn.functional.silu(X.float() @ g.float().t()) * (X.float() @ u.float().t())
    assert rel_err(y, e) < 2e-2


@pytest.mark.parametrize("M,N,K", [(2600, 4096, 14336), (2560, 4096, 4096), (700, 4096, 4096)])
def test_residual_gemm_every_height(M, N, K):
    """Residual projections (x += a W^T in place, the o / down projections) on
    the AGPR kernel at every tile height (algo 9..13 = plan codes 1..5) and
    through the production selector match the fp32 reference."""
    torch.manual_seed(11)
    X = torch.randn(M, K, device=DEV).bfloat16()
    W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    R = torch.randn(M, N, device=DEV).bfloat16()
    exp = X.float() @ W.float().t() + R.float()
    for algo in (-1, 9, 10, 11, 12, 13):
        y = R.clone()
        out = ops.gemm(X, W, R=y, out=y, algo=algo)
        assert out.data_ptr() == y.data_ptr()
        assert rel_err(out, exp) < 1e-2, algo


@pytest.mark.parametrize("M", [1024, 2600])
def test_qkv_rope_fused_every_height(M):
    """QKV + RoPE + paged K/V write fused in the AGPR epilogue (EPI 3) at every
    tile height the plan can pick gives the fp32 reference's q / K / V rows."""
    torch.manual_seed(12)
    L = ops.lib()
    Hq, Hkv, D, H, BS = 32, 8, 128, 4096, 64
    N = (Hq + 2 * Hkv) * D
    X = torch.randn(M, H, device=DEV).bfloat16()
    W = (torch.randn(N, H, device=DEV) / math.sqrt(H)).bfloat16()
    nb = (M + BS - 1) // BS + 1
    pos = torch.randint(0, 8000, (M,), device=DEV, dtype=torch.int32)
    slots = torch.randperm(nb * BS, device=DEV)[:M].to(torch.int32)
    cs = ref.rope_cos_sin(8192, D, 500000.0, DEV)
    qkv = ref.gemm(X, W).cpu()
    qr, kr, vr = (torch.zeros(M, Hq, D), torch.zeros(nb, Hkv, BS, D), torch.zeros(nb, Hkv, BS, D))
    ref.rope_kv(qkv, pos.cpu(), slots.cpu(), cs.cpu(), qr, kr, vr, Hq, Hkv, D)
    try:
        for code in (1, 2, 3, 4, 5):
            L.gemm_plan_set(N, H, [code] * 64)
            q = torch.empty(M, Hq, D, device=DEV, dtype=torch.bfloat16)
            kc = torch.zeros(nb, Hkv, BS, D, device=DEV, dtype=torch.bfloat16)
            vc = torch.zeros_like(kc)
            ops.qkv_rope(X, W, pos, slots, cs, q, kc, vc, Hq, Hkv, D)
            assert rel_err(q.cpu(), qr) < 1e-2, code
            assert rel_err(kc.cpu(), kr) < 1e-2 and rel_err(vc.cpu(), vr) < 1e-2, code
    finally:
        L.gemm_plan_clear()
        ops._load_gemm_plan(L)


# ---------------------------------------------------------------- fused RMSNorm
@pytest.mark.parametrize("M,N,K", [(1, 4096, 4096), (5, 4096, 14336), (24, 4096, 4096),
                                   (100, 4096, 4096), (300, 4096, 14336), (700, 4096, 4096),
                                   (2600, 4096, 4096), (2600, 4096, 14336)])
def test_fused_norm_residual_statistic(M, N, K):
    """Residual GEMMs (y += x W^T) with ``ss_out``: every path the dispatcher
    can take (skinny / stream / split-K 128^2 / flex / AGPR at every height,
    algo -1 and forced) adds each output row's sum of squares (int64 fixed
    point) matching the fp32 sum over the stored bf16 row; repeated runs give
    bit-identical statistics (integer atomics)."""
    torch.manual_seed(21)
    X = torch.randn(M, K, device=DEV).bfloat16()
    W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    R = torch.randn(M, N, device=DEV).bfloat16()
    algos = [-1, 0] + ([9, 10, 11, 12, 13] if M >= 256 else [])
    for algo in algos:
        outs = []
        for _ in range(2):
            y = R.clone()
            ss = torch.zeros(M, dtype=torch.int64, device=DEV)
            ops.gemm(X, W, R=y, out=y, algo=algo, ss_out=ss)
            exp = y.float().pow(2).sum(-1) * ref.SS_FIX
            assert ((ss.double() - exp.double()).abs() / exp.double()).max().item() < 1e-5, algo
            outs.append(ss)
        assert torch.equal(outs[0], outs[1]), algo
        assert rel_err(y, ref.gemm(X, W, R)) < 1e-2


@pytest.mark.parametrize("M", [3, 300, 2600])
def test_fused_norm_statistic_large_rows(M):
    """rows of |x| ~ 3e3 at H = 8192 (70B width).  At the old
    2^-28 unit such a row's sum of squares overflowed int64 and wrapped; the
    2^-20 unit with a clamped add keeps it exact to 1e-5 and positive, both in
    the residual GEMM epilogue and in the stand-alone norm kernel."""
    torch.manual_seed(23)
    N, K = 8192, 1024
    X = torch.randn(M, K, device=DEV).bfloat16()
    W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    R = (torch.randn(M, N, device=DEV) * 3e3).bfloat16()
    y = R.clone()
    ss = torch.zeros(M, dtype=torch.int64, device=DEV)
    ops.gemm(X, W, R=y, out=y, ss_out=ss)
    exp = y.double().pow(2).sum(-1) * ref.SS_FIX
    assert (ss > 0).all()
    assert ((ss.double() - exp).abs() / exp).max().item() < 1e-5
    ss2 = torch.zeros(M, dtype=torch.int64, device=DEV)
    ops.row_sumsq(y, ss2)
    assert (ss2 > 0).all() and ((ss2.double() - exp).abs() / exp).max().item() < 1e-5
    sc = ref.norm_row_scale(ss.cpu(), N, 1e-5)
    exp_sc = torch.rsqrt(y.cpu().double().pow(2).mean(-1) + 1e-5).float().unsqueeze(-1)
    assert torch.allclose(sc, exp_sc, rtol=1e-5)


@pytest.mark.parametrize("M", [1, 6, 20, 48, 200, 700, 2600])
def test_fused_norm_swiglu_and_qkv(M):
    """SwiGLU and QKV + RoPE with ``ss_in``: the accumulators of row m scaled
    by rsqrt(ss[m] / H + eps) equal the GEMMs of the explicitly RMS-normed
    rows (norm weight folded into W) against fp32, on every path the
    dispatcher picks at this M (and every AGPR height for QKV)."""
    torch.manual_seed(22)
    L = ops.lib()
    H, F, eps = 4096, 14336, 1e-5
    x = (torch.randn(M, H, device=DEV) * 3).bfloat16()
    gw = (torch.rand(H, device=DEV) + 0.5)                 # a non-trivial norm weight
    ss = ref.row_sumsq(x.cpu()).to(DEV)
    xn = x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + eps) * gw
    Wg = (torch.randn(2 * F, H, device=DEV) / math.sqrt(H)).bfloat16()
    Wf = (Wg.float() * gw).bfloat16()                      # folded
    y = ops.gemm_silu(x, Wf, ss_in=ss, eps=eps)
    g, u = ref.deinterleave_gate_up(Wg.float())
    e = torch.nn.functional.silu(xn @ g.t()) * (xn @ u.t())
    assert rel_err(y, e) < 2e-2
    Hq, Hkv, D, BS = 32, 8, 128, 64
    Wq = (torch.randn((Hq + 2 * Hkv) * D, H, device=DEV) / math.sqrt(H)).bfloat16()
    Wqf = (Wq.float() * gw).bfloat16()
    nb = (M + BS - 1) // BS + 1
    pos = torch.randint(0, 8000, (M,), device=DEV, dtype=torch.int32)
    slots = torch.randperm(nb * BS, device=DEV)[:M].to(torch.int32)
    cs = ref.rope_cos_sin(8192, D, 500000.0, DEV)
    qkv = (xn.cpu() @ Wq.float().cpu().t()).bfloat16()
    qr, kr, vr = (torch.zeros(M, Hq, D), torch.zeros(nb, Hkv, BS, D), torch.zeros(nb, Hkv, BS, D))
    ref.rope_kv(qkv, pos.cpu(), slots.cpu(), cs.cpu(), qr, kr, vr, Hq, Hkv, D)
    codes = (None, 1, 2, 3, 4, 5) if M >= 256 else (None,)
    # flex x split-K plan entries (the reduce applies the row scale, RoPE and
    # the K / V write: gemm.hip splitk_reduce_rope), M > 64 (below: the stream kernel)
    codes += tuple(("fs", fs) for fs in (16 * 5 + 4, 16 * 7 + 4, 16 * 6 + 2)) if M > 64 else ()
    try:
        for code in codes:
            if isinstance(code, tuple):
                L.gemm_plan_set(Wqf.shape[0], H, [0] * 64)
                L.gemm_plan_set_fsplit(Wqf.shape[0], H, [code[1]] * 64)
            elif code is not None:
                L.gemm_plan_set_fsplit(Wqf.shape[0], H, [-1] * 64)
                L.gemm_plan_set(Wqf.shape[0], H, [code] * 64)
            q = torch.empty(M, Hq, D, device=DEV, dtype=torch.bfloat16)
            kc = torch.zeros(nb, Hkv, BS, D, device=DEV, dtype=torch.bfloat16)
            vc = torch.zeros_like(kc)
            ops.qkv_rope(x, Wqf, pos, slots, cs, q, kc, vc, Hq, Hkv, D, ss_in=ss, eps=eps)
            assert rel_err(q.cpu(), qr) < 2e-2, code
            assert rel_err(kc.cpu(), kr) < 2e-2 and rel_err(vc.cpu(), vr) < 2e-2, code
    finally:
        L.gemm_plan_clear()
        ops._load_gemm_plan(L)


def test_fused_norm_qkv_fallback_rope_kv(monkeypatch):
    """QKV through the unfused path (plain GEMM into qkv scratch + rope_kv,
    MCP_QKV_ROPE_FUSED routing off via a shape the AGPR kernel rejects):
    rope_kv applies the row scale to q, K and V."""
    torch.manual_seed(23)
    M, H, eps = 100, 320, 1e-5              # M > 64: no stream path; K % 128 != 0: no AGPR path
    Hq, Hkv, D, BS = 4, 2, 128, 64
    x = torch.randn(M, H, device=DEV).bfloat16()
    ss = ref.row_sumsq(x.cpu()).to(DEV)
    xn = x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + eps)
    W = (torch.randn((Hq + 2 * Hkv) * D, H, device=DEV) / math.sqrt(H)).bfloat16()
    nb = 2
    pos = torch.arange(M, device=DEV, dtype=torch.int32)
    slots = torch.arange(M, device=DEV, dtype=torch.int32)
    cs = ref.rope_cos_sin(512, D, 500000.0, DEV)
    qkv = (xn.cpu() @ W.float().cpu().t()).bfloat16()
    qr, kr, vr = (torch.zeros(M, Hq, D), torch.zeros(nb, Hkv, BS, D), torch.zeros(nb, Hkv, BS, D))
    ref.rope_kv(qkv, pos.cpu(), slots.cpu(), cs.cpu(), qr, kr, vr, Hq, Hkv, D)
    q = torch.empty(M, Hq, D, device=DEV, dtype=torch.bfloat16)
    kc = torch.zeros(nb, Hkv, BS, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    ops.qkv_rope(x, W, pos, slots, cs, q, kc, vc, Hq, Hkv, D, ss_in=ss, eps=eps)
    assert rel_err(q.cpu(), qr) < 2e-2
    assert rel_err(kc.cpu(), kr) < 2e-2 and rel_err(vc.cpu(), vr) < 2e-2


@pytest.mark.parametrize("P", [64, 128, 192, 640, 4096, 4160])
def test_prefix_pass_block_table_walk(P, monkeypatch):
    """The prefix pass at 1, 2, 3, 10 and 64 key tiles and at 65 (past one
    VGPR of cached block-table entries: the cache refills) against fp32
    softmax attention, with a shuffled block table; 2100 query tokens give
    the 8-wave grid (more blocks than CUs)."""
    monkeypatch.setenv("MCP_ATTN_PREFIX_RT", "2")
    torch.manual_seed(13)
    Hq, Hkv, D, T = 32, 8, 128, 2100
    n_pre = P // 64
    kc, vc = _cache(n_pre + 2, Hkv)
    kc = (kc.float() * (1 + torch.arange(n_pre + 2, device=DEV).view(-1, 1, 1, 1) % 5)).bfloat16()
    pre_bt = (torch.randperm(n_pre + 2, device=DEV)[:n_pre]).to(torch.int32)
    q = torch.randn(T, Hq, D, device=DEV).bfloat16()
    out = torch.empty_like(q)
    lse = torch.empty(T, Hq, device=DEV, dtype=torch.float32)
    scale = 1 / math.sqrt(D)
    ops.lib().prefix_attention(q, kc, vc, out, lse, pre_bt, P, T, scale)
    G = Hq // Hkv
    k = kc[pre_bt.long()].float().permute(1, 0, 2, 3).reshape(Hkv, P, D)
    v = vc[pre_bt.long()].float().permute(1, 0, 2, 3).reshape(Hkv, P, D)
    s = torch.einsum("thgd,hpd->thgp", q.float().view(T, Hkv, G, D), k) * scale
    exp_o = torch.einsum("thgp,hpd->thgd", torch.softmax(s, -1), v).reshape(T, Hq, D)
    exp_lse = (torch.logsumexp(s, -1) / math.log(2)).reshape(T, Hq)
    assert rel_err(out, exp_o) < 2e-2
    assert torch.allclose(lse, exp_lse, atol=5e-2, rtol=1e-3)
    again = torch.empty_like(q)
    ops.lib().prefix_attention(q, kc, vc, again, lse, pre_bt, P, T, scale)
    assert torch.equal(out, again)


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("own_keys,q_lens", [([5, 200, 64, 65], [1, 1, 1, 2]),
                                              ([300, 130, 1100, 20, 700], [1, 9, 2, 16, 5]),
                                              ([3000, 64], [1, 1])])
def test_decode_kernel_own_span_mode(own_keys, q_lens, mode, monkeypatch):
    """The decode kernel in own-span mode (unsplit steps, MCP_ATTN_DECODE_OWN:
    1 = the 1-wave items on it, the 4-wave items on the work-list kernel; 2 =
    both): grid z over each sequence's own tiles after a 640-key cascade
    prefix, single- and multi-block own spans (last-arriver merge, prefix
    fold), against fp32 full attention; repeated launches bitwise equal."""
    monkeypatch.setattr(ops, "_DECODE_OWN", mode)
    monkeypatch.setenv("MCP_ATTN_CONCURRENT", "0")
    monkeypatch.setenv("MCP_KV_SPLIT", "0")
    torch.manual_seed(37)
    Hq, Hkv, D, BS, P_full = 32, 8, 128, 64, 640
    ctx = [P_full + k for k in own_keys]
    n_pre = P_full // BS
    own_blocks = [(k + BS - 1) // BS for k in own_keys]
    nb = n_pre + sum(own_blocks) + 2
    kc, vc = _cache(nb, Hkv)
    pre = list(range(n_pre))
    o = n_pre
    tables = []
    for nbk in own_blocks:
        tables.append(pre + list(range(o, o + nbk)))
        o += nbk
    bt = np.zeros((len(q_lens), max(len(t) for t in tables) + 3), np.int32)
    for i, t in enumerate(tables):
        bt[i, :len(t)] = t
    T = sum(q_lens)
    q = torch.randn(T, Hq, D, device=DEV).bfloat16()
    qs = np.concatenate([[0], np.cumsum(q_lens)[:-1]]).astype(np.int32)
    step = StepInputs(token_ids=np.zeros(T, np.int32), positions=np.zeros(T, np.int32),
                      slots=np.zeros(T, np.int32), q_start=qs,
                      q_len=np.asarray(q_lens, np.int32), ctx_len=np.asarray(ctx, np.int32),
                      block_table=bt, logit_rows=np.zeros(0, np.int32),
                      kv_begin=np.full(len(q_lens), P_full, np.int32),
                      pre_bt=np.asarray(pre, np.int32), pre_tokens=T)
    dev = pack(step, Hq // Hkv, DEV)
    dev.attn.kv_splits = 1
    dev.attn.own_tiles = max(own_blocks)
    exp = ref.paged_attention(q.cpu(), kc.cpu(), vc.cpu(), torch.from_numpy(qs),
                              torch.tensor(q_lens), torch.tensor(ctx), torch.from_numpy(bt),
                              1 / math.sqrt(D))
    outs = []
    for _ in range(2):
        out = ops.paged_attention(q, kc, vc, dev.attn, 1 / math.sqrt(D)).cpu()
        assert rel_err(out, exp) < 2e-2, (own_keys, q_lens)
        outs.append(out)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("M", [136, 257, 640])
def test_gemm_flex_swiglu(M):
    """The SwiGLU epilogue of every flex tile that has one (per-wave column
    spans of whole gate | up pairs), 2- and 4-stage forms, routed by a plan
    "flex" entry through ops.gemm_silu, with and without the fused RMSNorm
    row scale, against fp32 - ragged M included."""
    torch.manual_seed(17)
    L = ops.lib()
    H, F, eps = 512, 1536, 1e-5
    N = 2 * F
    x = (torch.randn(M, H, device=DEV) * 2).bfloat16()
    Wg = (torch.randn(N, H, device=DEV) / math.sqrt(H)).bfloat16()
    g, u = ref.deinterleave_gate_up(Wg.float())
    e_plain = torch.nn.functional.silu(x.float() @ g.t()) * (x.float() @ u.t())
    ss = ref.row_sumsq(x.cpu()).to(DEV)
    xn = x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + eps)
    e_norm = torch.nn.functional.silu(xn @ g.t()) * (xn @ u.t())
    cands = [c for c in range(L.gemm_flex_count()) if L.gemm_flex_silu_ok(c)]
    assert cands
    try:
        for c in cands + [32 + c for c in cands]:
            L.gemm_plan_set(N, H, [0] * 16)
            L.gemm_plan_set_flex(N, H, [c] * 16)
            assert L.gemm_plan_flex(M, N, H) == c
            assert rel_err(ops.gemm_silu(x, Wg), e_plain) < 2e-2, c
            assert rel_err(ops.gemm_silu(x, Wg, ss_in=ss, eps=eps), e_norm) < 2e-2, c
        # flex x split-K through the plan's "fsplit" entry: the reduce applies
        # the SwiGLU and the row scale
        L.gemm_plan_set_flex(N, H, [-1] * 16)
        for fs in (16 * 6 + 2, 16 * 12 + 4, 16 * 1 + 8):
            L.gemm_plan_set_fsplit(N, H, [fs] * 16)
            assert rel_err(ops.gemm_silu(x, Wg), e_plain) < 2e-2, fs
            assert rel_err(ops.gemm_silu(x, Wg, ss_in=ss, eps=eps), e_norm) < 2e-2, fs
    finally:
        L.gemm_plan_clear()
        ops._load_gemm_plan(L)


def test_weight_prefetch_in_graph():
    """The Infinity Cache prefetch (csrc/prefetch.hip) runs eagerly and as a
    forked side-stream branch of a captured hipGraph without touching its
    input; the GEMM after it is unchanged."""
    torch.manual_seed(31)
    W = torch.randn(4096, 1024, device=DEV).bfloat16()
    X = torch.randn(8, 1024, device=DEV).bfloat16()
    W0 = W.clone()
    ops.weight_prefetch_init(DEV)
    ops.weight_prefetch(W, -1, 64)
    ops.weight_prefetch(W, 12345, 8)                 # ragged length: the 16-B head only
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    out = torch.empty(8, 4096, device=DEV, dtype=torch.bfloat16)
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            ops.weight_prefetch(W, 1 << 20, 32)
        ops.gemm(X, W, out=out)
        cur.wait_stream(side)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(W, W0)
    assert rel_err(out, ref.gemm(X, W)) < 1e-2

