"""GPU parity: the HIP path (through the C ABI) against the reference-generated
golden vectors and the CPU oracle.

Bit-exact: MX codes/values/exponents, approximator operands, true and
approximate scores, top-k indices in torch's CPU order, prune masks.
Tolerance: the attention output, normwise relative error <= 1e-3 (north star;
SURVEY.md F7)."""
import os

import numpy as np
import pytest
import torch

from oracle import mx_oracle as O

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
OUT_TOL = 1e-3


def load(name):
    return np.load(os.path.join(G, name))


def dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


def host(t):
    return t.detach().cpu().numpy()


def same(a, b, what=""):
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    if a.dtype.kind == "f":
        ok = (a == b) | (np.isnan(a) & np.isnan(b))
    else:
        ok = a == b
    if not ok.all():
        bad = np.argwhere(~ok)
        raise AssertionError(f"{what}: {bad.shape[0]}/{ok.size} mismatches, first {bad[:4].tolist()}: "
                             f"{a[tuple(bad[0])]} vs {b[tuple(bad[0])]}")


@pytest.fixture(scope="module")
def M():
    import mx_quantization_amd as m
    return m


# ------------------------------------------------------------------ MFMA lane maps
def test_mfma_i8_lane_maps(M):
    from mx_quantization_amd.ops import selftest_mfma
    rng = np.random.default_rng(0)
    A = rng.integers(-128, 128, (16, 32)).astype(np.int8)
    B = rng.integers(-128, 128, (32, 16)).astype(np.int8)
    C = host(selftest_mfma(dev(A), dev(B)))
    same(C, A.astype(np.int32) @ B.astype(np.int32), "mfma 16x16x32 i8")


def test_mfma_i8_32x32x32_lane_maps(M):
    """the finishing kernel's P.V operand / accumulator maps (v_mfma_i32_32x32x32_i8)"""
    from mx_quantization_amd.ops import selftest_mfma32
    rng = np.random.default_rng(1)
    for lo, hi in ((-128, 128), (-127, 128), (0, 2)):
        A = rng.integers(lo, hi, (32, 32)).astype(np.int8)
        B = rng.integers(lo, hi, (32, 32)).astype(np.int8)
        C = host(selftest_mfma32(dev(A), dev(B)))
        same(C, A.astype(np.int32) @ B.astype(np.int32), "mfma 32x32x32 i8")


# ------------------------------------------------------------------ quantization
@pytest.mark.parametrize("elem,mbits", [("int8", 8), ("int4", 4), ("int2", 2)])
@pytest.mark.parametrize("rnd", ["nearest", "floor", "even"])
@pytest.mark.parametrize("flush", [False, True])
def test_quantize_boundary_vectors(M, elem, mbits, rnd, flush):
    d = load("quant_kat.npz")
    y = M.quantize_mx(dev(d["x"]), elem_mbits=mbits, block_size=32, axis=-1, round=rnd, flush=flush)
    same(host(y), d[f"y_{elem}_{rnd}_{int(flush)}"], f"{elem}/{rnd}/{flush}")


def test_quantize_hw_kat_and_scale_bits(M):
    d = load("quant_kat.npz")
    same(host(M.quantize_mx(dev(d["hw_x"]), 8, 10, 1)), d["hw_y"], "hw_test")
    same(host(M.quantize_mx(dev(d["x"]), 8, 32, -1, scale_bits=5)), d["y_int8_nearest_0_sb5"], "scale_bits 5")


@pytest.mark.parametrize("bs", [8, 9, 32, 64])
@pytest.mark.parametrize("ax", [-1, -2, 0])
def test_quantize_block_sizes_axes(M, bs, ax):
    d = load("quant_kat.npz")
    same(host(M.quantize_mx(dev(d["z"]), 8, bs, ax)), d[f"z_bs{bs}_ax{ax}"], f"bs{bs} ax{ax}")


def test_shared_exponents_and_bfloat(M):
    d = load("quant_kat.npz")
    from mx_quantization_amd.mx.mx_ops import _reshape_to_blocks, _shared_exponents
    xb, *_ = _reshape_to_blocks(dev(d["x"]), [-1], 32)
    same(host(_shared_exponents(xb, "max", axes=[-1])), d["sexp_max"], "sexp max")
    same(host(_shared_exponents(xb, "none", axes=[-1])), d["sexp_none"], "sexp none")
    same(host(M.quantize_bfloat(dev(d["bf_x"]), 16)), d["bf_y"], "bfloat16")


def test_exponent_rule_exhaustive_sample(M):
    """The device exponent rule on every float32 around every per-binade threshold
    and a dense sample elsewhere, against torch.log2 on the CPU."""
    lut = load("exp_lut.npz")
    parts = []
    for E in range(1, 255):
        t = int(min(lut["th_norm"][E], (1 << 23) - 1))
        parts.append(np.arange((E << 23) | max(0, t - 256), (E << 23) | min(1 << 23, t + 256), dtype=np.uint32))
    parts.append(np.arange(1, 1 << 23, 97, dtype=np.uint32))
    parts.append(np.random.default_rng(3).integers(1, 0x7F800000, 1 << 22).astype(np.uint32))
    b = np.concatenate(parts)
    x = b.view(np.float32)
    ref = torch.floor(torch.log2(torch.from_numpy(x))).numpy()
    got = host(M.shared_exponents(dev(x.reshape(-1, 1)), "none")).reshape(-1)
    same(got, ref, "floor(log2)")


# ------------------------------------------------------------------ top-k order
@pytest.mark.parametrize("name", ["deit", "deit30", "dit", "cross"])
def test_topk_ties_exact_order(M, name):
    d = load("topk_ties.npz")
    k = int(d[f"{name}_k"])
    vals, idx = M.topk(dev(d[f"{name}_pred"]), k)
    same(host(idx).astype(np.int16), d[f"{name}_idx"], name)
    same(host(vals), np.take_along_axis(d[f"{name}_pred"], host(idx), -1), name + " vals")


@pytest.mark.parametrize("n", [120, 197, 256])
def test_topk_adversarial_rows(M, n):
    d = load("topk_ties.npz")
    rows, ks, want = d[f"adv{n}_rows"], d[f"adv{n}_k"], d[f"adv{n}_idx"]
    for k in np.unique(ks):
        sel = ks == k
        _, idx = M.topk(dev(rows[sel]), int(k))
        same(host(idx).astype(np.int16), want[sel][:, :k], f"n{n} k{k}")


@pytest.mark.parametrize("n,k", [(197, 30), (197, 154), (256, 77), (256, 154), (512, 300), (120, 20), (300, 4)])
def test_topk_depth_limit_fallbacks_and_partial_sort(M, n, k):
    rows = np.stack([O.antiqsort_row(n, k)] + [np.random.default_rng(i).integers(0, 3, n).astype(np.float32)
                                                for i in range(7)])
    _, want = O.topk(rows, k)
    _, idx = M.topk(dev(rows), k)
    same(host(idx), want, f"n{n} k{k}")


def test_topk_random_small_alphabets_and_specials(M):
    rng = np.random.default_rng(11)
    for n in (5, 17, 64, 65, 127, 128, 129, 197, 256, 300, 511, 512):
        for k in sorted({1, 2, 3, min(n, 20), (n + 1) // 2, n}):
            rows = rng.integers(-2, 3, (32, n)).astype(np.float32)
            rows[rows == 2] = np.nan
            rows[rows == -2] = -0.0
            _, want = O.topk(rows, k)
            _, idx = M.topk(dev(rows), k)
            same(host(idx), want, f"n{n} k{k}")
            _, idx = M.topk(dev(rows), k, packed=False)  # the 64-bit pass alone
            same(host(idx), want, f"n{n} k{k} unpacked")


def test_topk_prune_mask_words(M):
    """mxa_topk's prune-mask output (scatter(1) at idx as bits) on tie-heavy rows."""
    d = load("topk_ties.npz")
    for name in ("deit", "dit", "cross"):
        k = int(d[f"{name}_k"])
        pred = d[f"{name}_pred"]
        n = pred.shape[-1]
        for packed in (True, False):
            _, idx, words = M.topk(dev(pred), k, return_mask=True, packed=packed)
            same(host(M.unpack_mask(words, n)), O.prune_mask(d[f"{name}_idx"].astype(np.int64), n), f"{name} {packed}")


@pytest.mark.parametrize("n", [33, 64, 65, 100, 197, 256, 512])
def test_topk_many_tie_rows(M, n):
    """thousands of rows with heavy ties: every window width of the group partition
    steps (4, 8, 16, 32 positions per lane), both sort-rank paths (k-1 <= 64 and > 64)"""
    rng = np.random.default_rng(n)
    for k in sorted({1, 2, 5, 16, 17, 20, 30, 32, 33, 48, 64} & set(range(1, n + 1))):
        rows = rng.integers(-6, 7, (700, n)).astype(np.float32) * np.float32(0.25)
        rows[:100] = rng.standard_normal((100, n)).astype(np.float32)
        _, want = O.topk(rows, k)
        _, idx = M.topk(dev(rows), k)
        same(host(idx), want, f"n{n} k{k}")


@pytest.mark.parametrize("n,k", [(1024, 20), (1024, 154), (700, 300), (1000, 999)])
def test_topk_rows_up_to_1024(M, n, k):
    """Rows longer than 512 (PixArt 512x512 self-attention: 1,024 tokens,
    MX_transformer_block.py:648-717, topk at :678): ex_pred-like tie rows, small
    alphabets and an antiqsort depth-limit row, against libstdc++."""
    rng = np.random.default_rng(n + k)
    q = rng.standard_normal((1, 8, 72), dtype=np.float32)
    kk = rng.standard_normal((1, n, 72), dtype=np.float32)
    aq, ak = O.approx_operands(q, kk, "ex_pred")
    rows = np.concatenate([O.exact_matmul_f32(aq, np.swapaxes(ak, -1, -2)).reshape(-1, n),
                           rng.integers(-3, 4, (8, n)).astype(np.float32), O.antiqsort_row(n, k)[None]])
    _, want = O.topk(rows, k)
    _, idx, words = M.topk(dev(rows), k, return_mask=True)
    same(host(idx), want, f"n{n} k{k}")
    same(host(M.unpack_mask(words, n)), O.prune_mask(want, n), f"n{n} k{k} mask")


# ------------------------------------------------------------------ approximators
@pytest.mark.parametrize("mode", ["ex_pred", "partial_Q", "partial_K", "MXINT4", "two_step_leading_ones", "true_ex"])
def test_approximator_operands(M, mode):
    d = load("attn_deit_tiny.npz")
    M.install_dropin()
    from funcs import exponent_approximation
    from mx.specs import apply_mx_specs
    specs = apply_mx_specs({"a_elem_format": "int8", "w_elem_format": "int8", "block_size": 32, "scale_bits": 8,
                            "bfloat": 32})
    obj = exponent_approximation(dev(d["q"]), dev(d["k"]), specs)
    fn = {"ex_pred": obj.exponent_based_sign, "true_ex": obj.exponent_based_sign_leading_ones}.get(
        mode, getattr(obj, mode, None))
    aq, ak = fn()
    same(host(aq)[..., :32, :], d[f"{mode}_k20/aq"], mode + " aq")
    same(host(ak)[..., :32, :], d[f"{mode}_k20/ak"], mode + " ak")


@pytest.mark.parametrize("mode", ["ex_pred", "partial_Q", "partial_K", "MXINT4", "two_step_leading_ones", "true_ex"])
def test_approximator_operands_special_blocks_vs_oracle(M, mode):
    """NaN / Inf blocks (true_ex maps them to +1 like zeros: examples :98-110), zero
    elements and rows, tiny and huge block scales, a ragged head dim."""
    rng = np.random.default_rng(17)
    q = rng.standard_normal((2, 3, 40, 72), dtype=np.float32)
    k = rng.standard_normal((2, 3, 40, 72), dtype=np.float32)
    q[0, 0, 3, 5], q[0, 1, 4, 40], k[1, 2, 6, 70] = np.nan, np.inf, -np.inf
    q[1, 0, :, ::5] = 0.0
    k[0, 2, 9, :] = 0.0
    q[1, 1] *= np.float32(2.0 ** -120)
    k[1, 1] *= np.float32(2.0 ** 90)
    M.install_dropin()
    from funcs import exponent_approximation
    from mx.specs import apply_mx_specs
    specs = apply_mx_specs({"a_elem_format": "int8", "w_elem_format": "int8", "block_size": 32, "scale_bits": 8,
                            "bfloat": 32})
    obj = exponent_approximation(dev(q), dev(k), specs)
    fn = {"ex_pred": obj.exponent_based_sign, "true_ex": obj.exponent_based_sign_leading_ones}.get(
        mode, getattr(obj, mode, None))
    aq, ak = fn()
    wq, wk = O.approx_operands(q, k, mode)
    same(host(aq), wq, mode + " aq")
    same(host(ak), wk, mode + " ak")


# ------------------------------------------------------------------ fused attention
CASES = [
    ("attn_deit_tiny.npz", "ex_pred_k20", dict(pred_mode="ex_pred", k_top=20)),
    ("attn_deit_tiny.npz", "dense", dict(top_k=False)),
    ("attn_deit_tiny.npz", "trueK_k30", dict(approx=False, k_top=30)),
    ("attn_deit_tiny.npz", "partial_Q_k20", dict(pred_mode="partial_Q", k_top=20)),
    ("attn_deit_tiny.npz", "partial_K_k20", dict(pred_mode="partial_K", k_top=20)),
    ("attn_deit_tiny.npz", "MXINT4_k20", dict(pred_mode="MXINT4", k_top=20)),
    ("attn_deit_tiny.npz", "two_step_leading_ones_k20", dict(pred_mode="two_step_leading_ones", k_top=20)),
    ("attn_deit_tiny.npz", "true_ex_k20", dict(pred_mode="true_ex", k_top=20)),
    ("attn_deit_tiny_peaky.npz", "ex_pred_k20", dict(pred_mode="ex_pred", k_top=20)),
    ("attn_dit.npz", "ex_pred_k154", dict(pred_mode="ex_pred", k_top=154)),
    ("attn_pixart_cross.npz", "MXINT4_k20", dict(pred_mode="MXINT4", k_top=20, flush_subnormals=True)),
    ("attn_pixart_cross.npz", "two_step_leading_ones_k20",
     dict(pred_mode="two_step_leading_ones", k_top=20, flush_subnormals=True)),
    ("attn_pixart_cross.npz", "ex_pred_k20", dict(pred_mode="ex_pred", k_top=20, flush_subnormals=True)),
]


@pytest.mark.parametrize("fname,tag,kw", CASES, ids=[f"{f[5:-4]}:{t}" for f, t, _ in CASES])
def test_fused_attention_vs_reference(M, fname, tag, kw):
    d = load(fname)
    bias = dev(d["bias"][:, :, None, :]) if "bias" in d.files else None  # (B,1,1,T)
    topk = kw.get("top_k", True)
    res = M.mx_topk_attention(dev(d["q"]), dev(d["k"]), dev(d["v"]), float(d["scale"]),
                              bias=bias, return_scores=True, return_mask=topk, **kw)
    out, idx, true_s, pred_s = res[:4]
    torch.cuda.synchronize()
    same(host(true_s), d["true"], "true scores")
    if f"{tag}/pred" in d.files:
        same(host(pred_s), d[f"{tag}/pred"], "approx scores")
        # the scores alone (mxa_approx_scores)
        alone = M.mx_approx_scores(dev(d["q"]), dev(d["k"]), kw["pred_mode"], bias=bias,
                                   flush_subnormals=kw.get("flush_subnormals", False))
        same(host(alone), d[f"{tag}/pred"], "mxa_approx_scores")
    if f"{tag}/idx" in d.files:
        same(host(idx), d[f"{tag}/idx"], "top-k idx")
        T = d["true"].shape[-1]
        # the kernel's prune-mask words (mask_out) against scatter(1) at the reference's idx
        same(host(M.unpack_mask(res[4], T)), O.prune_mask(d[f"{tag}/idx"], T), "prune mask")
    err = O.normwise_rel_err(host(out), d[f"{tag}/out"])
    assert err <= OUT_TOL, err


EXTRA = [
    ("elsa_deit_k20", dict(pred_mode="ELSA", k_top=20)),
    ("elsa_dit_k154", dict(pred_mode="ELSA", k_top=154)),
    ("bf16", dict(pred_mode="ex_pred", k_top=154, bfloat=16)),
]


@pytest.mark.parametrize("tag,kw", EXTRA, ids=[t for t, _ in EXTRA])
def test_fused_attention_extra_vs_reference(M, tag, kw):
    """ELSA scores (funcs/elsa_approximation.py) and the bfloat16 elementwise variant
    (DiT sample.py:42) against reference-generated vectors."""
    d = load("attn_extra.npz")
    g = lambda n: d[f"{tag}/{n}"]
    proj = dev(g("proj")) if kw["pred_mode"] == "ELSA" else None
    out, idx, true_s, pred_s, mask = M.mx_topk_attention(dev(g("q")), dev(g("k")), dev(g("v")), float(g("scale")),
                                                         return_scores=True, return_mask=True, elsa_proj=proj, **kw)
    torch.cuda.synchronize()
    same(host(true_s), g("true"), "true")
    same(host(pred_s), g("pred"), "pred")
    same(host(idx), g("idx"), "idx")
    T = g("true").shape[-1]
    same(host(M.unpack_mask(mask, T)), O.prune_mask(g("idx"), T), "mask")
    assert O.normwise_rel_err(host(out), g("out")) <= OUT_TOL
    if kw["pred_mode"] == "ELSA":  # the drop-in class on the same inputs
        M.install_dropin()
        from funcs import elsa_approximation
        from mx.specs import apply_mx_specs
        specs = apply_mx_specs({"a_elem_format": "int8", "w_elem_format": "int8", "block_size": 32,
                                "scale_bits": 8, "bfloat": 32})
        sc = elsa_approximation(Q=dev(g("q")), K=dev(g("k")), mx_specs=specs,
                                orthogonal_matrix=torch.from_numpy(g("proj"))).approximation_scores()
        same(host(sc), g("pred"), "elsa_approximation.approximation_scores")
    else:
        o2, _ = M.mx_topk_attention(dev(g("q")), dev(g("k")), dev(g("v")), float(g("scale")), top_k=False, bfloat=16)
        assert O.normwise_rel_err(host(o2), g("dense_out")) <= OUT_TOL


@pytest.mark.parametrize("D", [64, 72])
@pytest.mark.parametrize("mode", ["true_ex", "ELSA"])
def test_trueex_elsa_vs_oracle(M, mode, D):
    """true_ex (power-of-two codes + zero indicators) and ELSA (hashes, key norms)
    against the oracle: odd lengths, zero elements and rows, a NaN row."""
    rng = np.random.default_rng(D + len(mode))
    B, H, N = 2, 3, 129
    q = rng.standard_normal((B, H, N, D), dtype=np.float32)
    kk = rng.standard_normal((B, H, N, D), dtype=np.float32)
    v = rng.standard_normal((B, H, N, D), dtype=np.float32)
    q[0, 0, :, ::7] = 0.0          # zero elements (true_ex: exponent 0 -> +1)
    kk[0, 1, 5, :] = 0.0           # a zero key row (ELSA: zero norm scales query row 5)
    kk[1, 0, :, 3] *= np.float32(1e-4)
    q[1, 2, 7, 9] = np.nan
    proj = None
    if mode == "ELSA":
        from mx_quantization_amd.funcs import _create_structured_orthogonal_matrix
        torch.manual_seed(D)
        proj = _create_structured_orthogonal_matrix(D).numpy()
    res = M.mx_topk_attention(dev(q), dev(kk), dev(v), D ** -0.5, k_top=30, pred_mode=mode, return_scores=True,
                              elsa_proj=None if proj is None else dev(proj))
    got = [host(t) for t in res]
    r = O.attention(q, kk, v, D ** -0.5, k_top=30, pred_mode=mode, elsa_proj=proj)
    _check_vs_oracle(got, r, mode)


def test_fused_attention_strided_qkv_views(M):
    """q/k/v as permuted views of one packed qkv buffer (deit main.py:87-88, DiT models.py:156-157)."""
    d = load("attn_deit_tiny.npz")
    B, H, N, D = d["q"].shape
    qkv = np.stack([d["q"], d["k"], d["v"]], 0).transpose(1, 3, 0, 2, 4).copy()  # (B,N,3,H,D)
    t = dev(qkv).permute(2, 0, 3, 1, 4)
    q, k, v = t[0], t[1], t[2]
    assert not q.is_contiguous()
    out, idx = M.mx_topk_attention(q, k, v, float(d["scale"]), k_top=20)
    same(host(idx), d["ex_pred_k20/idx"], "idx")
    assert O.normwise_rel_err(host(out), d["ex_pred_k20/out"]) <= OUT_TOL


@pytest.mark.parametrize("cfg", ["deit_base", "dit"])
def test_fused_attention_full_size_vs_oracle(M, cfg):
    """BASELINE configs at full batch: every head's top-k indices against the oracle's
    libstdc++ top-k of the kernel's own approximate scores, a sample of heads fully
    (scores, indices, output) against the oracle."""
    if cfg == "deit_base":
        B, H, N, D, k, scale = 256, 12, 197, 64, 20, 64 ** -0.5
    else:
        B, H, N, D, k, scale = 64, 16, 256, 72, 154, 72 ** -0.5
    q, kk, v = (torch.from_numpy(np.random.default_rng(s).standard_normal((B, H, N, D), dtype=np.float32)).cuda()
                for s in (0, 1, 2))
    out, idx, true_s, pred_s = M.mx_topk_attention(q, kk, v, scale, k_top=k, return_scores=True)
    pred_h = host(pred_s)
    # the approximate scores of EVERY image against the oracle's (16 images at a time), and
    # every head's indices against the oracle's libstdc++ top-k of the oracle's own scores
    qh, kh = host(q), host(kk)
    pred_o = np.empty_like(pred_h)
    for b0 in range(0, B, 16):
        aq, ak = O.approx_operands(qh[b0:b0 + 16], kh[b0:b0 + 16], "ex_pred")
        pred_o[b0:b0 + 16] = O.exact_matmul_f32(aq, np.swapaxes(ak, -1, -2))
    same(pred_h, pred_o, "pred (every image)")
    _, want = O.topk(pred_o.reshape(-1, N), k)
    same(host(idx).reshape(-1, k), want, "idx (all heads, the oracle's scores)")
    for b in (0, B // 2, B - 1):
        r = O.attention(host(q[b:b + 1]), host(kk[b:b + 1]), host(v[b:b + 1]), scale, k_top=k)
        same(host(true_s[b:b + 1]), r["true"], "true")
        same(pred_h[b:b + 1], r["pred"], "pred")
        same(host(idx[b:b + 1]), r["idx"], "idx")
        assert O.normwise_rel_err(host(out[b:b + 1]), r["out"]) <= OUT_TOL


PATHS = ("split",)


def _attn_all_paths(M, q, k, v, scale, **kw):
    """Run the op (selection kernel + finishing kernel for top-k)."""
    res = [M.mx_topk_attention(dev(q), dev(k), dev(v), scale, return_scores=True, **kw)]
    torch.cuda.synchronize()
    return [[host(t) for t in r] for r in res]


def _check_vs_oracle(got, r, what):
    out, idx, true_s, pred_s = got
    same(true_s, r["true"], what + " true")
    same(pred_s, r["pred"], what + " pred")
    same(idx, r["idx"], what + " idx")
    nan_o, nan_r = np.isnan(out), np.isnan(r["out"])
    same(nan_o, nan_r, what + " NaN rows")
    fin = ~nan_r.any(-1)
    assert O.normwise_rel_err(out[fin], r["out"][fin]) <= OUT_TOL, what


@pytest.mark.parametrize("D", [32, 64, 72, 128])
@pytest.mark.parametrize("N,T,k", [(197, 197, 20), (256, 256, 154), (5, 64, 7), (1, 20, 5), (70, 130, 65)])
def test_expred_paths_vs_oracle(M, D, N, T, k):
    """The op against the oracle over head dims of 1..4 MX blocks, short and long
    rows, k in both top-k branches."""
    rng = np.random.default_rng(D * 1000 + N)
    B, H = 2, 3
    q = rng.standard_normal((B, H, N, D), dtype=np.float32)
    kk = rng.standard_normal((B, H, T, D), dtype=np.float32)
    v = rng.standard_normal((B, H, T, D), dtype=np.float32)
    scale = float(D) ** -0.5
    outs = _attn_all_paths(M, q, kk, v, scale, k_top=k)
    r = O.attention(q, kk, v, scale, k_top=k)
    for got, name in zip(outs, PATHS):
        _check_vs_oracle(got, r, name)


@pytest.mark.parametrize("k", [20, 100])
def test_expred_special_rows(M, k):
    """Zero K rows (exponent -126 blocks), a wide exponent spread, NaN / Inf
    inputs, rows whose true scores overflow, all-zero query rows, block exponents around
    the bounds of the ex_pred key loop's fast range; k on the gather
    finishing kernel (20) and on the MFMA one (100: every key's exact epilogue, its fp64
    and NaN branches)."""
    rng = np.random.default_rng(5)
    B, H, N, T, D = 2, 4, 197, 197, 64
    q = rng.standard_normal((B, H, N, D), dtype=np.float32)
    kk = rng.standard_normal((B, H, T, D), dtype=np.float32)
    v = rng.standard_normal((B, H, T, D), dtype=np.float32)
    kk[0, 0, 7, :] = 0.0                        # zero key row: exponent -126 blocks, head falls back
    kk[0, 1, 11, 32:] *= np.float32(2.0 ** 40)  # exponent spread > 24 bits
    q[0, 2, 3, 5] = np.nan                      # NaN row
    q[0, 2, 9, 40] = np.inf                     # Inf row
    kk[1, 0, 50, 3] = np.nan                    # NaN key: head's preds all NaN in block 0
    q[1, 1, 17, :] *= np.float32(2.0 ** 100)    # true scores overflow for this row
    kk[1, 1, :, :] *= np.float32(2.0 ** 30)
    q[1, 2, :4, :] = 0.0                        # zero query rows (all preds tie)
    # block exponents across the ex_pred key loop's fast range [-50, 61] (mxa_select.hpp
    # kExpFastLo / Hi): keys at 2^59..2^63, query rows at 2^-49..-53, one key's blocks split
    kk[1, 3, :40, :] *= (np.float32(2.0) ** np.arange(59, 64, dtype=np.float32).repeat(8))[:, None]
    q[1, 3, 40:80, :] *= (np.float32(2.0) ** -np.arange(49, 54, dtype=np.float32).repeat(8))[:, None]
    kk[1, 3, 100, 32:] *= np.float32(2.0 ** -60)
    outs = _attn_all_paths(M, q, kk, v, 0.125, k_top=k)
    r = O.attention(q, kk, v, 0.125, k_top=k)
    for got, name in zip(outs, PATHS):
        _check_vs_oracle(got, r, name)


@pytest.mark.parametrize("D", [32, 64, 72, 128])
@pytest.mark.parametrize("N,T", [(197, 197), (256, 256), (77, 120), (5, 20), (40, 300)])
def test_dense_branch_vs_oracle(M, D, N, T):
    """The dense branch (top_k=False, deit main.py:149-152, DiT models.py:218-225): true scores
    bit-exact, the output within tolerance, on the MFMA finishing kernel with every key kept
    (T <= 256) and on the v_dot4 row kernel (T = 300); special rows: NaN / Inf inputs, a row
    whose bias masks every key (-inf: softmax NaN), zero rows, a wide exponent spread."""
    rng = np.random.default_rng(D * 7 + T)
    B, H = 2, 3
    q = rng.standard_normal((B, H, N, D), dtype=np.float32)
    kk = rng.standard_normal((B, H, T, D), dtype=np.float32)
    v = rng.standard_normal((B, H, T, D), dtype=np.float32)
    q[0, 0, min(3, N - 1), 1] = np.nan
    q[0, 1, min(4, N - 1), 0] = np.inf
    kk[1, 0, 2, :] = 0.0
    q[1, 1, 0, :] = 0.0
    kk[1, 2, 1, D // 2:] *= np.float32(2.0 ** 30)
    bias = np.zeros((B, 1, N, T), np.float32)
    bias[:, :, :, T // 2:] = -10000.0
    bias[1, 0, min(2, N - 1), :] = -np.inf
    fk = M._native.lib().mxa_attention_finish_kernel
    for bb in (None, bias):
        out, idx, true_s, _ = M.mx_topk_attention(dev(q), dev(kk), dev(v), D ** -0.5, top_k=False, return_scores=True,
                                                  bias=None if bb is None else dev(bb))
        assert idx is None
        r = O.attention(q, kk, v, D ** -0.5, top_k=False, bias=bb)
        same(host(true_s), r["true"], "true")
        o, ro = host(out), r["out"]
        same(np.isnan(o), np.isnan(ro), "NaN rows")
        fin = ~np.isnan(ro).any(-1)
        assert O.normwise_rel_err(o[fin], ro[fin]) <= OUT_TOL
    if T <= 256:
        import ctypes
        p, _, _, _ = M.ops._attn_params(dev(q), dev(kk), dev(v), D ** -0.5, 0, "ex_pred", False, False, None, False, 0,
                                        None)
        p.out = 16  # the query launches nothing
        assert fk(ctypes.byref(p)) == 4  # MXA_FIN_DENSE_MFMA


@pytest.mark.parametrize("mode,k", [("ex_pred", 20), ("ex_pred", 100), ("MXINT4", 20)])
def test_packed_pass_fallback_rows(M, mode, k):
    """Scattered query rows whose approximate scores do not pack into 32-bit elements (the
    query's second MX block scaled by 2^20: every score needs more than 16 significant bits)
    go from the packed selection pass to the 64-bit pass, next to rows the packed pass and
    the one-lane tail finish, in the same workgroups.  Every head's idx and prune mask
    against the oracle's libstdc++ top-k of the oracle's scores (mxa_select.hpp select_item:
    the per-workgroup fallback flag)."""
    rng = np.random.default_rng(11)
    B, H, N, D = 8, 12, 197, 64
    q = rng.standard_normal((B, H, N, D), dtype=np.float32)
    kk = rng.standard_normal((B, H, N, D), dtype=np.float32)
    v = rng.standard_normal((B, H, N, D), dtype=np.float32)
    r = np.arange(N)
    for b in range(B):
        for h in range(H):
            rows = r[(r * 7 + 3 * h + b) % 13 == 0]
            q[b, h, rows, 32:] *= np.float32(2.0 ** 20)
    out, idx, _, pred_s, mask = M.mx_topk_attention(dev(q), dev(kk), dev(v), 0.125, k_top=k, pred_mode=mode,
                                                    return_scores=True, return_mask=True)
    aq, ak = O.approx_operands(q, kk, mode)
    pred_o = O.exact_matmul_f32(aq, np.swapaxes(ak, -1, -2))
    same(host(pred_s), pred_o, "pred")
    _, want = O.topk(pred_o.reshape(-1, N), k)
    same(host(idx).reshape(-1, k), want, "idx")
    same(host(M.unpack_mask(mask, N)).reshape(-1, N), O.prune_mask(want, N), "mask")
    ro = O.attention(q[:1], kk[:1], v[:1], 0.125, k_top=k, pred_mode=mode)
    assert O.normwise_rel_err(host(out[:1]), ro["out"]) <= OUT_TOL


@pytest.mark.parametrize("mode", ["MXINT4", "two_step_leading_ones", "partial_Q", "partial_K"])
@pytest.mark.parametrize("N,T,k", [(197, 197, 20), (77, 120, 77), (33, 256, 154)])
def test_approx_modes_all_paths_vs_oracle(M, mode, N, T, k):
    """Approximator-code scoring (v_dot4, EXP / EXION-MUL block combine) on both
    fused kernels, odd row counts."""
    rng = np.random.default_rng(7)
    B, H, D = 1, 2, 72
    q = rng.standard_normal((B, H, N, D), dtype=np.float32)
    kk = rng.standard_normal((B, H, T, D), dtype=np.float32)
    v = rng.standard_normal((B, H, T, D), dtype=np.float32)
    outs = _attn_all_paths(M, q, kk, v, 72 ** -0.5, k_top=k, pred_mode=mode)
    r = O.attention(q, kk, v, 72 ** -0.5, k_top=k, pred_mode=mode)
    for got, name in zip(outs, PATHS):
        _check_vs_oracle(got, r, name)


def test_pixart_cross_full_batch(M):
    B, H, N, T, D, k = 8, 16, 256, 120, 72, 20
    rng = np.random.default_rng(0)
    q = rng.standard_normal((B, H, N, D), dtype=np.float32)
    kk = rng.standard_normal((B, H, T, D), dtype=np.float32)
    v = rng.standard_normal((B, H, T, D), dtype=np.float32)
    bias = np.where(np.arange(T) < 60, 0.0, -10000.0).astype(np.float32)[None, None, None, :].repeat(B, 0)
    for mode in ("MXINT4", "two_step_leading_ones", "ex_pred"):
        out, idx = M.mx_topk_attention(dev(q), dev(kk), dev(v), 1 / np.sqrt(72), k_top=k, pred_mode=mode,
                                       bias=dev(bias), flush_subnormals=True)
        r = O.attention(q, kk, v, 1 / np.sqrt(72), k_top=k, pred_mode=mode, bias=bias, flush=True)
        same(host(idx), r["idx"], mode)  # all 8 images
        assert O.normwise_rel_err(host(out), r["out"]) <= OUT_TOL


# ------------------------------------------------------------------ mx.matmul / Linear drop-in
def test_mx_matmul_dropin(M):
    d = load("attn_deit_tiny.npz")
    mx, _ = M.install_dropin()
    specs = {"a_elem_format": "int8", "w_elem_format": "int8", "block_size": 32, "scale_bits": 8, "bfloat": 32}
    q, k = dev(d["q"]), dev(d["k"])
    t = mx.matmul(q, k.transpose(-2, -1), mx_specs=specs) * float(d["scale"])
    same(host(t), d["true"], "mx.matmul QK^T")
    a = np.random.default_rng(5).standard_normal((4, 37, 100), dtype=np.float32)
    b = np.random.default_rng(6).standard_normal((4, 100, 45), dtype=np.float32)
    same(host(mx.matmul(dev(a), dev(b), mx_specs=specs)), O.mx_matmul(a, b), "ragged mx.matmul")


def test_linear_dropin(M):
    mx, _ = M.install_dropin()
    specs = {"a_elem_format": "int8", "w_elem_format": "int8", "block_size": 32, "scale_bits": 8, "bfloat": 32}
    lin = mx.Linear(96, 80, bias=True, mx_specs=specs).cuda()
    x = torch.randn(2, 7, 96, device="cuda")
    y = lin(x)
    same(host(y), O.mx_linear(host(x), host(lin.weight), host(lin.bias)), "mx.Linear drop-in")


@pytest.mark.parametrize("case,mode,approx,k_top", [("ex_pred_k20", "ex_pred", True, 20),
                                                    ("partial_Q_k20", "partial_Q", True, 20),
                                                    ("MXINT4_k20", "MXINT4", True, 20),
                                                    ("trueK_k30", None, False, 30)])
def test_unchanged_glue_exact_topk(M, case, mode, approx, k_top):
    """The DeiT glue (main.py:100-152, tests/glue_deit.py) run unchanged on the drop-in
    modules, its own `torch.topk` call served by bind_exact_topk: idx bit-exact against the
    reference's (attn_deit_tiny.npz), the output within tolerance."""
    M.install_dropin()
    import glue_deit
    from mx.specs import apply_mx_specs
    d = load("attn_deit_tiny.npz")
    specs = apply_mx_specs({"a_elem_format": "int8", "w_elem_format": "int8", "block_size": 32, "scale_bits": 8,
                            "bfloat": 32, "shared_exp_method": "max", "round": "nearest"})
    assert M.bind_exact_topk(glue_deit) == 1
    try:
        out, idx = glue_deit.attention_core(dev(d["q"]), dev(d["k"]), dev(d["v"]), float(d["scale"]), k_top, specs,
                                            pred_mode=mode or "ex_pred", approx=approx)
    finally:
        M.unbind_exact_topk(glue_deit)
    torch.cuda.synchronize()
    same(host(idx), d[f"{case}/idx"], f"{case} idx through the module's torch.topk")
    assert O.normwise_rel_err(host(out), d[f"{case}/out"]) <= OUT_TOL
    assert glue_deit.torch is torch


def test_exact_topk_namespace_forwards(M):
    """The rebound name is torch for everything but topk; unsupported topk forms are torch's."""
    T = M.exact_topk_torch
    assert T.zeros is torch.zeros and T.cuda is torch.cuda and T.float32 is torch.float32
    x = torch.randn(3, 40, device="cuda")
    r = T.topk(x, 5, dim=-1, largest=False)
    same(host(r.indices), host(torch.topk(x, 5, dim=-1, largest=False).indices), "largest=False passthrough")
    v, i = T.topk(x, 5)
    _, want = O.topk(host(x), 5)
    same(host(i), want, "exact order")
    same(host(v), np.take_along_axis(host(x), want, -1), "values")


# ------------------------------------------------------------------ fused qkv projection
def test_qkv_attention_vs_reference(M):
    """mx.Linear qkv projection fused into operand production (mxa_qkv_attention) against
    the reference's Linear + attention chain (linear_qkv.npz)."""
    d = load("linear_qkv.npz")
    out, idx, qkv = M.mx_qkv_attention(dev(d["x"]), dev(d["W"]), dev(d["bias"]), 3, float(d["scale"]), k_top=20,
                                       return_qkv=True)
    torch.cuda.synchronize()
    same(host(qkv), d["qkv"], "qkv projection")
    same(host(idx), d["idx"], "idx")
    assert O.normwise_rel_err(host(out), d["out"]) <= OUT_TOL


@pytest.mark.parametrize("mode", ["ex_pred", "MXINT4", "two_step_leading_ones", "true_ex", "partial_Q", "ELSA"])
@pytest.mark.parametrize("B,N,C,H,k_top", [(2, 197, 768, 12, 20), (2, 197, 768, 12, 30), (1, 256, 1152, 16, 154),
                                           (3, 45, 96, 2, 20)])
def test_qkv_attention_vs_oracle_chain(M, mode, B, N, C, H, k_top):
    """The fused projection + attention against the oracle chained the same way (exact
    projection, split, attention) on every image, at the DeiT-base (k = 20 and the
    --topk 30 variant) and DiT-XL/2 (k = 154, the 0.6 x 256 of the bench) block widths and a
    ragged small case; NaN token row and zero weight row included."""
    D = C // H
    if mode == "ELSA" and D not in (64, 72):
        pytest.skip("ELSA's structured matrix exists for d = 64, 72 only")
    rng = np.random.default_rng(B * 1000 + N)
    x = rng.standard_normal((B, N, C), dtype=np.float32)
    W = (rng.standard_normal((3 * C, C), dtype=np.float32) * np.float32(0.05)).astype(np.float32)
    bias = (rng.standard_normal(3 * C, dtype=np.float32) * np.float32(0.1)).astype(np.float32)
    x[0, 3, 7] = np.nan
    W[5] = 0.0
    k = min(k_top, N)
    proj = None
    if mode == "ELSA":
        from mx_quantization_amd.funcs import _create_structured_orthogonal_matrix
        torch.manual_seed(D)
        proj = _create_structured_orthogonal_matrix(D).numpy()
    wq = M.LinearWeightMX(dev(W), D)
    out, idx, qkv = M.mx_qkv_attention(dev(x), wq, dev(bias), H, D ** -0.5, k_top=k, pred_mode=mode,
                                       return_qkv=True, elsa_proj=None if proj is None else dev(proj))
    torch.cuda.synchronize()
    want_qkv = O.mx_linear(x, W, bias)
    same(host(qkv), want_qkv, "qkv")
    # the operands the fused kernel produced equal those of the unfused op on its q, k, v
    q, kk, v = O.qkv_split(want_qkv, H)
    r = O.attention(q, kk, v, D ** -0.5, k_top=k, pred_mode=mode, elsa_proj=proj)
    same(host(idx), r["idx"], "idx vs oracle")
    o_fin = ~np.isnan(r["out"]).any(-1)
    assert O.normwise_rel_err(host(out)[o_fin], r["out"][o_fin]) <= OUT_TOL
    o2, i2 = M.mx_topk_attention(*(dev(np.ascontiguousarray(t)) for t in (q, kk, v)), D ** -0.5, k_top=k,
                                 pred_mode=mode, elsa_proj=None if proj is None else dev(proj))
    same(host(idx), host(i2), "idx vs unfused op")
    same(host(out), host(o2), "out vs unfused op")


@pytest.mark.parametrize("H", [4, 2])
def test_qkv_projection_spread_paths(M, H):
    """The fused projection's three accumulations in one launch, bit-exact against the
    oracle: exponent-folded digits (row and column spreads <= 8), shifted int32 sums (row
    spreads 9 .. smax, or a head whose weight columns spread 10), fp64 block sums (wider,
    up to the 34-bit span they hold exactly).
    Rows scale alternate 32-channel blocks by 2^s; one head's q columns by 2^10, another's
    k columns by 2^8 (the digit limit itself); H = 2 (D = 128) the widest head.  The first
    32-token tile has every 32-channel block normalised to one exponent before its shift
    (s <= 8), so its row spreads are the shifts themselves: the digit path for the head
    groups whose weight columns spread <= 8; later tiles spread 9 .. 30."""
    B, N, C = 2, 70, 256
    D = C // H
    rng = np.random.default_rng(11 + H)
    x = rng.standard_normal((B, N, C), dtype=np.float32)
    W = (rng.standard_normal((3 * C, C), dtype=np.float32) * np.float32(0.05)).astype(np.float32)
    bias = (rng.standard_normal(3 * C, dtype=np.float32) * np.float32(0.1)).astype(np.float32)
    odd = (np.arange(C) // 32) % 2 == 1
    blk = x[:, :32].reshape(B, 32, C // 32, 32)
    e = np.floor(np.log2(np.abs(blk).max(-1, keepdims=True)))
    x[:, :32] = (blk * np.float32(2.0) ** -e).reshape(B, 32, C).astype(np.float32)  # block max in [1, 2)
    shifts = [0, 3, 8, 9, 12, 20, 30]  # fp64 block sums are exact to a 34-bit span
    for t in range(N):
        s = shifts[(t // 5) % 3] if t < 32 else shifts[(t // 5) % len(shifts)]  # first tile: s <= 8
        x[:, t, odd] *= np.float32(2.0 ** s)
    W[0 * C + 0 * D: 0 * C + 0 * D + D][:, odd] *= np.float32(2.0 ** 10)  # head 0's q columns
    hk = min(1, H - 1)
    W[1 * C + hk * D: 1 * C + hk * D + D][:, odd] *= np.float32(2.0 ** 8)  # a head's k columns
    wq = M.LinearWeightMX(dev(W), D)
    out, idx, qkv = M.mx_qkv_attention(dev(x), wq, dev(bias), H, D ** -0.5, k_top=10, return_qkv=True)
    torch.cuda.synchronize()
    same(host(qkv), O.mx_linear(x, W, bias), "qkv across the accumulation paths")
    q, kk, v = (dev(np.ascontiguousarray(t)) for t in O.qkv_split(host(qkv), H))
    o2, i2 = M.mx_topk_attention(q, kk, v, D ** -0.5, k_top=10)
    same(host(idx), host(i2), "idx vs unfused op")
    same(host(out), host(o2), "out vs unfused op")


def test_qkv_weight_header_checked(M):
    """mxa_qkv_attention refuses a prepared weight whose header does not match the call
    (ADVICE r2): other settings, an unprepared buffer; a copy of a good one is accepted
    (its header is read once) and gives the same result."""
    rng = np.random.default_rng(7)
    x = dev(rng.standard_normal((1, 64, 128), dtype=np.float32))
    W = dev(rng.standard_normal((3 * 128, 128), dtype=np.float32) * np.float32(0.05))
    wq = M.LinearWeightMX(W, 64)
    o1, i1 = M.mx_qkv_attention(x, wq, None, 2, 0.125, k_top=10)
    cp = M.LinearWeightMX.__new__(M.LinearWeightMX)
    cp.__dict__.update(wq.__dict__)
    cp.buf = wq.buf.clone()
    o2, i2 = M.mx_qkv_attention(x, cp, None, 2, 0.125, k_top=10)
    same(host(i1), host(i2), "copied weight idx")
    same(host(o1), host(o2), "copied weight out")
    spoof = M.LinearWeightMX.__new__(M.LinearWeightMX)
    spoof.__dict__.update(wq.__dict__)
    spoof.bfloat = 16  # passes the Python check, the header says bfloat 0
    with pytest.raises(M.NativeError):
        M.mx_qkv_attention(x, spoof, None, 2, 0.125, k_top=10, bfloat=16)
    blank = M.LinearWeightMX.__new__(M.LinearWeightMX)
    blank.__dict__.update(wq.__dict__)
    blank.buf = torch.zeros_like(wq.buf)
    with pytest.raises(M.NativeError):
        M.mx_qkv_attention(x, blank, None, 2, 0.125, k_top=10)


def test_analysis_hooks_on_device_tensors(M):
    """total_chosen_k / diff_idx_analysis (funcs/analysis.py:56-110, :136-157) on device
    idx / scores -- as the --anal runs call them on the GPU outputs (deit main.py:134-145)
    -- against the reference's values (analysis.npz)."""
    from mx_quantization_amd.funcs import analysis as A
    d = load("analysis.npz")
    idx = dev(d["idx"])
    assert A.total_chosen_k(idx) == pytest.approx(float(d["chosen_k"]), rel=1e-12)
    assert A.diff_idx_analysis(dev(d["true_vals"]), dev(d["scores"])) == pytest.approx(float(d["diff"]), rel=1e-6)
    # and on the fused op's own device idx: the union coverage of a real top-k output
    dt = load("attn_deit_tiny.npz")
    _, gidx = M.mx_topk_attention(dev(dt["q"]), dev(dt["k"]), dev(dt["v"]), float(dt["scale"]), k_top=20)
    assert A.total_chosen_k(gidx) == pytest.approx(A.total_chosen_k(torch.from_numpy(dt["ex_pred_k20/idx"])),
                                                   rel=1e-12)
