"""Pin the CPU oracle (oracle/) against golden vectors generated from the reference.

Bit-exact: MX values / shared exponents, approximator operands, approximate and
true scores, top-k indices (torch order) and prune masks.  Tolerance (normwise,
SURVEY.md F7): the attention output.
"""
import os

import numpy as np
import pytest

from oracle import mx_oracle as O

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(G, name))


def same(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    if a.dtype.kind == "f":
        ok = (a == b) | (np.isnan(a) & np.isnan(b))
        bad = np.argwhere(~ok)
        assert ok.all(), f"{bad.shape[0]} mismatches, first at {bad[:3].tolist()}: {a[tuple(bad[0])]} vs {b[tuple(bad[0])]}"
    else:
        assert np.array_equal(a, b)


# ---------------------------------------------------------------- exponent rule
def test_exp_lut_matches_floor_log2():
    lut = load("exp_lut.npz")
    th = lut["th_norm"].astype(np.int64)
    rng = np.random.default_rng(1)
    bits = []
    for E in range(1, 255):
        t = int(min(th[E], (1 << 23) - 1))
        lo, hi = max(0, t - 64), min(1 << 23, t + 64)
        bits.append(np.arange((E << 23) | lo, (E << 23) | hi, dtype=np.uint32))
        bits.append(((E << 23) | rng.integers(0, 1 << 23, 256)).astype(np.uint32))
    bits.append(np.arange(1, 1 << 16, dtype=np.uint32))
    bits.append(np.arange((1 << 23) - 4096, 1 << 23, dtype=np.uint32))
    b = np.concatenate(bits)
    E = (b >> 23).astype(np.int64)
    M = (b & 0x7FFFFF).astype(np.int64)
    want = np.where(E > 0, E - 127 + (M >= th[E]), 0)
    sub = E == 0
    j = np.floor(np.log2(np.maximum(M[sub], 1))).astype(np.int64)
    want[sub] = -149 + j + (M[sub] >= lut["th_sub"].astype(np.int64)[j])
    got = O.floor_log2_f32(b.view(np.float32)).astype(np.int64)
    assert np.array_equal(want, got)


def test_device_closed_form_thresholds_match_lut():
    """The kernels' closed form (mxa_common.hpp floor_log2_abs_bits: the gap below
    2^23 by exponent octave) equals the bisected threshold table, entry by entry."""
    lut = load("exp_lut.npz")
    for E in range(1, 255):
        e = E - 127
        u = e if e >= 0 else -e - 1
        o = u.bit_length() - 1 if u >= 2 else 0
        gap = (0x2C160B05020100 >> (8 * o)) & 0xFF
        assert int(lut["th_norm"][E]) == (1 << 23) - gap, E
    for j in range(23):
        gap = 0 if j < 17 else (0x160B0B050201 >> (8 * (j - 17))) & 0xFF
        th = (2 << j) - gap
        assert int(lut["th_sub"][j]) == th, j


def test_exp_rule_vs_torch_sample():
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(2)
    b = rng.integers(1, 0x7F800000, 1 << 20).astype(np.uint32)
    x = b.view(np.float32)
    ref = torch.floor(torch.log2(torch.from_numpy(x))).numpy()
    same(O.floor_log2_f32(x), ref)


# ---------------------------------------------------------------- MX quantize
def test_hw_kat():
    d = load("quant_kat.npz")
    y = O.quantize_mx(d["hw_x"], "int8", 10, 1)[0]
    same(y, d["hw_y"])


@pytest.mark.parametrize("elem", ["int8", "int4", "int2"])
@pytest.mark.parametrize("rnd", ["nearest", "floor", "even"])
@pytest.mark.parametrize("flush", [False, True])
def test_quant_boundary_vectors(elem, rnd, flush):
    d = load("quant_kat.npz")
    y = O.quantize_mx(d["x"], elem, 32, -1, 8, rnd, flush)[0]
    same(y, d[f"y_{elem}_{rnd}_{int(flush)}"])


def test_quant_scale_bits5():
    d = load("quant_kat.npz")
    same(O.quantize_mx(d["x"], "int8", 32, -1, 5)[0], d["y_int8_nearest_0_sb5"])


@pytest.mark.parametrize("bs", [8, 9, 32, 64])
@pytest.mark.parametrize("ax", [-1, -2, 0])
def test_quant_block_axis(bs, ax):
    d = load("quant_kat.npz")
    same(O.quantize_mx(d["z"], "int8", bs, ax)[0], d[f"z_bs{bs}_ax{ax}"])


def test_shared_exponents():
    d = load("quant_kat.npz")
    Ab, _ = O.to_blocks(d["x"], -1, 32)
    same(O.shared_exponents(Ab, "max"), d["sexp_max"])
    same(O.shared_exponents(Ab, "none"), d["sexp_none"])


def test_bfloat16_elemwise():
    d = load("quant_kat.npz")
    same(O.quantize_bfloat(d["bf_x"], 16), d["bf_y"])


# ---------------------------------------------------------------- top-k order
@pytest.mark.parametrize("name", ["deit", "deit30", "dit", "cross"])
def test_topk_ties_exact_order(name):
    d = load("topk_ties.npz")
    k = int(d[f"{name}_k"])
    _, idx = O.topk(d[f"{name}_pred"], k)
    same(idx.astype(np.int16), d[f"{name}_idx"])


@pytest.mark.parametrize("n", [120, 197, 256])
def test_topk_adversarial(n):
    d = load("topk_ties.npz")
    rows, ks, want = d[f"adv{n}_rows"], d[f"adv{n}_k"], d[f"adv{n}_idx"]
    for r, k, w in zip(rows, ks, want):
        _, idx = O.topk(r[None], int(k))
        assert np.array_equal(idx[0].astype(np.int16), w[:k])


# ---------------------------------------------------------------- attention
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
    ("attn_pixart_cross.npz", "MXINT4_k20", dict(pred_mode="MXINT4", k_top=20, flush=True)),
    ("attn_pixart_cross.npz", "two_step_leading_ones_k20",
     dict(pred_mode="two_step_leading_ones", k_top=20, flush=True)),
    ("attn_pixart_cross.npz", "ex_pred_k20", dict(pred_mode="ex_pred", k_top=20, flush=True)),
]


@pytest.mark.parametrize("fname,tag,kw", CASES, ids=[f"{f[5:-4]}:{t}" for f, t, _ in CASES])
def test_attention_vs_reference(fname, tag, kw):
    d = load(fname)
    bias = d["bias"][:, :, None, :] if "bias" in d.files else None
    r = O.attention(d["q"], d["k"], d["v"], float(d["scale"]), bias=bias, **kw)
    same(r["true"], d["true"])
    if f"{tag}/pred" in d.files:
        same(r["pred"], d[f"{tag}/pred"])
        same(r["aq"][..., :32, :], d[f"{tag}/aq"])
        same(r["ak"][..., :32, :], d[f"{tag}/ak"])
    if f"{tag}/idx" in d.files:
        same(r["idx"], d[f"{tag}/idx"])
        T = d["true"].shape[-1]
        same(O.prune_mask(r["idx"], T), O.prune_mask(d[f"{tag}/idx"], T))
    err = O.normwise_rel_err(r["out"], d[f"{tag}/out"])
    # product bar (north star): 1e-3 normwise.  Softmax ulps flip P's MX rounding:
    # measured 3.9e-4 on the x3 "peaky" input, <=1e-6 elsewhere.
    assert err <= 1e-3, err
    if "mx_q" in d.files:
        same(O.quantize_mx(d["q"], "int8", 32, -1)[0][..., :64, :], d["mx_q"])
        same(O.quantize_mx(d["k"], "int8", 32, -1)[0][..., :64, :], d["mx_k"])
        same(O.quantize_mx(d["v"], "int8", 32, -2)[0][..., :64, :], d["mx_v"])


# ---------------------------------------------------------------- ELSA, bfloat16 (attn_extra.npz)
EXTRA = [
    ("elsa_deit_k20", dict(pred_mode="ELSA", k_top=20)),
    ("elsa_dit_k154", dict(pred_mode="ELSA", k_top=154)),
    ("bf16", dict(pred_mode="ex_pred", k_top=154, bfloat=16)),
]


@pytest.mark.parametrize("tag,kw", EXTRA, ids=[t for t, _ in EXTRA])
def test_attention_extra_vs_reference(tag, kw):
    d = load("attn_extra.npz")
    g = lambda n: d[f"{tag}/{n}"]
    proj = g("proj") if kw["pred_mode"] == "ELSA" else None
    r = O.attention(g("q"), g("k"), g("v"), float(g("scale")), elsa_proj=proj, **kw)
    same(r["true"], g("true"))
    same(r["pred"], g("pred"))
    same(r["idx"], g("idx"))
    assert O.normwise_rel_err(r["out"], g("out")) <= 1e-3
    if tag == "bf16":
        rd = O.attention(g("q"), g("k"), g("v"), float(g("scale")), top_k=False, bfloat=16)
        assert O.normwise_rel_err(rd["out"], g("dense_out")) <= 1e-3


@pytest.mark.parametrize("d", [64, 72])
def test_dropin_structured_orthogonal_matrix(d):
    """funcs._create_structured_orthogonal_matrix of the drop-in draws the same
    torch.randn stream and runs the same modified Gram-Schmidt arithmetic as
    funcs/elsa_approximation.py:5-58: bit-identical matrices for the same seed."""
    import torch
    from mx_quantization_amd.funcs import _create_structured_orthogonal_matrix
    ex = load("attn_extra.npz")
    tag = "elsa_deit_k20" if d == 64 else "elsa_dit_k154"
    torch.manual_seed(int(ex[f"{tag}/proj_seed"]))
    P = _create_structured_orthogonal_matrix(d).numpy()
    same(P, ex[f"{tag}/proj"])


def test_linear_qkv_chain_vs_reference():
    """The oracle's mx.Linear (exact-then-round) on the reference's qkv fixture, and the
    ex_pred attention chained on it (linear_qkv.npz from gen_golden.py)."""
    d = load("linear_qkv.npz")
    qkv = O.mx_linear(d["x"], d["W"], d["bias"])
    same(qkv, d["qkv"])
    q, k, v = O.qkv_split(qkv, 3)
    r = O.attention(q, k, v, float(d["scale"]), k_top=20)
    same(r["true"], d["true"])
    same(r["pred"], d["pred"])
    same(r["idx"], d["idx"])
    assert O.normwise_rel_err(r["out"], d["out"]) <= 1e-3


@pytest.mark.parametrize("dt", ["f16", "bf16"])
def test_dtype_exponent_rule_matches_reference_on_every_value(dt):
    """floor(log2) computed in float16 / bfloat16 (the reference's ops on tensors of
    those dtypes) restated per binade, against torch on every positive finite value."""
    d = np.load(os.path.join(G, "attn_dtype.npz"))
    got = O.floor_log2_dtype(d[f"{dt}/sexp_x"], dt)
    ref = d[f"{dt}/sexp_none"].astype(np.float64)
    assert np.array_equal(got, ref)


def test_oracle_linear_proj_golden():
    """oracle.mx_linear against the reference's mx.Linear (linear_proj.npz): the proj on the
    reference attention output at the DeiT-tiny / DiT-like widths and a ragged Linear."""
    d = np.load(os.path.join(G, "linear_proj.npz"))
    for tag in ("deit", "dit"):
        y = O.mx_linear(d[f"{tag}/attn_out"], d[f"{tag}/Wp"], d[f"{tag}/bp"])
        assert np.array_equal(y, d[f"{tag}/y"]), tag
    assert np.array_equal(O.mx_linear(d["ragged/x"], d["ragged/W"], d["ragged/b"]), d["ragged/y"])
