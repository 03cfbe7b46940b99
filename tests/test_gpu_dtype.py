"""GPU parity of the float16 / bfloat16 inputs and of torch.autocast, against vectors the
reference itself produced (tests/golden/gen_golden.py gen_dtype -> attn_dtype.npz).

The reference's ops follow their input's dtype (microxscaling/mx/mx_ops.py:85, :283;
elemwise_ops.py:146): shared exponents are floor(log2) computed in the dtype, a float16
all-zero block quantizes to NaN, and the matmuls return the dtype.  Under torch.autocast
(deit engine.py:97) the fp32 q / k / v keep fp32 quantization but the matmuls return the
autocast dtype and P = zeros_like(true scores) is of it (deit main.py:101-152).

Bit-exact: MX values, shared exponents, true / approximate scores, top-k indices, the NaN
pattern of the output.  Tolerance: the output, normwise over its finite elements, within
the dtype's rounding (float16 1e-3, bfloat16 8e-3: the reference's P.V order is unpinned,
SURVEY.md F7, and bfloat16 carries 8 significant bits)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TDT = {"f16": torch.float16, "bf16": torch.bfloat16}
TOL = {"f16": 1e-3, "bf16": 8e-3}


@pytest.fixture(scope="module")
def D():
    return np.load(os.path.join(G, "attn_dtype.npz"))


@pytest.fixture(scope="module")
def M():
    import mx_quantization_amd as m
    return m


def from_bits(bits, dt):
    return torch.from_numpy(np.ascontiguousarray(bits).view(np.int16)).view(TDT[dt]).cuda()


def to_f32(bits, dt):
    """uint16 bit patterns of the dtype -> float32 values (exact)."""
    return torch.from_numpy(np.ascontiguousarray(bits).view(np.int16)).view(TDT[dt]).float().numpy()


def host(t):
    return t.detach().float().cpu().numpy()


def same(a, b, what=""):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    ok = (a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else a == b
    if not ok.all():
        bad = np.argwhere(~ok)
        raise AssertionError(f"{what}: {bad.shape[0]}/{ok.size} mismatches, first {bad[:4].tolist()}: "
                             f"{a[tuple(bad[0])]} vs {b[tuple(bad[0])]}")


def out_close(got, ref, tol, what):
    """the NaN pattern bit-exact, the finite elements within tol normwise"""
    same(np.isnan(got), np.isnan(ref), what + " NaN pattern")
    fin = ~np.isnan(ref)
    if fin.any():
        g, r = got[fin].astype(np.float64), ref[fin].astype(np.float64)
        err = np.linalg.norm(g - r) / max(np.linalg.norm(r), 1e-30)
        assert err <= tol, f"{what}: normwise error {err:.3e} > {tol}"


@pytest.mark.parametrize("dt", ["f16", "bf16"])
def test_shared_exponents_every_value(M, D, dt):
    """_shared_exponents(method='none') on every positive finite value of the dtype."""
    x = from_bits(D[f"{dt}/sexp_x"], dt)
    got = M.shared_exponents(x, "none")
    assert got.dtype == TDT[dt]
    same(host(got), D[f"{dt}/sexp_none"], f"{dt} floor(log2)")


@pytest.mark.parametrize("dt", ["f16", "bf16"])
def test_quantize_mx_kats(M, D, dt):
    """quantize_mx_op on dtype tensors: random blocks, the float16 zero-block NaN, tiny
    and large blocks, inf / NaN, both axes, int4, subnormal flush."""
    from mx_quantization_amd.mx import mx_ops
    from mx_quantization_amd.mx.specs import apply_mx_specs
    base = dict(block_size=32, scale_bits=8, shared_exp_method="max", custom_cuda=False,
                mx_flush_fp32_subnorms=False)
    x = from_bits(D[f"{dt}/q_x"], dt)
    s = apply_mx_specs(base)
    for key, fmt, ax, spec in (("q_int8_ax1", "int8", -1, s), ("q_int4_ax1", "int4", -1, s),
                               ("q_int8_ax0", "int8", -2, s),
                               ("q_int8_flush", "int8", -1, apply_mx_specs(dict(base, mx_flush_fp32_subnorms=True)))):
        got = mx_ops.quantize_mx_op(x, spec, elem_format=fmt, axes=[ax])
        assert got.dtype == TDT[dt]
        same(host(got), D[f"{dt}/{key}"], f"{dt} {key}")
    if dt == "f16":  # the all-zero block of row 1 is NaN in float16 (0 / 2^-127 underflowed)
        assert np.isnan(D["f16/q_int8_ax1"][1, 32:64]).all()


@pytest.mark.parametrize("dt", ["f16", "bf16"])
@pytest.mark.parametrize("tag,mode,k_top", [("deit", "ex_pred", 20), ("deit", "MXINT4", 20),
                                            ("deit", "partial_Q", 20), ("dit", "ex_pred", 154)])
def test_attention_dtype_inputs(M, D, dt, tag, mode, k_top):
    q, k, v = (from_bits(D[f"{dt}/{tag}/{n}"], dt) for n in "qkv")
    sc = q.shape[-1] ** -0.5
    out, idx, true_s, pred_s = M.mx_topk_attention(q, k, v, sc, k_top=k_top, pred_mode=mode, return_scores=True)
    assert out.dtype == TDT[dt]
    pre = f"{dt}/{tag}/{mode}"
    if f"{pre}/true" in D.files:
        same(host(true_s), to_f32(D[f"{pre}/true"], dt), pre + " true")
    if f"{pre}/pred" in D.files:
        same(host(pred_s), to_f32(D[f"{pre}/pred"], dt), pre + " pred")
    same(host(idx), D[f"{pre}/idx"].astype(np.int64), pre + " idx")
    out_close(host(out), to_f32(D[f"{pre}/out"], dt), TOL[dt], pre + " out")


@pytest.mark.parametrize("dt", ["f16", "bf16"])
@pytest.mark.parametrize("tag", ["deit", "dit"])
def test_attention_dtype_dense(M, D, dt, tag):
    q, k, v = (from_bits(D[f"{dt}/{tag}/{n}"], dt) for n in "qkv")
    out, _ = M.mx_topk_attention(q, k, v, q.shape[-1] ** -0.5, top_k=False)
    out_close(host(out), to_f32(D[f"{dt}/{tag}/dense/out"], dt), TOL[dt], f"{dt}/{tag} dense")


@pytest.mark.parametrize("dt", ["f16", "bf16"])
@pytest.mark.parametrize("mode", ["ex_pred", "MXINT4", "dense"])
def test_attention_autocast(M, D, dt, mode):
    """fp32 q / k / v under torch.autocast: scores, P and out in the autocast dtype."""
    q, k, v = (torch.from_numpy(D[f"ac/{n}"]).cuda() for n in "qkv")
    pre = f"{dt}/ac/{mode}"
    if mode == "dense":
        out, _ = M.mx_topk_attention(q, k, v, 64 ** -0.5, top_k=False, autocast=TDT[dt])
        out_close(host(out), to_f32(D[f"{pre}/out"], dt), TOL[dt], pre)
        return
    out, idx, true_s, pred_s = M.mx_topk_attention(q, k, v, 64 ** -0.5, k_top=20, pred_mode=mode,
                                                   return_scores=True, autocast=TDT[dt])
    assert out.dtype == TDT[dt]
    if f"{pre}/true" in D.files:
        same(host(true_s), to_f32(D[f"{pre}/true"], dt), pre + " true")
        same(host(pred_s), to_f32(D[f"{pre}/pred"], dt), pre + " pred")
    same(host(idx), D[f"{pre}/idx"].astype(np.int64), pre + " idx")
    out_close(host(out), to_f32(D[f"{pre}/out"], dt), TOL[dt], pre + " out")


@pytest.mark.parametrize("dt", ["f16", "bf16"])
def test_qkv_attention_autocast_chain(M, D, dt):
    """mx.Linear qkv -> attention, both under torch.autocast, against the reference chain:
    projection bit-exact (fp32(dtype(x W^T)) + bias), idx bit-exact, out within tolerance."""
    x, W, b = (torch.from_numpy(D[f"acq/{n}"]).cuda() for n in ("x", "W", "bias"))
    out, idx, qkv = M.mx_qkv_attention(x, W, b, 3, 64 ** -0.5, k_top=20, pred_mode="ex_pred", return_qkv=True,
                                       autocast=TDT[dt])
    same(host(qkv), D[f"{dt}/acq/qkv"], f"{dt} autocast projection")
    same(host(idx), D[f"{dt}/acq/idx"].astype(np.int64), f"{dt} autocast chain idx")
    out_close(host(out), to_f32(D[f"{dt}/acq/out"], dt), TOL[dt], f"{dt} autocast chain out")


@pytest.mark.parametrize("dt", ["f16", "bf16"])
def test_mx_matmul_dtype(M, D, dt):
    from mx_quantization_amd.mx import matmul
    from mx_quantization_amd.mx.specs import apply_mx_specs
    s = apply_mx_specs(dict(block_size=32, scale_bits=8, shared_exp_method="max", custom_cuda=False,
                            a_elem_format="int8", w_elem_format="int8"))
    a, b = from_bits(D[f"{dt}/mm_a"], dt), from_bits(D[f"{dt}/mm_b"], dt)
    c = matmul(a, b, mx_specs=s, mode_config="aa")
    assert c.dtype == TDT[dt]
    out_close(host(c), D[f"{dt}/mm_c"], TOL[dt], f"{dt} mx.matmul")


def test_elsa_rejects_bias(M):
    """ELSA scores carry no bias in the reference (deit main.py:120-121)."""
    q = torch.randn(1, 2, 64, 64, device="cuda")
    with pytest.raises(ValueError, match="ELSA"):
        M.mx_approx_scores(q, q, "ELSA", bias=torch.zeros(64, 64, device="cuda"),
                           elsa_proj=torch.eye(64, device="cuda"))
