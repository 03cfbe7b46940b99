"""Generate the golden vectors in tests/golden/*.npz FROM THE REFERENCE ITSELF.

Run only in the build container (where /root/reference exists):

    python tests/golden/gen_golden.py

It imports the reference's own `mx` package (microxscaling/mx) and `funcs`
approximator API, and restates only the ~30 lines of attention-module glue
that cannot be imported (the workload modules need timm/diffusers, absent
here).  The glue follows workloads/deit/scripts/main.py:100-152,
workloads/DiT/models.py:168-225 and
workloads/PixArt/models/MX_transformer_block.py:792-859 line for line.

`exponent_based_sign()` raises in funcs/ (SURVEY.md F1), so ex_pred operands
are taken from partial_K() (Q side) and partial_Q() (K side) of fresh objects
and cross-checked against the working copy in
microxscaling/examples/deit/exponent_based_prediction.py.

Nothing from the reference is copied into the repo: only inputs and outputs.
"""
import importlib.util
import os
import sys

sys.dont_write_bytecode = True  # never write __pycache__ into the reference tree

import numpy as np
import torch

REF = os.environ.get("MXA_REFERENCE", "/root/reference")
sys.path.insert(0, os.path.join(REF, "microxscaling"))
sys.path.insert(0, REF)

import mx  # noqa: E402  (reference)
from mx.specs import apply_mx_specs  # noqa: E402
from mx.mx_ops import _quantize_mx, _shared_exponents, _reshape_to_blocks  # noqa: E402
from mx.elemwise_ops import quantize_elemwise_op  # noqa: E402
from funcs import exponent_approximation, elsa_approximation  # noqa: E402  (reference)
from funcs import _create_structured_orthogonal_matrix  # noqa: E402  (reference)

OUT = os.path.dirname(os.path.abspath(__file__))
torch.set_num_threads(8)

BASE_SPECS = {  # workloads/DiT/scripts/sample_ddp.py:51-67 (== deit main.py:716-736)
    'w_elem_format': 'int8', 'a_elem_format': 'int8', 'scale_bits': 8,
    'shared_exp_method': 'max', 'block_size': 32, 'bfloat': 32, 'fp': 0,
    'bfloat_subnorms': True, 'round': 'nearest', 'round_mx_output': 'nearest',
    'round_output': 'nearest', 'round_weight': 'nearest',
    'mx_flush_fp32_subnorms': False, 'custom_cuda': False, 'quantize_backprop': False,
}


def specs(**kw):
    d = dict(BASE_SPECS)
    d.update(kw)
    return apply_mx_specs(d)


def load_examples_module():
    path = os.path.join(REF, "microxscaling", "examples", "deit", "exponent_based_prediction.py")
    spec = importlib.util.spec_from_file_location("examples_ebp", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


EX = load_examples_module()


def approx_ops(q, k, s, mode):
    if mode == "ex_pred":
        aq = exponent_approximation(Q=q, K=k, mx_specs=s).partial_K()[0]
        ak = exponent_approximation(Q=q, K=k, mx_specs=s).partial_Q()[1]
        eq, ek = EX.exponent_approximation(q, k, s).exponent_based_sign()
        assert torch.equal(eq, aq) and torch.equal(ek, ak), "F2 cross-check failed"
        return aq, ak
    if mode == "true_ex":
        return EX.exponent_approximation(q, k, s).exponent_based_sign_leading_ones()
    obj = exponent_approximation(Q=q, K=k, mx_specs=s)
    return getattr(obj, mode)()


def attention_glue(q, k, v, s, scale, k_top, mode, top_k=True, approx=True, bias=None, proj=None):
    """The mx_quant branch of the patched attention forward (restated).  mode 'ELSA'
    takes the scores from elsa_approximation (orthogonal matrix `proj`), as the
    modules do (deit main.py:119-121, DiT models.py:187-189, PixArt :675-677)."""
    res = {}
    true_scores = mx.matmul(q, k.transpose(-2, -1), mx_specs=s, mode_config='aa')
    true_scores = true_scores * scale
    if bias is not None:
        true_scores += bias
    res["true"] = true_scores
    if top_k:
        if approx and mode == "ELSA":
            pred = elsa_approximation(Q=q, K=k, mx_specs=s, orthogonal_matrix=proj).approximation_scores()
            res["pred"] = pred
            _, idx = torch.topk(pred, k_top, dim=-1, largest=True, sorted=True)
            vals = true_scores.gather(dim=-1, index=idx)
        elif approx:
            aq, ak = approx_ops(q, k, s, mode)
            pred = aq @ ak.transpose(-2, -1)
            if bias is not None:
                pred = pred + bias
            res["aq"], res["ak"], res["pred"] = aq, ak, pred
            _, idx = torch.topk(pred, k_top, dim=-1, largest=True, sorted=True)
            vals = true_scores.gather(dim=-1, index=idx)
        else:
            vals, idx = torch.topk(true_scores, k_top, dim=-1, largest=True, sorted=True)
        res["idx"], res["vals"] = idx, vals
        attn = torch.zeros_like(true_scores)
        attn.scatter_(-1, idx, torch.softmax(vals, dim=-1).to(attn.dtype))
    else:
        attn = torch.softmax(true_scores, dim=-1)
    res["attn"] = attn
    res["out"] = mx.matmul(attn, v, mx_specs=s, mode_config='aa')
    # quantized operands of the dense GEMMs (for bit-level checks)
    from mx.mx_ops import quantize_mx_op  # reference op
    res["mx_q"] = quantize_mx_op(q, s, elem_format='int8', axes=[-1])
    res["mx_k"] = quantize_mx_op(k, s, elem_format='int8', axes=[-1])
    res["mx_v"] = quantize_mx_op(v, s, elem_format='int8', axes=[-2])
    return {kk: vv.numpy() for kk, vv in res.items()}


def rnd(shape, seed, mult=1.0):
    return (np.random.default_rng(seed).standard_normal(shape, dtype=np.float32) * np.float32(mult)).astype(np.float32)


def gen_attention():
    """One file per input set: inputs, scale and the mode-independent true scores once,
    then per-variant outputs keyed '<variant>/<name>'."""
    import math

    def pack(store, tag, r, keep=("pred", "aq", "ak", "idx", "out")):
        for kk in keep:
            if kk in r:
                # approximator operands are pinned on the first 32 rows of every head
                store[f"{tag}/{kk}"] = r[kk][..., :32, :] if kk in ("aq", "ak") else r[kk]

    # 1 DeiT-tiny single block (configs[0]): B1 H3 N197 d64, k=20; scale = 64**-0.5 (timm)
    for mult, fname in ((1.0, "attn_deit_tiny"), (3.0, "attn_deit_tiny_peaky")):
        q, k, v = (torch.from_numpy(rnd((1, 3, 197, 64), s, mult)) for s in (0, 1, 2))
        sc = 64 ** -0.5
        store = dict(q=q.numpy(), k=k.numpy(), v=v.numpy(), scale=np.float32(sc))
        r = attention_glue(q, k, v, specs(), sc, 20, "ex_pred")
        store.update(true=r["true"], mx_q=r["mx_q"][..., :64, :], mx_k=r["mx_k"][..., :64, :],
                     mx_v=r["mx_v"][..., :64, :])
        pack(store, "ex_pred_k20", r)
        if mult == 1.0:
            pack(store, "dense", attention_glue(q, k, v, specs(), sc, 20, "ex_pred", top_k=False), ("out",))
            pack(store, "trueK_k30", attention_glue(q, k, v, specs(), sc, 30, "ex_pred", approx=False),
                 ("idx", "out"))
            for mode in ("partial_Q", "partial_K", "MXINT4", "two_step_leading_ones", "true_ex"):
                pack(store, f"{mode}_k20", attention_glue(q, k, v, specs(), sc, 20, mode))
        np.savez_compressed(os.path.join(OUT, fname + ".npz"), **store)
        print("wrote", fname)
    # 3 DiT-XL/2 slice: B1 H2 N256 d72, k=154; scale = 72**-0.5 (models.py:130)
    q, k, v = (torch.from_numpy(rnd((1, 2, 256, 72), s)) for s in (0, 1, 2))
    sc = 72 ** -0.5
    r = attention_glue(q, k, v, specs(), sc, 154, "ex_pred")
    store = dict(q=q.numpy(), k=k.numpy(), v=v.numpy(), scale=np.float32(sc), true=r["true"])
    pack(store, "ex_pred_k154", r)
    np.savez_compressed(os.path.join(OUT, "attn_dit.npz"), **store)
    print("wrote attn_dit")
    # 5 PixArt cross-attn slice: q (1,2,256,72), k/v (1,2,120,72), 60 valid text tokens,
    #   bias = (1-mask)*-10000 (MX_pixart_transformer_2d.py:394-397), flush subnormals
    #   (text_local_inference_alpha.py:121), scale = 1/math.sqrt(72) (MX_transformer_block.py:791)
    q = torch.from_numpy(rnd((1, 2, 256, 72), 0))
    k = torch.from_numpy(rnd((1, 2, 120, 72), 1))
    v = torch.from_numpy(rnd((1, 2, 120, 72), 2))
    mask = torch.zeros(1, 120)
    mask[:, :60] = 1
    bias = ((1 - mask) * -10000.0).unsqueeze(1)  # (B,1,T)
    attn_bias = torch.zeros([256, 120]) + bias.unsqueeze(1).repeat(1, 2, 1, 1)  # (B,H,N,T)
    sc = 1 / math.sqrt(72)
    store = dict(q=q.numpy(), k=k.numpy(), v=v.numpy(), scale=np.float32(sc), bias=bias.numpy())
    for mode in ("MXINT4", "two_step_leading_ones", "ex_pred"):
        r = attention_glue(q, k, v, specs(mx_flush_fp32_subnorms=True), sc, 20, mode, bias=attn_bias)
        store["true"] = r["true"]
        pack(store, f"{mode}_k20", r)
    np.savez_compressed(os.path.join(OUT, "attn_pixart_cross.npz"), **store)
    print("wrote attn_pixart_cross")


def gen_attention_extra():
    """attn_extra.npz: ELSA (DeiT-tiny and DiT shapes; the orthogonal matrices made by
    the reference's _create_structured_orthogonal_matrix under fixed torch seeds, also
    kept as fixtures of the drop-in's own construction), and the bfloat16 variant
    (DiT sample.py:42 `bfloat=16`) of ex_pred attention at the DiT shape."""
    import math
    store = {}
    for tag, shape, k_top, seed in (("elsa_deit_k20", (1, 3, 197, 64), 20, 0), ("elsa_dit_k154", (1, 2, 256, 72), 154, 5)):
        d = shape[-1]
        torch.manual_seed(100 + d)
        proj = _create_structured_orthogonal_matrix(d)
        q, k, v = (torch.from_numpy(rnd(shape, seed + s_)) for s_ in (0, 1, 2))
        sc = d ** -0.5
        r = attention_glue(q, k, v, specs(), sc, k_top, "ELSA", proj=proj)
        store.update({f"{tag}/q": q.numpy(), f"{tag}/k": k.numpy(), f"{tag}/v": v.numpy(), f"{tag}/scale": np.float32(sc),
                      f"{tag}/proj": proj.numpy(), f"{tag}/proj_seed": np.int64(100 + d), f"{tag}/pred": r["pred"],
                      f"{tag}/idx": r["idx"], f"{tag}/out": r["out"], f"{tag}/true": r["true"]})
    # bfloat16 elementwise variant, DiT slice, ex_pred k=154 and the dense branch
    q, k, v = (torch.from_numpy(rnd((1, 2, 256, 72), 20 + s_)) for s_ in (0, 1, 2))
    sc = 72 ** -0.5
    r = attention_glue(q, k, v, specs(bfloat=16), sc, 154, "ex_pred")
    store.update({"bf16/q": q.numpy(), "bf16/k": k.numpy(), "bf16/v": v.numpy(), "bf16/scale": np.float32(sc),
                  "bf16/true": r["true"], "bf16/pred": r["pred"], "bf16/idx": r["idx"], "bf16/out": r["out"]})
    store["bf16/dense_out"] = attention_glue(q, k, v, specs(bfloat=16), sc, 154, "ex_pred", top_k=False)["out"]
    np.savez_compressed(os.path.join(OUT, "attn_extra.npz"), **store)
    print("wrote attn_extra")


def gen_linear_qkv():
    """linear_qkv.npz: the reference's mx.Linear qkv projection (linear.py:20-103) at the
    DeiT-tiny block shape (C = 192, 3 heads of 64; deit main.py:59-64, :87-88), then its
    ex_pred top-k attention on the reference's own q, k, v."""
    from mx import Linear
    x = torch.from_numpy(rnd((1, 197, 192), 30))
    W = torch.from_numpy(rnd((576, 192), 31, 0.08))
    bias = torch.from_numpy(rnd((576,), 32, 0.1))
    lin = Linear(192, 576, bias=True, mx_specs=specs())
    lin.weight.data = W.clone()
    lin.bias.data = bias.clone()
    with torch.no_grad():
        qkv = lin(x)
    q, k, v = qkv.reshape(1, 197, 3, 3, 64).permute(2, 0, 3, 1, 4)
    sc = 64 ** -0.5
    r = attention_glue(q.contiguous(), k.contiguous(), v.contiguous(), specs(), sc, 20, "ex_pred")
    np.savez_compressed(os.path.join(OUT, "linear_qkv.npz"), x=x.numpy(), W=W.numpy(), bias=bias.numpy(),
                        qkv=qkv.numpy(), scale=np.float32(sc), pred=r["pred"], idx=r["idx"], out=r["out"],
                        true=r["true"])
    print("wrote linear_qkv")


def gen_linear_proj():
    """linear_proj.npz: the reference's mx.Linear proj behind the attention (deit main.py:152-154,
    DiT models.py:225-227): x -> qkv Linear -> ex_pred top-k attention -> transpose/reshape ->
    proj Linear, at the DeiT-tiny block (3 heads of 64, k = 20) and a DiT-like block (4 heads of
    72, N = 256, k = 154: a 32-element block of C spans two heads); plus the proj Linear alone
    on given inputs (its exact-then-rounded product pinned bit for bit) and a ragged Linear
    (rows / features not multiples of 32)."""
    from mx import Linear
    store = {}
    for tag, (N, H, D, k_top, seed) in (("deit", (197, 3, 64, 20, 40)), ("dit", (256, 4, 72, 154, 50))):
        C = H * D
        x = torch.from_numpy(rnd((1, N, C), seed))
        W = torch.from_numpy(rnd((3 * C, C), seed + 1, 0.08))
        b = torch.from_numpy(rnd((3 * C,), seed + 2, 0.1))
        Wp = torch.from_numpy(rnd((C, C), seed + 3, 0.08))
        bp = torch.from_numpy(rnd((C,), seed + 4, 0.1))
        qkv_l = Linear(C, 3 * C, bias=True, mx_specs=specs())
        qkv_l.weight.data, qkv_l.bias.data = W.clone(), b.clone()
        proj_l = Linear(C, C, bias=True, mx_specs=specs())
        proj_l.weight.data, proj_l.bias.data = Wp.clone(), bp.clone()
        sc = D ** -0.5
        with torch.no_grad():
            qkv = qkv_l(x)
            q, k, v = qkv.reshape(1, N, 3, H, D).permute(2, 0, 3, 1, 4)
            r = attention_glue(q.contiguous(), k.contiguous(), v.contiguous(), specs(), sc, k_top, "ex_pred")
            xo = torch.from_numpy(r["out"]).transpose(1, 2).reshape(1, N, C)
            y = proj_l(xo)
        store.update({f"{tag}/x": x.numpy(), f"{tag}/W": W.numpy(), f"{tag}/b": b.numpy(), f"{tag}/Wp": Wp.numpy(),
                      f"{tag}/bp": bp.numpy(), f"{tag}/scale": np.float32(sc), f"{tag}/H": np.int64(H),
                      f"{tag}/k": np.int64(k_top), f"{tag}/idx": r["idx"], f"{tag}/attn_out": xo.numpy(),
                      f"{tag}/y": y.numpy()})
    xr = torch.from_numpy(rnd((37, 100), 60))
    Wr = torch.from_numpy(rnd((70, 100), 61, 0.1))
    br = torch.from_numpy(rnd((70,), 62, 0.1))
    lr = Linear(100, 70, bias=True, mx_specs=specs())
    lr.weight.data, lr.bias.data = Wr.clone(), br.clone()
    with torch.no_grad():
        store.update({"ragged/x": xr.numpy(), "ragged/W": Wr.numpy(), "ragged/b": br.numpy(), "ragged/y": lr(xr).numpy()})
    np.savez_compressed(os.path.join(OUT, "linear_proj.npz"), **store)
    print("wrote linear_proj")


def gen_analysis():
    """analysis.npz: the reference's funcs/analysis.py hooks (total_chosen_k :56-110,
    diff_idx_analysis :136-157, save_idx_file :22-29) on seeded top-k outputs."""
    import tempfile
    from funcs import total_chosen_k, diff_idx_analysis, save_idx_file
    g = torch.Generator().manual_seed(5)
    idx = torch.randint(0, 197, (3, 4, 197, 20), generator=g)
    true_vals = torch.rand((120, 2, 8, 20), generator=g)
    scores = torch.where(torch.rand((120, 2, 8, 20), generator=g) < 0.7, true_vals, torch.rand((120, 2, 8, 20), generator=g))
    with tempfile.TemporaryDirectory() as d:
        f = os.path.join(d, "idx.txt")
        save_idx_file(idx[:, :, :5, :], f, block_idx=3)
        text = open(f).read()
    # mismatch_analysis (:159-191): two save_idx_file outputs of a DiT-shaped layer (16 heads
    # x 256 tokens, so the token-255 / head-15 block stepping runs), indices from a small
    # alphabet so that both kept and missing entries occur
    from funcs import mismatch_analysis
    tk = torch.randint(0, 24, (2, 16, 256, 4), generator=g)  # save_idx_file writes batch entry 1 (:22-29)
    pk = torch.randint(0, 24, (2, 16, 256, 6), generator=g)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as d:
        ft, fp = os.path.join(d, "true.txt"), os.path.join(d, "pred.txt")
        save_idx_file(tk, ft, block_idx=0)
        save_idx_file(tk, ft, block_idx=1)  # a second block appended
        save_idx_file(pk, fp, block_idx=0)
        save_idx_file(pk, fp, block_idx=1)
        t_text, p_text = open(ft).read(), open(fp).read()
        os.chdir(d)
        try:
            res = mismatch_analysis(ft, fp)
            m_text = open(res).read()
        finally:
            os.chdir(cwd)
    np.savez_compressed(os.path.join(OUT, "analysis.npz"), idx=idx.numpy(), true_vals=true_vals.numpy(),
                        scores=scores.numpy(), chosen_k=np.float64(total_chosen_k(idx)),
                        diff=np.float64(diff_idx_analysis(true_vals, scores)), idx_text=np.array(text),
                        mm_true=np.array(t_text), mm_pred=np.array(p_text), mm_out=np.array(m_text),
                        mm_name=np.array(str(res)))
    print("wrote analysis")


def gen_quant_kat():
    """Known-answer + boundary vectors through the reference's _quantize_mx."""
    out = {}
    # test_corners_mx.py::test_mx_hw_test inputs (block 10, int8, nearest)
    hw = np.array([
        [1.0] * 10, [1.0] * 5 + [2.0] * 5, [-1.0] * 5 + [-2.0] * 5, [1.0] * 5 + [-2.0] * 5,
        [1.015625, 1.0234375, 1.03125, 1.0390625, 1.25, 1.2578125, 1.9375, 1.9453125, 1.984375, 1.9921875],
        [-1.984375, -1.9765625, -1.96875, -1.9609375, -1.9375, -1.9296875, -1.75, -1.7421875, -1.0, -1.9921875],
        [1.99609375, 1.98828125, 0.0, 0.00390625, 0.0078125, 0.01171875, -0.015625, -0.01171875, -0.0078125, -0.00390625],
    ], dtype=np.float32)
    out["hw_x"] = hw
    out["hw_y"] = _quantize_mx(torch.from_numpy(hw), 8, elem_format="int8", block_size=10, axes=1,
                               round="nearest").numpy()
    # F5 boundary set + corner blocks, 32-wide rows
    rng = np.random.default_rng(7)
    rows = []
    th = np.load(os.path.join(OUT, "exp_lut.npz"))["th_norm"]
    for E in range(1, 255):
        t = int(th[E])
        for M in sorted({max(0, t - 2), max(0, t - 1), min(t, (1 << 23) - 1), (1 << 23) - 1, 0}):
            mbits = np.uint32((E << 23) | M)
            blk = rng.standard_normal(32).astype(np.float32) * np.float32(0.3)
            blk = np.clip(blk, -0.99, 0.99) * mbits.view(np.float32)
            blk[rng.integers(32)] = mbits.view(np.float32) * (1 if rng.random() < 0.5 else -1)
            rows.append(blk.astype(np.float32))
    sub = np.array([1, 2, 3, 1 << 20, (1 << 23) - 1, (1 << 23) - 40], dtype=np.uint32)
    for s in sub:
        blk = np.zeros(32, np.float32)
        blk[:4] = s.view(np.float32)
        blk[4:8] = (s // 2).view(np.float32) if s > 1 else 0
        rows.append(blk)
    specials = [
        np.zeros(32, np.float32),
        np.full(32, 127.0 / 64, np.float32),
        np.linspace(-1, 1, 32, dtype=np.float32) * np.float32(1.9921875),
        (np.arange(32, dtype=np.float32) + np.float32(0.5)) / np.float32(64),  # half-way ties
        np.array([np.float32(3.4028235e38)] + [1.0] * 31, np.float32),
        np.array([np.inf] + [1.0] * 31, np.float32),
        np.array([-np.inf] + [1.0] * 31, np.float32),
        np.array([np.nan] + [1.0] * 31, np.float32),
        np.array([1e-38, -2e-39] + [0.0] * 30, np.float32),
    ]
    rows += specials
    for _ in range(64):
        rows.append((rng.standard_normal(32) * np.exp2(rng.integers(-140, 120))).astype(np.float32))
    X = np.stack(rows).astype(np.float32)
    out["x"] = X
    t = torch.from_numpy(X)
    for elem in ("int8", "int4", "int2"):
        for rnd_ in ("nearest", "floor", "even"):
            for flush in (False, True):
                y = _quantize_mx(t.clone(), 8, elem_format=elem, block_size=32, axes=[-1], round=rnd_,
                                 flush_fp32_subnorms=flush).numpy()
                out[f"y_{elem}_{rnd_}_{int(flush)}"] = y
    out["y_int8_nearest_0_sb5"] = _quantize_mx(t.clone(), 5, elem_format="int8", block_size=32, axes=[-1],
                                               round="nearest").numpy()
    # block sizes / axes through the spec-level op
    Z = rng.standard_normal((3, 70, 45)).astype(np.float32)
    out["z"] = Z
    for bs in (8, 9, 32, 64):
        for ax in (-1, -2, 0):
            out[f"z_bs{bs}_ax{ax}"] = _quantize_mx(torch.from_numpy(Z), 8, elem_format="int8", block_size=bs,
                                                   axes=[ax], round="nearest").numpy()
    # shared exponents (max / none) of the 32-blocks
    rb, *_ = _reshape_to_blocks(t, [-1], 32)
    out["sexp_max"] = _shared_exponents(rb, method="max", axes=[-1], ebits=0).numpy()
    out["sexp_none"] = _shared_exponents(rb, method="none", axes=[-1], ebits=0).numpy()
    # bfloat16 elementwise (DiT sample.py:42 variant) through quantize_elemwise_op
    bf = rng.standard_normal(4096).astype(np.float32) * np.exp2(rng.integers(-130, 125, 4096)).astype(np.float32)
    bf[:8] = [0.0, -0.0, np.inf, -np.inf, 3.3895314e38, 1.1754942e-38, 1e-45, 1.00390625]
    out["bf_x"] = bf
    out["bf_y"] = quantize_elemwise_op(torch.from_numpy(bf), specs(bfloat=16), round="nearest").numpy()
    np.savez_compressed(os.path.join(OUT, "quant_kat.npz"), **out)
    print("wrote quant_kat", X.shape)


def gen_topk_ties():
    """Tie-heavy ex_pred score rows + torch CPU topk order (pins F3/F4)."""
    out = {}
    cfgs = [("deit", (4, 12, 197, 64), (4, 12, 197, 64), 20), ("deit30", (2, 12, 197, 64), (2, 12, 197, 64), 30),
            ("dit", (2, 4, 256, 72), (2, 4, 256, 72), 154), ("cross", (2, 4, 256, 72), (2, 4, 120, 72), 20)]
    for name, qs, ks, k in cfgs:
        q = torch.from_numpy(rnd(qs, 10))
        kk = torch.from_numpy(rnd(ks, 11))
        aq, ak = approx_ops(q, kk, specs(), "ex_pred")
        pred = (aq @ ak.transpose(-2, -1)).reshape(-1, ks[-2])
        pred = pred[: 1024]
        _, idx = torch.topk(pred, k, dim=-1, largest=True, sorted=True)
        out[f"{name}_pred"] = pred.numpy()
        out[f"{name}_idx"] = idx.numpy().astype(np.int16)
        out[f"{name}_k"] = np.int64(k)
    # adversarial rows: constants, few distinct values, sorted, NaN/inf
    rng = np.random.default_rng(3)
    adv = []
    for n in (120, 197, 256):
        adv.append(np.zeros(n, np.float32))
        adv.append(np.arange(n, dtype=np.float32))
        adv.append(np.arange(n, dtype=np.float32)[::-1].copy())
        for nd in (2, 3, 5):
            for _ in range(8):
                adv.append(rng.integers(0, nd, n).astype(np.float32))
    advs = {}
    for i, r in enumerate(adv):
        n = r.shape[0]
        for k in (1, 2, 3, 20, 30, 77, 154):
            if k > n:
                continue
            _, idx = torch.topk(torch.from_numpy(r), k, largest=True, sorted=True)
            advs.setdefault(n, []).append((i, k, idx.numpy()))
    for n, lst in advs.items():
        rows = np.stack([adv[i] for i, _, _ in lst])
        ks_ = np.array([k for _, k, _ in lst])
        idxs = np.full((len(lst), n), -1, np.int16)
        for j, (_, k, idx) in enumerate(lst):
            idxs[j, :k] = idx
        out[f"adv{n}_rows"], out[f"adv{n}_k"], out[f"adv{n}_idx"] = rows, ks_, idxs
    np.savez_compressed(os.path.join(OUT, "topk_ties.npz"), **out)
    print("wrote topk_ties")


def _bits(t):
    """float16 / bfloat16 tensor -> its uint16 bit patterns (numpy holds no bfloat16)."""
    return t.contiguous().view(torch.int16).numpy().view(np.uint16)


def _f32(t):
    return t.float().numpy()  # exact: every float16 / bfloat16 value is a float32


def gen_dtype():
    """float16 / bfloat16 inputs (the reference's ops follow their input's dtype:
    mx_ops.py:85, :283, elemwise_ops.py:146) and torch.autocast around the attention
    glue (deit engine.py:97): exhaustive shared exponents, MX quantize KATs incl. the
    float16 zero-block NaN, attention cases, mx.matmul, and the autocast qkv chain."""
    from mx.mx_ops import quantize_mx_op
    out = {}
    s = specs()
    for name, dt, lim in (("f16", torch.float16, 0x7C00), ("bf16", torch.bfloat16, 0x7F80)):
        # every positive finite value: floor(log2(x)) in the dtype (method 'none')
        u = torch.arange(0, lim, dtype=torch.int32).to(torch.int16)
        x = u.view(dt)
        out[f"{name}/sexp_x"] = _bits(x)
        out[f"{name}/sexp_none"] = _f32(_shared_exponents(x, method="none"))
        # quantize KATs: random blocks + specials (zero block, tiny, large, inf/nan), both axes
        rng = np.random.default_rng(5)
        a = rng.standard_normal((6, 96), dtype=np.float32) * np.float32(3.0)
        a[1, 32:64] = 0.0                        # all-zero block
        a[2, :32] *= np.float32(2.0 ** -20)      # tiny block (float16 subnormals)
        a[3, 64:] *= np.float32(2.0 ** 10)       # large block
        a[4, 5] = np.inf
        a[5, 40] = np.nan
        a[0, :32] = np.linspace(-1, 1, 32, dtype=np.float32) * np.float32(1.9921875)
        at = torch.from_numpy(a).to(dt)
        out[f"{name}/q_x"] = _bits(at)
        out[f"{name}/q_int8_ax1"] = _f32(quantize_mx_op(at, s, elem_format="int8", axes=[-1]))
        out[f"{name}/q_int4_ax1"] = _f32(quantize_mx_op(at, s, elem_format="int4", axes=[-1]))
        out[f"{name}/q_int8_ax0"] = _f32(quantize_mx_op(at, s, elem_format="int8", axes=[-2]))
        out[f"{name}/q_int8_flush"] = _f32(quantize_mx_op(at, specs(mx_flush_fp32_subnorms=True),
                                                          elem_format="int8", axes=[-1]))
        # the attention glue on dtype tensors (DeiT-tiny, DiT slice)
        for tag, shp, k_top, modes in (("deit", (1, 3, 197, 64), 20, ("ex_pred", "MXINT4", "partial_Q")),
                                       ("dit", (1, 2, 256, 72), 154, ("ex_pred",))):
            q = torch.from_numpy(rnd(shp, 20)).to(dt)
            kk = torch.from_numpy(rnd(shp, 21)).to(dt)
            v = torch.from_numpy(rnd(shp, 22)).to(dt)
            out[f"{name}/{tag}/q"], out[f"{name}/{tag}/k"], out[f"{name}/{tag}/v"] = _bits(q), _bits(kk), _bits(v)
            sc = shp[-1] ** -0.5
            for mode in modes:
                r = attention_glue_t(q, kk, v, s, sc, k_top, mode)
                keys = ("idx", "out") if mode != "ex_pred" else (("true", "pred", "idx", "out") if tag == "deit" else
                                                                 ("pred", "idx", "out"))
                for key in keys:
                    out[f"{name}/{tag}/{mode}/{key}"] = r[key]
            out[f"{name}/{tag}/dense/out"] = attention_glue_t(q, kk, v, s, sc, k_top, "ex_pred", top_k=False)["out"]
        # mx.matmul on dtype tensors
        a2 = torch.from_numpy(rnd((2, 40, 72), 30)).to(dt)
        b2 = torch.from_numpy(rnd((2, 72, 24), 31)).to(dt)
        out[f"{name}/mm_a"], out[f"{name}/mm_b"] = _bits(a2), _bits(b2)
        out[f"{name}/mm_c"] = _f32(mx.matmul(a2, b2, mx_specs=s, mode_config="aa"))
        # torch.autocast around the fp32 attention (deit engine.py:97 + main.py:101-152)
        shp = (1, 3, 197, 64)
        q, kk, v = (torch.from_numpy(rnd(shp, sd)) for sd in (40, 41, 42))
        out["ac/q"], out["ac/k"], out["ac/v"] = q.numpy(), kk.numpy(), v.numpy()
        with torch.autocast("cpu", dtype=dt):
            for mode in ("ex_pred", "MXINT4"):
                r = attention_glue_t(q, kk, v, s, 64 ** -0.5, 20, mode)
                for key in (("true", "pred", "idx", "out") if mode == "ex_pred" else ("idx", "out")):
                    out[f"{name}/ac/{mode}/{key}"] = r[key]
            out[f"{name}/ac/dense/out"] = attention_glue_t(q, kk, v, s, 64 ** -0.5, 20, "ex_pred", top_k=False)["out"]
        # the autocast qkv chain: mx.Linear (autocast) -> split -> attention (autocast)
        rng = np.random.default_rng(50)
        C, H = 192, 3
        x = torch.from_numpy(rng.standard_normal((1, 197, C), dtype=np.float32))
        lin = mx.Linear(C, 3 * C, bias=True, mx_specs=s)
        with torch.no_grad():
            lin.weight.copy_(torch.from_numpy(rng.standard_normal((3 * C, C), dtype=np.float32) * np.float32(C ** -0.5)))
            lin.bias.copy_(torch.from_numpy(rng.standard_normal(3 * C, dtype=np.float32) * np.float32(0.02)))
            out["acq/x"], out["acq/W"], out["acq/bias"] = x.numpy(), lin.weight.numpy().copy(), lin.bias.numpy().copy()
            with torch.autocast("cpu", dtype=dt):
                qkv = lin(x)
                qq, kq, vq = qkv.reshape(1, 197, 3, H, C // H).permute(2, 0, 3, 1, 4)
                r = attention_glue_t(qq, kq, vq, s, (C // H) ** -0.5, 20, "ex_pred")
            out[f"{name}/acq/qkv"] = qkv.numpy()
            for key in ("idx", "out"):
                out[f"{name}/acq/{key}"] = r[key]
    np.savez_compressed(os.path.join(OUT, "attn_dtype.npz"), **out)
    print("wrote attn_dtype")


def attention_glue_t(q, k, v, s, scale, k_top, mode, top_k=True):
    """attention_glue for float16 / bfloat16 / autocast: the same glue, outputs as float32
    arrays of the dtype's values (idx int64)."""
    res = {}
    true_scores = mx.matmul(q, k.transpose(-2, -1), mx_specs=s, mode_config='aa')
    true_scores = true_scores * scale
    res["true"] = true_scores
    if top_k:
        aq, ak = approx_ops(q, k, s, mode)
        pred = aq @ ak.transpose(-2, -1)
        res["pred"] = pred
        _, idx = torch.topk(pred, k_top, dim=-1, largest=True, sorted=True)
        vals = true_scores.gather(dim=-1, index=idx)
        res["idx"] = idx
        attn = torch.zeros_like(true_scores)
        attn.scatter_(-1, idx, torch.softmax(vals, dim=-1).to(attn.dtype))
    else:
        attn = torch.softmax(true_scores, dim=-1)
    res["out"] = mx.matmul(attn, v, mx_specs=s, mode_config='aa')
    # compact: idx int16, the rest as uint16 bit patterns of the 16-bit dtype (float32 when it is float32)
    return {kk: (vv.numpy().astype(np.int16) if vv.dtype == torch.int64 else
                 (vv.numpy() if vv.dtype == torch.float32 else _bits(vv))) for kk, vv in res.items()}


if __name__ == "__main__":
    which = sys.argv[1:] or ["quant_kat", "topk_ties", "attention", "attention_extra", "linear_qkv", "linear_proj", "analysis",
                             "dtype"]
    for w in which:
        globals()["gen_" + w]()
