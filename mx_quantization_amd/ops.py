"""torch-facing wrappers over the C ABI.  torch only allocates and supplies the
stream; every byte of arithmetic happens in libmxa.so on the MI355X."""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import torch

from . import _native as N
from ._native import check, lib, require_device, stream_ptr

_WS: dict = {}
_ELSA_COS: dict = {}


def _workspace(device: torch.device, nbytes: int) -> torch.Tensor:
    key = (device, stream_ptr(device))
    buf = _WS.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
        _WS[key] = buf
    return buf


def _f32(t: torch.Tensor, name: str) -> torch.Tensor:
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32 (got {t.dtype})")
    return t


def _dt(t: torch.Tensor, name: str) -> int:
    """MXA_DT_* of a float32 / float16 / bfloat16 tensor.  The kernels read the tensor in
    its own dtype and follow the reference's dtype rules (include/mxa.h MXA_DT_*)."""
    try:
        return N.DTYPES[t.dtype]
    except KeyError:
        raise TypeError(f"{name} must be float32, float16 or bfloat16 (got {t.dtype})") from None


def autocast_dtype(device_type: str = "cuda"):
    """torch.autocast's lower-precision dtype when it is enabled for `device_type`, else None."""
    if torch.is_autocast_enabled(device_type):
        return torch.get_autocast_dtype(device_type)
    return None


def _split(shape, axis):
    axis = axis % len(shape) if len(shape) else 0
    outer = 1
    for s in shape[:axis]:
        outer *= s
    inner = 1
    for s in shape[axis + 1:]:
        inner *= s
    return outer, (shape[axis] if len(shape) else 1), inner


def quantize_mx(A: torch.Tensor, elem_mbits: int = 8, block_size: int = 32, axis: int = -1, scale_bits: int = 8,
                round: str = "nearest", flush: bool = False, bfloat: int = 0, want_codes: bool = False):
    """MX block quantization along one axis (mx_ops.py:180-306).  Returns the
    dequantized tensor, plus (codes int8, block exponents int16) if want_codes."""
    dev = require_device(A)
    dt = _dt(A, "A")
    A = A.contiguous()
    y = torch.empty_like(A)
    outer, L, inner = _split(tuple(A.shape), axis)
    codes = exps = None
    if want_codes:
        bs = L if block_size == 0 else block_size
        codes = torch.empty(A.shape, dtype=torch.int8, device=dev)
        exps = torch.empty((outer, (L + bs - 1) // max(bs, 1), inner), dtype=torch.int16, device=dev)
    if A.numel():
        check(lib().mxa_quantize_mx(A.data_ptr(), y.data_ptr(), codes.data_ptr() if want_codes else None,
                                    exps.data_ptr() if want_codes else None, outer, L, inner, block_size,
                                    elem_mbits, scale_bits, N.ROUND_MODES[round], int(flush), int(bfloat), dt,
                                    stream_ptr(dev)), "mxa_quantize_mx")
    return (y, codes, exps) if want_codes else y


def shared_exponents(A: torch.Tensor, method: str = "max", axis: int = -1, block_size: int = 0,
                     ebits: int = 0) -> torch.Tensor:
    """_shared_exponents (mx_ops.py:49-99) for one axis; 'max' keeps the axis as
    the block count (size 1 when block_size covers the axis)."""
    dev = require_device(A)
    dt = _dt(A, "A")
    A = A.contiguous()
    outer, L, inner = _split(tuple(A.shape), axis)
    if method == "none":
        out = torch.empty_like(A)
        m = 1
    elif method == "max":
        bs = L if block_size == 0 else block_size
        shape = list(A.shape)
        shape[axis % A.dim()] = (L + bs - 1) // bs
        out = torch.empty(shape, dtype=A.dtype, device=dev)
        m = 0
    else:
        raise ValueError(f"Unrecognized shared exponent selection method {method}")
    if A.numel():
        check(lib().mxa_shared_exponents(A.data_ptr(), out.data_ptr(), outer, L, inner, block_size, m, ebits, dt,
                                         stream_ptr(dev)), "mxa_shared_exponents")
    return out


def quantize_bfloat(A: torch.Tensor, bfloat: int = 16, round: str = "nearest", allow_denorm: bool = True):
    """bfloatX elementwise quantization (elemwise_ops.py:201-216)."""
    dev = require_device(A)
    dt = _dt(A, "A")
    A = A.contiguous()
    y = torch.empty_like(A)
    if A.numel():
        check(lib().mxa_quantize_bfloat(A.data_ptr(), y.data_ptr(), A.numel(), int(bfloat), N.ROUND_MODES[round],
                                        int(allow_denorm), dt, stream_ptr(dev)), "mxa_quantize_bfloat")
    return y


OP_KINDS = {"sign": N.MXA_OP_SIGN, "mxint8": N.MXA_OP_MXINT8, "mxint4": N.MXA_OP_MXINT4,
            "exion": N.MXA_OP_EXION, "true_ex": N.MXA_OP_TRUE_EX}


def approx_values(X: torch.Tensor, kind: str, flush: bool = False, bfloat: int = 0) -> torch.Tensor:
    """Approximator operand values along the last axis (funcs/exponent_based_prediction.py)."""
    dev = require_device(X)
    dt = _dt(X, "X")
    X = X.contiguous()
    out = torch.empty_like(X)
    d = X.shape[-1]
    rows = X.numel() // d if d else 0
    if rows:
        check(lib().mxa_approx_values(X.data_ptr(), out.data_ptr(), rows, d, d, d, OP_KINDS[kind], int(flush),
                                      int(bfloat), dt, stream_ptr(dev)), "mxa_approx_values")
    return out


def topk(vals: torch.Tensor, k: int, return_mask: bool = False, packed: bool = True):
    """torch.topk(vals, k, dim=-1, largest=True, sorted=True) with torch's CPU
    index order (TopKImpl.h:45-86), computed on the device.  Returns (values, idx),
    plus the prune mask as packed words (..., ceil(n/32)) int32 if return_mask.

    packed (rows of <= 256 values): try the packed 32-bit pass first (mxa_topk_ws) -- the
    fast path for approximate scores, whose values leave the low mantissa byte free; rows
    that do not pack are redone by the 64-bit pass.  For arbitrary float rows (almost none
    pack) packed=False runs the 64-bit pass alone: DeiT-base-sized random rows 0.79 ms
    against 1.05 ms through the packed attempt (profiles/r06v1_ab_topk_fp32.txt)."""
    dev = require_device(vals)
    dt = _dt(vals, "vals")
    vals = vals.contiguous()
    n = vals.shape[-1]
    rows = vals.numel() // n if n else 0
    idx = torch.empty(vals.shape[:-1] + (k,), dtype=torch.int64, device=dev)
    out = torch.empty(vals.shape[:-1] + (k,), dtype=vals.dtype, device=dev)
    mask = torch.empty(vals.shape[:-1] + ((n + 31) // 32,), dtype=torch.int32, device=dev) if return_mask else None
    if rows:
        # the workspace path (rows of <= 256 values: the fused op's packed selection pass
        # and one-lane tail); 0 bytes: mxa_topk alone
        mp = mask.data_ptr() if return_mask else None
        if not packed:  # the 64-bit pass alone
            check(lib().mxa_topk(vals.data_ptr(), rows, n, n, k, idx.data_ptr(), out.data_ptr(), mp, dt,
                                 stream_ptr(dev)), "mxa_topk")
            return (out, idx, mask) if return_mask else (out, idx)
        wsb = lib().mxa_topk_workspace_bytes(rows, n, k)
        if wsb < 0:
            raise ValueError(f"topk: invalid shape rows={rows} n={n} k={k}")
        ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
        check(lib().mxa_topk_ws(vals.data_ptr(), rows, n, n, k, idx.data_ptr(), out.data_ptr(), mp, dt, ws.data_ptr(),
                                wsb, stream_ptr(dev)), "mxa_topk")
    return (out, idx, mask) if return_mask else (out, idx)


def unpack_mask(words: torch.Tensor, n: int) -> torch.Tensor:
    """Packed prune-mask words (..., ceil(n/32)) -> bool (..., n) (bit j%32 of word j/32)."""
    bits = torch.arange(32, device=words.device, dtype=torch.int32)
    m = (words.unsqueeze(-1) >> bits) & 1
    return m.reshape(words.shape[:-1] + (-1,))[..., :n].bool()


def mx_matmul(a: torch.Tensor, b: torch.Tensor, elem_mbits_a: int = 8, elem_mbits_b: int = 8, flush: bool = False,
              bfloat: int = 0, out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """MX matmul forward (matmul.py:31-100): a (..., M, K) along K, b (..., K, Nc) along K.
    Each operand is quantized in its own dtype; the product is rounded once to out_dtype
    (default: the operands' dtype, which must then agree -- torch.matmul's rule; under
    torch.autocast the caller passes the autocast dtype)."""
    dev = require_device(a, b)
    adt, bdt = _dt(a, "in1"), _dt(b, "in2")
    if out_dtype is None:
        if a.dtype != b.dtype:
            raise RuntimeError(f"expected both operands to have the same dtype, got {a.dtype} and {b.dtype}")
        out_dtype = a.dtype
    cdt = N.DTYPES[out_dtype]
    if a.dim() < 2 or b.dim() < 2:
        raise ValueError("mx matmul needs >= 2-D operands")
    batch_shape = torch.broadcast_shapes(a.shape[:-2], b.shape[:-2])
    M, K = a.shape[-2:]
    K2, Nc = b.shape[-2:]
    if K != K2:
        raise ValueError(f"inner dimensions differ: {K} vs {K2}")
    a = a.expand(batch_shape + (M, K)).contiguous()
    b = b.expand(batch_shape + (K, Nc))
    # b the transpose of a row-major (..., Nc, K) tensor (the callers' k.transpose(-2, -1)):
    # quantized from that layout along K (mxa_matmul_bt), no copy
    bt = b.transpose(-2, -1)
    transposed = bt.is_contiguous()
    if not transposed:
        b = b.contiguous()
    batch = 1
    for s in batch_shape:
        batch *= s
    c = torch.empty(batch_shape + (M, Nc), dtype=out_dtype, device=dev)
    if batch == 0 or M == 0 or Nc == 0:
        return c
    if K == 0:
        return c.zero_()
    nbytes = lib().mxa_matmul_workspace_bytes(batch, M, K, Nc)
    ws = _workspace(dev, nbytes)
    fn, bp = (lib().mxa_matmul_bt, bt.data_ptr()) if transposed else (lib().mxa_matmul, b.data_ptr())
    check(fn(a.data_ptr(), bp, c.data_ptr(), batch, M, K, Nc, M * K, K * Nc, elem_mbits_a, elem_mbits_b, int(flush),
             int(bfloat), adt, bdt, cdt, ws.data_ptr(), ws.numel(), stream_ptr(dev)), "mxa_matmul")
    return c


def _strides3(t: torch.Tensor, name: str):
    if t.dim() != 4:
        raise ValueError(f"{name} must be (B, H, rows, D)")
    if t.stride(3) != 1:
        raise ValueError(f"{name} must be contiguous in its last (head_dim) axis")
    return (t.stride(0), t.stride(1), t.stride(2))


def elsa_cos_table(d: int) -> torch.Tensor:
    """cos(clamp(pi/d * h - 0.127, 0)) for hamming distances h = 0..d, computed the way
    funcs/elsa_approximation.py:138-143 computes it (fp32 torch ops on the host, torch's
    CPU cosf).  A (d+1)-entry constant of the approximator; the per-pair scores are
    formed on the device."""
    h = torch.arange(d + 1, dtype=torch.float32)
    est = (torch.pi / d) * h
    return torch.cos(torch.clamp(est - 0.127, min=0))


def _attn_params(q, k, v, scale, k_top, pred_mode, top_k, approx, bias, flush_subnormals, bfloat, elsa_proj,
                 autocast=None):
    """autocast: None, or the torch.autocast dtype (float16 / bfloat16) under which the
    reference's matmuls return that dtype (include/mxa.h score_dtype)."""
    dev = require_device(q, k, v, bias, elsa_proj)
    dt = _dt(q, "q")
    for t, nm in ((k, "k"),) + (((v, "v"),) if v is not None else ()):
        if t.dtype != q.dtype:
            raise TypeError(f"{nm} must have q's dtype {q.dtype} (got {t.dtype})")
    sdt = 0
    if autocast is not None and autocast != torch.float32:
        if autocast not in (torch.float16, torch.bfloat16):
            raise TypeError(f"autocast dtype must be float16 or bfloat16 (got {autocast})")
        sdt = N.DTYPES[autocast]
    if approx and pred_mode == "ELSA" and bias is not None:
        # elsa_approximation.approximation_scores adds no bias (deit main.py:120-121, DiT
        # models.py:188-189, PixArt :676-677): ranking ELSA scores plus a bias would differ
        raise ValueError("pred_mode 'ELSA' takes no bias: the reference's ELSA scores are unbiased")
    B, H, Nq, D = q.shape
    Bk, Hk, T, Dk = k.shape
    if (Bk, Hk, Dk) != (B, H, D) or (v is not None and tuple(v.shape) != (B, H, T, D)):
        raise ValueError(f"shape mismatch q{tuple(q.shape)} k{tuple(k.shape)} "
                         f"v{None if v is None else tuple(v.shape)}")
    if top_k and not (0 < k_top <= T):
        raise ValueError(f"k={k_top} out of range for {T} keys")
    if approx and pred_mode not in N.PRED_MODES:
        raise ValueError(f"pred_mode {pred_mode!r} not supported by the fused op "
                         f"(supported: {sorted(N.PRED_MODES)})")
    keep = []  # tensors whose storage the call reads
    p = N.AttnParams()
    p.q, p.k = q.data_ptr(), k.data_ptr()
    p.v = v.data_ptr() if v is not None else None
    p.q_strides[:] = _strides3(q, "q")
    p.k_strides[:] = _strides3(k, "k")
    if v is not None:
        p.v_strides[:] = _strides3(v, "v")
    p.B, p.H, p.N, p.T, p.D = B, H, Nq, T, D
    p.k_top = int(k_top) if top_k else 0
    p.scale = float(torch.tensor(scale, dtype=torch.float32).item())  # torch: python scale -> fp32 operand
    p.pred_mode = N.PRED_MODES.get(pred_mode, 0)
    p.top_k, p.approx = int(bool(top_k)), int(bool(approx))
    p.flush_subnormals, p.bfloat = int(bool(flush_subnormals)), int(bfloat)
    p.dtype, p.score_dtype = dt, sdt
    if bias is not None:
        if bias.dtype != q.dtype:
            raise TypeError(f"bias must have q's dtype {q.dtype} (got {bias.dtype})")
        bias4 = bias
        while bias4.dim() < 4:
            bias4 = bias4.unsqueeze(0)
        bias4 = bias4.expand(B, H, Nq, T)
        p.bias = bias4.data_ptr()
        p.bias_strides[:] = tuple(bias4.stride())
    if approx and pred_mode == "ELSA":
        if elsa_proj is None:
            raise ValueError("pred_mode 'ELSA' needs the caller's orthogonal matrix (elsa_proj)")
        if Nq != T:
            # elsa_approximation.py:142-143 broadcasts the key norms over the query rows
            raise RuntimeError(f"ELSA scores need N == T (got N={Nq}, T={T}): the reference's key-norm "
                               f"broadcast (funcs/elsa_approximation.py:142) fails otherwise")
        proj = _f32(elsa_proj, "elsa_proj").contiguous()
        if tuple(proj.shape) != (D, D):
            raise ValueError(f"elsa_proj must be ({D}, {D})")
        ck = (D, dev)
        if ck not in _ELSA_COS:
            _ELSA_COS[ck] = elsa_cos_table(D).to(dev)
        cos = _ELSA_COS[ck]
        keep += [proj, cos]
        p.elsa_proj, p.elsa_cos = proj.data_ptr(), cos.data_ptr()
    return p, dev, (B, H, Nq, T, D), keep


def _out_dtype(q, autocast):
    return autocast if autocast in (torch.float16, torch.bfloat16) else q.dtype


def mx_topk_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float, k_top: int = 20,
                      pred_mode: str = "ex_pred", top_k: bool = True, approx: bool = True,
                      bias: Optional[torch.Tensor] = None, flush_subnormals: bool = False, bfloat: int = 0,
                      return_scores: bool = False, out: Optional[torch.Tensor] = None,
                      return_mask: bool = False, elsa_proj: Optional[torch.Tensor] = None,
                      autocast: Optional[torch.dtype] = None):
    """The fused hot path (include/mxa.h mxa_attention): q (B,H,N,D), k/v (B,H,T,D)
    float32, float16 or bfloat16 (strided views of a packed qkv are fine; the ops follow
    the tensors' dtype as the reference's do).  autocast: the torch.autocast dtype the
    reference's matmuls would return (scores, P and out in it).  Returns (out (B,H,N,D),
    idx (B,H,N,k_top) int64 or None[, true, pred][, mask words (B,H,N,ceil(T/32))]);
    true / pred are float32 tensors holding the score-dtype values."""
    p, dev, (B, H, Nq, T, D), keep = _attn_params(q, k, v, scale, k_top, pred_mode, top_k, approx and top_k, bias,
                                                  flush_subnormals, bfloat, elsa_proj, autocast)
    odt = _out_dtype(q, autocast)
    if out is None:
        out = torch.empty((B, H, Nq, D), dtype=odt, device=dev)
    elif out.dtype != odt:
        raise TypeError(f"out must be {odt} (got {out.dtype})")
    p.out = out.data_ptr()
    p.out_strides[:] = (out.stride(0), out.stride(1), out.stride(2))
    if out.stride(3) != 1:
        raise ValueError("out must be contiguous in its last axis")
    idx = torch.empty((B, H, Nq, k_top), dtype=torch.int64, device=dev) if top_k else None
    p.idx_out = idx.data_ptr() if idx is not None else None
    mask = None
    if return_mask:
        if not top_k:
            raise ValueError("the prune mask exists on the top-k path only")
        mask = torch.empty((B, H, Nq, (T + 31) // 32), dtype=torch.int32, device=dev)
        p.mask_out = mask.data_ptr()
    true_s = pred_s = None
    if return_scores:
        true_s = torch.empty((B, H, Nq, T), dtype=torch.float32, device=dev)
        pred_s = torch.full((B, H, Nq, T), float("nan"), dtype=torch.float32, device=dev)
        p.true_out, p.pred_out = true_s.data_ptr(), pred_s.data_ptr()
    nbytes = lib().mxa_attention_workspace_bytes(ctypes.byref(p))
    if nbytes < 0:
        raise ValueError("bad attention shape")
    ws = _workspace(dev, nbytes)
    p.workspace, p.workspace_bytes = ws.data_ptr(), ws.numel()
    check(lib().mxa_attention(ctypes.byref(p), stream_ptr(dev)), "mxa_attention")
    res = (out, idx) + ((true_s, pred_s) if return_scores else ()) + ((mask,) if return_mask else ())
    return res


def mx_approx_scores(q: torch.Tensor, k: torch.Tensor, pred_mode: str = "ex_pred",
                     bias: Optional[torch.Tensor] = None, flush_subnormals: bool = False, bfloat: int = 0,
                     elsa_proj: Optional[torch.Tensor] = None, autocast: Optional[torch.dtype] = None) -> torch.Tensor:
    """pred = aQ @ aK^T (+ bias) of the approximator `pred_mode` (or ELSA's
    approximation_scores), (B,H,N,T) in the score dtype -- include/mxa.h mxa_approx_scores."""
    p, dev, (B, H, Nq, T, D), keep = _attn_params(q, k, None, 1.0, 0, pred_mode, False, True, bias,
                                                  flush_subnormals, bfloat, elsa_proj, autocast)
    pred = torch.empty((B, H, Nq, T), dtype=torch.float32, device=dev)
    p.pred_out = pred.data_ptr()
    nbytes = lib().mxa_attention_workspace_bytes(ctypes.byref(p))
    ws = _workspace(dev, nbytes)
    p.workspace, p.workspace_bytes = ws.data_ptr(), ws.numel()
    check(lib().mxa_approx_scores(ctypes.byref(p), stream_ptr(dev)), "mxa_approx_scores")
    odt = _out_dtype(q, autocast)
    return pred if odt == torch.float32 else pred.to(odt)  # the values are exact in odt


class LinearWeightMX:
    """A Linear weight (out_features, in_features) as MXINT8 codes + block exponents
    along in_features on the device (mxa_linear_weight_prep), MFMA-ready in column
    groups of group_width (qkv: the head dim): prepared once, reused by every fused
    call (the weights are constant at inference)."""

    def __init__(self, weight: torch.Tensor, group_width: int, flush_subnormals: bool = False, bfloat: int = 0):
        dev = require_device(weight)
        w = _f32(weight.detach(), "weight").contiguous()
        self.out_features, self.in_features = w.shape
        self.group_width = int(group_width)
        nbytes = lib().mxa_linear_weight_bytes(self.out_features, self.in_features, self.group_width)
        if nbytes < 0:
            raise ValueError(f"group_width {group_width} does not divide out_features {self.out_features}")
        self.buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        check(lib().mxa_linear_weight_prep(w.data_ptr(), self.out_features, self.in_features, self.group_width,
                                           int(bool(flush_subnormals)), int(bfloat), self.buf.data_ptr(),
                                           stream_ptr(dev)), "mxa_linear_weight_prep")
        self.flush, self.bfloat = bool(flush_subnormals), int(bfloat)


def _prepared(weight, group_width: int, flush_subnormals: bool, bfloat: int) -> "LinearWeightMX":
    wq = weight if isinstance(weight, LinearWeightMX) else LinearWeightMX(weight, group_width, flush_subnormals, bfloat)
    if (wq.flush, wq.bfloat) != (bool(flush_subnormals), int(bfloat)):
        raise ValueError("the prepared weight was quantized with other flush / bfloat settings")
    return wq


def mx_linear(x: torch.Tensor, weight, bias: Optional[torch.Tensor] = None, flush_subnormals: bool = False,
              bfloat: int = 0, autocast: Optional[torch.dtype] = None) -> torch.Tensor:
    """mx.Linear forward (microxscaling/mx/linear.py:20-103; include/mxa.h mxa_linear):
    x (..., in_features) float32, weight an (out, in) tensor or a LinearWeightMX (any group
    width); out (..., out) float32 = bf(fl32(MX(x) @ MX(W)^T)) [+ bf(bias)], every product
    the exact sum rounded once.  autocast: the product rounded to float16 / bfloat16 before
    the fp32 bias add (F.linear under torch.autocast)."""
    dev = require_device(x, bias)
    x = _f32(x, "x")
    wq = _prepared(weight, weight.shape[0] if not isinstance(weight, LinearWeightMX) else 1, flush_subnormals, bfloat)
    if x.shape[-1] != wq.in_features:
        raise ValueError(f"x has {x.shape[-1]} features, the weight {wq.in_features}")
    x2 = x.reshape(-1, x.shape[-1])
    if x2.stride(-1) != 1:
        x2 = x2.contiguous()
    rows = x2.shape[0]
    out = torch.empty((rows, wq.out_features), dtype=torch.float32, device=dev)
    if rows == 0:
        return out.reshape(x.shape[:-1] + (wq.out_features,))
    ac = 0
    if autocast is not None and autocast != torch.float32:
        ac = N.DTYPES[autocast]
    bptr = None
    if bias is not None:
        bias = _f32(bias, "bias").contiguous()
        bptr = bias.data_ptr()
    nbytes = lib().mxa_linear_workspace_bytes(rows, wq.in_features, wq.out_features)
    ws = _workspace(dev, nbytes)
    check(lib().mxa_linear(x2.data_ptr(), rows, wq.in_features, x2.stride(0), wq.buf.data_ptr(), wq.out_features,
                           bptr, out.data_ptr(), out.stride(0), int(bool(flush_subnormals)), int(bfloat), ac,
                           ws.data_ptr(), ws.numel(), stream_ptr(dev)), "mxa_linear")
    out = out.reshape(x.shape[:-1] + (wq.out_features,))
    if ac and bias is None:  # F.linear's autocast dtype (the values are already rounded to it)
        out = out.to(autocast)
    return out


def _proj_params(proj_weight, proj_bias, C: int, rows: int, flush_subnormals: bool, bfloat: int, dev):
    """(ProjParams, y (rows, out_features), keep) for the proj Linear behind the attention."""
    wp = _prepared(proj_weight, proj_weight.shape[0] if not isinstance(proj_weight, LinearWeightMX) else 1,
                   flush_subnormals, bfloat)
    if wp.in_features != C:
        raise ValueError(f"proj weight takes {wp.in_features} features, the attention gives H*D = {C}")
    pj = N.ProjParams()
    pj.wq, pj.out_features = wp.buf.data_ptr(), wp.out_features
    keep = [wp]
    if proj_bias is not None:
        pb = _f32(proj_bias, "proj_bias").contiguous()
        keep.append(pb)
        pj.bias = pb.data_ptr()
    y = torch.empty((rows, wp.out_features), dtype=torch.float32, device=dev)
    pj.y, pj.y_row_stride = y.data_ptr(), y.stride(0)
    return pj, y, keep


def mx_topk_attention_proj(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float, proj_weight,
                           proj_bias: Optional[torch.Tensor] = None, k_top: int = 20, pred_mode: str = "ex_pred",
                           approx: bool = True, bias: Optional[torch.Tensor] = None, flush_subnormals: bool = False,
                           bfloat: int = 0, elsa_proj: Optional[torch.Tensor] = None):
    """The top-k attention core with the proj mx.Linear fused behind it (include/mxa.h
    mxa_attention_proj): y = proj(out.transpose(1, 2).reshape(B, N, H*D)) as (B, N, out)
    float32, plus idx (B,H,N,k).  float32 q, k, v (views fine)."""
    p, dev, (B, H, Nq, T, D), keep = _attn_params(q, k, v, scale, k_top, pred_mode, True, approx, bias,
                                                  flush_subnormals, bfloat, elsa_proj)
    if p.dtype != N.DT_F32:
        raise TypeError("the fused proj takes float32 q, k, v")
    idx = torch.empty((B, H, Nq, k_top), dtype=torch.int64, device=dev)
    p.idx_out = idx.data_ptr()
    pj, y, keep2 = _proj_params(proj_weight, proj_bias, H * D, B * Nq, flush_subnormals, bfloat, dev)
    nbytes = lib().mxa_attention_proj_workspace_bytes(ctypes.byref(p), None, ctypes.byref(pj))
    if nbytes < 0:
        raise ValueError("bad attention shape")
    ws = _workspace(dev, nbytes)
    p.workspace, p.workspace_bytes = ws.data_ptr(), ws.numel()
    check(lib().mxa_attention_proj(ctypes.byref(p), None, ctypes.byref(pj), stream_ptr(dev)), "mxa_attention_proj")
    return y.reshape(B, Nq, -1), idx


def mx_qkv_attention(x: torch.Tensor, weight, bias: Optional[torch.Tensor], num_heads: int, scale: float,
                     k_top: int = 20, pred_mode: str = "ex_pred", top_k: bool = True, approx: bool = True,
                     flush_subnormals: bool = False, bfloat: int = 0, return_qkv: bool = False,
                     elsa_proj: Optional[torch.Tensor] = None, autocast: Optional[torch.dtype] = None,
                     proj_weight=None, proj_bias: Optional[torch.Tensor] = None):
    """The qkv mx.Linear fused into the attention core (include/mxa.h mxa_qkv_attention):
    x (B, N, C) float32 tokens; weight a (3C', C) tensor or a LinearWeightMX; returns
    (out (B,H,N,D), idx (B,H,N,k) or None[, qkv (B,N,3C') fp32 projection]).
    autocast (float16 / bfloat16): torch.autocast around the module -- the projection's
    product is rounded to it before the fp32 bias add, and the attention's matmuls return
    it (the output is of that dtype)."""
    dev = require_device(x, bias, elsa_proj)
    x = _f32(x, "x")
    if x.dim() != 3 or x.stride(2) != 1:
        raise ValueError("x must be (B, N, C) with contiguous C")
    B, Ntok, C = x.shape
    out_f = weight.out_features if isinstance(weight, LinearWeightMX) else weight.shape[0]
    if out_f % (3 * num_heads):
        raise ValueError(f"weight rows {out_f} are not 3 * heads * head_dim")
    D = out_f // (3 * num_heads)
    wq = weight if isinstance(weight, LinearWeightMX) else LinearWeightMX(weight, D, flush_subnormals, bfloat)
    if wq.in_features != C or wq.group_width != D:
        raise ValueError(f"weight ({wq.out_features}, {wq.in_features}) / group {wq.group_width} does not fit "
                         f"x C={C}, heads={num_heads}")
    if (wq.flush, wq.bfloat) != (bool(flush_subnormals), int(bfloat)):
        raise ValueError("the prepared weight was quantized with other flush / bfloat settings")
    if top_k and not (0 < k_top <= Ntok):
        raise ValueError(f"k={k_top} out of range for {Ntok} keys")
    if approx and top_k and pred_mode not in N.PRED_MODES:
        raise ValueError(f"pred_mode {pred_mode!r} not supported")
    # q / k / v are produced inside the call: stand-in views carry the shapes only
    shape_q = torch.empty((D,), device=dev).as_strided((B, num_heads, Ntok, D), (0, 0, 0, 1))
    p, _, _, keep = _attn_params(shape_q, shape_q, shape_q, scale, k_top, pred_mode, top_k, approx and top_k, None,
                                 flush_subnormals, bfloat, elsa_proj, autocast)
    p.q = p.k = p.v = None
    out = torch.empty((B, num_heads, Ntok, D), dtype=_out_dtype(x, autocast), device=dev)
    p.out = out.data_ptr()
    p.out_strides[:] = (out.stride(0), out.stride(1), out.stride(2))
    idx = torch.empty((B, num_heads, Ntok, k_top), dtype=torch.int64, device=dev) if top_k else None
    p.idx_out = idx.data_ptr() if idx is not None else None
    xp = N.QkvParams()
    xp.x, xp.x_row_stride, xp.C, xp.wq = x.data_ptr(), x.stride(1), C, wq.buf.data_ptr()
    xp.autocast_dtype = p.score_dtype
    if B > 1 and x.stride(0) != Ntok * x.stride(1):
        raise ValueError("x rows must be evenly strided over (B, N)")
    if bias is not None:
        bias = _f32(bias, "bias").contiguous()
        xp.bias = bias.data_ptr()
    qkv = torch.empty((B, Ntok, wq.out_features), dtype=torch.float32, device=dev) if return_qkv else None
    xp.qkv_out = qkv.data_ptr() if return_qkv else None
    if proj_weight is not None:
        # ... then the proj mx.Linear on the attention output (mxa_attention_proj): (y, idx[, qkv])
        if not top_k or autocast not in (None, torch.float32):
            raise ValueError("the fused proj runs on the float32 top-k path")
        pj, y, keep2 = _proj_params(proj_weight, proj_bias, num_heads * D, B * Ntok, flush_subnormals, bfloat, dev)
        p.out = None
        nbytes = lib().mxa_attention_proj_workspace_bytes(ctypes.byref(p), ctypes.byref(xp), ctypes.byref(pj))
        if nbytes < 0:
            raise ValueError("bad shape")
        ws = _workspace(dev, nbytes)
        p.workspace, p.workspace_bytes = ws.data_ptr(), ws.numel()
        check(lib().mxa_attention_proj(ctypes.byref(p), ctypes.byref(xp), ctypes.byref(pj), stream_ptr(dev)),
              "mxa_attention_proj")
        y = y.reshape(B, Ntok, -1)
        return (y, idx, qkv) if return_qkv else (y, idx)
    nbytes = lib().mxa_qkv_attention_workspace_bytes(ctypes.byref(p), ctypes.byref(xp))
    if nbytes < 0:
        raise ValueError("bad shape")
    ws = _workspace(dev, nbytes)
    p.workspace, p.workspace_bytes = ws.data_ptr(), ws.numel()
    check(lib().mxa_qkv_attention(ctypes.byref(p), ctypes.byref(xp), stream_ptr(dev)), "mxa_qkv_attention")
    return (out, idx, qkv) if return_qkv else (out, idx)


def selftest_mfma(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    dev = require_device(a, b)
    c = torch.empty((16, 16), dtype=torch.int32, device=dev)
    check(lib().mxa_selftest_mfma(a.contiguous().data_ptr(), b.contiguous().data_ptr(), c.data_ptr(),
                                  stream_ptr(dev)), "mxa_selftest_mfma")
    return c


def selftest_mfma32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """C = A (32x32 int8) @ B (32x32 int8) by one v_mfma_i32_32x32x32_i8 through the
    finishing kernel's lane maps."""
    dev = require_device(a, b)
    c = torch.empty((32, 32), dtype=torch.int32, device=dev)
    check(lib().mxa_selftest_mfma32(a.contiguous().data_ptr(), b.contiguous().data_ptr(), c.data_ptr(),
                                    stream_ptr(dev)), "mxa_selftest_mfma32")
    return c
