"""ORACLE — test infrastructure only.

CPU restatement (numpy, float32-exact) of the reference's MX-quantized,
approximator-pruned top-k attention path.  Only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
module, and only as the checker: the product path (mx_quantization_amd) never
imports it and fails loudly without its HIP extension.

Every function cites the reference lines it restates.  Paths are relative to
the reference root (d9bjo0522/mx_quantization @ 2025-12-12):

  MX quantize        microxscaling/mx/mx_ops.py:49-99, :102-174, :180-306
  element rounding   microxscaling/mx/elemwise_ops.py:45-86, :92-180, :201-216
  formats            microxscaling/mx/formats.py:61-125
  mx.matmul          microxscaling/mx/matmul.py:31-100
  approximators      funcs/exponent_based_prediction.py:12-318
                     microxscaling/examples/deit/exponent_based_prediction.py:98-178
  attention glue     workloads/deit/scripts/main.py:100-152,
                     workloads/DiT/models.py:168-225,
                     workloads/PixArt/models/MX_transformer_block.py:648-717, :792-859
  top-k              torch aten/src/ATen/native/TopKImpl.h:45-86 (oracle/topk_ref.cpp)

Parity is pinned by tests/golden/*.npz (generated from the reference itself
by tests/golden/gen_golden.py) — see tests/test_oracle_golden.py.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

F32 = np.float32
F64 = np.float64

_HERE = os.path.dirname(os.path.abspath(__file__))

# formats.py:61-125 -- (ebits, mbits, emax, max_norm) for the integer formats
_INT_FORMATS = {
    "int8": (0, 8, 0, 127.0 / 64.0),
    "int4": (0, 4, 0, 7.0 / 4.0),
    "int2": (0, 2, 0, 1.0),
}
FP32_MIN_NORMAL = F32(2.0 ** -126)  # formats.py:9


# ---------------------------------------------------------------------------
# exponent rule: torch.floor(torch.log2(x)) on float32  
# ---------------------------------------------------------------------------
def floor_log2_f32(x: np.ndarray) -> np.ndarray:
    """torch.floor(torch.log2(x)) for float32 x (x >= 0 or NaN).

    torch's float32 log2 == fl32(log2((double)x)) for every float32 (verified
    exhaustively by tools/gen_exp_lut.py --torch)."""
    x = np.asarray(x, dtype=F32)
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.floor(np.log2(x.astype(F64)).astype(F32)).astype(F32)


def floor_log2_dtype(bits: np.ndarray, dtype: str) -> np.ndarray:
    """torch.floor(torch.log2(x)) for float16 / bfloat16 x >= 0 given as uint16 bit
    patterns, as float64 (-inf for a float16 zero: mx_ops.py:85's FP32_MIN_NORMAL
    underflows to 0 in float16; bfloat16 zero -> -126 like float32).

    log2 is rounded to the dtype: it reaches the next integer for the top `gap`
    mantissa codes of a binade, gap depending on the octave of the exponent (float16:
    0, 1, 2, 5; bfloat16: 0, 1, 2, 5, 10, 21, 40), and for dtype subnormals from a
    per-leading-bit threshold.  The same rule as mxa_common.hpp floor_log2_dt; pinned
    against torch by tests/test_oracle_golden.py on every value (dtype_exp in
    tests/golden/attn_dtype.npz)."""
    b = np.asarray(bits, dtype=np.uint16).astype(np.int64) & 0x7FFF
    if dtype == "f16":
        mb, bias, gaps = 10, 15, (0, 1, 2, 5)
        sub_thr = {7: 255, 8: 511, 9: 1022}
        inf_bits = 0x7C00
    else:
        mb, bias, gaps = 7, 127, (0, 1, 2, 5, 10, 21, 40)
        sub_thr = {1: 3, 2: 6, 3: 12, 4: 23, 5: 54, 6: 108}
        inf_bits = 0x7F80
    out = np.zeros(b.shape, dtype=F64)
    for i, v in np.ndenumerate(b):
        E, M = int(v) >> mb, int(v) & ((1 << mb) - 1)
        if v >= inf_bits:
            out[i] = np.inf if v == inf_bits else np.nan
        elif v == 0:
            out[i] = -np.inf if dtype == "f16" else -126.0
        elif E:
            e = E - bias
            u = e if e >= 0 else -e - 1
            o = u.bit_length() - 1 if u >= 2 else 0
            out[i] = e + (1 if M + gaps[o] >= (1 << mb) else 0)
        else:
            j = M.bit_length() - 1
            e = (1 - bias - mb) + j
            out[i] = e + (1 if M >= sub_thr.get(j, 2 << j) else 0)
    return out


def _pow2(e: np.ndarray) -> np.ndarray:
    """2**e for float32 e holding integers or NaN (torch `2 ** tensor`)."""
    e = np.asarray(e, dtype=F32)
    out = np.full(e.shape, np.nan, dtype=F32)
    fin = np.isfinite(e)
    out[fin] = np.ldexp(F32(1.0), e[fin].astype(np.int32)).astype(F32)
    return out


# ---------------------------------------------------------------------------
# blocking (mx_ops.py:102-174), restricted to one axis
# ---------------------------------------------------------------------------
def to_blocks(A: np.ndarray, axis: int, block_size: int):
    """Move `axis` last, zero-pad to a multiple of block_size, view (..., nb, bs)."""
    A = np.moveaxis(np.asarray(A, dtype=F32), axis, -1)
    L = A.shape[-1]
    bs = L if block_size == 0 else block_size
    nb = max(1, -(-L // bs))
    pad = nb * bs - L
    if pad:
        A = np.concatenate([A, np.zeros(A.shape[:-1] + (pad,), dtype=F32)], axis=-1)
    return A.reshape(A.shape[:-1] + (nb, bs)), L


def from_blocks(Ab: np.ndarray, L: int, axis: int) -> np.ndarray:
    A = Ab.reshape(Ab.shape[:-2] + (Ab.shape[-2] * Ab.shape[-1],))[..., :L]
    return np.moveaxis(A, -1, axis)


def shared_exponents(Ab: np.ndarray, method: str = "max", ebits: int = 0) -> np.ndarray:
    """mx_ops.py:49-99 with axes=[-1] on a blocked view."""
    if method == "max":
        m = np.max(np.abs(Ab), axis=-1, keepdims=True)  # NaN propagates like torch.max
    elif method == "none":
        m = np.abs(Ab)
    else:
        raise ValueError(method)
    m = m.astype(F32)
    e = floor_log2_f32(m + FP32_MIN_NORMAL * (m == 0).astype(F32))
    if ebits > 0:
        emax = 2 ** (ebits - 1) - 1
        e = e.copy()
        e[e > emax] = np.nan
        e[e < -emax] = -emax
    return e


# ---------------------------------------------------------------------------
# element rounding (elemwise_ops.py:45-86) and MX quantize (mx_ops.py:180-306)
# ---------------------------------------------------------------------------
def round_mantissa(A: np.ndarray, rnd: str) -> np.ndarray:
    A = A.astype(F32)
    s = np.sign(A).astype(F32)
    a = np.abs(A)
    if rnd == "nearest":
        return (s * np.floor(a + F32(0.5))).astype(F32)
    if rnd == "floor":
        return (s * np.floor(a)).astype(F32)
    if rnd == "even":
        d = (a - F32(0.5)).astype(F32)
        mask = (np.mod(d, F32(2.0)) == 0).astype(F32)
        return (s * (np.floor(a + F32(0.5)) - mask)).astype(F32)
    raise ValueError(rnd)


def quantize_mx(A, elem="int8", block_size=32, axis=-1, scale_bits=8, rnd="nearest",
                flush=False):
    """_quantize_mx python branch (mx_ops.py:276-300) for the integer formats.

    Returns (values f32 same shape as A, codes int32 blocked (..., nb, bs),
    shared exponents f32 (..., nb, 1) after clamp [NaN = overflow])."""
    ebits, mbits, emax, max_norm = _INT_FORMATS[elem]
    Ab, L = to_blocks(A, axis, block_size)
    e = shared_exponents(Ab, "max", 0)
    if flush:
        Ab = (Ab * (e > -127).astype(F32)).astype(F32)
    e = (e - F32(emax)).astype(F32)
    scale_emax = 2 ** (scale_bits - 1) - 1
    e[e > scale_emax] = np.nan
    e[e < -scale_emax] = -scale_emax
    p2 = _pow2(e)
    with np.errstate(invalid="ignore", over="ignore"):
        As = (Ab / p2).astype(F32)
        # _quantize_elemwise_core (elemwise_ops.py:92-180), exp_bits == 0
        out = (As * F32(2.0 ** (mbits - 2))).astype(F32)
        out = round_mantissa(out, rnd)
        codes = np.clip(out, -(2 ** (mbits - 1) - 1), 2 ** (mbits - 1) - 1)
        out = (out / F32(2.0 ** (mbits - 2))).astype(F32)
        out = np.clip(out, F32(-max_norm), F32(max_norm)).astype(F32)
        out[As == np.inf] = np.inf
        out[As == -np.inf] = -np.inf
        vals = (out * p2).astype(F32)
    codes = np.where(np.isfinite(codes), codes, 0).astype(np.int32)
    return from_blocks(vals, L, axis), codes, e


def quantize_bfloat(A, bfloat=16, rnd="nearest", allow_denorm=True):
    """_quantize_bfloat (elemwise_ops.py:201-216) -> _quantize_elemwise_core."""
    if bfloat in (0, 32):
        return np.asarray(A, dtype=F32)
    A = np.asarray(A, dtype=F32)
    bits = bfloat - 7
    max_norm = F32(2.0 ** 127 * float(2 ** (bits - 1) - 1) / 2 ** (bits - 2))
    with np.errstate(invalid="ignore", over="ignore"):
        out = A.copy()
        if not allow_denorm:
            out = ((np.abs(A) >= F32(2.0 ** -126)).astype(F32) * A).astype(F32)
        pe = floor_log2_f32(np.abs(A) + (A == 0).astype(F32))
        pe = np.maximum(pe, F32(-126))
        p2 = _pow2(pe)
        out = (out / p2 * F32(2.0 ** (bits - 2))).astype(F32)
        out = round_mantissa(out, rnd)
        out = (out / F32(2.0 ** (bits - 2)) * p2).astype(F32)
        out = np.where(np.abs(out) > max_norm, np.sign(out) * np.inf, out).astype(F32)
        out[A == np.inf] = np.inf
        out[A == -np.inf] = -np.inf
    return out


# ---------------------------------------------------------------------------
# approximators (funcs/exponent_based_prediction.py)
# ---------------------------------------------------------------------------
class ExponentApproximation:
    """exponent_approximation.__init__ (funcs/exponent_based_prediction.py:12-38)
    on float32 numpy Q, K of shape (..., rows, d); quantized along the last axis."""

    def __init__(self, Q, K, block_size=32, elem="int8", flush=False, bfloat=32):
        self.Q = quantize_bfloat(Q, bfloat)
        self.K = quantize_bfloat(K, bfloat)
        self.block_size, self.flush = block_size, flush
        self.MX_Q, self.codes_Q, self.e_Q = quantize_mx(self.Q, elem, block_size, -1, flush=flush)
        self.MX_K, self.codes_K, self.e_K = quantize_mx(self.K, elem, block_size, -1, flush=flush)
        self.bQ, self.L = to_blocks(self.MX_Q, -1, block_size)
        self.bK, _ = to_blocks(self.MX_K, -1, block_size)
        self.sQ = shared_exponents(self.bQ, "max", 0)  # :35-36, unclamped
        self.sK = shared_exponents(self.bK, "max", 0)

    def _undo(self, Ab):
        return from_blocks(Ab.astype(F32), self.L, -1)

    @staticmethod
    def _exp_sign(b, s):
        sign = np.where(b < 0, F32(-1), F32(1)).astype(F32)
        return (sign * _pow2(np.broadcast_to(s, b.shape))).astype(F32)

    def exponent_based_sign(self):
        """Intended semantics: examples/deit/exponent_based_prediction.py:135-161
        == partial_K Q-side (:284-293) + partial_Q K-side (:309-313)."""
        return self._undo(self._exp_sign(self.bQ, self.sQ)), self._undo(self._exp_sign(self.bK, self.sK))

    def partial_K(self):  # :274-300
        return self._undo(self._exp_sign(self.bQ, self.sQ)), self.MX_K.copy()

    def partial_Q(self):  # :302-318
        return self.MX_Q.copy(), self._undo(self._exp_sign(self.bK, self.sK))

    def MXINT4(self):  # :179-272
        return (quantize_mx(self.Q, "int4", self.block_size, -1, flush=self.flush)[0],
                quantize_mx(self.K, "int4", self.block_size, -1, flush=self.flush)[0])

    @staticmethod
    def _two_step(b, s):
        """two_step_leading_ones (EXION) funcs/exponent_based_prediction.py:96-177, incl.
        the quirk that the approximation multiplies by the exponent itself (:126-127)."""
        with np.errstate(invalid="ignore", over="ignore"):
            sign = np.sign(b).astype(F32)
            es = np.broadcast_to(s, b.shape).astype(F32)
            raw = ((b / _pow2(es)) * F32(64)).astype(F32)
            l1 = shared_exponents(np.abs(raw), "none", 0)
            r1 = (raw - _pow2(l1)).astype(F32)
            t = np.where(r1 < 0, F32(0), r1).astype(F32)
            l2 = shared_exponents(t, "none", 0)
            return ((sign * es) * (_pow2(l1) + _pow2(l2)) / F32(64)).astype(F32)

    def two_step_leading_ones(self):
        return self._undo(self._two_step(self.bQ, self.sQ)), self._undo(self._two_step(self.bK, self.sK))

    @staticmethod
    def _true_ex(b):
        """exponent_based_sign_leading_ones: examples/deit/exponent_based_prediction.py:163-178,
        get_true_exponents :98-110 (zeros -> exponent 0 -> +1)."""
        sign = np.where(b < 0, F32(-1), F32(1)).astype(F32)
        a = np.abs(b)
        te = np.zeros_like(a)
        nz = a > 0
        te[nz] = floor_log2_f32(a[nz])
        return (sign * _pow2(te)).astype(F32)

    def exponent_based_sign_leading_ones(self):
        return self._undo(self._true_ex(self.bQ)), self._undo(self._true_ex(self.bK))


PRED_MODES = ("ex_pred", "partial_Q", "partial_K", "MXINT4", "two_step_leading_ones", "true_ex", "ELSA")


def elsa_cos_table(d):
    """cos(clamp(fl32(pi/d) * h - 0.127, 0)), h = 0..d: funcs/elsa_approximation.py:138-143
    evaluated with torch's own fp32 ops (torch.cos on the CPU is not correctly rounded
    on every entry, and the reference's scores carry its values)."""
    import torch
    h = torch.arange(d + 1, dtype=torch.float32)
    return torch.cos(torch.clamp((torch.pi / d) * h - 0.127, min=0)).numpy()


def elsa_scores(Q, K, proj, block_size=32, flush=False, bfloat=32):
    """elsa_approximation(Q, K).approximation_scores() (funcs/elsa_approximation.py:68-143):
    MXINT8 of Q, K along d (:83-96); hash bit j = (MX . P[j] >= 0) (:105-112, the
    products exact in float64); hamming distance over d bits (:128-137); the cosine of
    the corrected angle from the table above; scaled by ||MX_K[row n]|| for query row n
    (:126, :142-143: the key norms broadcast over the QUERY axis, so N == T)."""
    mq = quantize_mx(quantize_bfloat(Q, bfloat), "int8", block_size, -1, flush=flush)[0]
    mk = quantize_mx(quantize_bfloat(K, bfloat), "int8", block_size, -1, flush=flush)[0]
    if mq.shape[-2] != mk.shape[-2]:
        raise RuntimeError("ELSA scores need N == T (elsa_approximation.py:142)")
    P = np.asarray(proj, F32).astype(F64)
    with np.errstate(invalid="ignore"):
        hq = (mq.astype(F64) @ P.T) >= 0
        hk = (mk.astype(F64) @ P.T) >= 0
    d = Q.shape[-1]
    ham = (hq[..., :, None, :] != hk[..., None, :, :]).sum(-1)
    with np.errstate(invalid="ignore", over="ignore"):
        knorm = np.sqrt((mk.astype(F64) ** 2).sum(-1)).astype(F32)
    return (knorm[..., :, None] * elsa_cos_table(d)[ham]).astype(F32)


def approx_operands(Q, K, mode, block_size=32, flush=False, bfloat=32):
    ea = ExponentApproximation(Q, K, block_size, flush=flush, bfloat=bfloat)
    fn = {
        "ex_pred": ea.exponent_based_sign,
        "partial_Q": ea.partial_Q,
        "partial_K": ea.partial_K,
        "MXINT4": ea.MXINT4,
        "two_step_leading_ones": ea.two_step_leading_ones,
        "true_ex": ea.exponent_based_sign_leading_ones,
    }[mode]
    return fn()


def exact_matmul_f32(A, B):
    """fl32(exact A @ B): float64 accumulation of products that are exact in
    float64 (SURVEY.md F6 -- equals the reference's fp32 matmul on these operands)."""
    return np.matmul(A.astype(F64), B.astype(F64)).astype(F32)


def mx_matmul(A, B, elem="int8", block_size=32, flush=False, bfloat=32):
    """mx.matmul forward (matmul.py:31-100): in1 quantized along -1, in2 along -2.
    Exact-then-round (bit-exact for QK^T; P.V only within tolerance)."""
    qa = quantize_mx(quantize_bfloat(A, bfloat), elem, block_size, -1, flush=flush)[0]
    qb = quantize_mx(quantize_bfloat(B, bfloat), elem, block_size, -2, flush=flush)[0]
    return quantize_bfloat(exact_matmul_f32(qa, qb), bfloat)


def mx_linear(x, W, bias=None, elem="int8", block_size=32, flush=False, bfloat=32):
    """mx.Linear forward (microxscaling/mx/linear.py:20-103): bf(fl32(MX(bf(x)) @ MX(bf(W))^T)),
    then bf(out + bf(bias)); both operands MX-quantized along in_features.
    Exact-then-round (the reference's fp32 GEMM order is unpinned: equal within rounding)."""
    qx = quantize_mx(quantize_bfloat(x, bfloat), elem, block_size, -1, flush=flush)[0]
    qw = quantize_mx(quantize_bfloat(W, bfloat), elem, block_size, -1, flush=flush)[0]
    out = quantize_bfloat(exact_matmul_f32(qx, np.swapaxes(qw, -1, -2)), bfloat)
    if bias is not None:
        out = quantize_bfloat((out + quantize_bfloat(np.asarray(bias, F32), bfloat)).astype(F32), bfloat)
    return out


def qkv_split(qkv, H):
    """qkv.reshape(B, N, 3, H, D).permute(2, 0, 3, 1, 4) (deit main.py:87-88, DiT models.py:156-157)."""
    B, N, C3 = qkv.shape
    t = qkv.reshape(B, N, 3, H, C3 // (3 * H)).transpose(2, 0, 3, 1, 4)
    return t[0], t[1], t[2]


# ---------------------------------------------------------------------------
# top-k (oracle/topk_ref.cpp)
# ---------------------------------------------------------------------------
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "build", "libmxa_oracle.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", _HERE])
        lib = ctypes.CDLL(path)
        lib.oracle_topk_f32.restype = ctypes.c_int
        lib.oracle_topk_f32.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                        ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_void_p]
        lib.oracle_antiqsort.restype = ctypes.c_int
        lib.oracle_antiqsort.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
        _LIB = lib
    return _LIB


def antiqsort_row(n: int, k: int) -> np.ndarray:
    """A row that exhausts introselect/introsort's depth limit (McIlroy adversary run
    against libstdc++, oracle/topk_ref.cpp) -- exercises the heap fallbacks."""
    out = np.zeros(n, dtype=F32)
    if _lib().oracle_antiqsort(n, k, 1, out.ctypes.data) != 0:
        raise ValueError("oracle_antiqsort failed")
    return out


def topk(vals: np.ndarray, k: int, largest=True, sorted=True):
    """torch.topk(vals, k, dim=-1) on CPU: (values f32, indices int64) in torch's order."""
    vals = np.ascontiguousarray(vals, dtype=F32)
    n = vals.shape[-1]
    rows = int(np.prod(vals.shape[:-1]))
    idx = np.zeros(vals.shape[:-1] + (k,), dtype=np.int64)
    out = np.zeros(vals.shape[:-1] + (k,), dtype=F32)
    rc = _lib().oracle_topk_f32(vals.ctypes.data, rows, n, n, k, int(largest), int(sorted),
                                idx.ctypes.data, out.ctypes.data)
    if rc != 0:
        raise ValueError("oracle_topk_f32 failed")
    return out, idx


def softmax_f32(x, axis=-1):
    x = x.astype(F32)
    m = np.max(x, axis=axis, keepdims=True)
    with np.errstate(invalid="ignore", over="ignore"):
        e = np.exp((x - m).astype(F32)).astype(F32)
        return (e / np.sum(e, axis=axis, keepdims=True, dtype=F32)).astype(F32)


# ---------------------------------------------------------------------------
# the attention core (caller glue restated)
# ---------------------------------------------------------------------------
def attention(q, k, v, scale, k_top=20, pred_mode="ex_pred", top_k=True, approx=True,
              bias=None, block_size=32, flush=False, bfloat=32, elsa_proj=None):
    """The mx_quant branch of QuantizedAttention.forward (deit main.py:100-152) /
    DiT Attention.forward (models.py:168-225) / MXCrossAttention.forward
    (MX_transformer_block.py:792-859), from q,k,v (…,N,d),(…,T,d) to the
    pre-projection output (…,N,d).  `bias` broadcasts to (…,N,T) (PixArt mask)."""
    q = np.asarray(q, F32)
    k = np.asarray(k, F32)
    v = np.asarray(v, F32)
    res = {}
    true = mx_matmul(q, np.swapaxes(k, -1, -2), block_size=block_size, flush=flush, bfloat=bfloat)
    true = (true * F32(scale)).astype(F32)
    if bias is not None:
        bias = np.broadcast_to(np.asarray(bias, F32), true.shape)
        true = (true + bias).astype(F32)
    res["true"] = true
    if top_k:
        if approx and pred_mode == "ELSA":
            pred = elsa_scores(q, k, elsa_proj, block_size, flush=flush, bfloat=bfloat)
            res["pred"] = pred
            _, idx = topk(pred, k_top)
            vals = np.take_along_axis(true, idx, axis=-1)
        elif approx:
            aq, ak = approx_operands(q, k, pred_mode, block_size, flush=flush, bfloat=bfloat)
            pred = exact_matmul_f32(aq, np.swapaxes(ak, -1, -2))
            if bias is not None:
                pred = (pred + bias).astype(F32)
            res["aq"], res["ak"], res["pred"] = aq, ak, pred
            _, idx = topk(pred, k_top)
            vals = np.take_along_axis(true, idx, axis=-1)
        else:
            vals, idx = topk(true, k_top)
        res["idx"], res["vals"] = idx, vals
        p = softmax_f32(vals)
        attn = np.zeros_like(true)
        np.put_along_axis(attn, idx, p, axis=-1)
    else:
        attn = softmax_f32(true)
    res["attn"] = attn
    res["out"] = mx_matmul(attn, v, block_size=block_size, flush=flush, bfloat=bfloat)
    return res


def prune_mask(idx: np.ndarray, T: int) -> np.ndarray:
    """scatter(1) at idx -- equivalently examples/deit/top_k.py:16-42."""
    m = np.zeros(idx.shape[:-1] + (T,), dtype=bool)
    np.put_along_axis(m, idx, True, axis=-1)
    return m


def normwise_rel_err(a, b) -> float:
    a = np.asarray(a, F64)
    b = np.asarray(b, F64)
    den = np.linalg.norm(b.ravel())
    return float(np.linalg.norm((a - b).ravel()) / (den if den > 0 else 1.0))
