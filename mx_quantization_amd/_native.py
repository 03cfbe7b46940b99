"""ctypes binding of libmxa.so (the C ABI declared in include/mxa.h).

torch is imported first on purpose: libmxa.so needs libamdhip64.so.7, and the
dynamic loader then binds it to the runtime torch already loaded, so torch's
streams and device pointers are valid inside the library.

There is no fallback: if the library is missing or fails to load, every op
raises.  Build it with `python -m mx_quantization_amd.build_native`.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede loading libmxa.so, see module doc)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MXA_LIB") or os.path.join(_HERE, "libmxa.so")  # MXA_LIB: tools only

c_i32, c_i64, c_f32, c_vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p

MXA_OK = 0
MXA_OP_SIGN, MXA_OP_MXINT8, MXA_OP_MXINT4, MXA_OP_EXION, MXA_OP_TRUE_EX = range(5)
ABI_VERSION = 6
DT_F32, DT_F16, DT_BF16 = 0, 1, 2
DTYPES = {torch.float32: DT_F32, torch.float16: DT_F16, torch.bfloat16: DT_BF16}
PATH_NAMES = {2: "rows_fused", 3: "rows_split"}  # mxa_attention_path
# mxa_attention_finish_kernel: the finishing kernel and the engines of QK^T / P.V
FIN_KERNELS = {1: ("finish16_kernel", "v_dot4 (kept keys)", "v_mfma_i32_16x16x32_i8"),
               2: ("finish_kernel", "v_dot4 (kept keys)", "v_mfma_i32_32x32x32_i8"),
               3: ("finish_qk_kernel", "v_mfma_i32_16x16x32_i8 (every key, prune mask in the softmax)",
                   "v_mfma_i32_16x16x32_i8"),
               4: ("finish_qk_kernel (dense: every key kept)", "v_mfma_i32_16x16x32_i8", "v_mfma_i32_16x16x32_i8"),
               5: ("dense_rows_kernel", "v_dot4", "v_dot4")}
PRED_MODES = {"ex_pred": 0, "partial_Q": 1, "partial_K": 2, "MXINT4": 3, "two_step_leading_ones": 4,
              "true_ex": 5, "ELSA": 6}
ROUND_MODES = {"nearest": 0, "floor": 1, "even": 2}


class AttnParams(ctypes.Structure):
    """mirror of struct mxa_attn_params (include/mxa.h)"""
    _fields_ = [
        ("q", c_vp), ("k", c_vp), ("v", c_vp),
        ("q_strides", c_i64 * 3), ("k_strides", c_i64 * 3), ("v_strides", c_i64 * 3),
        ("B", c_i32), ("H", c_i32), ("N", c_i32), ("T", c_i32), ("D", c_i32),
        ("k_top", c_i32), ("scale", c_f32), ("pred_mode", c_i32), ("top_k", c_i32), ("approx", c_i32),
        ("flush_subnormals", c_i32), ("bfloat", c_i32),
        ("bias", c_vp), ("bias_strides", c_i64 * 4),
        ("out", c_vp), ("out_strides", c_i64 * 3),
        ("idx_out", c_vp), ("true_out", c_vp), ("pred_out", c_vp), ("mask_out", c_vp),
        ("elsa_proj", c_vp), ("elsa_cos", c_vp),
        ("workspace", c_vp), ("workspace_bytes", c_i64),
        ("dtype", c_i32), ("score_dtype", c_i32),
    ]


class QkvParams(ctypes.Structure):
    """mirror of struct mxa_qkv_params (include/mxa.h)"""
    _fields_ = [("x", c_vp), ("x_row_stride", c_i64), ("C", c_i32), ("wq", c_vp), ("bias", c_vp),
                ("qkv_out", c_vp), ("autocast_dtype", c_i32)]


class ProjParams(ctypes.Structure):
    """mirror of struct mxa_proj_params (include/mxa.h)"""
    _fields_ = [("wq", c_vp), ("out_features", c_i32), ("bias", c_vp), ("y", c_vp), ("y_row_stride", c_i64)]


PROJ_STAGES = 6  # MXA_PROJ_STAGES

_SIGS = {
    "mxa_abi_version": (c_i32, []),
    "mxa_status_string": (ctypes.c_char_p, [c_i32]),
    "mxa_quantize_mx": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i32, c_i32, c_i32, c_i32, c_i32,
                                c_i32, c_i32, c_vp]),
    "mxa_shared_exponents": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp]),
    "mxa_quantize_bfloat": (c_i32, [c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp]),
    "mxa_approx_values": (c_i32, [c_vp, c_vp, c_i64, c_i32, c_i64, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp]),
    "mxa_topk": (c_i32, [c_vp, c_i64, c_i32, c_i64, c_i32, c_vp, c_vp, c_vp, c_i32, c_vp]),
    "mxa_topk_workspace_bytes": (c_i64, [c_i64, c_i32, c_i32]),
    "mxa_topk_ws": (c_i32, [c_vp, c_i64, c_i32, c_i64, c_i32, c_vp, c_vp, c_vp, c_i32, c_vp, c_i64, c_vp]),
    "mxa_attention_workspace_bytes": (c_i64, [ctypes.POINTER(AttnParams)]),
    "mxa_attention": (c_i32, [ctypes.POINTER(AttnParams), c_vp]),
    "mxa_approx_scores": (c_i32, [ctypes.POINTER(AttnParams), c_vp]),
    "mxa_attention_path": (c_i32, [ctypes.POINTER(AttnParams)]),
    "mxa_attention_finish_kernel": (c_i32, [ctypes.POINTER(AttnParams)]),
    "mxa_attention_timed": (c_i32, [ctypes.POINTER(AttnParams), c_vp, c_i32, ctypes.POINTER(c_f32)]),
    "mxa_linear_weight_bytes": (c_i64, [c_i32, c_i32, c_i32]),
    "mxa_linear_weight_prep": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp]),
    "mxa_qkv_attention_workspace_bytes": (c_i64, [ctypes.POINTER(AttnParams), ctypes.POINTER(QkvParams)]),
    "mxa_qkv_attention": (c_i32, [ctypes.POINTER(AttnParams), ctypes.POINTER(QkvParams), c_vp]),
    "mxa_qkv_attention_timed": (c_i32, [ctypes.POINTER(AttnParams), ctypes.POINTER(QkvParams), c_vp, c_i32,
                                        ctypes.POINTER(c_f32)]),
    "mxa_linear_workspace_bytes": (c_i64, [c_i64, c_i32, c_i32]),
    "mxa_linear": (c_i32, [c_vp, c_i64, c_i32, c_i64, c_vp, c_i32, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_vp, c_i64,
                           c_vp]),
    "mxa_attention_proj_workspace_bytes": (c_i64, [ctypes.POINTER(AttnParams), ctypes.POINTER(QkvParams),
                                                   ctypes.POINTER(ProjParams)]),
    "mxa_attention_proj": (c_i32, [ctypes.POINTER(AttnParams), ctypes.POINTER(QkvParams), ctypes.POINTER(ProjParams),
                                   c_vp]),
    "mxa_attention_proj_timed": (c_i32, [ctypes.POINTER(AttnParams), ctypes.POINTER(QkvParams),
                                         ctypes.POINTER(ProjParams), c_vp, c_i32, ctypes.POINTER(c_f32)]),
    "mxa_matmul": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_i64, c_i64, c_i32, c_i32, c_i32, c_i32,
                           c_i32, c_i32, c_i32, c_vp, c_i64, c_vp]),
    "mxa_matmul_workspace_bytes": (c_i64, [c_i64, c_i32, c_i32, c_i32]),
    "mxa_matmul_bt": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_i64, c_i64, c_i32, c_i32, c_i32, c_i32,
                              c_i32, c_i32, c_i32, c_vp, c_i64, c_vp]),
    "mxa_selftest_mfma": (c_i32, [c_vp, c_vp, c_vp, c_vp]),
    "mxa_selftest_mfma32": (c_i32, [c_vp, c_vp, c_vp, c_vp]),
}
EXPORTS = tuple(_SIGS)

_lib = None


class NativeError(RuntimeError):
    pass


def lib():
    """The loaded library (raises NativeError when absent -- no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(f"{LIB_PATH} is missing: build it with `python -m mx_quantization_amd.build_native`")
        try:
            handle = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - depends on the box
            raise NativeError(f"cannot load {LIB_PATH}: {e}") from e
        for name, (res, args) in _SIGS.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        if handle.mxa_abi_version() != ABI_VERSION:
            raise NativeError("libmxa.so ABI version mismatch")
        _lib = handle
    return _lib


def check(status: int, what: str) -> None:
    if status != MXA_OK:
        msg = lib().mxa_status_string(status).decode()
        raise NativeError(f"{what} failed: {msg} (status {status})")


def stream_ptr(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_device(*tensors: torch.Tensor) -> torch.device:
    """The product path runs on the MI355X only; CPU tensors are an error, not a fallback."""
    dev = None
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise NativeError("mx_quantization_amd ops run on a HIP device; got a CPU tensor "
                              "(the CPU restatement lives in oracle/ and is test infrastructure only)")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise NativeError("tensors on different devices")
    return dev
