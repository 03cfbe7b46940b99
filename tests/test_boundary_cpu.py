"""CPU checks of the drop-in boundary: the C-ABI library loads and exports every
symbol include/mxa.h declares, the Python surfaces import under the reference's
names, and the product path refuses CPU tensors (no fallback)."""
import os

import numpy as np
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "mxa.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mxa_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from mx_quantization_amd import _native as N
    lib = N.lib()
    syms = declared_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(N.EXPORTS), "ctypes signatures out of sync with include/mxa.h"
    assert lib.mxa_abi_version() == N.ABI_VERSION == 6


def test_status_strings_and_arg_errors():
    from mx_quantization_amd import _native as N
    lib = N.lib()
    assert lib.mxa_status_string(0) == b"ok"
    # argument validation happens before any launch, so these run without a GPU
    assert lib.mxa_quantize_mx(None, None, None, None, 1, 1, 1, 32, 8, 8, 0, 0, 0, 0, None) == -1
    assert lib.mxa_quantize_mx(1, 1, None, None, 1, 1, 1, 32, 5, 8, 0, 0, 0, 0, None) == -2  # fp formats
    assert lib.mxa_quantize_mx(1, 1, None, None, 1, 1, 1, 32, 8, 8, 0, 0, 0, 7, None) == -1  # bad dtype
    assert lib.mxa_topk(1, 1, 1100, 1100, 3, 1, None, None, 0, None) == -2  # n > 1024
    assert lib.mxa_topk(1, 1, 10, 10, 11, 1, None, None, 0, None) == -1  # k > n
    assert lib.mxa_topk(1, 1, 10, 10, 3, 1, None, None, 5, None) == -1  # bad dtype
    p = N.AttnParams()
    assert lib.mxa_attention_workspace_bytes(p) == -1
    assert lib.mxa_attention(p, None) == -1


def test_workspace_formula():
    import ctypes
    from mx_quantization_amd import _native as N
    p = N.AttnParams()
    p.B, p.H, p.N, p.T, p.D = 256, 12, 197, 197, 64
    p.top_k, p.approx, p.k_top, p.pred_mode = 1, 1, 20, 0
    nbytes = N.lib().mxa_attention_workspace_bytes(ctypes.byref(p))
    # per head: Q,K codes + exponents + sign words (2 x 197 x (64 + 4 + 4 + 8) B),
    # V^T codes + exponents (64 x 224 + 7 x 64 x 2 B), kept indices (197 x 20 x 2 B: the
    # 16-bit copy for callers without idx), the one-lane tail's records (197 x (48 + 4) x 4 B:
    # k = 20 takes the 48-position prefix), the packed pass's flags (13 x 4 B: one per 16 rows)
    per_head = 2 * 197 * (64 + 4 + 4 + 8) + 64 * 224 + 7 * 64 * 2 + 197 * 20 * 2 + 197 * 52 * 4 + 13 * 4
    assert 3072 * per_head <= nbytes < 3072 * per_head + 17 * 256


def test_dropin_import_surface():
    import mx_quantization_amd as m
    mx, funcs = m.install_dropin()
    from mx import Linear, matmul  # noqa: F401  (deit main.py:36)
    from mx.elemwise_ops import quantize_elemwise_op  # noqa: F401
    from mx.mx_ops import quantize_mx_op, _shared_exponents, _reshape_to_blocks, _undo_reshape_to_blocks  # noqa
    from funcs import (exponent_approximation, elsa_approximation, save_idx_file, save_diff_score_file,  # noqa
                       diff_idx_analysis, init_analysis_files, _create_structured_orthogonal_matrix,
                       _modified_gram_schmidt, total_chosen_k, create_file, mismatch_analysis, write_data)
    assert mx.__name__ == "mx_quantization_amd.mx"


def test_reshape_to_blocks_matches_reference_shapes():
    from mx_quantization_amd.mx.mx_ops import _reshape_to_blocks, _undo_reshape_to_blocks
    x = torch.randn(2, 3, 197, 72)
    b, axes, orig, padded = _reshape_to_blocks(x, [-1], 32)
    assert tuple(b.shape) == (2, 3, 197, 3, 32) and axes == [3]
    assert torch.equal(_undo_reshape_to_blocks(b, padded, orig, axes), x)
    b, axes, orig, padded = _reshape_to_blocks(x, [-2], 32)
    assert tuple(b.shape) == (2, 3, 7, 32, 72)
    assert torch.equal(_undo_reshape_to_blocks(b, padded, orig, axes), x)


def test_specs_semantics():
    from mx_quantization_amd.mx.specs import MxSpecs, apply_mx_specs, finalize_mx_specs
    s = apply_mx_specs({"a_elem_format": "int8", "block_size": 32})
    assert isinstance(s, MxSpecs) and s["scale_bits"] == 0 and s["round"] == "nearest"
    with pytest.raises(KeyError):
        apply_mx_specs({"nope": 1})
    assert finalize_mx_specs({}) is None
    f = finalize_mx_specs({"a_elem_format": "int8", "round": "floor"})
    assert f["round_output"] == "floor" and f["a_elem_format_bp"] == "int8"


def test_product_refuses_cpu_tensors():
    import mx_quantization_amd as m
    from mx_quantization_amd import NativeError
    x = torch.zeros(2, 64)
    with pytest.raises(NativeError):
        m.topk(x, 3)
    with pytest.raises(NativeError):
        m.quantize_mx(x)
    q = torch.zeros(1, 1, 8, 64)
    with pytest.raises(NativeError):
        m.mx_topk_attention(q, q, q, 0.125, k_top=4)


def _params(B, H, Nq, T, D, k, mode="ex_pred", top_k=1):
    from mx_quantization_amd import _native as nat
    p = nat.AttnParams()
    p.q = p.k = p.v = p.out = 16  # non-null placeholders: the path query launches nothing
    p.B, p.H, p.N, p.T, p.D, p.k_top = B, H, Nq, T, D, k
    p.pred_mode, p.top_k, p.approx, p.scale = nat.PRED_MODES[mode], top_k, 1, 0.125
    return p


def test_attention_path_selection_is_host_logic():
    """mxa_attention_path: selection + finishing kernels for top-k at every bench
    shape, the dense row kernel for top_k=False (no launch, no GPU)."""
    import ctypes
    from mx_quantization_amd import _native as N
    lib = N.lib()
    split, fused = 3, 2
    for shape in [(256, 12, 197, 197, 64, 20), (64, 16, 256, 256, 72, 154), (1, 3, 197, 197, 64, 20)]:
        assert lib.mxa_attention_path(ctypes.byref(_params(*shape))) == split, shape
    assert lib.mxa_attention_path(ctypes.byref(_params(8, 16, 256, 120, 72, 20, "MXINT4"))) == split
    assert lib.mxa_attention_path(ctypes.byref(_params(1, 3, 197, 197, 64, 20, top_k=0))) == fused
    assert lib.mxa_attention_path(ctypes.byref(_params(1, 1, 10, 600, 64, 5))) == -2  # T > 512
    assert lib.mxa_attention_path(ctypes.byref(_params(1, 1, 10, 60, 160, 5))) == -2  # D > 128


def test_finishing_kernel_selection_is_host_logic():
    """mxa_attention_finish_kernel: which finishing kernel (and so which engines for QK^T /
    P.V) each bench shape and the dense branch run -- the value bench.py's mfma.engine
    reports (no launch, no GPU)."""
    import ctypes
    from mx_quantization_amd import _native as N
    fk = lambda *a, **kw: N.lib().mxa_attention_finish_kernel(ctypes.byref(_params(*a, **kw)))
    assert fk(256, 12, 197, 197, 64, 20) == 1            # DeiT-base k = 20: finish16_kernel
    assert fk(64, 16, 256, 256, 72, 154) == 3            # DiT-XL/2 k = 154: finish_qk_kernel (MFMA QK^T)
    assert fk(8, 16, 256, 120, 72, 20, "MXINT4") == 1    # PixArt cross
    assert fk(1, 2, 100, 300, 64, 100) == 2              # T > 256, k > 64: the 32-row gather kernel
    assert fk(256, 12, 197, 197, 64, 20, top_k=0) == 4   # dense DeiT-base: MFMA for both contractions
    assert fk(64, 16, 256, 256, 72, 154, top_k=0) == 4   # dense DiT-XL/2
    assert fk(1, 2, 100, 300, 64, 20, top_k=0) == 5      # dense, T > 256: the v_dot4 row kernel
    assert fk(1, 1, 10, 600, 64, 5) == -2                # T > 512
    assert set(N.FIN_KERNELS) == {1, 2, 3, 4, 5}


def test_analysis_hooks_vs_reference():
    """The drop-in funcs/analysis.py hooks against the reference's own outputs
    (tests/golden/analysis.npz from gen_golden.py): total_chosen_k, diff_idx_analysis,
    save_idx_file's text."""
    import tempfile
    from mx_quantization_amd.funcs import analysis as A
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "analysis.npz"))
    idx = torch.from_numpy(d["idx"])
    assert A.total_chosen_k(idx) == pytest.approx(float(d["chosen_k"]), rel=1e-12)
    assert A.diff_idx_analysis(torch.from_numpy(d["true_vals"]), torch.from_numpy(d["scores"])) == \
        pytest.approx(float(d["diff"]), rel=1e-6)
    with tempfile.TemporaryDirectory() as t:
        f = os.path.join(t, "idx.txt")
        A.save_idx_file(idx[:, :, :5, :], f, block_idx=3)
        assert open(f).read() == str(d["idx_text"])


def test_mismatch_analysis_vs_reference(tmp_path, monkeypatch):
    """funcs.mismatch_analysis (analysis.py:159-191) rewrites the true-index file into
    ./mismatch_idx.txt, token by token; checked against the file the reference wrote
    for the same two save_idx_file outputs (tests/golden/analysis.npz)."""
    from mx_quantization_amd.funcs import analysis as A
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "analysis.npz"))
    ft, fp = tmp_path / "true.txt", tmp_path / "pred.txt"
    ft.write_text(str(d["mm_true"]))
    fp.write_text(str(d["mm_pred"]))
    monkeypatch.chdir(tmp_path)
    res = A.mismatch_analysis(str(ft), str(fp))
    assert str(res) == str(d["mm_name"])
    assert (tmp_path / str(res)).read_text() == str(d["mm_out"])


def test_linear_and_proj_entry_points_validate_without_gpu():
    """mxa_linear / mxa_attention_proj reject bad arguments before any HIP call, and the
    workspace formulas: mxa_linear holds whole 32-row blocks of MFMA-ready codes; the
    fused proj adds the proj input (codes + exponents, plus the fp32 copy when D % 32 != 0)
    to the attention's workspace."""
    import ctypes
    from mx_quantization_amd import _native as N
    lib = N.lib()
    assert lib.mxa_linear(None, 10, 64, 64, None, 32, None, None, 32, 0, 0, 0, None, 0, None) == -1
    assert lib.mxa_linear(1, 10, 64, 63, 1, 32, None, 1, 32, 0, 0, 0, None, 0, None) == -1  # row stride < in
    assert lib.mxa_linear(1, 10, 64, 64, 1, 32, None, 1, 32, 0, 7, 0, None, 0, None) == -1  # bad bfloat
    assert lib.mxa_linear_workspace_bytes(0, 64, 32) == -1
    w = lib.mxa_linear_workspace_bytes(37, 100, 70)
    assert w >= 64 * 128 + 37 * 4 * 2  # 2 row blocks x 4 K-blocks x 32 B, plus exponents
    p = N.AttnParams()
    p.B, p.H, p.N, p.T, p.D = 2, 12, 197, 197, 64
    p.top_k, p.approx, p.k_top, p.pred_mode = 1, 1, 20, 0
    pj = N.ProjParams()
    pj.out_features = 768
    base = lib.mxa_attention_workspace_bytes(ctypes.byref(p))
    with_proj = lib.mxa_attention_proj_workspace_bytes(ctypes.byref(p), None, ctypes.byref(pj))
    tokens32 = (2 * 197 + 31) // 32 * 32
    assert with_proj >= base + tokens32 * 768 + 2 * 197 * 24 * 2
    p.D, p.H = 72, 16  # a 32-block of C spans two heads: + the fp32 output copy
    pj.out_features = 1152
    base72 = lib.mxa_attention_workspace_bytes(ctypes.byref(p))
    assert lib.mxa_attention_proj_workspace_bytes(ctypes.byref(p), None, ctypes.byref(pj)) >= base72 + 2 * 197 * 1152 * 4
    assert lib.mxa_attention_proj(ctypes.byref(p), None, None, None) == -1  # no proj params
    pj.wq = None
    assert lib.mxa_attention_proj(ctypes.byref(p), None, ctypes.byref(pj), None) == -1  # no weight


def test_exact_topk_bind_cpu():
    """bind_exact_topk rebinds only a module-level `torch` that is torch itself; the
    namespace forwards everything else; CPU tensors get torch's own topk (the reference's
    CPU path)."""
    import types

    import torch

    import mx_quantization_amd as M
    mod = types.ModuleType("glue")
    mod.torch = torch
    other = {"torch": "not torch"}
    assert M.bind_exact_topk(mod, other) == 1
    assert mod.torch is M.exact_topk_torch and other["torch"] == "not torch"
    assert mod.torch.softmax is torch.softmax and mod.torch.return_types is torch.return_types
    x = torch.randn(4, 50)
    r = mod.torch.topk(x, 7, dim=-1, largest=True, sorted=True)
    w = torch.topk(x, 7)
    assert torch.equal(r.indices, w.indices) and torch.equal(r.values, w.values)
    M.unbind_exact_topk(mod)
    assert mod.torch is torch


def test_committed_profiles_name_current_kernels():
    """The bench line's roofline.traffic / limiter come from the committed profiles of
    bench.PROFILE_TAG (profiles/<tag>_{rocprof,traffic,pmc}_*): every kernel they name
    must be a kernel of the current library, and each main-line profile must hold the
    current selection kernel family -- so a kernel change without new profiles fails."""
    import glob
    import json
    import subprocess

    import bench
    lib = os.path.join(ROOT, "mx_quantization_amd", "libmxa.so")
    if not os.path.exists(lib):
        pytest.skip("libmxa.so not built")
    syms = subprocess.run(["nm", "-C", lib], capture_output=True, text=True, check=True).stdout
    kernels = {ln.split(" ", 2)[2] for ln in syms.splitlines() if " mxa::" in ln and ln.count(" ") >= 2}
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"{bench.PROFILE_TAG}_*")))
    assert files, f"no committed profiles for PROFILE_TAG {bench.PROFILE_TAG}"
    named = set()
    for f in files:
        if f.endswith(".csv"):
            import csv
            with open(f) as fh:
                named |= {r["Name"] for r in csv.DictReader(fh) if "mxa::" in r["Name"]}
        elif "_traffic_" in f and f.endswith(".json"):
            with open(f) as fh:
                named |= {k for k in json.load(fh)["kernels"] if "mxa::" in k}
        elif "_pmc_" in f and f.endswith(".json"):
            with open(f) as fh:
                named |= {k for k in json.load(fh) if "mxa::" in k}
    missing = sorted(n for n in named if n not in kernels)
    assert not missing, f"profiles name kernels the library does not have: {missing[:4]}"
    for cfg in ("deit_base", "dit_xl2"):
        with open(os.path.join(ROOT, "profiles", f"{bench.PROFILE_TAG}_traffic_{cfg}.json")) as fh:
            sel = [k for k in json.load(fh)["kernels"] if bench.stage_of_kernel(k) == "select"]
        assert len(sel) == 1 and sel[0] in kernels, sel


def _header_params():
    """{function: [parameter declarations]} of every extern entry point in include/mxa.h."""
    import re
    src = open(os.path.join(ROOT, "include", "mxa.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    out = {}
    for m in re.finditer(r"\b(?:int|int64_t|int32_t|const char\*|void)\s+\**(mxa_\w+)\s*\(([^)]*)\)\s*;", src):
        args = [a.strip() for a in m.group(2).split(",") if a.strip() and a.strip() != "void"]
        out[m.group(1)] = args
    return out


def _ctype_of_decl(decl):
    """The ctypes type a C parameter declaration binds to (pointers -> c_void_p)."""
    import ctypes
    d = decl.replace("const ", "").strip()
    if "*" in d or d.startswith("hipStream_t"):
        return ctypes.c_void_p
    base = d.split()[0]
    return {"int64_t": ctypes.c_int64, "int32_t": ctypes.c_int32, "int": ctypes.c_int32, "float": ctypes.c_float,
            "uint32_t": ctypes.c_uint32}[base]


def test_integration_stubs_match_abi():
    """Every reference-side ctypes stub in INTEGRATION.md (`_lib.<fn>.argtypes = [...]`)
    has the argument count and order of include/mxa.h and of _native._SIGS, and every
    call of such a stub in the document passes that many arguments."""
    import ast
    import ctypes
    import re
    from mx_quantization_amd import _native
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    hdr = _header_params()
    stubs = re.findall(r"_lib\.(mxa_\w+)\.argtypes\s*=\s*(\[[^\]]*\])", doc)
    assert stubs, "no ctypes stubs found in INTEGRATION.md"
    alias = {"ctypes.c_void_p": ctypes.c_void_p, "ctypes.c_int64": ctypes.c_int64, "ctypes.c_int32": ctypes.c_int32,
             "ctypes.c_float": ctypes.c_float, "ctypes.c_uint32": ctypes.c_uint32}
    for fn, lst in stubs:
        names = [t.strip() for t in lst.strip("[]").split(",") if t.strip()]
        types = [alias[n] for n in names]
        assert fn in hdr, f"{fn}: not declared in include/mxa.h"
        want = [_ctype_of_decl(d) for d in hdr[fn]]
        assert types == want, f"{fn}: INTEGRATION.md stub {names} != include/mxa.h {hdr[fn]}"
        sig = _native._SIGS[fn][1]
        assert [t for t in sig] == want, f"{fn}: _native._SIGS disagrees with include/mxa.h"
        # every call of the stub in the document passes len(want) arguments
        for call in re.finditer(r"_lib\." + fn + r"\(", doc):
            i, depth = call.end(), 1
            while depth:
                depth += {"(": 1, ")": -1}.get(doc[i], 0)
                i += 1
            node = ast.parse("f(" + doc[call.end():i], mode="eval").body
            assert len(node.args) == len(want), f"{fn}: a call in INTEGRATION.md passes {len(node.args)} arguments"


def test_native_sigs_match_header():
    """_native._SIGS binds every include/mxa.h entry point with its parameter types."""
    from mx_quantization_amd import _native
    hdr = _header_params()
    import ctypes

    def norm(t):  # a typed pointer binds like c_void_p
        return ctypes.c_void_p if isinstance(t, type) and issubclass(t, ctypes._Pointer) else t

    for fn, params in hdr.items():
        assert fn in _native._SIGS, f"{fn} not bound in _native._SIGS"
        assert [norm(t) for t in _native._SIGS[fn][1]] == [_ctype_of_decl(d) for d in params], fn
