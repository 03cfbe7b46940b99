"""Build libmxa.so (the HIP kernels + C ABI of include/mxa.h) for gfx950, in-tree.

    python -m mx_quantization_amd.build_native      (or __graft_entry__.build())

hipcc cross-compiles without a GPU.  The library links the HIP runtime by
SONAME (libamdhip64.so.7); when torch is imported first the process reuses
torch's runtime, so torch streams and device pointers are valid in it.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libmxa.so")
# (source, object suffix, defines): mxa_sel.hip is compiled seven times, the dispatcher and
# one score mode's selection kernels each (MXA_SEL_PART), so that the parts build in parallel
UNITS = [("mxa_quant.hip", "", ()), ("mxa_attn.hip", "", ()), ("mxa_sel.hip", "", ("MXA_SEL_PART=0",))]
UNITS += [("mxa_sel.hip", f"_p{i}", (f"MXA_SEL_PART={i}",)) for i in range(1, 7)]
# mxa_fin.hip: the dispatch + dense kernel (part 0) and the 32-row finishing kernel per NB (1..4)
UNITS += [("mxa_fin.hip", "", ("MXA_FIN_PART=0",))] + [("mxa_fin.hip", f"_p{i}", (f"MXA_FIN_PART={i}",)) for i in range(1, 5)]
# the 16-row finishing kernel: float32 and float16 / bfloat16 instantiations (MXA_F16_XDT)
UNITS += [("mxa_fin16.hip", f"_x{i}", (f"MXA_F16_XDT={i}",)) for i in range(2)]
UNITS += [("mxa_proj.hip", "", ()), ("mxa_gemm.hip", "", ())]
# the MFMA finishing kernel's float32 and float16 / bfloat16 instantiations (MXA_FQ_XDT)
UNITS += [("mxa_fin_qk.hip", f"_x{i}", (f"MXA_FQ_XDT={i}",)) for i in range(2)]
SOURCES = sorted({u[0] for u in UNITS})
HEADERS = ["mxa_common.hpp", "mxa_kernels.hpp", "mxa_prep.hpp", "mxa_proj.hpp", "mxa_proj_args.hpp", "mxa_finish.hpp",
           "mxa_order.hpp", "mxa_topk_grp.hpp", "mxa_topk_wave.hpp", "mxa_finish16.hpp", "mxa_finish_qk.hpp", "mxa_tail.hpp", "mxa_gemm.hpp", "mxa_dot.hpp", "mxa_select.hpp", "mxa_rows2.hpp", "mxa_modes.hpp", "mxa_launch.hpp",
           "../../include/mxa.h"]
ARCH = os.environ.get("MXA_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


OBJDIR = os.path.join(HERE, "build")  # per-unit objects + dependency files (git-ignored)


def _stale(lib=LIB):
    """The library is stale when it is missing or older than any source / header of
    csrc/ or include/ (globbed, so a new header counts without being listed) or this file."""
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    import glob
    deps = glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.hpp"))
    deps += glob.glob(os.path.join(HERE, "..", "include", "*.h")) + [os.path.abspath(__file__)]
    return any(os.path.getmtime(d) > t for d in deps)


def _obj_stale(obj, dep, cmd_file, cmd):
    """An object is rebuilt when it, its dependency list or its command line is missing or
    older than any file the compiler read for it (hipcc -MD)."""
    if not (os.path.exists(obj) and os.path.exists(dep) and os.path.exists(cmd_file)):
        return True
    with open(cmd_file) as f:
        if f.read() != " ".join(cmd):
            return True
    with open(dep) as f:
        files = f.read().replace("\\\n", " ").split()
    t = os.path.getmtime(obj)
    files = [x for x in files[1:] if not x.endswith(":")]
    return any(not os.path.exists(x) or os.path.getmtime(x) > t for x in files + [os.path.abspath(__file__)])


def build(force=False, verbose=True, defines=(), tag="", only=()):
    """defines / tag: a tools-only variant (e.g. defines=("MXA_SEL_SKIP=1",), tag="skip1"
    -> libmxa_skip1.so, loaded by tools through MXA_LIB); never the product.  only: the
    source files the variant recompiles (the other units link the product's objects, which
    must be built).  Units whose object is up to date (by hipcc's dependency list) are not
    recompiled unless force."""
    lib = LIB.replace("libmxa.so", f"libmxa_{tag}.so") if tag else LIB
    if not force and not _stale(lib):
        return lib
    os.makedirs(OBJDIR, exist_ok=True)
    objs, procs = [], []
    for src, suffix, unit_defs in UNITS:  # one hipcc per translation unit, in parallel
        if tag and only and src not in only:
            objs.append(os.path.join(OBJDIR, src.replace(".hip", f"{suffix}.o")))
            continue
        stem = src.replace(".hip", f"{suffix}{'_' + tag if tag else ''}")
        obj, dep = os.path.join(OBJDIR, stem + ".o"), os.path.join(OBJDIR, stem + ".d")
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
               "-Wall", "-Wno-unused-function", "-I", os.path.join(HERE, "..", "include"),
               "-c", os.path.join(CSRC, src), "-o", obj] + [f"-D{d}" for d in tuple(unit_defs) + tuple(defines)]
        objs.append(obj)
        cmd_file = obj + ".cmd"
        if not force and not _obj_stale(obj, dep, cmd_file, cmd):
            continue
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((subprocess.Popen(cmd + ["-MD", "-MF", dep]), cmd, cmd_file))
    bad = [c for p, c, _ in procs if p.wait() != 0]
    for p, c, cf in procs:
        if p.returncode == 0:
            with open(cf, "w") as f:
                f.write(" ".join(c))
    if bad:
        raise subprocess.CalledProcessError(1, bad[0])
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib + ".tmp"] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(lib + ".tmp", lib)
    return lib


if __name__ == "__main__":
    defs = [a[2:] for a in sys.argv[1:] if a.startswith("-D")]
    tags = [a[6:] for a in sys.argv[1:] if a.startswith("--tag=")]
    only = [x for a in sys.argv[1:] if a.startswith("--only=") for x in a[7:].split(",")]
    print(build(force="--force" in sys.argv, defines=defs, tag=tags[0] if tags else "", only=tuple(only)))
