"""Drop-in for the reference's `mx` package (microxscaling/mx/__init__.py) --
the names the patched attention modules and `funcs` import.  The remaining
modules of the MS MX emulation library (conv, norms, activations, ...) are not
on the attention path and are not part of this build."""
from .specs import MxSpecs, add_mx_args, finalize_mx_specs, get_mx_specs, get_backwards_mx_specs  # noqa: F401
from .specs import apply_mx_specs  # noqa: F401
from .linear import Linear, linear  # noqa: F401
from .matmul import matmul  # noqa: F401
from .elemwise_ops import _quantize_bfloat as quantize_bfloat  # noqa: F401

_SUBMODULES = ("specs", "formats", "mx_ops", "elemwise_ops", "matmul", "linear")
