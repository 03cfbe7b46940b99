"""Drop-in for the reference's `funcs` package (funcs/__init__.py:11-14): the
names the patched attention modules import."""
from .exponent_based_prediction import exponent_approximation  # noqa: F401
from .elsa_approximation import (  # noqa: F401
    elsa_approximation,
    _create_structured_orthogonal_matrix,
    _modified_gram_schmidt,
)
from .utils import write_data  # noqa: F401
from .analysis import (  # noqa: F401
    create_file,
    diff_idx_analysis,
    init_analysis_files,
    mismatch_analysis,
    save_diff_score_file,
    save_idx_file,
    total_chosen_k,
)

_SUBMODULES = ("exponent_based_prediction", "elsa_approximation", "analysis", "utils")
