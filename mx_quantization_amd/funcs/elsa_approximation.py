"""ELSA baseline approximator -- import surface of funcs/elsa_approximation.py.

ELSA (random structured orthogonal projection -> sign hashes -> Hamming
distance -> cosine estimate, funcs/elsa_approximation.py:5-146) is not in the
BASELINE configs; it is SURVEY.md §8f "next" row 3.  The names exist so the
patched modules import unchanged; calling them raises."""


def _not_built(*_a, **_k):
    raise NotImplementedError("ELSA approximator is not built yet (SURVEY.md §8f row 3)")


_modified_gram_schmidt = _not_built
_create_structured_orthogonal_matrix = _not_built


class elsa_approximation:
    def __init__(self, *a, **k):
        _not_built()

    def approximation_scores(self):
        _not_built()
