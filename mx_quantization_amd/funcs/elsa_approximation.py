"""ELSA approximator -- drop-in for funcs/elsa_approximation.py.

`elsa_approximation(Q, K, mx_specs, orthogonal_matrix)` keeps the reference's
constructor and `approximation_scores()`; the scores come from libmxa.so
(mxa_approx_scores with MXA_PRED_ELSA): MXINT8 of Q and K along d, sign hashes
against the caller's orthogonal matrix (elsa_prep_kernel), Hamming distance by
popcount and the cosine of the corrected angle (selection kernel's ELSA mode).
The fused path takes the same mode: mx_topk_attention(..., pred_mode="ELSA",
elsa_proj=P).

Semantics kept from the reference, quirks included:
  * the scores of query row n are scaled by the norm of KEY row n
    (`key_norms.unsqueeze(-1)`, :126, :142-143) -- so N must equal T, as in the
    reference, where the broadcast fails otherwise;
  * the cosine table holds torch's CPU cosf values of the (d+1) corrected angles
    (ops.elsa_cos_table), which is what the reference's scores carry.

`_modified_gram_schmidt` / `_create_structured_orthogonal_matrix` build the
random projection once per model on the host, as the reference does (:5-58);
they consume the torch RNG and run the same floating-point sequence, so a given
seed gives the reference's matrix bit for bit (tests/test_oracle_golden.py).
"""
from __future__ import annotations

import torch

from .. import ops
from ..mx.elemwise_ops import quantize_elemwise_op
from ..mx.mx_ops import quantize_mx_op


def _modified_gram_schmidt(dim: int) -> torch.Tensor:
    """Orthonormal rows from torch.randn(dim, dim) by modified Gram-Schmidt (:5-29)."""
    vecs = torch.randn(dim, dim)
    basis = torch.zeros_like(vecs)
    for i in range(dim):
        v = vecs[i]
        for j in range(i):
            v = v - torch.dot(basis[j], v) * basis[j]
        n = torch.norm(v)
        if n < 1e-10:
            raise RuntimeError("Vectors are not linearly independent.")
        basis[i] = v / n
    return basis


def _create_structured_orthogonal_matrix(dim) -> torch.Tensor:
    """d x d orthogonal projection as a Kronecker product of small MGS factors (:31-58):
    d = 64 -> 4 (x) 4 (x) 4, d = 72 -> 8 (x) 9."""
    if dim == 64:
        a1, a2, a3 = (_modified_gram_schmidt(4) for _ in range(3))
        return torch.kron(torch.kron(a1, a2), a3)
    if dim == 72:
        print("Using Gram-Schmidt and 8x8 ⊗ 9x9 Kronecker product for 72x72 matrix.")
        a1 = _modified_gram_schmidt(8)
        a2 = _modified_gram_schmidt(9)
        return torch.kron(a1, a2)
    raise ValueError(f"No structured matrix construction defined for d={dim}. "
                     "Please add a suitable factorization in _create_structured_orthogonal_matrix.")


class elsa_approximation:
    """funcs/elsa_approximation.py:60-143 on the device."""

    def __init__(self, Q, K, mx_specs, orthogonal_matrix=None):
        if mx_specs["block_size"] != 32:
            raise NotImplementedError("ELSA is built for 32-element MX blocks")
        self.device, self.dtype = Q.device, Q.dtype
        self.mx_specs = mx_specs
        self.Q, self.K = Q, K
        self.d = Q.shape[-1]
        self.k = K.shape[-1]
        self.query_hashes = self.key_hashes = self.key_norms = None
        self.theta_bias = 0.127
        self.projection_matrix = orthogonal_matrix.to(self.device) if orthogonal_matrix is not None else None
        self._bfloat = int(mx_specs.get("bfloat", 0) or 0)
        self._flush = bool(mx_specs["mx_flush_fp32_subnorms"])

    def _mx(self, X):
        return quantize_mx_op(quantize_elemwise_op(X, self.mx_specs, round=self.mx_specs["round_output"]),
                              self.mx_specs, elem_format=self.mx_specs["a_elem_format"], axes=[-1],
                              round=self.mx_specs["round_mx_output"])

    @property
    def MX_Q(self):
        return self._mx(self.Q)

    @property
    def MX_K(self):
        return self._mx(self.K)

    def compute_hashes(self, matrix: torch.Tensor) -> torch.Tensor:
        """(matrix @ P^T >= 0), the reference's helper (:105-113).  Not on the hot path:
        approximation_scores() forms the hashes inside libmxa.so."""
        return torch.matmul(matrix, self.projection_matrix.T) >= 0

    def approximation_scores(self) -> torch.Tensor:
        if self.projection_matrix is None:
            raise ValueError("elsa_approximation needs the orthogonal matrix")
        if self.Q.dtype != torch.float32 or self.K.dtype != torch.float32:
            # the reference projects float16 / bfloat16 rows in that dtype (sign flips near 0
            # that the exact fp64 projection here does not reproduce): float32 only
            raise NotImplementedError("ELSA scores are built for float32 Q / K")
        return ops.mx_approx_scores(self.Q, self.K, "ELSA", flush_subnormals=self._flush,
                                    bfloat=self._bfloat, elsa_proj=self.projection_matrix.float())
