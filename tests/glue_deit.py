"""The mx_quant branch of the DeiT attention forward, as a workload module holds it
(workloads/deit/scripts/main.py:100-152, restated): it imports `torch`, `matmul` and
`exponent_approximation` at module level and calls `torch.topk` itself.  Test helper
(not a test file): test_gpu_parity.py rebinds its `torch` with bind_exact_topk."""
import torch

from mx import matmul
from funcs import exponent_approximation


def attention_core(q, k, v, scale, k_top, mx_specs, pred_mode="ex_pred", approx=True):
    true_scores = matmul(q, k.transpose(-2, -1), mx_specs=mx_specs, mode_config="aa") * scale
    if approx:
        ea = exponent_approximation(Q=q, K=k, mx_specs=mx_specs)
        aq, ak = {"ex_pred": ea.exponent_based_sign, "partial_Q": ea.partial_Q, "partial_K": ea.partial_K,
                  "two_step_leading_ones": ea.two_step_leading_ones, "MXINT4": ea.MXINT4}[pred_mode]()
        pred_scores = aq @ ak.transpose(-2, -1)
        _, idx = torch.topk(pred_scores, k_top, dim=-1, largest=True, sorted=True)
        vals = true_scores.gather(dim=-1, index=idx)
    else:
        vals, idx = torch.topk(true_scores, k_top, dim=-1, largest=True, sorted=True)
    attn = torch.zeros_like(true_scores)
    attn.scatter_(-1, idx, torch.softmax(vals, dim=-1).to(attn.dtype))
    return matmul(attn, v, mx_specs=mx_specs, mode_config="aa"), idx
