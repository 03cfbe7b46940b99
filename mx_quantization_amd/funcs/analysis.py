"""Approximation-quality hooks -- funcs/analysis.py surface (the `--anal` runs).
File writers and index statistics; torch ops on whatever device idx lives on."""
from __future__ import annotations

import ast
import os
import re
from pathlib import Path

import torch


def create_file(output_file):
    d = os.path.dirname(output_file)
    if d:
        os.makedirs(d, exist_ok=True)
    open(output_file, "w").close()


def save_idx_file(idx, output_file, block_idx=None):
    """Per head / token index lists of batch element 1 (analysis.py:22-29)."""
    _, H, N, _ = idx.shape
    with open(output_file, "a") as f:
        f.write(f"Cross-attention Block {block_idx}\n")
        for h in range(H):
            f.write(f" Head {h}:\n")
            for n in range(N):
                f.write(f"  Token {n:3d}: {idx[1, h, n, :].tolist()}\n")


def save_diff_score_file(diff_score, output_file, block_idx=None):
    with open(output_file, "a") as f:
        f.write(f"{diff_score}\n")


def init_analysis_files(attn_type, anal_dir, k, approx_flag, pred_mode, total_timestep):
    """File-name table per timestep (analysis.py:35-54)."""
    d = f"{anal_dir}/{attn_type}"
    d = f"{d}/{pred_mode}" if approx_flag else f"{d}/true"
    table = {}
    for t in range(total_timestep):
        table[t] = {
            "idx": f"{d}/top{k}_idx_t{t}.txt",
            "vals": f"{d}/top{k}_vals_t{t}.txt",
            "diff_idx": f"{d}/top{k}_diff_idx_t{t}.txt",
        }
        create_file(table[t]["diff_idx"])
    return table


def total_chosen_k(pred_idx):
    """Mean over (batch, head) of |unique chosen keys| / rows (analysis.py:56-110),
    vectorised on idx's device: the union of the rows' prune masks per (batch, head)
    (scatter), its popcount, instead of a torch.unique per head."""
    B, H = pred_idx.shape[0], pred_idx.shape[1]
    rows = pred_idx.shape[-2]
    flat = pred_idx.reshape(B, H, -1).long()
    T = int(flat.max().item()) + 1 if flat.numel() else 1
    union = torch.zeros((B, H, T), dtype=torch.bool, device=pred_idx.device)
    union.scatter_(-1, flat, True)
    cov = union.sum(dim=-1).to(torch.float64) / rows
    return float(cov.mean().item())


def diff_idx_analysis(true_idx: torch.Tensor, pred_idx: torch.Tensor):
    """Share of the true top-k score mass the predicted top-k keeps, over the first
    100 batch entries (analysis.py:136-157)."""
    present = torch.isin(true_idx, pred_idx)
    kept = torch.where(present, true_idx, torch.zeros_like(true_idx))
    ratio = kept.sum(dim=-1, keepdim=True) / true_idx.sum(dim=-1, keepdim=True)
    return ratio[0:100, :, :, 0].sum().item() / (100 * ratio.shape[1] * ratio.shape[2])


def parse_tokens(path, token_re):
    """{block: {head: {token: list}}} from save_idx_file output."""
    tokens = {}
    block_idx = head_idx = 0
    with Path(path).open() as f:
        for line in f:
            m = token_re.search(line)
            if not m:
                continue
            tid = int(m.group(2))
            tokens.setdefault(block_idx, {}).setdefault(head_idx, {})[tid] = ast.literal_eval(m.group(3))
            if tid == 255 and head_idx == 15:
                head_idx, block_idx = 0, block_idx + 1
            elif tid == 255:
                head_idx += 1
    return tokens


def mismatch_analysis(true_top20_file, pred_top60_file):
    """Per token, the true top-k indices missing from the predicted list (analysis.py:159-191):
    rewrites the true file with each `Token n: [...]` line replaced by `Token n: <count>:
    [missing, in true order]` (other lines kept), into ./mismatch_idx.txt, and returns
    that path.  Blocks / heads advance at token 255 / head 15 as in parse_tokens."""
    true_top20_file = Path(true_top20_file)
    pred_top60_file = Path(pred_top60_file)
    token_re = re.compile(r"(Token\s+(\d+):\s*)(\[[^\]]*\])")
    true_t = parse_tokens(true_top20_file, token_re)
    pred_t = parse_tokens(pred_top60_file, token_re)
    diff_lines = []
    block_idx = head_idx = 0
    with true_top20_file.open() as src:
        for line in src:
            m = token_re.search(line)
            if not m:
                diff_lines.append(line)
                continue
            tid = int(m.group(2))
            pred = pred_t[block_idx][head_idx][tid]
            diff = [x for x in true_t[block_idx][head_idx][tid] if x not in pred]
            diff_lines.append(f"{m.group(1)}{len(diff)}: {diff}\n")
            if tid == 255 and head_idx == 15:
                head_idx, block_idx = 0, block_idx + 1
            elif tid == 255:
                head_idx += 1
    out_file = Path("mismatch_idx.txt")
    out_file.write_text("".join(diff_lines))
    print(f"Diff file written to: {out_file}")
    return out_file
