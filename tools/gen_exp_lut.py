"""Generate the per-binade threshold table for the MX shared-exponent rule.

The reference computes a block's shared exponent as

    e = floor(torch.log2(m + 2**-126 * (m == 0)))        (mx_ops.py:83-87)

on float32 tensors.  `torch.log2` on float32 is NOT the exponent field of m:
for the top few ulps just below 2^(E+1) the float32-rounded log2 equals E+1,
so the floor is E+1.  The rule that reproduces torch on every
positive float32 is  floor(fl32(log2((double) m))).

This script turns that rule into a threshold table:

  * normal m (biased exponent field E in 1..254, mantissa M):
        e = E - 127 + (M >= TH_NORM[E])          (TH_NORM[E] == 2^23: never bumps)
  * subnormal m (E == 0, M > 0), j = floor(log2 M):
        e = -149 + j + (M >= TH_SUB[j])

Thresholds are found by bisection (the rule is monotone in m) and then checked
EXHAUSTIVELY over every positive finite float32 against numpy's float64 log2
(the restatement of torch's float32 log2).  With --torch the
exhaustive check is repeated against torch.log2 itself.

Output: tests/golden/exp_lut.npz.  The HIP kernels evaluate the same thresholds
in closed form (the distance below 2^23 depends only on the exponent's octave,
mxa_common.hpp floor_log2_abs_bits); tests/test_oracle_golden.py checks that
closed form against this table.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rule_f64(bits_u32: np.ndarray) -> np.ndarray:
    x = bits_u32.view(np.float32).astype(np.float64)
    return np.floor(np.log2(x).astype(np.float32)).astype(np.int32)


def find_threshold(base_bits: int, lo: int, hi: int, target: int) -> int:
    """Smallest mantissa offset in [lo, hi) whose rule value == target, else hi."""
    vals = rule_f64(np.array([base_bits + hi - 1], dtype=np.uint32))
    if vals[0] != target:
        return hi
    a, b = lo, hi - 1  # rule(b) == target
    while a < b:
        mid = (a + b) // 2
        if rule_f64(np.array([base_bits + mid], dtype=np.uint32))[0] == target:
            b = mid
        else:
            a = mid + 1
    return a


def build_tables():
    th_norm = np.full(256, 1 << 23, dtype=np.int64)
    for E in range(1, 255):
        th_norm[E] = find_threshold(E << 23, 0, 1 << 23, E - 126)
    th_sub = np.full(23, 1 << 23, dtype=np.int64)
    for j in range(23):
        lo, hi = 1 << j, 1 << (j + 1)
        th_sub[j] = find_threshold(0, lo, hi, -149 + j + 1)
    return th_norm, th_sub


def table_rule(bits_u32: np.ndarray, th_norm, th_sub) -> np.ndarray:
    E = (bits_u32 >> 23).astype(np.int64)
    M = (bits_u32 & 0x7FFFFF).astype(np.int64)
    out = np.empty(bits_u32.shape, dtype=np.int32)
    nrm = E > 0
    out[nrm] = (E[nrm] - 127 + (M[nrm] >= th_norm[E[nrm]])).astype(np.int32)
    sub = ~nrm
    if np.any(sub):
        Ms = M[sub]
        j = np.floor(np.log2(Ms)).astype(np.int64)
        out[sub] = (-149 + j + (Ms >= th_sub[j])).astype(np.int32)
    return out


def exhaustive_check(th_norm, th_sub, use_torch=False, chunk=1 << 25):
    if use_torch:
        import torch
    bad = 0
    start, stop = 1, 0x7F800000  # every positive finite float32 (subnormal + normal)
    for s in range(start, stop, chunk):
        e = min(s + chunk, stop)
        b = np.arange(s, e, dtype=np.uint32)
        want = table_rule(b, th_norm, th_sub)
        if use_torch:
            t = torch.from_numpy(b.view(np.float32))
            ref = torch.floor(torch.log2(t)).numpy().astype(np.int32)
        else:
            ref = rule_f64(b)
        bad += int(np.count_nonzero(want != ref))
    return bad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true", help="exhaustive check vs float64 rule")
    ap.add_argument("--torch", action="store_true", help="exhaustive check vs torch.log2")
    args = ap.parse_args()
    th_norm, th_sub = build_tables()
    bumped = int(np.sum((1 << 23) - np.minimum(th_norm[1:255], 1 << 23)))
    print(f"binades with a bump: {int(np.sum(th_norm[1:255] < (1 << 23)))}, bumped floats: {bumped}")
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "exp_lut.npz"),
                        th_norm=th_norm.astype(np.int32), th_sub=th_sub.astype(np.int32))
    if args.check:
        print("mismatches vs float64 rule:", exhaustive_check(th_norm, th_sub))
    if args.torch:
        print("mismatches vs torch.log2:", exhaustive_check(th_norm, th_sub, use_torch=True))


if __name__ == "__main__":
    sys.exit(main())
