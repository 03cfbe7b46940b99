#!/bin/bash
# GEMM / projection parity subset, then the qkv and qkv+proj bench lines (deit, dit)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread -k "${PYK:-qkv or proj or linear or matmul}" > gpurun_out/pt2.log 2>&1
rc=$?; tail -4 gpurun_out/pt2.log; [ $rc -eq 0 ] || exit $rc
LINES=${LINES:-qkv,qkvproj} CFGS="${CFGS:-deit_base dit_xl2}" bash tools/gpu_libs_qkv.sh
