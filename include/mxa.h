/*
 * mxa.h -- C ABI of the MI355X-native MX top-k attention library (libmxa.so).
 *
 * Plain pointers, sizes and a hipStream_t; no torch types.  Every device
 * pointer is a gfx950 device allocation; every call is asynchronous on
 * `stream` and returns an MXA_* status (0 = OK, < 0 = error, nothing launched).
 * No global state: calls are reentrant; one call per stream at a time.
 *
 * Each entry point names the reference interface it replaces.  Reference
 * paths are relative to d9bjo0522/mx_quantization (snapshot 2025-12-12).
 * The reference's own native boundary is the pybind module
 * microxscaling/mx/cpp/funcs.cpp:234-242 (7 functions), JIT-built by
 * microxscaling/mx/custom_extensions.py:11-19; its Python fallbacks in
 * mx_ops.py / elemwise_ops.py are what the workloads actually run.
 */
#ifndef MXA_H_
#define MXA_H_

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MXA_ABI_VERSION 6  /* 6: mxa_matmul_bt */

/* status codes */
#define MXA_OK 0
#define MXA_ERR_ARG (-1)          /* bad shape / pointer / option */
#define MXA_ERR_UNSUPPORTED (-2)  /* valid for the reference, not implemented here */
#define MXA_ERR_LAUNCH (-3)       /* HIP launch error */
#define MXA_ERR_WORKSPACE (-4)    /* workspace too small */

/* storage dtypes of tensor arguments.  The reference's ops follow their input's dtype
 * (microxscaling/mx/mx_ops.py:85, :283; elemwise_ops.py:146): on float16 / bfloat16
 * tensors the shared exponent is floor(log2) computed in that dtype, a float16 all-zero
 * block quantizes to NaN (2^-126 underflows: log2(0) = -inf, scale 2^-127 = 0, 0/0),
 * and every op's result is a tensor of that dtype. */
#define MXA_DT_F32 0
#define MXA_DT_F16 1
#define MXA_DT_BF16 2

/* rounding modes: microxscaling/mx/formats.py:12-16 (RoundingMode) */
#define MXA_ROUND_NEAREST 0
#define MXA_ROUND_FLOOR 1
#define MXA_ROUND_EVEN 2

/* approximator kinds, per operand side.
 * funcs/exponent_based_prediction.py:44-318 and
 * microxscaling/examples/deit/exponent_based_prediction.py:135-178 */
#define MXA_OP_SIGN 0     /* exp-sign:  (mx<0 ? -1 : +1) * 2^e_block        (ex_pred, partial_*) */
#define MXA_OP_MXINT8 1   /* MXINT8 values                                    (partial_* MX side) */
#define MXA_OP_MXINT4 2   /* MXINT4 values (Sanger)                           (MXINT4)            */
#define MXA_OP_EXION 3    /* two_step_leading_ones incl. its e*(...) quirk    (EXION)             */
#define MXA_OP_TRUE_EX 4  /* exponent_based_sign_leading_ones (values only)   (true_ex)           */

/* prediction modes of the fused op (the caller's `pred_mode`) */
#define MXA_PRED_EX_PRED 0
#define MXA_PRED_PARTIAL_Q 1
#define MXA_PRED_PARTIAL_K 2
#define MXA_PRED_MXINT4 3
#define MXA_PRED_EXION 4
#define MXA_PRED_TRUE_EX 5  /* exponent_based_sign_leading_ones (PixArt MX_transformer_block.py:663-664)   */
#define MXA_PRED_ELSA 6     /* elsa_approximation.approximation_scores (funcs/elsa_approximation.py:115-143);
                               self-attention only (N == T): the reference scales row n by the norm of
                               key row n (:126, :142-143), which broadcasts only when N == T         */

int mxa_abi_version(void);
const char* mxa_status_string(int status);

/*
 * MX block quantization of a contiguous tensor viewed as (outer, axis_len, inner),
 * blocks of `block_size` along the middle axis (0 = whole axis), integer element
 * formats with elem_mbits in {8, 4, 2} (int8 / int4 / int2).
 * Replaces quantize_mx_op -> _quantize_mx (microxscaling/mx/mx_ops.py:180-341)
 * and the reference's native quantize_mx_func_cpp / quantize_mx_by_tile_func_cuda
 * (microxscaling/mx/cpp/funcs.cpp:23-98, :177-231; mx.cu:116-287).
 *   y      : dequantized values, same layout as x (required)
 *   codes  : element codes, same layout as x (nullable)
 *   exps   : block scale exponents (outer, nblocks, inner), INT16_MIN = NaN (nullable)
 *   bfloat : elementwise pre-rounding of x (0/32 = none, 16 = bfloat16; quantize_elemwise_op)
 *   dtype  : MXA_DT_* of x and y
 */
int mxa_quantize_mx(const void* x, void* y, int8_t* codes, int16_t* exps,
                    int64_t outer, int64_t axis_len, int64_t inner, int32_t block_size,
                    int32_t elem_mbits, int32_t scale_bits, int32_t round_mode,
                    int32_t flush_subnormals, int32_t bfloat, int32_t dtype, hipStream_t stream);

/*
 * Shared exponents of the blocks of a (outer, axis_len, inner) tensor.
 * Replaces _shared_exponents (microxscaling/mx/mx_ops.py:49-99).
 *   method 0 = "max" -> out (outer, nblocks, inner); 1 = "none" -> out like x.
 *   ebits > 0 applies the [-emax, emax] / NaN clamp of :90-97.  x and out: dtype (MXA_DT_*).
 */
int mxa_shared_exponents(const void* x, void* out, int64_t outer, int64_t axis_len, int64_t inner,
                         int32_t block_size, int32_t method, int32_t ebits, int32_t dtype, hipStream_t stream);

/*
 * Elementwise bfloatX quantization.  Replaces quantize_elemwise_op / _quantize_bfloat
 * (microxscaling/mx/elemwise_ops.py:201-277) and quantize_elemwise_func_cuda
 * (microxscaling/mx/cpp/elemwise.cu:12-95).
 */
int mxa_quantize_bfloat(const void* x, void* y, int64_t n, int32_t bfloat, int32_t round_mode,
                        int32_t allow_denorm, int32_t dtype, hipStream_t stream);

/*
 * Approximator operand values along the last axis (rows x d, leading dims ld_x / ld_out),
 * MX block size 32.  Replaces the tensors returned by exponent_approximation's methods
 * (funcs/exponent_based_prediction.py:44-318): op_kind MXA_OP_*.  x and out: dtype.
 */
int mxa_approx_values(const void* x, void* out, int64_t rows, int32_t d, int64_t ld_x,
                      int64_t ld_out, int32_t op_kind, int32_t flush_subnormals, int32_t bfloat,
                      int32_t dtype, hipStream_t stream);

/*
 * torch.topk(vals, k, dim=-1, largest=True, sorted=True) with torch's CPU index
 * order (aten TopKImpl.h:45-86 -> libstdc++ nth_element + sort / partial_sort),
 * as called at workloads/deit/scripts/main.py:123, workloads/DiT/models.py:194,
 * workloads/PixArt/models/MX_transformer_block.py:678, :825.
 * rows x n with leading dim ld; n <= 1024 (PixArt 512x512 self-attention rows:
 * MX_transformer_block.py:648-717, 1,024 tokens).  out_vals nullable.
 * out_mask (nullable): the prune mask zeros.scatter_(-1, idx, 1) of the callers
 * (deit main.py:147-148; examples/deit/top_k.py:16-42) as rows x ceil(n/32)
 * words, bit j%32 of word j/32 set iff j is kept.  vals / out_vals: dtype (MXA_DT_*).
 */
int mxa_topk(const void* vals, int64_t rows, int32_t n, int64_t ld, int32_t k,
             int64_t* out_idx, void* out_vals, uint32_t* out_mask, int32_t dtype, hipStream_t stream);

/*
 * mxa_topk with a device workspace (the same results): rows of <= 256 values go through
 * the packed 32-bit selection pass and the one-lane tail (the fused op's selection
 * engine), which stage per-row state in the workspace.  mxa_topk_workspace_bytes:
 * the bytes it needs (0: no workspace path for this shape -- mxa_topk_ws then runs
 * mxa_topk; -1: invalid arguments).  workspace: 16-B aligned device memory.
 */
int64_t mxa_topk_workspace_bytes(int64_t rows, int32_t n, int32_t k);
int mxa_topk_ws(const void* vals, int64_t rows, int32_t n, int64_t ld, int32_t k,
                int64_t* out_idx, void* out_vals, uint32_t* out_mask, int32_t dtype,
                void* workspace, int64_t workspace_bytes, hipStream_t stream);

/*
 * The fused hot path: MXINT8 true scores, approximate scores, top-k prune,
 * softmax over the kept scores, MXINT8 P.V -- the mx_quant branch of
 *   QuantizedAttention.forward  workloads/deit/scripts/main.py:100-152
 *   Attention.forward           workloads/DiT/models.py:168-225
 *   MXSelfAttention.forward     workloads/PixArt/models/MX_transformer_block.py:648-717
 *   MXCrossAttention.forward    workloads/PixArt/models/MX_transformer_block.py:792-859
 * from q (B,H,N,D), k/v (B,H,T,D) to the pre-projection output (B,H,N,D).
 * Strides are in elements for the (b,h,row) dims; the D dim must be contiguous.
 */
typedef struct mxa_attn_params {
  const void* q;           /* dtype `dtype`                                                 */
  const void* k;
  const void* v;
  int64_t q_strides[3];
  int64_t k_strides[3];
  int64_t v_strides[3];
  int32_t B, H, N, T, D;
  int32_t k_top;           /* kept keys per query row (top_k != 0)                         */
  float scale;             /* float32(head_dim ** -0.5) as the caller computes it          */
  int32_t pred_mode;       /* MXA_PRED_*                                                   */
  int32_t top_k;           /* 0: dense softmax (blocks excluded from top-k)                */
  int32_t approx;          /* 0: top-k on the true scores (approx_flag / ex_pred False)    */
  int32_t flush_subnormals;/* mx_specs["mx_flush_fp32_subnorms"]                           */
  int32_t bfloat;          /* mx_specs["bfloat"]: 0/32 none, 16 bfloat16                   */
  const void* bias;        /* additive score bias (PixArt mask), dtype `dtype`, nullable   */
  int64_t bias_strides[4]; /* (b,h,n,t) element strides, 0 = broadcast                     */
  void* out;               /* (B,H,N,D) output, dtype: score_dtype ? score_dtype : dtype   */
  int64_t out_strides[3];
  int64_t* idx_out;        /* (B,H,N,k_top) contiguous int64, nullable                     */
  float* true_out;         /* optional (B,H,N,T) contiguous true scores (tests)            */
  float* pred_out;         /* optional (B,H,N,T) contiguous approximate scores            */
  uint32_t* mask_out;      /* optional prune mask (B,H,N,ceil(T/32)) words: bit t%32 of word
                              t/32 set iff key t is kept (zeros.scatter_(-1, idx, 1))      */
  const float* elsa_proj;  /* MXA_PRED_ELSA: (D,D) row-major orthogonal matrix P of the
                              caller; hash bit j = (MX(x) . P[j] >= 0)  (:105-112)           */
  const float* elsa_cos;   /* MXA_PRED_ELSA: (D+1) floats cos(clamp(pi/D*h - 0.127, 0)), the
                              caller's torch.cos values (:138-143); nullable: computed on the
                              device, correctly rounded                                    */
  void* workspace;         /* device scratch of mxa_attention_workspace_bytes() bytes     */
  int64_t workspace_bytes;
  int32_t dtype;           /* MXA_DT_* of q, k, v, bias: their MX quantization follows it   */
  int32_t score_dtype;     /* 0: the GEMM outputs (true / approximate scores, P, out) are in
                              `dtype` (the ops on tensors of that dtype); MXA_DT_F16 / BF16:
                              torch.autocast -- the fp32 q, k, v operands' matmuls return that
                              dtype, P = zeros_like(true scores) is of it and is quantized by its
                              rules (deit main.py:101, :118, :147; engine.py:97).  true_out /
                              pred_out hold those dtype values as float32.                  */
} mxa_attn_params;

int64_t mxa_attention_workspace_bytes(const mxa_attn_params* p);
int mxa_attention(const mxa_attn_params* p, hipStream_t stream);

/*
 * The approximate scores alone: pred = aQ @ aK^T (+ bias) for p->pred_mode into
 * p->pred_out (required, (B,H,N,T) contiguous) -- what the callers compute from
 * exponent_approximation's operands (deit main.py:101-118, DiT models.py:176-190,
 * PixArt MX_transformer_block.py:658-677, :805-822) or ELSA's approximation_scores,
 * without the top-k, softmax or P.V.  v and out are ignored (may be null).
 */
int mxa_approx_scores(const mxa_attn_params* p, hipStream_t stream);

/*
 * Which kernels mxa_attention(p) runs (no launch; the workspace may be null):
 *   MXA_PATH_ROWS_SPLIT  selection kernel (scores + top-k) then finishing kernel
 *                        (gather, softmax, MX(P), P.V on int8 MFMA) -- top_k != 0
 *   MXA_PATH_ROWS_FUSED  one row kernel for all of it -- the dense branch (top_k == 0)
 * or a negative MXA_ERR_* for invalid parameters.
 */
#define MXA_PATH_ROWS_FUSED 2
#define MXA_PATH_ROWS_SPLIT 3
int mxa_attention_path(const mxa_attn_params* p);

/*
 * Which finishing kernel mxa_attention(p) runs, and so on which engines its two dense
 * contractions (QK^T, P.V: microxscaling/mx/matmul.py:68-76, :85-88 as the callers use them,
 * workloads/deit/scripts/main.py:124-152, workloads/DiT/models.py:194-225) run (no launch):
 *   MXA_FIN_GATHER16    finish16_kernel: kept-key QK^T on v_dot4, P.V on v_mfma_i32_16x16x32_i8
 *   MXA_FIN_GATHER32    finish_kernel: kept-key QK^T on v_dot4, P.V on v_mfma_i32_32x32x32_i8
 *   MXA_FIN_MFMA        finish_qk_kernel: every key's QK^T and P.V on v_mfma_i32_16x16x32_i8
 *                       (the prune mask applied in the softmax)
 *   MXA_FIN_DENSE_MFMA  the dense branch (top_k == 0) on finish_qk_kernel, every key kept
 *   MXA_FIN_DENSE_ROWS  the dense branch on dense_rows_kernel (T > 256): v_dot4 for both
 * or a negative MXA_ERR_* for invalid parameters.
 */
#define MXA_FIN_GATHER16 1
#define MXA_FIN_GATHER32 2
#define MXA_FIN_MFMA 3
#define MXA_FIN_DENSE_MFMA 4
#define MXA_FIN_DENSE_ROWS 5
int mxa_attention_finish_kernel(const mxa_attn_params* p);

/*
 * Measurement entry point (bench.py): runs mxa_attention `iters` times on `stream`
 * recording HIP events between the kernels, synchronizes the stream, and writes
 * the mean milliseconds of each stage to stage_ms[MXA_ATTN_STAGES]:
 *   0 the operand builders (Q, K rows and V columns, one launch; for mxa_qkv_attention_timed
 *   the x quantization + projection)  1, 2 empty  3 scores+top-k (on MXA_PATH_ROWS_FUSED: 0)
 *   4 gather+softmax+P+P.V (on MXA_PATH_ROWS_FUSED: the dense row kernel)
 * Host-synchronizing: not for use inside graph capture.
 */
#define MXA_ATTN_STAGES 5
#define MXA_ATTN_STAGES_PLUS1 6
int mxa_attention_timed(const mxa_attn_params* p, hipStream_t stream, int32_t iters, float* stage_ms);

/*
 * The fused MX Linear qkv projection in front of the attention core: the patched
 * modules' `qkv = self.qkv(x).reshape(B, N, 3, H, D)` (workloads/deit/scripts/main.py:87-88,
 * workloads/DiT/models.py:156-157) with self.qkv an mx.Linear (microxscaling/mx/linear.py:
 * 20-103: out = bf(fl32(MX(bf(x)) @ MX(bf(W))^T)); out = bf(out + bf(bias))), feeding the
 * attention's MX operands directly -- the fp32 q / k / v never reach HBM.
 *
 * mxa_linear_weight_prep: W (out_features, in_features) fp32 row-major -> MXINT8 codes +
 * block exponents along in_features into `wq` (mxa_linear_weight_bytes bytes, 16-B
 * aligned; once per weight), laid out MFMA-ready in column groups of group_width
 * (the qkv projection: out_features = 3 * H * D, group_width = D -- one head's q, k or v).
 * The buffer starts with a header recording out_features, in_features, group_width,
 * flush_subnormals and bfloat; mxa_qkv_attention returns MXA_ERR_ARG for a buffer whose
 * header does not match (3*H*D, C, D, p->flush_subnormals, p->bfloat).  A buffer prepared
 * in another process (or copied) has its header read once, synchronously -- so not
 * inside a stream capture: call once before capturing.
 *
 * mxa_qkv_attention: mxa_attention with q, k, v produced from x (p->q, p->k, p->v are
 * ignored; self-attention, p->N == p->T).  The projection is exact-then-rounded (the
 * reference's fp32 GEMM order is unpinned: equal within fp32 rounding).
 */
typedef struct mxa_qkv_params {
  const float* x;        /* (B*N, C) tokens, row stride x_row_stride (elements)            */
  int64_t x_row_stride;
  int32_t C;             /* in_features                                                     */
  const void* wq;        /* mxa_linear_weight_prep output for W (3*H*D, C), group_width D    */
  const float* bias;     /* (3*H*D) or null                                                 */
  float* qkv_out;        /* optional (B*N, 3*H*D) fp32 projection (tests)                   */
  int32_t autocast_dtype;/* 0, or MXA_DT_F16 / BF16: torch.autocast's F.linear -- the product
                            rounded to that dtype, then + bias in fp32 (linear.py:88-101 under
                            autocast: the fp16 output + fp32 bias promotes to fp32)         */
} mxa_qkv_params;

int64_t mxa_linear_weight_bytes(int32_t out_features, int32_t in_features, int32_t group_width);
int mxa_linear_weight_prep(const float* w, int32_t out_features, int32_t in_features, int32_t group_width,
                           int32_t flush_subnormals, int32_t bfloat, void* wq, hipStream_t stream);
int64_t mxa_qkv_attention_workspace_bytes(const mxa_attn_params* p, const mxa_qkv_params* x);
int mxa_qkv_attention(const mxa_attn_params* p, const mxa_qkv_params* x, hipStream_t stream);
/* mxa_attention_timed for the fused projection path (stage 0 = x quantize + projection) */
int mxa_qkv_attention_timed(const mxa_attn_params* p, const mxa_qkv_params* x, hipStream_t stream, int32_t iters,
                            float* stage_ms);

/*
 * mx.Linear forward (microxscaling/mx/linear.py:20-103) on a prepared weight:
 *   out = bf(fl32(MX(bf(x), along in_features) @ MX(bf(W), along in_features)^T));
 *   out = bf(out + bf(bias))          (bf = quantize_elemwise_op: bfloat rounding or none)
 * x (rows, in_features) fp32 at x_row_stride; wq from mxa_linear_weight_prep(W, out_features,
 * in_features, any group_width, flush_subnormals, bfloat) -- MXA_ERR_ARG if its header
 * differs; out (rows, out_features) fp32 at out_row_stride.  Every product is the exact sum
 * rounded once (the reference's MKL sgemm order is unpinned: equal within fp32 rounding).
 * autocast_dtype: 0, or MXA_DT_F16 / BF16 (torch.autocast: the product rounded to that
 * dtype before the fp32 bias add).  The patched modules' proj Linear (deit main.py:154, DiT
 * models.py:227) and every Linear of the mx.Linear drop-in.
 */
int64_t mxa_linear_workspace_bytes(int64_t rows, int32_t in_features, int32_t out_features);
int mxa_linear(const float* x, int64_t rows, int32_t in_features, int64_t x_row_stride, const void* wq,
               int32_t out_features, const float* bias, float* out, int64_t out_row_stride,
               int32_t flush_subnormals, int32_t bfloat, int32_t autocast_dtype, void* workspace,
               int64_t workspace_bytes, hipStream_t stream);

/*
 * The attention core with the proj Linear fused behind it: the patched modules'
 *   x = attn_out.transpose(1, 2).reshape(B, N, C);  x = self.proj(x)
 * (workloads/deit/scripts/main.py:152-154, workloads/DiT/models.py:225-227; proj an
 * mx.Linear, microxscaling/mx/linear.py:20-103) after mxa_attention (xq == NULL) or
 * mxa_qkv_attention (xq != NULL).  With D % 32 == 0 (float32, no autocast) the finishing
 * kernel MX-quantizes each 32-column P.V tile straight into the proj's input codes -- the
 * fp32 attention output never reaches HBM; otherwise (a 32-element block of C spans two
 * heads) the output goes through a workspace copy and the row quantizer.  p->out is not
 * written (may be NULL); y (B*N, out_features) fp32 at y_row_stride.  Top-k path only.
 */
typedef struct mxa_proj_params {
  const void* wq;        /* mxa_linear_weight_prep output for W_proj (out_features, H*D)      */
  int32_t out_features;
  const float* bias;     /* (out_features) or null                                           */
  float* y;              /* (B*N, out_features) rows at y_row_stride                         */
  int64_t y_row_stride;
} mxa_proj_params;

int64_t mxa_attention_proj_workspace_bytes(const mxa_attn_params* p, const mxa_qkv_params* xq,
                                           const mxa_proj_params* pj);
int mxa_attention_proj(const mxa_attn_params* p, const mxa_qkv_params* xq, const mxa_proj_params* pj,
                       hipStream_t stream);
/* mxa_attention_timed for it: stage_ms[MXA_PROJ_STAGES] -- slots 0..4 as mxa_attention_timed
 * (slot 0 the x quantize + qkv projection when xq != NULL), slot 5 the proj Linear (with
 * the row quantizer when the output went through the workspace) */
#define MXA_PROJ_STAGES 6
int mxa_attention_proj_timed(const mxa_attn_params* p, const mxa_qkv_params* xq, const mxa_proj_params* pj,
                             hipStream_t stream, int32_t iters, float* stage_ms);

/*
 * mx.matmul forward (microxscaling/mx/matmul.py:31-100, :211-222): in1 (batch, M, K)
 * quantized along K, in2 (batch, K, Nc) quantized along K, fp32 result (batch, M, Nc)
 * contiguous.  Integer formats, block size 32.  a_dtype / b_dtype (MXA_DT_*): each operand's
 * MX quantization follows its dtype; c is the exact product rounded once to c_dtype (the
 * operands' dtype, or torch.autocast's: P (float16) @ V (float32) under autocast, deit
 * main.py:152 with engine.py:97).
 */
int mxa_matmul(const void* a, const void* b, void* c, int64_t batch, int32_t M, int32_t K,
               int32_t Nc, int64_t a_batch_stride, int64_t b_batch_stride, int32_t elem_mbits_a,
               int32_t elem_mbits_b, int32_t flush_subnormals, int32_t bfloat, int32_t a_dtype,
               int32_t b_dtype, int32_t c_dtype, void* workspace, int64_t workspace_bytes, hipStream_t stream);
int64_t mxa_matmul_workspace_bytes(int64_t batch, int32_t M, int32_t K, int32_t Nc);
/* mxa_matmul with in2 given transposed: bt (batch, Nc, K) row-major, i.e. in2 = bt^T (the
 * k.transpose(-2, -1) view of deit main.py:101, DiT models.py:169), quantized along K as in
 * mxa_matmul -- no copy of the transposed operand.  Same workspace (mxa_matmul_workspace_bytes). */
int mxa_matmul_bt(const void* a, const void* bt, void* c, int64_t batch, int32_t M, int32_t K,
                  int32_t Nc, int64_t a_batch_stride, int64_t bt_batch_stride, int32_t elem_mbits_a,
                  int32_t elem_mbits_b, int32_t flush_subnormals, int32_t bfloat, int32_t a_dtype,
                  int32_t b_dtype, int32_t c_dtype, void* workspace, int64_t workspace_bytes, hipStream_t stream);

/* Self-tests of the int8 MFMA operand/accumulator lane maps the kernels rely on:
 * C = A * B computed by one MFMA, row-major int8 operands, int32 result; the host
 * compares.  mxa_selftest_mfma: v_mfma_i32_16x16x32_i8 (A 16x32, B 32x16; mx.matmul);
 * mxa_selftest_mfma32: v_mfma_i32_32x32x32_i8 (A 32x32, B 32x32; the finishing
 * kernel's P.V). */
int mxa_selftest_mfma(const int8_t* a, const int8_t* b, int32_t* c, hipStream_t stream);
int mxa_selftest_mfma32(const int8_t* a, const int8_t* b, int32_t* c, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* MXA_H_ */
