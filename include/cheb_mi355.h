/*
 * cheb_mi355.h -- C ABI of libcheb_mi355.so, the MI355X (gfx950) Chebyshev
 * spectral graph-convolution path.
 *
 * Drop-in boundary for the reference's filter plug-in
 *   lib/graph_conv.py:144-176  GraphConv.chebyshev5(x, L, Fout, K)
 *   lib/models.py:192-224      cgcnn.chebyshev5 (identical copy)
 *   lib/filter.py:45-95        cheby_conv(x, L, lmax, feat_out, K, W)
 * plus the ops adjacent to it on the path:
 *   lib/graph_conv.py:201-218  mpool1 / apool1
 *   lib/coarsening.py:219-240  perm_data
 *   lib/graph_model.py:293-298 Adam (compute_gradients -> apply_gradients),
 *                              with the data-parallel all-reduce inserted between.
 *
 * Conventions
 *   - Every function returns int status (CG_OK == 0); on failure
 *     cg_last_error() returns a thread-local message.  No C++ exception
 *     crosses the ABI.
 *   - Tensor pointers are DEVICE pointers owned by the caller (e.g. a torch
 *     tensor's data_ptr()), fp32, dense row-major, 16-byte aligned.
 *   - Calls are asynchronous on the given hipStream_t (passed as void*;
 *     NULL = the legacy default stream).  No call allocates or synchronises
 *     inside the compute entry points, so they may be captured in a hipGraph.
 *   - A plan is not thread-safe; use one process per GPU.
 *   - Shapes use the reference's names: N samples, M vertices, Fin / Fout
 *     features, K Chebyshev order.
 */
#ifndef CHEB_MI355_H
#define CHEB_MI355_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  CG_OK = 0,
  CG_ERR_ARG = 1,          /* bad shape / null pointer / inconsistent CSR          */
  CG_ERR_HIP = 2,          /* a HIP runtime call failed                            */
  CG_ERR_UNSUPPORTED = 3,  /* shape not supported by the requested kernel path     */
  CG_ERR_ALLOC = 4,        /* device allocation failed                             */
  CG_ERR_COMM = 5          /* RCCL failure                                         */
};

/* Kernel path selection for cg_plan_set_path (default CG_PATH_AUTO). */
enum {
  CG_PATH_AUTO = 0,     /* resident path when it fits, streaming otherwise          */
  CG_PATH_RESIDENT = 1, /* one workgroup per sample, whole recurrence in LDS        */
  CG_PATH_STREAM = 2    /* one launch per Chebyshev step + MFMA GEMMs (any size)    */
};

/* Kernel variant for cg_plan_set_variant (default CG_VARIANT_AUTO).  Every
 * variant computes the same result (the basis bit-exactly); they exist for
 * A/B measurement and as independent cross-checks in the tests. */
enum {
  CG_VARIANT_AUTO = 0,       /* fastest kernels that fit (cheb_fast when it applies)  */
  CG_VARIANT_CLASSIC = 1,    /* classic resident kernels (cheb_resident)              */
  CG_VARIANT_UNFUSED_DW = 2, /* fast kernels, dW by the separate streaming GEMM       */
  CG_VARIANT_NARROW = 3,     /* streaming path in the sample-major layout even where
                                the wide-column layout (Fin < 8) would apply          */
  CG_VARIANT_STEPS = 4       /* streaming path with one launch per Chebyshev step even
                                where the channel-group resident kernels apply
                                (M <= 1024, Fin % 8 == 0)                             */
};

/* Kernel-selection options for cg_set_option (process-wide, read at every
 * launch; no environment variables are read by the library).  The defaults are
 * the measured-faster choices; every alternative computes the same result
 * (bitwise, or y to fp32 rounding for CG_OPT_GRP16).  Values marked [ablation
 * build] are accepted only by the `make debug` library (the kernels behind them
 * lost every A/B); the release library returns CG_ERR_ARG
 * for them. */
enum {
  CG_OPT_DW_DIRECT = 0, /* 1: k_dw_direct where a chunk has >= 256 rows and the grid fills
                           the chip (default); 0: k_dw_slabs; [ablation build] 2:
                           k_dw_direct whatever the wave count, 3: as 2 with one-float
                           basis loads only                                           */
  CG_OPT_DW_W2 = 1,     /* 1: the two-waves-per-SIMD build of k_dw_direct where it fits
                           (default); [ablation build] 0: the one-wave build          */
  CG_OPT_DW_WAVES = 2,  /* waves per k_dw_slabs block: 8 (default) or 4               */
  CG_OPT_SPMM_PW = 3,   /* 1: resident SpMMs read CSR metadata two entries per LDS
                           access (default); [ablation build] 0: one entry per access */
  CG_OPT_GRP16 = 4,     /* 1: 16-channel group forward where it applies (default);
                           0: the 8-channel one                                       */
  CG_OPT_GRP_PC = 5,    /* 1: k_grp_clen with register-packed columns (default);
                           [ablation build] 0: columns from LDS                       */
  CG_OPT_CLEN_DY = 6,   /* 1: fused-dBasis Clenshaw k_grp_clen_dy, tiles pipelined
                           (default); [ablation build] 2: each order group's tiles up
                           front; 0: row-GEMM dBasis planes + k_grp_clen              */
  CG_OPT_SEQ_XPRE = 7,  /* 1: the gconv-LSTM x basis of all steps formed up front,
                           one launch with the recurrence in LDS where it fits
                           (default); 2: up front by one streaming launch per
                           order; 0: recomputed inside k_lstm_seq                     */
  CG_OPT_DW_X3 = 8,     /* 1: dW GEMMs with 65-128 dy columns (the gconv-LSTM's gates)
                           on the bf16 matrix pipe, every f32 operand split exactly
                           into three bf16 terms, six products accumulated in f32
                           (f32-accurate; not bitwise the f32 kernels) (default);
                           0: the f32-MFMA kernels                                    */
  CG_OPT_GEMM_X3 = 9,   /* 1: the same three-term split for the fast backward's dBasis
                           and fused dW (config B), the streaming path's skinny row
                           GEMMs (y = basis W, dBasis = dy W^T) and the gconv-LSTM BPTT
                           step's D_k = dpre Wh_k^T (f32-accurate; not bitwise the f32
                           kernels) (default); 0: f32 MFMA                            */
  CG_OPT_COUNT = 10
};

typedef struct cg_plan cg_plan;
typedef struct cg_comm cg_comm;

/* Set / read a kernel-selection option (CG_OPT_*); CG_ERR_ARG for an unknown
 * option or a value outside its range.  Thread-safe (relaxed atomics); a launch
 * reads the value current when it is enqueued. */
int cg_set_option(int32_t option, int32_t value);
int cg_get_option(int32_t option, int32_t* value);

/* ABI version (major*10000 + minor*100 + patch). */
int cg_version(void);
/* Message for the last non-zero status on this thread ("" if none). */
const char* cg_last_error(void);

/* ---------------------------------------------------------------------------
 * Plan: the rescaled Laplacian L~ = L/(lmax/2) - I as host CSR (int32 row
 * pointers / column indices sorted within each row, i.e. the row-major order
 * tf.sparse_reorder gives at lib/graph_conv.py:153; fp32 values), copied to
 * the device once -- the analogue of the TF graph constant built at
 * lib/graph_conv.py:148-153.  L~^T is needed by the backward (adjoint_a SpMM);
 * pass NULL for t_* to have it built on the host inside the call (L~ is not
 * bit-symmetric in fp32, so it is transposed exactly, never assumed symmetric).
 * ------------------------------------------------------------------------- */
int cg_plan_create(cg_plan** plan, int device, int32_t M, int64_t nnz,
                   const int32_t* rowptr, const int32_t* col, const float* val,
                   const int32_t* t_rowptr, const int32_t* t_col, const float* t_val);
int cg_plan_destroy(cg_plan* plan);
int cg_plan_set_path(cg_plan* plan, int path);
int cg_plan_set_variant(cg_plan* plan, int variant);
/* Which path cg_cheb_forward/backward would take for this shape (CG_PATH_*). */
int cg_plan_query_path(const cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                       int* path);

/* Device workspace the forward / backward need for this shape (bytes; may be 0).
 * The forward's workspace is dead once the forward call has been enqueued and
 * executed, so one buffer of max(fwd, bwd) bytes may serve both calls of a
 * training step on one stream. */
int cg_cheb_workspace_bytes(const cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                            size_t* fwd_bytes, size_t* bwd_bytes);

/* ---------------------------------------------------------------------------
 * Forward of chebyshev5 / cheby_conv (lib/graph_conv.py:155-176):
 *   x     [N][M][Fin]            input signals
 *   W     [Fin*K][Fout]          filter weights, row index fin*K + k (:174)
 *   basis [N*M][Fin*K]           OUT: Chebyshev basis in the layout of :172
 *                                (column fin*K + k); saved for the backward.
 *                                Bit-exact to the reference's fp32 recurrence.
 *   y     [N][M][Fout]           OUT: basis @ W (:175-176); NULL => basis only
 *                                (chebyshev2 / lib/graph.py::chebyshev analogue)
 * ------------------------------------------------------------------------- */
int cg_cheb_forward(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                    const float* x, const float* W, float* basis, float* y,
                    void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Backward (TF autodiff of the above via lib/graph_model.py:296):
 *   dy [N][M][Fout], basis (from forward), W  ->
 *   dx [N][M][Fin]  (NULL to skip), dW [Fin*K][Fout]  (overwritten, not accumulated;
 *   NULL to skip -- e.g. a recurrent caller that sums dW over time steps with
 *   one cg_weight_grad call; dx and dW may not both be NULL)
 *   basis may be NULL when dW is NULL (a dx-only call never reads it).
 * dW = basis^T dy ; dBasis = dy W^T ; reverse recurrence over L~^T.
 * ------------------------------------------------------------------------- */
int cg_cheb_backward(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                     const float* dy, const float* basis, const float* W,
                     float* dx, float* dW, void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Residual GraphConv block epilogues (lib/graph_conv.py:234-262):
 *   y = act(basis W + residual)       residual [N][M][Fout] or NULL, act CG_ACT_*
 * i.e. `x = self.filter(x, ...)`, `x = x + x_identity`, `x = b1relu(x)` in one
 * pass (the resident and streaming kernels apply it in their y store).
 * Backward through it: dz = dy * act'(y) with y the forward's OUTPUT (ReLU:
 * y > 0), written to dz (required when act != NONE; also the gradient of the
 * residual input), then the filter backward on dz.  dx_accumulate != 0 adds
 * the filter's input gradient into dx (dx += ...) -- the gradient sum of a
 * tensor that feeds both a filter and a residual branch.
 * ------------------------------------------------------------------------- */
enum { CG_ACT_NONE = 0, CG_ACT_RELU = 1, CG_ACT_TANH = 2 /* bias_act only */ };
int cg_cheb_forward_ex(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                       const float* x, const float* W, const float* residual, int32_t act,
                       float* basis, float* y, void* workspace, size_t ws_bytes, void* stream);
int cg_cheb_backward_ex(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                        const float* dy, const float* y, int32_t act, const float* basis,
                        const float* W, float* dx, int32_t dx_accumulate, float* dW, float* dz,
                        void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Basis layouts.  The basis is the forward's saved tensor (the x of
 * lib/graph_conv.py:172 that TF keeps for the matmul gradient at :175); its
 * layout is the caller's choice per call pair:
 *   CG_BASIS_ROWS    [N*M][Fin*K]   (:172; every path; the default of the calls above)
 *   CG_BASIS_ORDERS  [N][Fin*K][Mb] (Mb = M rounded up to 32; rows >= M hold 0):
 *                    one contiguous plane per Chebyshev order, so the fast forward
 *                    stores each order pair while the recurrence runs instead of
 *                    after it.  Only for Fin <= 2 where the fast resident forward
 *                    AND the fused-dW fast backward apply (else CG_ERR_UNSUPPORTED),
 *                    and the backward must compute dx with dW.
 *   CG_BASIS_PLANES  [K][N*M][Fin]: plane k is T_k in the layout of x (plane 0
 *                    a copy of x), so each streaming Chebyshev step writes its
 *                    own plane and the rows-layout assembly of the last step
 *                    (a read of T_0..T_{K-2} and a write of the whole basis)
 *                    disappears; the contraction and dW read the planes.  Only
 *                    where forward and backward both run the sample-major
 *                    streaming path with Fin a multiple of 16 and K >= 2 (the
 *                    ResGNN hidden layers), else CG_ERR_UNSUPPORTED.
 *                    x may BE plane 0 (x == basis): a caller whose producer
 *                    writes the filter input straight into plane 0 (e.g. the
 *                    previous layer's y) then pays no copy of x -- T_0 is read
 *                    in place, and the backward reads plane 0 as before.
 * Same values either way (bit-exact basis, y and dx; dW sums its per-wave row
 * chunks in another grouping, so it agrees to fp32 rounding; with the planes
 * layout y sums its inner dimension in another order, agreeing to fp32
 * rounding, and dW is bitwise the rows layout's).
 * cg_cheb_basis_elems: floats the basis buffer of that layout holds, or
 * CG_ERR_UNSUPPORTED where the layout does not apply.
 * ------------------------------------------------------------------------- */
enum { CG_BASIS_ROWS = 0, CG_BASIS_ORDERS = 1, CG_BASIS_PLANES = 2 };
int cg_cheb_basis_elems(const cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                        int32_t layout, int64_t* elems);
int cg_cheb_forward_layout(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                           const float* x, const float* W, const float* residual, int32_t act,
                           int32_t layout, float* basis, float* y, void* workspace,
                           size_t ws_bytes, void* stream);
int cg_cheb_backward_layout(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                            const float* dy, const float* y, int32_t act, int32_t layout,
                            const float* basis, const float* W, float* dx, int32_t dx_accumulate,
                            float* dW, float* dz, void* workspace, size_t ws_bytes, void* stream);
/* MSE loss of lib/graph_model.py:255, tf.reduce_mean(tf.square(labels - logits)),
 * over n elements: *loss (device scalar) and dpred = 2 (pred - labels) / n
 * (NULL to skip).  Fixed-order reduction (bitwise reproducible). */
int cg_mse_loss_workspace_bytes(int64_t n, size_t* bytes);
int cg_mse_loss(const float* pred, const float* labels, int64_t n, float* loss, float* dpred,
                void* workspace, size_t ws_bytes, void* stream);
/* The same, and the loss moving average of lib/graph_model.py:265-273
 * (tf.train.ExponentialMovingAverage(decay).apply([loss]), zero-debiased as TF
 * 1.0-1.3 does for a Tensor; the reference pins no TF version, its notebooks are
 * Python 3.4-3.6 / 2017; TF >= 1.4's zero_debias=False default is NOT what this
 * computes -- unpinned): ema = device float[3] {biased, average, local_step},
 * zero-initialised by the caller, updated in place; average is loss_average. */
int cg_mse_loss_ema(const float* pred, const float* labels, int64_t n, float* loss, float* dpred,
                    float* ema, float decay, void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Stacked-input ResGNN, GraphConv._inference with stack_num > 1
 * (lib/graph_conv.py:272-303): the input's channel groups feed separate
 * residual networks whose outputs merge as X = sum_i relu(net_i) * w_i,
 * w_i [M][F] (tf.get_variable 'final_merge/W_i/weights') broadcast over N.
 *   cg_slice_channels:  out [rows][c1-c0] = x[rows][C][c0:c1]
 *   cg_stack_merge_forward:  y = (accumulate ? y : 0) + relu(out_i) * w_i
 *   cg_stack_merge_backward: dout_i = out_i > 0 ? dy * w_i : 0 and
 *       dw_i[m][f] = sum_n relu(out_i[n][m][f]) dy[n][m][f] (n ascending);
 *       either output may be NULL.
 * ------------------------------------------------------------------------- */
int cg_slice_channels(const float* x, int64_t rows, int32_t C, int32_t c0, int32_t c1, float* out,
                      void* stream);
int cg_stack_merge_forward(int32_t N, int32_t M, int32_t F, const float* out_i, const float* w_i,
                           int32_t accumulate, float* y, void* stream);
int cg_stack_merge_backward(int32_t N, int32_t M, int32_t F, const float* dy, const float* out_i,
                            const float* w_i, float* dout_i, float* dw_i, void* stream);

/* ---------------------------------------------------------------------------
 * Weight gradient of the contraction on its own (the tf.matmul gradient of
 * lib/graph_conv.py:175 / lib/filter.py:93): dW = basis^T dy over R rows,
 * basis [R][FinK], dy [R][Fout], dW [FinK][Fout].  Fixed-order, bitwise
 * reproducible reduction; accumulate != 0 adds into dW (dW += ...), so
 * recurrent callers can sum the gradient of a weight shared over time steps.
 * ------------------------------------------------------------------------- */
int cg_weight_grad_workspace_bytes(int64_t R, int32_t FinK, int32_t Fout, size_t* bytes);
int cg_weight_grad(int64_t R, int32_t FinK, int32_t Fout, const float* basis, const float* dy,
                   float* dW, int32_t accumulate, void* workspace, size_t ws_bytes, void* stream);
/* The same for a basis in the planes layout: K planes [R][Fin] plane_stride
 * floats apart (plane k = T_k), dW [Fin*K][Fout] in the row order fin*K + k
 * (lib/graph_conv.py:174); workspace as cg_weight_grad_workspace_bytes(R,
 * Fin*K, Fout).  One pass over dy for all K orders (the gconv-LSTM's h-weight
 * gradient summed over every time step). */
int cg_weight_grad_planes(int64_t R, int32_t Fin, int32_t K, int32_t Fout, const float* planes,
                          int64_t plane_stride, const float* dy, float* dW, int32_t accumulate,
                          void* workspace, size_t ws_bytes, void* stream);
/* The three weight gradients of a gconv-LSTM layer in ONE pass over dpre
 * [R][4H] (lib/gconv_lstm.py:183-207's two cheby_conv weights and the gate
 * bias, summed over every step of the layer; R = T*N*M):
 *   dWh [H*K][4H] (row c*K + k) = sum_k T_k(h)^T dpre, h planes: K planes
 *       [R][H] h_plane_stride floats apart (rows of a step without an h-conv
 *       must hold zeros);
 *   dWx [Fin*K][4H] (row f*K + k) from the x planes [R][Fin] likewise;
 *   db [4H] = column sums of dpre.
 * Fixed-order reduction (bitwise reproducible).  4H <= 256, Fin*K < 64. */
int cg_lstm_weight_grads_workspace_bytes(int64_t R, int32_t H, int32_t Fin, int32_t K,
                                         size_t* bytes);
int cg_lstm_weight_grads(int64_t R, int32_t H, int32_t Fin, int32_t K, const float* h_planes,
                         int64_t h_plane_stride, const float* x_planes, int64_t x_plane_stride,
                         const float* dpre, float* dWh, float* dWx, float* db, void* workspace,
                         size_t ws_bytes, void* stream);
/* db[c] (+)= sum_r dy[r][c] -- gradient of a broadcast bias add, dy [R][C]. */
int cg_bias_grad_workspace_bytes(int64_t R, int32_t C, size_t* bytes);
int cg_bias_grad(int64_t R, int32_t C, const float* dy, float* db, int32_t accumulate,
                 void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Bias + activation of the GraphConv model (lib/graph_conv.py:178-199):
 *   y[i] = act(x[i] + bias[i % bias_len])       bias NULL: no add
 * b1relu / b1tanh: bias_len = F (one bias per filter, [1,1,F]); b2relu:
 * bias_len = M*F ([1,M,F]); fc (:220-226): bias_len = Mout.  act is
 * CG_ACT_NONE / RELU / TANH; x and y may alias.  n % bias_len == 0.
 * Backward: dz = dy * act'(y) from the forward OUTPUT y (TF ReluGrad /
 * TanhGrad: dy (1 - y^2)); db (+)= column sums of dz viewed [n/bias_len][bias_len]
 * (fixed order; NULL to skip).  dz and dy may alias.
 * ------------------------------------------------------------------------- */
int cg_bias_act_forward(int64_t n, int32_t bias_len, const float* x, const float* bias,
                        int32_t act, float* y, void* stream);
int cg_bias_act_workspace_bytes(int64_t n, int32_t bias_len, size_t* bytes);
int cg_bias_act_backward(int64_t n, int32_t bias_len, const float* dy, const float* y, int32_t act,
                         float* dz, float* db, int32_t accumulate, void* workspace,
                         size_t ws_bytes, void* stream);
/* C[M][N] = op(A) op(B), fp32 on MFMA (v_mfma_f32_32x32x2_f32), row-major with
 * leading dimensions; trans_a: A stored [K][lda], trans_b: B stored [N][ldb].
 * The tf.matmul of fc (lib/graph_conv.py:225) and of the Fourier transforms. */
int cg_gemm_f32(int32_t trans_a, int32_t trans_b, int32_t M, int32_t N, int32_t K, const float* A,
                int32_t lda, const float* B, int32_t ldb, float* C, int32_t ldc, void* stream);

/* ---------------------------------------------------------------------------
 * Fourier (spectral) filter, lib/graph_conv.py:83-111 (filter_in_fourier,
 * fourier; lib/models.py:129-159; lib/filter.py fourier_conv):
 *   U [M][M] = eigenvectors of L in columns (lib/graph.py:148 fourier(),
 *              U[j][m] = component j of eigenvector m), resident on device
 *   W [M][Fout][Fin] (the reference's _weight_variable([M, Fout, Fin]))
 *   x [N][M][Fin] -> y [N][M][Fout]:  y_n = U (W . (U^T x_n)) per frequency
 * xhat [N][Fin][M] receives U^T x (kept for the backward, which returns
 * dx = U W^T U^T dy-style gradients and dW[m][fo][fin] = sum_n dYh xhat,
 * fixed order over n).  dx / dW may be NULL. */
int cg_fourier_workspace_bytes(int32_t N, int32_t M, int32_t Fin, int32_t Fout, size_t* fwd_bytes,
                               size_t* bwd_bytes);
int cg_fourier_forward(int32_t N, int32_t M, int32_t Fin, int32_t Fout, const float* U,
                       const float* W, const float* x, float* xhat, float* y, void* workspace,
                       size_t ws_bytes, void* stream);
int cg_fourier_backward(int32_t N, int32_t M, int32_t Fin, int32_t Fout, const float* U,
                        const float* W, const float* xhat, const float* dy, float* dx, float* dW,
                        void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * gconv-LSTM cell pointwise part (lib/gconv_lstm.py:77-221, GConvLSTMCell).
 * The cell's eight cheby_conv calls are two chebyshev5 calls with the four
 * gate weights concatenated: gx = cheb(x; [Wzxt|Wixt|Wfxt|Woxt]) and
 * gh = cheb(h; [Wzht|Wiht|Wfht|Woht]), each [R][4H] with R = N*M rows and
 * gate blocks z | i | f | o of H columns.  Then per (r, j):
 *   a_q = (gx_q + gh_q) + b_q                      (:186, :193, :200, :207)
 *   REFERENCE gates: z = tan(a_z), i = sigmoid, f = sigmoid, o = tanh(a_o)
 *   STANDARD gates:  z = tanh(a_z), o = sigmoid(a_o)
 *   c' = f*c + i*z ;  h' = o*tanh(c')              (:215, :218)
 * gh, bias, c may be NULL (zero: the zero state of :71-76).  act [R][4H]
 * receives the gate activations (z|i|f|o) for the backward; may be NULL.
 * ------------------------------------------------------------------------- */
enum { CG_LSTM_GATES_REFERENCE = 0, CG_LSTM_GATES_STANDARD = 1 };
int cg_lstm_cell_forward(int64_t R, int32_t H, int32_t gates, const float* gx, const float* gh,
                         const float* bias, const float* c, float* c_out, float* h_out, float* act,
                         void* stream);
/* Backward of the pointwise part: dh + dh_rec = gradient w.r.t. h' (the
 * step's output gradient and the recurrent one from step t+1's h-conv,
 * summed in-kernel), dc = gradient w.r.t. c' (any of the three NULL = 0);
 * act, c (NULL = 0), c_out from the forward.  Writes
 * dpre [R][4H] = dLoss/d(a_z | a_i | a_f | a_o) (the dy of both gate
 * contractions and of the bias) and dc_prev [R][H] = dLoss/dc (NULL to skip). */
int cg_lstm_cell_backward(int64_t R, int32_t H, int32_t gates, const float* dh,
                          const float* dh_rec, const float* dc,
                          const float* act, const float* c, const float* c_out, float* dpre,
                          float* dc_prev, void* stream);

/* One time step of the cell's h path in ONE launch (the four h-gate
 * cheby_conv calls of GConvLSTMCell.__call__, lib/gconv_lstm.py:183-207, plus
 * the pointwise update above): the Chebyshev basis of h_prev [N][M][H] is
 * built in LDS, gh = basis Wh on MFMA (Wh [K*H][4H], row c*K + k -- the four
 * gate weights concatenated), a = (gx + gh) + bias, then c_out, h_out, act as
 * cg_lstm_cell_forward.  planes (NULL to skip) receives T_1 .. T_{K-1} of
 * h_prev, plane k-1 at planes + (k-1)*plane_stride, each [N][M][H] (the
 * backward's weight gradient reads them).  c_prev / bias may be NULL (zero).
 * Needs H == 32, M <= 1024 and the LDS of K (cg_lstm_hconv_supported);
 * replaces cg_cheb_forward(h) + cg_lstm_cell_forward for one step. */
int cg_lstm_hconv_supported(const cg_plan* plan, int32_t H, int32_t K, int32_t* supported);
int cg_lstm_hconv_step(cg_plan* plan, int32_t N, int32_t H, int32_t K, int32_t gates,
                       const float* h_prev, const float* c_prev, const float* gx, const float* Wh,
                       const float* bias, float* c_out, float* h_out, float* act, float* planes,
                       int64_t plane_stride, void* stream);

/* ---------------------------------------------------------------------------
 * gconv-LSTM layer, H = 32, M <= 1024 (lib/gconv_lstm.py:609-627 glstm_layer
 * -> static_rnn over GConvLSTMCell, :77-221):
 *
 * cg_lstm_seq_forward: ALL T steps of one layer in ONE cooperative launch
 * (two workgroups per sample, one per 16 hidden units, exchanging h through a
 * per-step flag; c kept in registers; L~ and Wh staged in LDS once).
 *   gx [T][N][M][4H]  the x-conv of every step (chebyshev5 of the [T*N] batch)
 *   h0, c0 [N][M][H]  initial state, NULL = zero state (step 0 then has no h-conv)
 *   hs, cs [T][N][M][H] OUT: h_t and c_t;  act [T][N][M][H][4] OUT (nullable):
 *   gate activations UNIT-major, act[r][4u + g] with g = z|i|f|o (each lane's
 *   4 units leave as one 64-byte record; cg_lstm_bwd_step reads it with
 *   act_unit_major = 1);  planes (required for K > 1): T_k of h_{t-1} for
 *   k = 1..K-1 at (k-1)*plane_stride + [T][N][M][H] (steps with an h-conv
 *   only; each workgroup computes the orders of its own 16 channels and reads
 *   its partner's from here)
 *   workspace: cg_lstm_seq_workspace_bytes (the pairs' step counters).
 *   A pair hand-off that times out (a partner workgroup not co-resident, e.g.
 *   CUs held by another stream's kernel) ends the launch instead of hanging:
 *   the lost workgroups write NaN into every hs / cs / act entry they still
 *   owed and set the plan's STICKY fault word.
 * cg_lstm_seq_fault: the plan's fault word over every sequence launch so far.
 *   wait = 1 blocks until the last launch has completed; wait = 0 never blocks
 *   and reports *fault = -1 while it is still in flight.  *fault = 1 (and
 *   CG_ERR_HIP) when a hand-off timed out; clear = 1 then resets the word.
 * cg_lstm_seq_status: (compatibility) synchronises the stream, then
 *   cg_lstm_seq_fault(plan, 1, 0, status); the workspace is not read.
 * cg_lstm_bwd_step: one BPTT step in ONE launch: dpre (the gradient of the
 *   gate pre-activations, [N][M][4H]), dc_prev and dh_prev = the h-conv's
 *   input gradient (reverse Chebyshev recurrence over L~^T of dpre Wh^T).
 *   dh / dh_rec / dc / c_prev nullable (= 0), dc_prev nullable.  K <= 4.
 *   act_unit_major: 0 = act [N][M][4H] gate-major (cg_lstm_cell_forward /
 *   cg_lstm_hconv_step), 1 = unit-major [N][M][H][4] (cg_lstm_seq_forward*).
 *   dh_prev = NULL: the step ran no h-conv (a zero-state layer's step 0): dpre
 *   and dc_prev only, bitwise cg_lstm_cell_backward on the same act values.
 * ------------------------------------------------------------------------- */
int cg_lstm_seq_supported(const cg_plan* plan, int32_t H, int32_t K, int32_t* supported);
int cg_lstm_seq_workspace_bytes(const cg_plan* plan, int32_t N, size_t* bytes);
int cg_lstm_seq_forward(cg_plan* plan, int32_t T, int32_t N, int32_t H, int32_t K, int32_t gates,
                        const float* gx, const float* Wh, const float* bias, const float* h0,
                        const float* c0, float* hs, float* cs, float* act, float* planes,
                        int64_t plane_stride, void* workspace, size_t ws_bytes, void* stream);
/* The same with the x-conv fused in (feat_in <= 8): xs [T][N][M][Fin] instead of
 * gx, Wx [K*Fin][4H] (row fin*K + k); xplanes OUT: the x basis T_k(x_t),
 * k = 0..K-1, at k*xplane_stride + [T][N][M][Fin] (the backward's dWx). */
int cg_lstm_seq_x_supported(const cg_plan* plan, int32_t Fin, int32_t H, int32_t K,
                            int32_t* supported);
int cg_lstm_seq_forward_x(cg_plan* plan, int32_t T, int32_t N, int32_t Fin, int32_t H, int32_t K,
                          int32_t gates, const float* xs, const float* Wx, float* xplanes,
                          int64_t xplane_stride, const float* Wh, const float* bias,
                          const float* h0, const float* c0, float* hs, float* cs, float* act,
                          float* planes, int64_t plane_stride, void* workspace, size_t ws_bytes,
                          void* stream);
int cg_lstm_seq_fault(cg_plan* plan, int32_t wait, int32_t clear, int32_t* fault);
int cg_lstm_seq_status(const cg_plan* plan, int32_t N, const void* workspace, int32_t* status,
                       void* stream);
/* (The failure-detection test hook cg_plan_set_seq_fault_test is declared in
 * cheb_mi355_testing.h, not here: it is for the library's own tests.) */
int cg_lstm_bwd_step(cg_plan* plan, int32_t N, int32_t H, int32_t K, int32_t gates, const float* dh,
                     const float* dh_rec, const float* dc, const float* act,
                     int32_t act_unit_major, const float* c_prev, const float* c_out,
                     const float* Wh, float* dpre, float* dc_prev, float* dh_prev, void* stream);

/* ---------------------------------------------------------------------------
 * Training-loop pieces of the gconv-LSTM models:
 * cg_dropout_forward / _backward: tf.nn.rnn_cell.DropoutWrapper(cell,
 *   output_keep_prob) of glstm_layer (lib/gconv_lstm.py:616, :623), i.e. TF 1.x
 *   tf.nn.dropout: y = (x / keep) * floor(keep + u), u ~ U[0,1) drawn from a
 *   counter hash of (seed, element index) -- the backward regenerates the mask
 *   from the same seed: dx = (dy * floor(keep + u)) / keep.  (TF's random
 *   stream itself is not reproducible here; the semantics are.)  Element i
 *   draws from the splitmix64 finaliser of seed + 0x9E3779B97F4A7C15 * (i + 1)
 *   (mod 2^64), so the slice starting at element o of a tensor dropped under
 *   seed s is dropped identically as its own tensor under seed
 *   s + 0x9E3779B97F4A7C15 * o (GLSTMModel drops only the last step this way).
 * cg_clip_by_norm: tf.clip_by_norm(t, clip_norm) then tf.check_numerics of
 *   gconvRNN.Model._build_optim (lib/gconvRNN.py:392-402), in place on one
 *   gradient tensor: t = (t * clip_norm) / max(||t||_2, clip_norm), the norm a
 *   fixed-order sum; *nonfinite (device int, nullable) is set to 1 when any
 *   clipped value is NaN or Inf (the caller raises, as check_numerics does).
 * ------------------------------------------------------------------------- */
int cg_dropout_forward(const float* x, int64_t n, float keep_prob, uint64_t seed, float* y,
                       void* stream);
int cg_dropout_backward(const float* dy, int64_t n, float keep_prob, uint64_t seed, float* dx,
                        void* stream);
int cg_clip_by_norm(float* t, int64_t n, float clip_norm, int32_t* nonfinite, void* stream);

/* ---------------------------------------------------------------------------
 * perm_data (lib/coarsening.py:219-240) on device:
 *   out[n][i][f] = perm[i] < M_in ? x[n][perm[i]][f] : 0   (fake vertices are 0)
 * x [N][M_in][F], perm [M_out] (int32), out [N][M_out][F].
 * ------------------------------------------------------------------------- */
int cg_perm_gather(const float* x, const int32_t* perm, int32_t N, int32_t M_in, int32_t M_out,
                   int32_t F, float* out, void* stream);

/* mpool1 (lib/graph_conv.py:201-209): window = stride = p along vertices,
 * y [N][M/p][F]; argmax [N][M/p][F] = absolute vertex index of the FIRST
 * maximum in window order (TF-1.x CPU MaxPoolGrad tie rule). M % p == 0. */
int cg_maxpool_forward(const float* x, int32_t N, int32_t M, int32_t F, int32_t p,
                       float* y, int32_t* argmax, void* stream);
/* dx [N][M][F] = dy routed to argmax, 0 elsewhere (fully overwritten). */
int cg_maxpool_backward(const float* dy, const int32_t* argmax, int32_t N, int32_t M, int32_t F,
                        int32_t p, float* dx, void* stream);
/* apool1 (lib/graph_conv.py:211-218) and its gradient. */
int cg_avgpool_forward(const float* x, int32_t N, int32_t M, int32_t F, int32_t p, float* y,
                       void* stream);
int cg_avgpool_backward(const float* dy, int32_t N, int32_t M, int32_t F, int32_t p, float* dx,
                        void* stream);

/* TF-1.x Adam update (lib/graph_model.py:293-298) on n fp32 parameters;
 * grad is multiplied by grad_scale first (1/world_size after an all-reduce
 * SUM).  step is 1-based. */
int cg_adam_update(float* param, const float* grad, float* m, float* v, int64_t n, float lr,
                   float beta1, float beta2, float eps, int32_t step, float grad_scale,
                   void* stream);
/* The other update rules gconvRNN.Model._build_optim selects
 * (lib/gconvRNN.py:381-389: "sgd" / "rmsprop"), as TF 1.x's training ops apply
 * them, on n fp32 parameters with grad multiplied by grad_scale first:
 *   cg_sgd_update     (GradientDescentOptimizer): param -= g * lr
 *   cg_rmsprop_update (RMSPropOptimizer, not centered; TF 1.x defaults rho 0.9,
 *     momentum 0, eps 1e-10, ms initialised to ONES, mom to zeros):
 *     ms += (g^2 - ms)(1 - rho); mom = mom*momentum + (g*lr)/sqrt(ms + eps);
 *     param -= mom */
int cg_sgd_update(float* param, const float* grad, int64_t n, float lr, float grad_scale,
                  void* stream);
int cg_rmsprop_update(float* param, const float* grad, float* ms, float* mom, int64_t n, float lr,
                      float rho, float momentum, float eps, float grad_scale, void* stream);

/* cg_cheb_backward followed by cg_adam_update(W, dW, m, v, ...) with the
 * optimizer step applied by the dW reduction itself -- for a training step
 * with no gradient exchange between them (one GPU; lib/graph_model.py:277-298,
 * `optimizer.minimize` = compute_gradients + apply_gradients).  dW receives the
 * same (bitwise) gradient as cg_cheb_backward; W, m, v are updated in place
 * after every read of W by the backward (stream order).  dW, W, m, v required. */
int cg_cheb_backward_adam(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                          const float* dy, const float* basis, float* W, float* dx, float* dW,
                          float* m, float* v, float lr, float beta1, float beta2, float eps,
                          int32_t step, float grad_scale, void* workspace, size_t ws_bytes,
                          void* stream);
/* The exchange step's Adam moved into the forward that consumes it (data-parallel
 * step: forward, backward, dW all-reduce, then this call of the NEXT step):
 *   W_out = ApplyAdam(W, grad * grad_scale; m, v) -> m_out, v_out  (lib/graph_model.py:293-298)
 *   basis, y = chebyshev5(x; W_out)                                (lib/graph_conv.py:155-176)
 * The fast kernels apply the update in their prologue (every workgroup computes
 * the same W_out; no separate Adam launch); other paths run k_adam first.  W_out,
 * m_out, v_out are written out of place and must not alias W, grad, m, v
 * (double-buffer them across steps).  Bitwise the result of cg_adam_update on
 * copies of W, m, v followed by cg_cheb_forward_layout. */
int cg_cheb_forward_adam(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                         const float* x, const float* W, const float* grad, const float* m,
                         const float* v, float lr, float beta1, float beta2, float eps,
                         int32_t step, float grad_scale, float* W_out, float* m_out, float* v_out,
                         int32_t layout, float* basis, float* y, void* workspace,
                         size_t ws_bytes, void* stream);
/* The same with the basis in a chosen layout (CG_BASIS_*, see cg_cheb_basis_elems). */
int cg_cheb_backward_adam_layout(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                                 int32_t layout, const float* dy, const float* basis, float* W,
                                 float* dx, float* dW, float* m, float* v, float lr, float beta1,
                                 float beta2, float eps, int32_t step, float grad_scale,
                                 void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Graph coarsening (host code; no device work).
 * Greedy Graclus matching of one level, lib/coarsening.py:119-165
 * (metis_one_level): rr/cc/vv are the nnz COO triplets of W in the order
 * metis() produced them (rows ascending), rid is the visit order of length
 * n_visit, weights the per-vertex Graclus weights.  The pairing weight
 * vv * (1/w_i + 1/w_j) is evaluated in the precision of vv/weights (f32: the
 * NumPy-2 float32 arithmetic of :152; f64 for float64 graphs), first strict
 * maximum wins.  cluster_id has N = rr[nnz-1] + 1 entries; *n_clusters
 * receives max(cluster_id) + 1.
 * ------------------------------------------------------------------------- */
int cg_graclus_match_f32(int64_t nnz, const int32_t* rr, const int32_t* cc, const float* vv,
                         int32_t n_visit, const int64_t* rid, const float* weights,
                         int32_t* cluster_id, int32_t* n_clusters);
int cg_graclus_match_f64(int64_t nnz, const int32_t* rr, const int32_t* cc, const double* vv,
                         int32_t n_visit, const int64_t* rid, const double* weights,
                         int32_t* cluster_id, int32_t* n_clusters);
/* Binary-tree vertex order of lib/coarsening.py:167-214 (compute_perm).
 * parents: `levels` arrays concatenated, level l has sizes[l] entries
 * (sizes[levels] = number of coarsest vertices = max(parents[levels-1]) + 1).
 * perm_out receives the orders of level 0..levels concatenated; the order of
 * level l has sizes_out[l] = n_coarsest * 2^(levels-l) entries.  perm_cap is
 * the capacity of perm_out in entries (>= n_coarsest * (2^(levels+1) - 1)). */
int cg_compute_perm(int32_t levels, const int32_t* sizes, const int32_t* parents,
                    int32_t* perm_out, int64_t perm_cap, int32_t* sizes_out);

/* ---------------------------------------------------------------------------
 * Data-parallel gradient exchange over RCCL (xGMI), for callers that do not
 * use torch.distributed.  One communicator per process/GPU; the unique id is
 * created on rank 0 and shipped by the caller (file, socket, store).
 * ------------------------------------------------------------------------- */
int cg_comm_unique_id(unsigned char id[128]);
int cg_comm_init(cg_comm** comm, int nranks, int rank, const unsigned char id[128], int device);
int cg_allreduce_sum_f32(cg_comm* comm, float* buf, size_t count, void* stream);
int cg_comm_destroy(cg_comm* comm);
/* Ranks the communicator spans (ncclCommCount): lets a caller prove the
 * exchange it times really ran over N ranks. */
int cg_comm_count(const cg_comm* comm, int* nranks);
/* Asynchronous communicator error (ncclCommGetAsyncError), polled by the
 * caller after a failed or timed-out step (SURVEY.md §5 failure detection):
 * *async_status = 0 when healthy, else the RCCL result code; the status
 * returned is CG_ERR_COMM (message in cg_last_error()) when an error is
 * pending.  With abort_on_error != 0 a pending error also aborts the
 * communicator (ncclCommAbort) so blocked ranks return. */
int cg_comm_async_error(cg_comm* comm, int* async_status, int abort_on_error);

#ifdef __cplusplus
}
#endif
#endif /* CHEB_MI355_H */
