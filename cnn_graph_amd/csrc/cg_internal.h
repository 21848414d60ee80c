// Internal declarations shared by the HIP translation units of libcheb_mi355.
// Not part of the public ABI (that is include/cheb_mi355.h).
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace cg {

constexpr int kWave = 64;
#ifndef CG_RESIDENT_THREADS
#define CG_RESIDENT_THREADS 1024
#endif
constexpr int kResidentThreads = CG_RESIDENT_THREADS;  // 1024: 16 waves, four per SIMD
constexpr int kLdsBytes = 160 * 1024;  // gfx950 LDS per CU

// Padded LDS row stride for a vertex vector: >= M, == 1 (mod 32) so that the
// 32 lanes of a half-wave writing 32 different rows at one vertex hit 32
// different banks (ds_write_b32 banks are (addr/4) mod 32).
__host__ __device__ inline int lds_vertex_stride(int M) { return ((M + 31) / 32) * 32 + 1; }
__host__ __device__ inline size_t align16(size_t b) { return (b + 15) & ~size_t(15); }

// Kernel-selection options (cg_set_option, CG_OPT_* in include/cheb_mi355.h):
// process-wide, read by the launch code at every launch
enum Opt { kOptDwDirect = 0, kOptDwW2, kOptDwWaves, kOptSpmmPw, kOptGrp16, kOptGrpPc, kOptClenDy,
           kOptSeqXpre, kOptDwX3, kOptGemmX3, kOptCount };
int option(Opt o);

// Timing-ablation switches (bits 0-7 forward resident kernel, 8-15 backward,
// 22 skip dW, 23 skip the slab reduction; outputs are WRONG when set).  They
// exist only in the ablation build (`make debug`, -DCG_DEBUG, a separate .so
// that scripts/ablate.py loads through CG_LIB_PATH): in the release library
// there is no such state and every CG_DBG test folds to false at compile time.
#ifdef CG_DEBUG
extern int g_debug_flags;
#define CG_DBG(flags, bit) (((flags) & (bit)) != 0)
inline int debug_flags() { return g_debug_flags; }
// tuning overrides of the ablation build (cg_debug_set_param); -1 = default
extern int g_debug_params[8];
inline int debug_param(int i, int dflt) { return g_debug_params[i] >= 0 ? g_debug_params[i] : dflt; }
// per-workgroup phase timestamps (cg_debug_set_ts): slot s of workgroup b at
// ts[b * 8 + s], wall clock (s_memrealtime), written by thread 0
extern unsigned long long* g_debug_ts;
#define CG_TS(ts, slot)                                                              \
  do {                                                                               \
    if ((ts) && threadIdx.x == 0) (ts)[blockIdx.x * 8 + (slot)] = wall_clock64();    \
  } while (0)
#else
constexpr int debug_param(int, int dflt) { return dflt; }
#define CG_DBG(flags, bit) false
constexpr int debug_flags() { return 0; }
#define CG_TS(ts, slot) ((void)0)
#endif

// Stage n values into LDS with U loads in flight per thread: the plain
// `for (e = tid; e < n; e += NT) lds[e] = ld(e)` loop is compiled load ->
// s_waitcnt vmcnt(0) -> ds_write per iteration (one L2 round trip each; 20 of
// them for a K = 20 weight block).  Same values, same places.
template <int U, int NT, typename LD, typename ST>
__device__ __forceinline__ void stage_lds(int n, LD&& ld, ST&& st) {
  for (int e0 = int(threadIdx.x); e0 < n; e0 += U * NT) {
    float v[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int e = e0 + q * NT;
      v[q] = e < n ? ld(e) : 0.f;
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int e = e0 + q * NT;
      if (e < n) st(e, v[q]);
    }
  }
}

// CSR values and 16-bit columns into LDS, U loads of each in flight per thread
// (one load per iteration leaves every iteration a full memory latency)
template <int U, int NT>
__device__ __forceinline__ void stage_csr_lds(int nnz, const float* __restrict__ val,
                                              const int* __restrict__ col, float* s_val,
                                              unsigned short* s_col) {
  for (int e0 = int(threadIdx.x); e0 < nnz; e0 += U * NT) {
    float v[U];
    int c[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int e = e0 + q * NT;
      v[q] = e < nnz ? val[e] : 0.f;
      c[q] = e < nnz ? col[e] : 0;
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int e = e0 + q * NT;
      if (e < nnz) {
        s_val[e] = v[q];
        s_col[e] = static_cast<unsigned short>(c[q]);
      }
    }
  }
}

// ---- resident (LDS) path ---------------------------------------------------
struct ResidentGeom {
  int nnz;         // nonzeros of L~ (== of L~^T); the resident path needs nnz >= 1
  int rpt;        // CSR rows per thread (ceil(M / 1024)), template arg
  int nt;          // 32-wide tiles over Fout (forward), template arg
  int maxnnz;      // register slots per row of L~ (forward), template arg
  int maxnnzT;     // register slots per row of L~^T (backward), template arg
  size_t fwd_lds;  // dynamic LDS bytes of the forward kernel
  size_t bwd_lds;  // dynamic LDS bytes of the backward kernel
  bool stage;      // forward stages the sample's basis in LDS and stores it coalesced
  bool fwd_ok;
  bool bwd_ok;
};
ResidentGeom resident_geometry(int M, int nnz, int max_row_nnz, int max_row_nnzT, int Fin, int K,
                               int Fout);
// Register slots per row (ELL width) the resident kernels use for this graph.
int resident_slot_width(int M, int max_row_nnz);

// Device image of a sparse operand in "thread-slot" order for the resident
// kernels (built on the host by cheb_abi.cpp::build_slots).  Slot t in
// [0, S), S = RPT*1024, owns row[t] (-1 = idle) with len[t] entries starting
// at CSR offset beg[t]; col/val are [width][S] (column-major, padding
// col = M -> a zero word, val = 0); wlen[q*16 + w] is the max len over the
// 64 slots of wave w in slot group q.
struct SlotLayout {
  const int* row;
  const int* len;
  const int* beg;
  const int* col;
  const float* val;
  const int* wlen;
  int S;
  int width;
};
struct ResidentFwdArgs {
  int M, Fin, K, Fout, Mp, dbg;
  const float* res;  // y epilogue: y = act(basis W + res) (res may be NULL)
  int act;           // 0 = none, 1 = ReLU
  SlotLayout E;                        // L~
  const int* col;                      // CSR columns / values of L~ (tails)
  const float* val;
  const float* x;
  const float* W;
  float* basis;
  float* y;
};
struct ResidentBwdArgs {
  int M, Fin, K, Fout, Mp, dbg;
  int dx_acc;  // dx += result instead of dx = result
  SlotLayout E;                        // L~^T
  const int* col;                      // CSR of L~^T (tails)
  const float* val;
  const float* dy;
  const float* W;
  float* dx;
};
hipError_t launch_resident_forward(const ResidentGeom& g, int N, const ResidentFwdArgs& a,
                                   hipStream_t s);
hipError_t launch_resident_backward(const ResidentGeom& g, int N, const ResidentBwdArgs& a,
                                    hipStream_t s);

// ---- fast resident path (cheb_fast.hip): M <= 1024, rows <= 16 nnz, Fin in {1,2,4}
constexpr int kFastWidth = 16;  // register slots per row
// Device image of a sparse operand for the fast kernels (built on the host by
// cheb_abi.cpp::build_fast_image).  Thread t owns row[t] (-1 = idle); its
// own ring record is rpos[t] and its CSR entries gather records
// cpos[j/2][t] >> (16 * (j & 1)) & 0xffff (j < 16: two 16-bit record indices
// per word, column-major; padding gathers the zero record zpos with val 0).
// mpos[m] is the record of vertex m (m < 32*ceil(M/32); zpos past M);
// wlen[w] the max row length of wave w.  Records: P (>= M + 2, incl. the zero
// record and a dummy record that idle lanes write).
struct FastImage {
  const int* row;
  const int* rpos;   // own record, copy 0 (written every step)
  const int* rpos1;  // own record, copy 1 (written every step)
  const int* rposr;  // own record copy read as T_{k-2}
  const int* cpos;
  const float* val;
  const int* wlen;
  const int* mpos;
  const int* pos0;   // [M] copy-0 record of vertex m (T_0 initialisation)
  const int* pos1;   // [M] copy-1 record of vertex m
  int zpos;          // first of the 32 zero records (positions zpos .. zpos+31)
  int P;
};
// Host-side layout plan (lds_layout.cpp): thread->row assignment, two bank-
// aware record copies per vertex, per-gather copy choice.
struct FastLayout {
  std::vector<int> row, wlen, cpos, rpos0, rpos1, rposr, mpos, pos0, pos1;
  int P = 0, zero_base = 0, dummy_base = 0;
  long gather_cycles = 0, gather_ideal = 0;  // modelled LDS cycles of one step's gathers
};
void plan_fast_layout(int M, const int32_t* rp, const int32_t* ci, FastLayout* out);
struct FastGeom {
  int nt;            // 32-wide Fout tiles (forward)
  bool dw_fused;     // backward computes the dW partial in-kernel (FinK, Fout <= 32)
  size_t dscratch;   // bytes of the backward's dBasis / dW-reduce LDS region
  size_t fwd_lds, bwd_lds;
  size_t fwd_lds_ob;  // forward with the orders-layout basis (no LDS staging of it)
  bool fwd_ok, bwd_ok, fwd_ok_ob;
};
FastGeom fast_geometry(int M, int P, int max_row_nnz, int max_row_nnzT, int Fin, int K, int Fout);
struct FastFwdArgs {
  int M, Fin, K, Fout, dbg;
  const float* res;  // y epilogue: y = act(basis W + res) (res may be NULL)
  int act;           // 0 = none, 1 = ReLU
  FastImage E;  // L~
  const float* x;
  const float* W;
  float* basis;
  float* y;
  int bord;  // 0: basis [N*M][Fin*K]; else the orders layout [N][Fin*K][bord] (bord = Mb)
  unsigned long long* ts;  // ablation build: phase timestamps (CG_TS), else NULL
  // Adam in the prologue (cg_cheb_forward_adam), when ad_grad != NULL: the
  // contraction uses W' = ApplyAdam(W, grad) computed by every workgroup
  // alike; workgroup 0 stores W', m', v' (out-of-place: the others still read
  // W, m, v)
  const float* ad_grad;
  const float* ad_m;
  const float* ad_v;
  float* ad_W;
  float* ad_mo;
  float* ad_vo;
  float ad_lr_t, ad_b1, ad_b2, ad_eps, ad_scale;
};
struct FastBwdArgs {
  int M, Fin, K, Fout, Mp, dbg;
  int dx_acc;  // dx += result instead of dx = result
  size_t dscratch_bytes;
  FastImage E;  // L~^T
  const float* dy;
  const float* basis;  // read by the fused dW
  const float* W;
  float* dx;
  float* dw_slab;      // [N][FinK][Fout] per-sample dW partials, or NULL (no fused dW)
  int bord;            // basis layout, as FastFwdArgs::bord
  unsigned long long* ts;  // ablation build: phase timestamps (CG_TS), else NULL
  int x3;              // dBasis = dy W^T on the split-bf16 matrix pipe (CG_OPT_GEMM_X3)
};
hipError_t launch_fast_forward(const FastGeom& g, int N, const FastFwdArgs& a, hipStream_t s);
hipError_t launch_fast_backward(const FastGeom& g, int N, const FastBwdArgs& a, hipStream_t s);

// ---- streaming path ----------------------------------------------------------
// One Chebyshev step over all (sample, row) pairs in the sample-major layout
// (T_k [N][M][Fin], T_0 = x).  last: also assemble the basis [N*M][Fin*K]
// from x, slots (T_1..T_{K-2}, N*M*Fin floats apart) and the new T_{K-1}.
// rperm: row visiting order (NULL = natural).
hipError_t launch_cheb_step(const int* rowptr, const int* col, const float* val, const int* rperm,
                            const float* Tp, const float* Tpp, float* Tout, const float* x,
                            const float* slots, float* basis, int N, int M, int Fin, int K, int k,
                            bool last, hipStream_t s);
// Reverse step G_k = D_k + c L~^T G_{k+1} - G_{k+2} (sample-major; k = 0 -> dx).
hipError_t launch_clenshaw(const int* trowptr, const int* tcol, const float* tval, const int* rperm,
                           const float* Gn1, const float* Gn2, float* Gout, const float* Dk, int N,
                           int M, int Fin, int K, int k, int dx_acc, hipStream_t s);
// ---- wide-column streaming path (cheb_wide.hip): Fin < 8, vertex-major [M][Fin*N]
struct WideGeom {
  int G;    // column groups (8: one per XCD under round-robin placement, or 1)
  int CB;   // columns per group
  int pl;   // floats per lane (1, 2, 4)
  int rpb;  // rows per 256-thread block
  bool ok;
};
WideGeom wide_geometry(int N, int Fin, int M);
// mode 0: out = L~ Tp; 1: out = 2 L~ Tp - Tpp; 2: out = Dk + c L~ Tp [- Tpp]
// (Tp NULL: the sum is +0).  Planes are [M][B], B = Fin*N.
hipError_t launch_wide_step(const WideGeom& g, const int* rowptr, const int* col, const float* val,
                            const int* rperm, const float* Tp, const float* Tpp, const float* Dk,
                            float* out, int M, int B, int mode, float c, hipStream_t s);
// The last forward step fused with the basis assembly (Fin == 1, natural row
// order): planes T_0..T_{K-2} in, basis [N][M][K] out.
bool wide_last_ok(const WideGeom& g, int Fin, int K, bool rperm);
hipError_t launch_wide_last(const WideGeom& g, const int* rowptr, const int* col, const float* val,
                            const float* planes, int64_t plane, float* basis, int M, int N, int K,
                            hipStream_t s);
// dst[p][q][n] = src[p][n][q] (P planes; Q = M*Fin) and the reverse, dst[n][q] (+)= src[q][n]
hipError_t launch_sm_to_vm(const float* src, int P, int N, int64_t Q, float* dst, hipStream_t s);
hipError_t launch_vm_to_sm(const float* src, int N, int64_t Q, float* dst, int accumulate,
                           hipStream_t s);
// Backward dense pass of the wide path, one read of dy: D planes
// D[k*plane + m*Fin*N + fin*N + n] = sum_f dy[n][m][f] W[fin*K+k][f] and per-block
// dW partials slab[b][FinK][Fout] (wide_dypass_blocks of them; reduce after).
bool wide_dypass_ok(int FinK, int Fout);
int wide_dypass_blocks(int N, int M);
hipError_t launch_wide_dypass(const float* dy, const float* basis, const float* W, int N, int M,
                              int Fin, int K, int Fout, float* D, int64_t plane, float* slab,
                              hipStream_t s);
// basis[n][m][fin*K + k] = T[k*plane + m*Fin*N + fin*N + n]
hipError_t launch_wide_assemble(const float* T, int64_t plane, int N, int M, int Fin, int K,
                                float* basis, hipStream_t s);

// ---- channel-group resident kernels (cheb_group.hip): M <= 1024, Fin % 8 == 0 ----
// One workgroup per (sample, 8 channels) runs the whole recurrence in LDS.
bool grp_ok(int M, int64_t nnz, int Fin, int K, int Fout);
size_t grp_partial_bytes(int N, int M, int Fin, int Fout);
// forward, planes basis layout: basis planes [K][N*M][Fin] (plane 0 = x) and,
// when y != NULL, y = act(basis W + res) via per-group partials yp
// (grp_partial_bytes of workspace)
hipError_t launch_grp_fwd(const int* rowptr, const int* col, const float* val, const int* order,
                          int64_t nnz, int N,
                          int M, int Fin, int K, int Fout, const float* x, const float* W,
                          float* basis, float* yp, const float* res, int act, float* y,
                          hipStream_t s);
// backward: the whole reverse recurrence from the k-major dBasis planes D; dx (+)= G_0
hipError_t launch_grp_clen(const int* trowptr, const int* tcol, const float* tval, const int* order,
                           int64_t nnzT,
                           int N, int M, int Fin, int K, const float* D, float* dx, int dx_acc,
                           hipStream_t s);
// the same with dBasis = dy W^T computed in the kernel (bitwise the row GEMM's
// planes; no D planes): Fout 2, 32 or 64 and the W rows fit the LDS (grp_clen_dy_ok)
bool grp_clen_dy_ok(int M, int64_t nnzT, int K, int Fout);
hipError_t launch_grp_clen_dy(const int* trowptr, const int* tcol, const float* tval,
                              const int* order, int64_t nnzT, int N, int M, int Fin, int K,
                              int Fout, const float* dy, const float* W, float* dx, int dx_acc,
                              hipStream_t s);

// C[Mg x Ng] (+)= op(A)[Mg x Kg] * op(B)[Kg x Ng]; fp32 in/out on MFMA f32.
// trans_a: A stored [Kg][lda] (A^T row-major); trans_b: B stored [Ng][ldb].
// splits > 1: the K range is cut into `splits` slices, slice s writes
// C + s*Mg*ldc (a partial slab, reduced later by launch_reduce_slabs).
// Skinny row GEMM on MFMA (persistent, B staged in LDS): for p < planes,
// C[p*c_plane + r*ldc + j] = sum_k A[r*lda + k] * B[p*bs_p + k*bs_k + j*bs_j],
// r < R, k < Kc, j < Nc.  rowgemm_ok says whether the shape is supported.
bool rowgemm_ok(int Kc, int lda, int Nc);
// Epilogue (planes == 1 use): C = act(C + res), res [R][ldc] or NULL, act 1 = ReLU.
// pfin > 0 (planes == 1, no epilogue): one pass over A computes Nc = P*pfin
// columns, column jj being column jj % pfin of plane jj / pfin (B and C alike),
// so A is read once for all planes instead of once per plane.
// apl_fin > 0 (planes == 1): A is a basis in the planes layout, K = bmapK
// planes of [R][apl_fin] apl_stride floats apart (inner index kk = k*apl_fin +
// fin), B the [Fin*K][Nc] weight in its own row order fin*K + k.
hipError_t launch_rowgemm(const float* A, int64_t R, int Kc, int lda, const float* B, int64_t bs_k,
                          int64_t bs_j, int64_t bs_p, int planes, int Nc, float* C, int ldc,
                          int64_t c_plane, hipStream_t s, const float* res = nullptr, int act = 0,
                          int pfin = 0, int apl_fin = 0, int64_t apl_stride = 0, int bmapK = 0);
// remapK > 0: write C in the k-major [remapK][Mg][Ng/remapK] layout instead
// (column fin*K + k -> plane k), splits must be 1.
hipError_t launch_gemm_f32(bool trans_a, bool trans_b, int Mg, int Ng, int Kg, const float* A,
                           int lda, const float* B, int ldb, float* C, int ldc, int splits,
                           hipStream_t s, int remapK = 0);
// dW = basis^T dy as per-chunk partial slabs ([dw_chunks(R)][FinK][Fout]),
// R = N*M basis rows; reduce with launch_reduce_slabs.
int dw_chunks(int64_t R);
// pl_fin > 0: basis in the planes layout (K planes of [R][pl_fin], pl_stride
// floats apart); the slabs keep the rows layout's [Fin*K][Fout] order.
// xb != NULL: x_fin*K more planes columns from xb (x_stride apart) and a
// column of ones after the FinK basis columns (the gconv-LSTM's dWx and db in
// the same pass over dy); the slabs are then [FinK + x_fin*K + 1][Fout].
// Small dW (config A: R = N*M rows of a few columns): ONE 256-thread block
// forms dW = basis^T dy (rows layout) straight into `out` in a fixed order (no
// slabs, no reduction launch).  dw_small_ok says whether the shape qualifies.
bool dw_small_ok(int64_t R, int FinK, int Fout);
bool dw_small_aligned(const float* basis, const float* dy);  // both 16-byte aligned
hipError_t launch_dw_small(const float* basis, const float* dy, int64_t R, int FinK, int Fout,
                           float* out, hipStream_t s);
hipError_t launch_dw_slabs(const float* basis, const float* dy, int64_t R, int FinK, int Fout,
                           float* slab, hipStream_t s, int pl_fin = 0, int64_t pl_stride = 0,
                           int K = 0, const float* xb = nullptr, int x_fin = 0,
                           int64_t x_stride = 0);
// Number of K slices launch_gemm_f32 actually uses for `splits` requested.
int gemm_effective_splits(int Kg, int splits);
hipError_t launch_reduce_slabs(const float* slab, int nslab, int64_t count, float* out,
                               hipStream_t s);
// Same fixed-order reduction, then out[i] = out[i] + sum (accumulate != 0).
hipError_t launch_reduce_slabs3(const float* slab, int nslab, int64_t count, float* out0,
                                int64_t n0, float* out1, int64_t n01, float* out2, hipStream_t s);
hipError_t launch_reduce_slabs_acc(const float* slab, int nslab, int64_t count, float* out,
                                   int accumulate, hipStream_t s);

// ---- elementwise epilogues and the MSE loss (epilogue.hip) ---------------------
// y = act(y + res) in place (res may be NULL); act 1 = ReLU
hipError_t launch_act_fwd(float* y, const float* res, int act, int64_t n, hipStream_t s);
// dz = y > 0 ? dy : 0 (gradient through ReLU given its output y)
hipError_t launch_relu_bwd(const float* dy, const float* y, float* dz, int64_t n, hipStream_t s);
// y = act(x + bias[i % blen]) (bias may be NULL); act 0 none, 1 ReLU, 2 tanh
hipError_t launch_bias_act_fwd(const float* x, const float* bias, int64_t blen, int act, int64_t n,
                               float* y, hipStream_t s);
// dz = dy * act'(y) given the activation's output y
hipError_t launch_bias_act_bwd(const float* dy, const float* y, int act, int64_t n, float* dz,
                               hipStream_t s);
// loss = mean((labels - pred)^2) (fixed-order reduction); dpred = 2 (pred - labels) / n
int mse_chunks(int64_t n);
// ema: optional float[3] {biased, average, local_step} of the loss moving
// average (ExponentialMovingAverage(decay), zero-debiased), updated in place
hipError_t launch_mse(const float* pred, const float* labels, int64_t n, float* slab, float* loss,
                      float* dpred, hipStream_t s, float* ema = nullptr, float decay = 0.9f);
// stacked-input ResGNN pieces (lib/graph_conv.py:272-303)
hipError_t launch_slice_channels(const float* x, int64_t rows, int C, int c0, int c1, float* out,
                                 hipStream_t s);
hipError_t launch_stack_merge_fwd(const float* o, const float* w, int N, int64_t MF, int accumulate,
                                  float* y, hipStream_t s);
hipError_t launch_dropout(const float* x, float* y, int64_t n, float keep, unsigned long long seed,
                          int bwd, hipStream_t s);
hipError_t launch_clip_norm(float* t, int64_t n, float c, int* nonfinite, hipStream_t s);
hipError_t launch_stack_merge_bwd(const float* dy, const float* o, const float* w, int N, int64_t MF,
                                  float* d_o, float* dw, hipStream_t s);

// ---- gconv-LSTM cell (lstm.hip) ------------------------------------------------
// gates: 0 = reference gate functions (tan / sigmoid / sigmoid / tanh,
// lib/gconv_lstm.py:188-209), 1 = standard LSTM (tanh / ... / sigmoid).
hipError_t launch_lstm_fwd(int gates, int64_t R, int H, const float* gx, const float* gh,
                           const float* bias, const float* c, float* c_out, float* h_out,
                           float* act, hipStream_t s);
hipError_t launch_lstm_bwd(int gates, int64_t R, int H, const float* dh, const float* dh_rec,
                           const float* dc,
                           const float* act, const float* c, const float* c_out, float* dpre,
                           float* dc_prev, hipStream_t s, int act_um = 0);
// One time step's h path of the gconv-LSTM in one launch (lstm_fused.hip):
// the Chebyshev basis of h_prev in LDS, gh = basis Wh on MFMA, the gate
// update; planes (nullable) receive T_1..T_{K-1} of h_prev ([N][M][H] each,
// `plane` floats apart).  H == 32, M <= 1024.
size_t lstm_hstep_lds(int M, int K);
bool lstm_hstep_ok(int M, int H, int K);
hipError_t launch_lstm_hstep(int gates, int N, int M, int K, const int* rowptr, const int* col,
                             const float* val, const float* h_prev, const float* c_prev,
                             const float* gx, const float* Wh, const float* bias, float* c_out,
                             float* h_out, float* act, float* planes, int64_t plane,
                             hipStream_t s);
// The gconv-LSTM layer forward over all T steps in ONE cooperative launch and
// the BPTT step in one launch (lstm_seq.hip).  H == 32, M <= 1024.
// xfin: feat_in of a fused x-conv (0: gx precomputed)
size_t lstm_seq_lds(int M, int K, int64_t nnz, int xfin);
bool lstm_seq_ok(int M, int H, int K, int64_t nnz, int xfin = 0);
size_t lstm_bstep_lds(int M, int K, int64_t nnzT, bool x3);
bool lstm_bstep_ok(int M, int H, int K, int64_t nnzT);
// workgroup pairs of the persistent forward (min(N, CUs / 2))
int lstm_seq_pairs(int N, int device);
// flags: 2P + 1 ints (pair step counters, then the status word), zeroed here
hipError_t launch_lstm_seq(int gates, int T, int N, int M, int K, int64_t nnz, const int* rowptr,
                           const int* col, const float* val, const int* order, const float* xs,
                           const float* Wx, int Fin, float* xplanes, int64_t xpstride, const float* gx, const float* Wh,
                           const float* bias, const float* h0, const float* c0, float* hs,
                           float* cs, float* act, float* planes, int64_t pstride, int* flags,
                           int* status, int P, hipStream_t s, int inject_t = -1,
                           int max_row_nnz = 1 << 30);
hipError_t launch_lstm_bstep(int gates, int N, int M, int K, const int* trowptr, const int* tcol,
                             const float* tval, const int* order, int64_t nnzT, const float* dh, const float* dh_rec,
                             const float* dc, const float* act, int act_um, const float* c_prev,
                             const float* c_out, const float* Wh, float* dpre, float* dc_prev,
                             float* dh_prev, hipStream_t s);
// Column sums of A [R][C] as [colsum_chunks(R)][C] partial slabs.
int colsum_chunks(int64_t R);
hipError_t launch_colsum_slabs(const float* A, int64_t R, int C, float* slab, hipStream_t s);

// ---- Fourier filter (fourier.hip) -----------------------------------------------
// out[b][c][r] = in[b][r][c] for b < B, r < R, c < C (LDS-tiled)
hipError_t launch_transpose_batched(const float* in, int64_t B, int R, int C, float* out,
                                    hipStream_t s);
// Yh[n][fo][m] = sum_fin W[m][fo][fin] Xh[n][fin][m]   (per-vertex filter)
hipError_t launch_fourier_mix(const float* Xh, const float* W, int N, int M, int Fin, int Fout,
                              float* Yh, hipStream_t s);
// dXh[n][fin][m] = sum_fo W[m][fo][fin] dYh[n][fo][m]
hipError_t launch_fourier_mix_t(const float* dYh, const float* W, int N, int M, int Fin, int Fout,
                                float* dXh, hipStream_t s);
// dW[m][fo][fin] = sum_n dYh[n][fo][m] Xh[n][fin][m]   (fixed order over n)
hipError_t launch_fourier_dw(const float* dYh, const float* Xh, int N, int M, int Fin, int Fout,
                             float* dW, hipStream_t s);

// ---- misc ----------------------------------------------------------------------
hipError_t launch_perm_gather(const float* x, const int32_t* perm, int N, int M_in, int M_out,
                              int F, float* out, hipStream_t s);
hipError_t launch_maxpool_fwd(const float* x, int N, int M, int F, int p, float* y, int32_t* arg,
                              hipStream_t s);
hipError_t launch_maxpool_bwd(const float* dy, const int32_t* arg, int N, int M, int F, int p,
                              float* dx, hipStream_t s);
hipError_t launch_avgpool_fwd(const float* x, int N, int M, int F, int p, float* y, hipStream_t s);
hipError_t launch_avgpool_bwd(const float* dy, int N, int M, int F, int p, float* dx,
                              hipStream_t s);
hipError_t launch_sgd(float* param, const float* grad, int64_t n, float lr, float grad_scale,
                      hipStream_t s);
hipError_t launch_rmsprop(float* param, const float* grad, float* ms, float* mom, int64_t n, float lr,
                          float rho, float momentum, float eps, float grad_scale, hipStream_t s);
hipError_t launch_adam(float* param, const float* grad, float* m, float* v, int64_t n, float lr_t,
                       float beta1, float beta2, float eps, float grad_scale, hipStream_t s);
// One Adam step applied by the slab reduction that produces its gradient.
struct AdamStep {
  float* param;
  float* m;
  float* v;
  float lr_t, beta1, beta2, eps, grad_scale;
};
// TF-1.x ApplyAdam on one element (lib/graph_model.py:293-298), one rounding
// per operation (no FMA contraction, as TF's CPU functor): the single
// definition k_adam, k_reduce_slabs_adam and the Adam-in-forward prologue of
// cheb_fwd_fast share, so all three agree bitwise.
struct AdamElem {
  float p, m, v;
};
__device__ __forceinline__ AdamElem adam_math(float p0, float m0, float v0, float grad,
                                              float grad_scale, float lr_t, float beta1,
                                              float beta2, float eps) {
#pragma clang fp contract(off)
  const float g = grad * grad_scale;
  const float mi = m0 + (g - m0) * (1.f - beta1);
  const float vi = v0 + (g * g - v0) * (1.f - beta2);
  return AdamElem{p0 - lr_t * mi / (sqrtf(vi) + eps), mi, vi};
}
// grad[i] = sum_z slab[z][i] in k_reduce_slabs' order (bitwise the same dW),
// then the k_adam update of element i, in one launch.
hipError_t launch_reduce_slabs_adam(const float* slab, int nslab, int64_t count, float* grad,
                                    const AdamStep& a, hipStream_t s);

}  // namespace cg
