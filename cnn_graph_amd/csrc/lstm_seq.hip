// gconv-LSTM layer on gfx950: the T-step forward in ONE persistent launch and
// the backprop-through-time step in ONE launch per step
// (lib/gconv_lstm.py:609-627 glstm_layer -> static_rnn over GConvLSTMCell,
// :77-221), H = 32 hidden units, M <= 1024 vertices.
//
// Per time step the cell computes (the x-conv either fused in -- feat_in <= 8:
// the recurrence of x_t in the same LDS slots, Wx on the same MFMAs -- or
// precomputed for all steps at once by the time-batched chebyshev5 call, gx):
//   T_0 = h, T_1 = L~ h, T_k = 2 L~ T_{k-1} - T_{k-2}       (cheby_conv, :183-207)
//   a = (gx + sum_k T_k Wh_k) + b
//   z = tan(a_z), i = sigmoid(a_i), f = sigmoid(a_f), o = tanh(a_o)   (reference)
//   c' = f c + i z ;  h' = o tanh(c')                              (:215, :218)
//
// k_lstm_seq (forward, all T steps, one cooperative launch)
//   Two 512-thread workgroups per sample (8 waves, 256 registers per lane): workgroup u owns hidden units
//   [16u, 16u + 16) (64 of the 128 gate columns); blocks b and b + 8 share an
//   XCD under round-robin placement, so a pair's hand-off stays in one L2
//   (speed only -- the hand-off protocol is agent-scope and placement-free).
//   Each workgroup runs the whole Chebyshev recurrence of h (one 8-channel
//   quarter at a time, two [M][8] LDS slots, CSR of L~ staged once in LDS,
//   each wave's gathers unrolled to its longest row: lds_spmm.h)
//   and the gate contraction on v_mfma_f32_32x32x2_f32 TRANSPOSED
//   (gates x rows = Wh^T T^T): the B operand is the lane's own T_k values
//   straight from the SpMM (no LDS read), and the accumulator leaves each
//   lane ALL FOUR gates of 4 units of one row, so the LSTM update is in-lane
//   (no shuffles); c_{t-1} is read back by the lane that stored it.
//   Hand-off per step: every lane stores its h' (the output hs[t]) with sc1
//   (write-through) stores, each wave drains (s_waitcnt vmcnt(0)), the
//   workgroup barrier, then ONE lane stores the step counter sc1 into the
//   pair's flag; the partner polls it (sc1 loads, s_sleep, bounded by a
//   wall-clock timeout: a workgroup that times out writes NaN into every hs /
//   cs / act entry it still owed -- its units of this and every later step and
//   sample -- sets the plan's sticky fault word and ends), joins a
//   barrier, and reads the other half of h with sc1 loads
//   (MI355X_MICROARCH.md §inter-workgroup visibility, table row 1).  A
//   workgroup does its OWN two quarters first, so the partner's half has
//   half a step to arrive.  All workgroups are co-resident (at most one
//   pair per two CUs); more samples than pairs are
//   processed by the same pairs in turn.  The grid never exceeds the
//   occupancy query's resident workgroups (checked at launch).
//
// k_xbasis (the x basis of every step, one launch before k_lstm_seq<true>)
//   One 1024-thread workgroup per CU runs the whole K-order recurrence of a
//   few samples' x in LDS, each thread's CSR row in registers; planes bitwise
//   the streaming k_cheb_step launches' (CG_OPT_SEQ_XPRE = 2 keeps those).
//
// k_lstm_bstep (backward, one launch per step, two workgroups per sample)
//   dpre = TF autodiff of the pointwise update (the expressions of
//   lstm.hip::k_lstm_bwd, so dpre is bitwise the unfused kernel's), then
//   D_k = dpre Wh_k^T on v_mfma_f32_16x16x4_f32 (again transposed: each lane
//   computes dpre for 8 units x 4 gates of one row and feeds it as the B
//   operand), then the reverse (Clenshaw) recurrence over the explicit L~^T
//   G_{K-1} = D_{K-1}, G_k = (D_k + c L~^T G_{k+1}) - G_{k+2} (c = 2, 1 at
//   k = 0) with G in one [M][16] LDS slot and L~^T staged in LDS; workgroup u owns h channels
//   [16u, 16u + 16) of dh_prev = G_0 and stores the dpre / dc_prev of its
//   units.  The h-weight gradient is summed afterwards per Chebyshev order
//   over all steps from the forward's planes (one GEMM per order).
#include "cg_internal.h"
#include "split_bf16.h"
#include "lds_spmm.h"
#include "lstm_gates.h"

namespace cg {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kST = 512;   // threads per workgroup: 8 waves, 2 per SIMD (256 VGPRs)
constexpr int kH = 32;     // hidden units
constexpr int kQ = 8;      // channels per forward SpMM pass (a quarter of H)
constexpr int kBS = 16;    // channels per backward workgroup (half of H)
constexpr int kRT = 4;     // forward: 32-row tiles per wave (8 waves x 4 x 32 = 1024 rows)
constexpr int kRB = 8;     // backward: 16-row tiles per wave (8 x 8 x 16 = 1024 rows)
constexpr int kSeqStaticLds = 64;  // k_lstm_seq's static __shared__ bytes (upper bound)

__device__ __forceinline__ float sigm(float a) { return gate_sigmoid(a); }

// agent-scope relaxed accesses: global_load/store ... sc1 (L1 bypass)
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __uint_as_float(__hip_atomic_load(reinterpret_cast<unsigned*>(const_cast<float*>(p)),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// 16 bytes as two 8-byte agent-scope accesses (global_load/store_dwordx2 sc1)
__device__ __forceinline__ float4 ld16_sc1(const float* p) {
  unsigned long long* q = reinterpret_cast<unsigned long long*>(const_cast<float*>(p));
  const unsigned long long a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return make_float4(__uint_as_float(unsigned(a)), __uint_as_float(unsigned(a >> 32)),
                     __uint_as_float(unsigned(b)), __uint_as_float(unsigned(b >> 32)));
}
__device__ __forceinline__ void st16_sc1(float* p, float4 v) {
  unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
  __hip_atomic_store(q, (unsigned long long)(__float_as_uint(v.x)) | ((unsigned long long)(__float_as_uint(v.y)) << 32),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(q + 1, (unsigned long long)(__float_as_uint(v.z)) | ((unsigned long long)(__float_as_uint(v.w)) << 32),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// 16-byte agent-scope accesses as buffer_load/store_dwordx4 ... sc1 (aux 16)
// through a descriptor over one [M][32] slab; the 8-byte forms above move
// 0.54-0.70x the bytes per instruction (MI355X_MICROARCH.md fence table)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slab_rsrc(const float* p, int M) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0, M * kH * 4, 0x00020000);
}
__device__ __forceinline__ float4 bld16_sc1(__amdgpu_buffer_rsrc_t r, int off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off * 4, 0, 16);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                     __uint_as_float(v.w));
}
__device__ __forceinline__ float4 bld16(__amdgpu_buffer_rsrc_t r, int off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off * 4, 0, 0);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                     __uint_as_float(v.w));
}
__device__ __forceinline__ void bst16(__amdgpu_buffer_rsrc_t r, int off, float4 v) {
  u32x4 w;
  w.x = __float_as_uint(v.x);
  w.y = __float_as_uint(v.y);
  w.z = __float_as_uint(v.z);
  w.w = __float_as_uint(v.w);
  __builtin_amdgcn_raw_buffer_store_b128(w, r, off * 4, 0, 0);
}
__device__ __forceinline__ void bst16_sc1(__amdgpu_buffer_rsrc_t r, int off, float4 v) {
  u32x4 w;
  w.x = __float_as_uint(v.x);
  w.y = __float_as_uint(v.y);
  w.z = __float_as_uint(v.z);
  w.w = __float_as_uint(v.w);
  __builtin_amdgcn_raw_buffer_store_b128(w, r, off * 4, 0, 16);
}

static int seq_xpre() { return option(kOptSeqXpre); }

struct SeqArgs {
  const int* rowptr;  // L~ (CSR, sorted columns)
  const int* col;
  const float* val;
  const int* order;   // rows by decreasing length (lane -> row)
  int M, Mr, K, N, T, gates, nnz, P, pair_xcd;
  const float* gx;    // [T][N][M][128] x-conv gate pre-activations (when xs == NULL)
  const float* xs;    // [T][N][M][Fin] inputs, Fin <= 8: the x-conv fused in (gx unused)
  const float* Wx;    // [K*Fin][128], row fin*K + k (with xs)
  float* xplanes;     // T_k of x_t, k = 0..K-1 at k*xpstride + [T][N][M][Fin] (with xs)
  int64_t xpstride;
  int Fin;
  const float* Wh;    // [K*32][128], row c*K + k
  const float* bias;  // [128] or NULL
  const float* h0;    // [N][M][32] or NULL (zero state: step 0 has no h-conv)
  const float* c0;    // [N][M][32] or NULL
  float* hs;          // [T][N][M][32]
  float* cs;          // [T][N][M][32]
  float* act;         // [T][N][M][32][4] gate activations z|i|f|o per unit (unit-major), or NULL
  float* planes;      // T_k of h_{t-1} at (k-1)*pstride + [T][N][M][32], or NULL
  int64_t pstride;
  int* flags;         // [P][2] step counters (zeroed before the launch)
  int* status;        // the plan's sticky fault word (host-mapped): set to 1 when a hand-off
                      // times out, never cleared by a launch
  unsigned long long timeout;  // wall-clock ticks
  int dbg;            // ablation build only (CG_DBG): 1 no MFMA, 2 no SpMM, 4 no gate math,
                      // 8 no partner wait, 16 no gx / c loads, 32 no plane stores,
                      // 64 no act stores, 128 no c stores, 256 no h stores
  unsigned long long* ts;  // ablation build: phase stamps of step 1 (CG_TS), else NULL
  int xpre;           // 1: xplanes already hold T_k(x_t) for every step (launch_lstm_seq's
                      // pre-pass): the x contraction reads them, no x recurrence in the loop
  int inject_t;       // fault injection (cg_plan_set_seq_fault_test, tests only): >= 0 makes workgroup
                      // 0 of pair 0 stop publishing its step counter from that step on
};

// A timed-out workgroup's outputs: NaN in every hs / cs / act entry of its
// units [16u, 16u + 16) from step t0 of sample n0 on, and every step of the
// pair's later samples, so nothing downstream can consume unwritten memory
__device__ void lstm_seq_poison(const SeqArgs& A, int n0, int t0, int u) {
  const float qnan = __builtin_nanf("");
  const int M = A.M;
  for (int n = n0; n < A.N; n += A.P)
    for (int t = (n == n0 ? t0 : 0); t < A.T; ++t) {
      const int64_t rb = (int64_t(t) * A.N + n) * M;
      for (int e = threadIdx.x; e < M * 16; e += kST) {
        const int64_t o = (rb + (e >> 4)) * kH + 16 * u + (e & 15);
        A.hs[o] = qnan;
        A.cs[o] = qnan;
      }
      if (A.act)
        for (int e = threadIdx.x; e < M * 64; e += kST) A.act[(rb + (e >> 6)) * 128 + 64 * u + (e & 63)] = qnan;
    }
}

// REF: the reference gate set (z = tan, o = tanh), a template parameter so the
// epilogue carries one gate set, not both behind selects
template <bool XPRE, bool REF>
__global__ __launch_bounds__(kST) void k_lstm_seq(SeqArgs A) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ int s_abort;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = lane & 31, hh = lane >> 5;
  const int M = A.M, K = A.K, N = A.N, T = A.T;
  int pair, u;
  if (A.pair_xcd) {
    const int b = blockIdx.x;
    pair = (b >> 4) * 8 + (b & 7);
    u = (b >> 3) & 1;
  } else {
    pair = blockIdx.x >> 1;
    u = blockIdx.x & 1;
  }
  float* slot0 = smem;
  float* slot1 = smem + A.Mr * kQ;
  float* s_W = slot1 + A.Mr * kQ;  // [K][q 4][s 4][hh 2][ct 2][i 32]
  float* s_Wx = s_W + K * 2048;  // [K][s 4][hh 2][ct 2][i 32] x-conv A operands (xs != NULL)
  float* s_b = s_Wx + (A.xs ? K * 512 : 0);  // [128] bias (zeros when NULL)
  float* s_val = s_b + 128;
  unsigned short* s_col = reinterpret_cast<unsigned short*>(s_val + A.nnz);
  // the lanes' rows, [rt][tid]: the epilogue reads its store offsets from here
  // (an LDS read waits for no store; a spilled offset's scratch reload waits
  // for every store before it -- the write-through h store above all)
  int* s_rowt = reinterpret_cast<int*>(reinterpret_cast<char*>(s_col) +
                                       align16(size_t(A.nnz) * 2 + kSpmmSlack));
  // A operands of the transposed contraction: lane (i, hh) of MFMA step s in
  // quarter q, order k holds Wh[(8q + 4hh + s) K + k][gate column of tile
  // row i] -- tile ct's rows i = 8 g + m are gate g, unit 16u + 8ct + m
  stage_lds<8, kST>(K * 2048, [&](int e) {
    const int i = e & 31, ct = (e >> 5) & 1, h2 = (e >> 6) & 1, s = (e >> 7) & 3;
    const int q = (e >> 9) & 3, k = e >> 11;
    const int ch = 8 * q + 4 * h2 + s;
    const int gcol = (i >> 3) * 32 + 16 * u + 8 * ct + (i & 7);
    return A.Wh[int64_t(ch * K + k) * 128 + gcol];
  }, [&](int e, float v) { s_W[e] = v; });
  if (A.xs) {
    // x channel c = 2s + hh of MFMA step s (zero past Fin): Fin <= 2 needs
    // one step per order, not four
    stage_lds<8, kST>(K * 512, [&](int e) {
      const int i = e & 31, ct = (e >> 5) & 1, h2 = (e >> 6) & 1, s = (e >> 7) & 3, k = e >> 9;
      const int c = 2 * s + h2;
      const int gcol = (i >> 3) * 32 + 16 * u + 8 * ct + (i & 7);
      return c < A.Fin ? A.Wx[int64_t(c * K + k) * 128 + gcol] : 0.f;
    }, [&](int e, float v) { s_Wx[e] = v; });
  }
  for (int e = tid; e < 128; e += kST) s_b[e] = A.bias ? A.bias[e] : 0.f;
  stage_csr_lds<8, kST>(A.nnz, A.val, A.col, s_val, s_col);
  if (tid == 0) s_abort = 0;
  if (tid < 2 * kQ) (tid < kQ ? slot0 : slot1)[M * kQ + (tid & (kQ - 1))] = 0.f;  // zero row M
  // lane (tile rt, j) owns row order[(wave + 8 rt) * 32 + j]: rows dealt by
  // decreasing length, so a tile's rows have nearly equal lengths
  // the SpMM lanes take the same 32 rows of a tile as (row lane / 2, half
  // lane % 2): an 8-lane LDS access group gathers 4 whole 32-byte records
  const int js = lane >> 1, hs2 = lane & 1;
  int row[kRT], rowS[kRT], rb[kRT], re[kRT], wl[kRT];
  bool rv[kRT], rvS[kRT];
#pragma unroll
  for (int rt = 0; rt < kRT; ++rt) {
    const int idx = (wave + 8 * rt) * 32 + j;
    rv[rt] = idx < M;
    row[rt] = rv[rt] ? A.order[idx] : M;
    const int idxS = (wave + 8 * rt) * 32 + js;
    rvS[rt] = idxS < M;
    rowS[rt] = rvS[rt] ? A.order[idxS] : M;
    rb[rt] = rvS[rt] ? A.rowptr[rowS[rt]] : 0;
    re[rt] = rvS[rt] ? A.rowptr[rowS[rt] + 1] : 0;
    wl[rt] = wave_max(re[rt] - rb[rt]);  // the tile's longest row: its unrolled gather count
    s_rowt[rt * kST + tid] = row[rt];
  }
  __syncthreads();

  int* my_flag = A.flags + 2 * pair + u;
  const int* partner_flag = A.flags + 2 * pair + (1 - u);
  for (int n = pair, it = 0; n < N; n += A.P, ++it) {
    const int base = it * T;
    for (int t = 0; t < T; ++t) {
      const bool stamp = (t == 1 && it == 0);
      if (stamp) CG_TS(A.ts, 0);
      f32x16 acc[kRT][2];
#pragma unroll
      for (int rt = 0; rt < kRT; ++rt)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[rt][ct][e] = 0.f;
      const bool has_h = t > 0 || A.h0;
      const float* hsrc = (t == 0) ? A.h0 + int64_t(n) * M * kH
                                   : A.hs + (int64_t(t - 1) * N + n) * M * kH;
      float* pl_t = A.planes + (int64_t(t) * N + n) * M * kH;  // plane k at + (k-1)*pstride
      const __amdgpu_buffer_rsrc_t r_hsrc = slab_rsrc(hsrc, M);
      const __amdgpu_buffer_rsrc_t r_hout = slab_rsrc(A.hs + (int64_t(t) * N + n) * M * kH, M);
      // gates^T += Wh_k^T T_k^T over quarter q's 8 channels; B operand: the
      // lane's own rows of T_k (tk, channels 8q + 4hh .. +3)
      auto contract = [&](int q, int k, const float4* tk) {
        const float* wq = s_W + (k * 4 + q) * 512 + hh * 64 + j;
#pragma unroll
        for (int s = 0; s < 4 && !CG_DBG(A.dbg, 1); ++s) {
          const float a0 = wq[s * 128], a1 = wq[s * 128 + 32];
#pragma unroll
          for (int rt = 0; rt < kRT; ++rt) {
            const float b = (&tk[rt].x)[s];
            acc[rt][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b, acc[rt][0], 0, 0, 0);
            acc[rt][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b, acc[rt][1], 0, 0, 0);
          }
        }
      };
      // the x quarter's contraction: MFMA step s takes channel 2s + hh of the
      // lane's rows straight from the LDS slot, steps past Fin skipped
      auto contract_x = [&](int k, const float* cur) {
        const float* wq = s_Wx + k * 512 + hh * 64 + j;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          if (2 * s >= A.Fin || CG_DBG(A.dbg, 1)) break;
          const float a0 = wq[s * 128], a1 = wq[s * 128 + 32];
#pragma unroll
          for (int rt = 0; rt < kRT; ++rt) {
            const float b = cur[row[rt] * kQ + 2 * s + hh];
            acc[rt][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b, acc[rt][0], 0, 0, 0);
            acc[rt][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b, acc[rt][1], 0, 0, 0);
          }
        }
      };
      // XPRE with feat_in <= 2: the x contraction runs behind the partner's
      // quarters, its loads issued after the publish drain (issued here they
      // would wait, one by one, for the previous epilogue's stores)
      const bool x_late = XPRE && A.Fin <= 2 && K <= 4;
      if (XPRE && x_late) {
        // contracted behind the partner's quarters (below)
      } else if (XPRE) {
        // the x basis of step t, precomputed for all steps: MFMA step s takes
        // channel 2s + hh of the lane's rows straight from plane k (L2)
        const int Fin = A.Fin;
        for (int k = 0; k < K; ++k) {
          const float* xp = A.xplanes + int64_t(k) * A.xpstride + (int64_t(t) * N + n) * M * Fin;
          // buffer loads: a padding row or a channel past Fin reads past the
          // plane's range, which returns 0 -- no branch (a conditional load
          // compiles to one with a vmcnt(0) wait behind every load)
          const __amdgpu_buffer_rsrc_t rx =
              __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xp), 0, M * Fin * 4, 0x00020000);
          const float* wq = s_Wx + k * 512 + hh * 64 + j;
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            if (2 * s >= Fin || CG_DBG(A.dbg, 1)) break;
            const int c = 2 * s + hh;
            float b[kRT];
#pragma unroll
            for (int rt = 0; rt < kRT; ++rt) {
              const int xo = (rv[rt] && c < Fin) ? (row[rt] * Fin + c) * 4 : M * Fin * 4;
              b[rt] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rx, xo, 0, 0));
            }
            const float a0 = wq[s * 128], a1 = wq[s * 128 + 32];
#pragma unroll
            for (int rt = 0; rt < kRT; ++rt) {
              acc[rt][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b[rt], acc[rt][0], 0, 0, 0);
              acc[rt][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b[rt], acc[rt][1], 0, 0, 0);
            }
          }
        }
      } else if (A.xs) {
        // the fused x-conv: the recurrence of x_t (Fin <= 8 channels in one
        // 8-channel slot, the rest zero) and its contraction with Wx; both
        // workgroups run it, workgroup 0 keeps the x basis planes
        const int Fin = A.Fin;
        const float* xt = A.xs + (int64_t(t) * N + n) * M * Fin;
        float* xp = A.xplanes + (int64_t(t) * N + n) * M * Fin;
#pragma unroll
        for (int rt = 0; rt < kRT; ++rt) {
          if (!rvS[rt]) continue;
          float v[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const int ch = 4 * hs2 + c;
            v[c] = ch < Fin ? xt[int64_t(rowS[rt]) * Fin + ch] : 0.f;
            if (ch < Fin && u == 0) xp[int64_t(rowS[rt]) * Fin + ch] = v[c];
          }
          *reinterpret_cast<float4*>(slot0 + rowS[rt] * kQ + 4 * hs2) = make_float4(v[0], v[1], v[2], v[3]);
        }
        __syncthreads();
        for (int k = 0; k < K; ++k) {
          const float* cur = (k & 1) ? slot1 : slot0;
          contract_x(k, cur);
          if (k + 1 < K) {
            float* nxt = (k & 1) ? slot0 : slot1;
#pragma unroll
            for (int rt = 0; rt < kRT; ++rt) {
              if (!rvS[rt]) continue;
              if (4 * hs2 >= Fin) {  // channels past Fin stay zero
                *reinterpret_cast<float4*>(nxt + rowS[rt] * kQ + 4 * hs2) = make_float4(0.f, 0.f, 0.f, 0.f);
                continue;
              }
              float4 sm;
              with_row_len(wl[rt], [&](auto lc) {
                sm = lds_row_spmm_w<decltype(lc)::value>(cur, kQ, 4 * hs2, s_col, s_val, rb[rt], re[rt], M);
              });
              float4* own = reinterpret_cast<float4*>(nxt + rowS[rt] * kQ + 4 * hs2);
              if (k >= 1) {
                const float4 p = *own;
                sm = make_float4(2.f * sm.x - p.x, 2.f * sm.y - p.y, 2.f * sm.z - p.z, 2.f * sm.w - p.w);
              }
              *own = sm;
              if (u == 0) {
                float* dst = xp + int64_t(k + 1) * A.xpstride + int64_t(rowS[rt]) * Fin;
                const float sv[4] = {sm.x, sm.y, sm.z, sm.w};
#pragma unroll
                for (int c = 0; c < 4; ++c)
                  if (4 * hs2 + c < Fin) dst[4 * hs2 + c] = sv[c];
              }
            }
            __syncthreads();
          }
        }
      }
      if (has_h) {
        // the two OWN quarters (units 16u .. 16u+15): the recurrence in LDS,
        // T_1 .. T_{K-1} leave as basis planes (write-through: the partner reads them)
        for (int qq = 0; qq < 2; ++qq) {
          const int q = 2 * u + qq;
          // all tiles' loads in flight together; a padding lane (row M) reads
          // past the slab (the descriptor's range check returns 0) and
          // rewrites the zero row with 0
          // quarter 2u at t > 0: h_{t-1} is already in slot 0 (the previous
          // epilogue wrote it there: no global load behind its stores)
          if (!(qq == 0 && t > 0 && (XPRE || !A.xs))) {  // (the fused x recurrence reuses slot 0)
            float4 v[kRT];
#pragma unroll
            for (int rt = 0; rt < kRT; ++rt) {
              const int off = row[rt] * kH + 8 * q + 4 * hh;
              v[rt] = (t > 0) ? bld16_sc1(r_hsrc, off) : bld16(r_hsrc, off);
            }
#pragma unroll
            for (int rt = 0; rt < kRT; ++rt)
              *reinterpret_cast<float4*>(slot0 + row[rt] * kQ + 4 * hh) = v[rt];
          }
          __syncthreads();
          for (int k = 0; k < K; ++k) {
            const float* cur = (k & 1) ? slot1 : slot0;
            float4 tk[kRT];
#pragma unroll
            for (int rt = 0; rt < kRT; ++rt)
              tk[rt] = *reinterpret_cast<const float4*>(cur + row[rt] * kQ + 4 * hh);
            contract(q, k, tk);
            if (k + 1 < K) {
              // T_{k+1} of this lane's rows / channels: CSR order from +0
              float* nxt = (k & 1) ? slot0 : slot1;
#pragma unroll
              for (int rt = 0; rt < kRT; ++rt) {
                if (!rvS[rt] || CG_DBG(A.dbg, 2)) continue;
                // one row per length switch here: the paired form (as in the
                // BPTT step) measured 1-1.5 % slower on config E (profiles/r04_final2)
                float4 sm;
                with_row_len(wl[rt], [&](auto lc) {
                  sm = lds_row_spmm_w<decltype(lc)::value>(cur, kQ, 4 * hs2, s_col, s_val, rb[rt], re[rt], M);
                });

                float s0 = sm.x, s1 = sm.y, s2 = sm.z, s3 = sm.w;
                float4* own = reinterpret_cast<float4*>(nxt + rowS[rt] * kQ + 4 * hs2);
                if (k >= 1) {  // T_{k-1} of this row: the slot being overwritten
                  const float4 p = *own;
                  s0 = 2.f * s0 - p.x;
                  s1 = 2.f * s1 - p.y;
                  s2 = 2.f * s2 - p.z;
                  s3 = 2.f * s3 - p.w;
                }
                const float4 o = make_float4(s0, s1, s2, s3);
                *own = o;
                if (!CG_DBG(A.dbg, 32))
                  bst16_sc1(slab_rsrc(pl_t + int64_t(k) * A.pstride, M), rowS[rt] * kH + 8 * q + 4 * hs2, o);
              }
              __syncthreads();
            }
          }
        }
      }
      if (stamp) CG_TS(A.ts, 1);
      // publish: h_{t-1} of this workgroup's units (stored by the previous
      // step's epilogue, drained here -- its stores overlapped the own
      // quarters above) and the own quarters' planes of step t
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0 && !(A.inject_t >= 0 && pair == 0 && u == 0 && base + t >= A.inject_t))
        __hip_atomic_store(my_flag, base + t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (has_h) {
        if (!CG_DBG(A.dbg, 8)) {
          // the partner's quarters of step t: wait for its counter
          if (tid == 0) {
            const int need = base + t + 1;
            const unsigned long long t0 = wall_clock64();
            while (__hip_atomic_load(const_cast<int*>(partner_flag), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT) < need) {
              __builtin_amdgcn_s_sleep(1);
              if (wall_clock64() - t0 > A.timeout) {
                s_abort = 1;
                __hip_atomic_store(A.status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
              }
            }
          }
          __syncthreads();
          if (s_abort) {  // every thread of the workgroup: poison what it owed, end
            lstm_seq_poison(A, n, t, u);
            return;
          }
        }
        if (stamp) CG_TS(A.ts, 2);
        // the partner's two quarters: T_0 = its half of h_{t-1}, T_k its planes
        // (sc1 loads, no recurrence here: it computed them)
        // items it = (qq, k), qq-major; item it + 1's loads are in flight
        // during item it's MFMAs (two register sets, alternating)
        // the row offsets recomputed here from an opaque copy of row[]: offsets
        // precomputed outside the time loop would be spilled, and each reload
        // (a vector-memory load, in order with the loads before it) would
        // serialise these loads one L2 round trip at a time
        int prow[kRT];
#pragma unroll
        for (int rt = 0; rt < kRT; ++rt) {
          prow[rt] = row[rt] * kH + 4 * hh;
          asm volatile("" : "+v"(prow[rt]));
        }
        auto ldq = [&](int it, float4 (&tk)[kRT]) {
          const int q = 2 * (1 - u) + it / K, k = it % K;
          const float* src = (k == 0) ? hsrc : pl_t + int64_t(k - 1) * A.pstride;
          const __amdgpu_buffer_rsrc_t r_src = slab_rsrc(src, M);
#pragma unroll
          for (int rt = 0; rt < kRT; ++rt) {  // row M: past the slab, reads 0
            const int off = prow[rt] + 8 * q;
            tk[rt] = bld16_sc1(r_src, off);  // (h0 too: one form, no branch per load)
          }
        };
        const int nit = 2 * K;
        float4 tka[kRT], tkb[kRT];
        ldq(0, tka);
        for (int it = 0; it < nit; it += 2) {
          ldq(it + 1, tkb);  // nit is even
          contract(2 * (1 - u) + it / K, it % K, tka);
          if (it + 2 < nit) ldq(it + 2, tka);
          contract(2 * (1 - u) + (it + 1) / K, (it + 1) % K, tkb);
        }
      }
      if (x_late) {
        // the x basis of step t (channel hh of the lane's rows; a padding row or
        // a channel past Fin reads past the plane's range: 0), all orders' loads
        // together
        const int Fin = A.Fin;
        float xb[4][kRT];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (k >= K) break;
          const float* xp = A.xplanes + int64_t(k) * A.xpstride + (int64_t(t) * N + n) * M * Fin;
          const __amdgpu_buffer_rsrc_t rx =
              __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xp), 0, M * Fin * 4, 0x00020000);
#pragma unroll
          for (int rt = 0; rt < kRT; ++rt) {
            const int xo = (rv[rt] && hh < Fin) ? (row[rt] * Fin + hh) * 4 : M * Fin * 4;
            xb[k][rt] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rx, xo, 0, 0));
          }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (k >= K || CG_DBG(A.dbg, 1)) break;
          const float* wq = s_Wx + k * 512 + hh * 64 + j;
          const float a0 = wq[0], a1 = wq[32];
#pragma unroll
          for (int rt = 0; rt < kRT; ++rt) {
            acc[rt][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, xb[k][rt], acc[rt][0], 0, 0, 0);
            acc[rt][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, xb[k][rt], acc[rt][1], 0, 0, 0);
          }
        }
      }
      if (stamp) CG_TS(A.ts, 3);
      // c_{t-1} of every tile, loaded together before the first store of the
      // epilogue (a load behind stores waits for them: vmcnt counts both):
      // this lane's own store of the previous step (same address, same lane)
      // or the initial state; buffer loads, a padding row (M) reads 0
      float4 cva[kRT][2];
      {
        const float* csrc = t > 0 ? A.cs + (int64_t(t - 1) * N + n) * M * kH
                                  : (A.c0 ? A.c0 + int64_t(n) * M * kH : A.cs);
        const __amdgpu_buffer_rsrc_t r_c = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(csrc), 0, (t > 0 || A.c0) && !CG_DBG(A.dbg, 16) ? M * kH * 4 : 0,
            0x00020000);
#pragma unroll
        for (int rt = 0; rt < kRT; ++rt)
#pragma unroll
          for (int ct = 0; ct < 2; ++ct)
            cva[rt][ct] = bld16(r_c, row[rt] * kH + 16 * u + 8 * ct + 4 * hh);
      }
      // gate update: lane (row, hh) of tile (rt, ct) holds gates g = 0..3 of
      // units 16u + 8ct + 4hh + m in acc[rt][ct][4g + m]
      // (c and act leave through buffer stores over the step's slabs: 32-bit
      // offsets from the row instead of a 64-bit address per tile)
      const int64_t slab0 = (int64_t(t) * N + n) * M;
      const __amdgpu_buffer_rsrc_t r_cout = slab_rsrc(A.cs + slab0 * kH, M);
      const __amdgpu_buffer_rsrc_t r_act = __builtin_amdgcn_make_buffer_rsrc(
          A.act ? A.act + slab0 * 128 : A.cs, 0, A.act && !CG_DBG(A.dbg, 64) ? M * 512 : 0, 0x00020000);
#pragma unroll
      for (int rt = 0; rt < kRT; ++rt) {
        if (!rv[rt]) continue;
        int erow = s_rowt[rt * kST + tid];  // == row[rt]
        asm volatile("" : "+v"(erow));
        const int64_t rr = slab0 + erow;
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          // one tile's gate math at a time (interleaving tiles costs registers
          // the kernel does not have: spills, whose reloads wait for the stores)
          __builtin_amdgcn_sched_barrier(0);
          int lq = threadIdx.x;  // 4hh re-derived per tile (a hoisted copy would spill)
          asm volatile("" : "+v"(lq));
          const int u0 = 16 * u + 8 * ct + ((lq >> 3) & 4);
          float4 gv[4];
#pragma unroll
          for (int g = 0; g < 4; ++g)
            gv[g] = (XPRE || CG_DBG(A.dbg, 16) || A.xs) ? make_float4(0.f, 0.f, 0.f, 0.f)
                                                : *reinterpret_cast<const float4*>(A.gx + rr * 128 + g * 32 + u0);
          const float4 cv = cva[rt][ct];
          float c[4] = {cv.x, cv.y, cv.z, cv.w};
          float hn[4], zz[4], ii[4], ff[4], oo[4];
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            const float gz = (&gv[0].x)[m], gi = (&gv[1].x)[m], gf = (&gv[2].x)[m],
                        go = (&gv[3].x)[m];
            float az = gz + acc[rt][ct][m], ai = gi + acc[rt][ct][4 + m];
            float af = gf + acc[rt][ct][8 + m], ao = go + acc[rt][ct][12 + m];
            if (A.bias) {
              az = az + s_b[u0 + m];
              ai = ai + s_b[32 + u0 + m];
              af = af + s_b[64 + u0 + m];
              ao = ao + s_b[96 + u0 + m];
            }
            float z, ig, fg, o, cn;
            if (CG_DBG(A.dbg, 4)) {
              z = az;
              ig = ai;
              fg = af;
              o = ao;
              cn = c[m] + az;
              c[m] = cn;
              hn[m] = ao * cn;
            } else {
              z = REF ? gate_tan(az) : gate_tanh(az);
              ig = sigm(ai);
              fg = sigm(af);
              o = REF ? gate_tanh(ao) : sigm(ao);
              cn = fg * c[m] + ig * z;
              c[m] = cn;
              hn[m] = o * gate_tanh(cn);
            }
            zz[m] = z;
            ii[m] = ig;
            ff[m] = fg;
            oo[m] = o;
          }
          // the tile's store offsets, formed here from the LDS row (laundered:
          // hoisted lane constants would spill, and their reloads wait for stores)
          int ec = erow * kH + u0, ea = erow * 128 + 4 * u0;
          asm volatile("" : "+v"(ec), "+v"(ea));
          if (!CG_DBG(A.dbg, 128)) bst16(r_cout, ec, make_float4(c[0], c[1], c[2], c[3]));
          // h_t of quarter 2u + ct into its slot (channels 4hh .. 4hh+3): quarter
          // 2u is the next step's T_0; both leave write-through after the tiles
          int es = erow * kQ + (ct == 0 ? 0 : A.Mr * kQ) + ((lq >> 3) & 4);  // slot0 / slot1
          asm volatile("" : "+v"(es));
          *reinterpret_cast<float4*>(smem + es) = make_float4(hn[0], hn[1], hn[2], hn[3]);
          // unit-major act: the 4 gates of a unit side by side, the lane's 4
          // units one contiguous 64-byte record (no act: a 0-byte range)
#pragma unroll
          for (int m = 0; m < 4; ++m)
            bst16(r_act, ea + 4 * m, make_float4(zz[m], ii[m], ff[m], oo[m]));
        }
      }
      // h_t of the lane's own slots (its own writes above), write-through: the
      // last vector-memory ops of the step, so no load of this step waits for
      // them (the next publish drains them, a quarter recurrence later)
      if (!CG_DBG(A.dbg, 256)) {
#pragma unroll
        for (int rt = 0; rt < kRT; ++rt) {
          if (!rv[rt]) continue;
          int erow = s_rowt[rt * kST + tid];
          asm volatile("" : "+v"(erow));
#pragma unroll
          for (int ct = 0; ct < 2; ++ct) {
            int lq = threadIdx.x;
            asm volatile("" : "+v"(lq));
            const int h4 = (lq >> 3) & 4;  // 4hh
            const int eh = erow * kH + 16 * u + 8 * ct + h4;
            const int es = erow * kQ + (ct == 0 ? 0 : A.Mr * kQ) + h4;
            bst16_sc1(r_hout, eh, *reinterpret_cast<const float4*>(smem + es));
          }
        }
      }
      if (stamp) CG_TS(A.ts, 4);
    }
  }
}

struct BStepArgs {
  const int* trowptr;  // L~^T (exact transpose, CSR)
  const int* tcol;
  const float* tval;
  const int* order;    // rows of L~^T by decreasing length (lane -> row)
  int M, Mr, N, gates, pair_xcd, nnz, act_um;
  const float* dh;      // [N][M][32] gradient of h' from above, or NULL
  const float* dh_rec;  // [N][M][32] gradient of h' from step t+1's h-conv, or NULL
  const float* dc;      // [N][M][32] gradient of c', or NULL
  const float* act;     // [N][M][128]: [g][32] (gate-major) or [32][g] (unit-major, act_um)
  const float* c_prev;  // [N][M][32] or NULL (zero state)
  const float* c_out;   // [N][M][32]
  const float* Wh;      // [K*32][128]
  float* dpre;          // [N][M][128]
  float* dc_prev;       // [N][M][32] or NULL
  float* dh_prev;       // [N][M][32]
  int dbg;              // ablation build only: 1 no MFMA, 2 no phase-A loads, 4 no recurrence,
                        // 8 no dpre / dc_prev stores
  unsigned long long* ts;  // ablation build: phase stamps (CG_TS), else NULL
};

// X3: D_k = dpre Wh_k^T on v_mfma_f32_16x16x32_bf16 with the exact three-term
// split of split_bf16.h (2.7x the f32 matrix rate, f32-accurate; Wh_k's terms
// staged once in LDS as A fragments [k][gate block 4][term 3][lane 64] x 16 B:
// lane (i, q) holds Wh_k[16u + i][32 kb + 8q + j]); the lane's dpre of gate kb,
// units 8q .. 8q+7, is exactly its B fragment of k-block kb.
template <int K, bool X3>
__global__ __launch_bounds__(kST) void k_lstm_bstep(BStepArgs A) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int jr = lane & 15, q = lane >> 4;
  const int M = A.M;
  CG_TS(A.ts, 0);
  int n, u;
  if (A.pair_xcd) {
    const int b = blockIdx.x;
    n = (b >> 4) * 8 + (b & 7);
    u = (b >> 3) & 1;
  } else {
    n = blockIdx.x >> 1;
    u = blockIdx.x & 1;
  }
  float* slot = smem;                // [Mr][16] G_{k+1} (row M: zeros)
  float* s_W = slot + A.Mr * kBS;   // [K][s 32][q 4][i 16] (X3: fragments, above)
  float* s_val = s_W + K * (X3 ? 3072 : 2048);
  unsigned short* s_col = reinterpret_cast<unsigned short*>(s_val + A.nnz);
  // A operand of MFMA step s, order o: lane (i, q) holds Wh[(16u + i) K + o][g]
  // with g the gate column (s % 4) * 32 + 8q + s / 4 -- the column whose dpre
  // lane (row, q) supplies as the B operand at that step
  // the prologue's loads in two round trips, not one per staging loop (each
  // L2 round trip at launch is ~1-2 us, paid by every one of the T-1 launches):
  // the lanes' rows, Wh and the first kCsr1 * kST CSR entries together, then
  // the row extents, which need the rows
  // lane (tile rt, jr) owns row order[wave * 128 + 16 rt + jr]
  int rows[kRB], rb[kRB], re[kRB], wl[kRB];
#pragma unroll
  for (int rt = 0; rt < kRB; ++rt) {
    const int idx = wave * 128 + rt * 16 + jr;
    rows[rt] = idx < M ? A.order[idx] : M;
  }
  constexpr int kWq = X3 ? 1 : K * 2048 / kST, kCsr1 = 16;
  constexpr int kWf = X3 ? (K * 256 + kST - 1) / kST : 1;  // X3: fragments per thread
  float wv[kWq], cv[kCsr1];
  float4 wf[kWf][2];
  int cc[kCsr1];
  if constexpr (X3) {
#pragma unroll
    for (int qd = 0; qd < kWf; ++qd) {
      const int e = tid + qd * kST;  // fragment (o, kb, lane l)
      const int l = e & 63, kb = (e >> 6) & 3, o = e >> 8;
      const float* src = A.Wh + int64_t((16 * u + (l & 15)) * K + (o < K ? o : 0)) * 128 + kb * 32 + 8 * (l >> 4);
      wf[qd][0] = *reinterpret_cast<const float4*>(src);
      wf[qd][1] = *reinterpret_cast<const float4*>(src + 4);
    }
  } else {
#pragma unroll
    for (int qd = 0; qd < kWq; ++qd) {
      const int e = tid + qd * kST;
      const int i = e & 15, qq = (e >> 4) & 3, s = (e >> 6) & 31, o = e >> 11;
      wv[qd] = A.Wh[int64_t((16 * u + i) * K + o) * 128 + (s & 3) * 32 + 8 * qq + (s >> 2)];
    }
  }
#pragma unroll
  for (int qd = 0; qd < kCsr1; ++qd) {
    const int e = tid + qd * kST;
    cv[qd] = e < A.nnz ? A.tval[e] : 0.f;
    cc[qd] = e < A.nnz ? A.tcol[e] : 0;
  }
#pragma unroll
  for (int rt = 0; rt < kRB; ++rt) {
    rb[rt] = rows[rt] < M ? A.trowptr[rows[rt]] : 0;
    re[rt] = rows[rt] < M ? A.trowptr[rows[rt] + 1] : 0;
  }
  if constexpr (X3) {
    x3::bf16x8* fw = reinterpret_cast<x3::bf16x8*>(s_W);
#pragma unroll
    for (int qd = 0; qd < kWf; ++qd) {
      const int e = tid + qd * kST;
      if (e < K * 256) {
        const float v[8] = {wf[qd][0].x, wf[qd][0].y, wf[qd][0].z, wf[qd][0].w,
                            wf[qd][1].x, wf[qd][1].y, wf[qd][1].z, wf[qd][1].w};
        const x3::Split3 sp = x3::split3(v);
        x3::bf16x8* d = fw + ((e >> 6) * 3) * 64 + (e & 63);  // (o * 4 + kb) * 3 terms
        d[0] = sp.hi;
        d[64] = sp.mid;
        d[128] = sp.lo;
      }
    }
  } else {
#pragma unroll
    for (int qd = 0; qd < kWq; ++qd) s_W[tid + qd * kST] = wv[qd];
  }
#pragma unroll
  for (int qd = 0; qd < kCsr1; ++qd) {
    const int e = tid + qd * kST;
    if (e < A.nnz) {
      s_val[e] = cv[qd];
      s_col[e] = static_cast<unsigned short>(cc[qd]);
    }
  }
  if (A.nnz > kCsr1 * kST) {
    const int rest = A.nnz - kCsr1 * kST;
    stage_csr_lds<8, kST>(rest, A.tval + kCsr1 * kST, A.tcol + kCsr1 * kST, s_val + kCsr1 * kST,
                          s_col + kCsr1 * kST);
  }
  if (tid < kBS) slot[M * kBS + tid] = 0.f;
#pragma unroll
  for (int rt = 0; rt < kRB; ++rt) wl[rt] = wave_max(re[rt] - rb[rt]);
  __syncthreads();
  CG_TS(A.ts, 1);
  f32x4 acc[kRB][K];
#pragma unroll
  for (int rt = 0; rt < kRB; ++rt)
#pragma unroll
    for (int o = 0; o < K; ++o) acc[rt][o] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool ref = A.gates == 0;
  const bool own = (q >> 1) == u;  // this lane's units are stored by this workgroup
  // phase A: dpre of units 8q .. 8q+7 of the lane's rows, and D_o
#pragma unroll
  for (int rt = 0; rt < kRB; ++rt) {
    const int row = rows[rt];
    float dp[4][8];
    if (row < M && !CG_DBG(A.dbg, 2)) {
      const int64_t rr = int64_t(n) * M + row;
      const int64_t hb = rr * kH + 8 * q;
      float av[4][8], cp[8], co[8], dhv[8], dcv[8];
      if (A.act_um) {  // units 8q .. 8q+7: one contiguous 128-byte record
        const float* ap = A.act + rr * 128 + 32 * q;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          const float4 x = *reinterpret_cast<const float4*>(ap + 4 * m);
          av[0][m] = x.x; av[1][m] = x.y; av[2][m] = x.z; av[3][m] = x.w;
        }
      } else {
        const float* ap = A.act + rr * 128 + 8 * q;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 x0 = *reinterpret_cast<const float4*>(ap + g * 32);
          const float4 x1 = *reinterpret_cast<const float4*>(ap + g * 32 + 4);
          av[g][0] = x0.x; av[g][1] = x0.y; av[g][2] = x0.z; av[g][3] = x0.w;
          av[g][4] = x1.x; av[g][5] = x1.y; av[g][6] = x1.z; av[g][7] = x1.w;
        }
      }
      auto ld8 = [&](const float* base, float* out) {
        if (base) {
          const float4 x0 = *reinterpret_cast<const float4*>(base + hb);
          const float4 x1 = *reinterpret_cast<const float4*>(base + hb + 4);
          out[0] = x0.x; out[1] = x0.y; out[2] = x0.z; out[3] = x0.w;
          out[4] = x1.x; out[5] = x1.y; out[6] = x1.z; out[7] = x1.w;
        } else {
#pragma unroll
          for (int m = 0; m < 8; ++m) out[m] = 0.f;
        }
      };
      ld8(A.c_prev, cp);
      ld8(A.c_out, co);
      ld8(A.dh, dhv);
      ld8(A.dc, dcv);
      float dhr[8];
      ld8(A.dh_rec, dhr);
      float dcp[8];
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        // the expressions (and their order) of lstm.hip::k_lstm_bwd
        const float z = av[0][m], i = av[1][m], f = av[2][m], o = av[3][m];
        const float tc = gate_tanh(co[m]);
        float dh = A.dh ? dhv[m] : 0.f;
        if (A.dh_rec) dh = dh + dhr[m];
        float dcn = dh * o * (1.f - tc * tc);
        if (A.dc) dcn = dcn + dcv[m];
        const float d_o = dh * tc;
        const float d_i = dcn * z, d_z = dcn * i, d_f = dcn * cp[m];
        dp[0][m] = ref ? d_z * (1.f + z * z) : d_z * (1.f - z * z);
        dp[1][m] = d_i * (i * (1.f - i));
        dp[2][m] = d_f * (f * (1.f - f));
        dp[3][m] = ref ? d_o * (1.f - o * o) : d_o * (o * (1.f - o));
        dcp[m] = dcn * f;
      }
      if (own && !CG_DBG(A.dbg, 8)) {
        float* dq = A.dpre + rr * 128 + 8 * q;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          *reinterpret_cast<float4*>(dq + g * 32) = make_float4(dp[g][0], dp[g][1], dp[g][2], dp[g][3]);
          *reinterpret_cast<float4*>(dq + g * 32 + 4) =
              make_float4(dp[g][4], dp[g][5], dp[g][6], dp[g][7]);
        }
        if (A.dc_prev) {
          *reinterpret_cast<float4*>(A.dc_prev + hb) = make_float4(dcp[0], dcp[1], dcp[2], dcp[3]);
          *reinterpret_cast<float4*>(A.dc_prev + hb + 4) = make_float4(dcp[4], dcp[5], dcp[6], dcp[7]);
        }
      }
    } else {
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int m = 0; m < 8; ++m) dp[g][m] = 0.f;
    }
    // D_o^T[channel 16u + i][row] += Wh_o[.][g] dpre[row][g]
    if constexpr (X3) {
      const x3::bf16x8* fw = reinterpret_cast<const x3::bf16x8*>(s_W) + lane;
#pragma unroll
      for (int kb = 0; kb < 4 && !CG_DBG(A.dbg, 1); ++kb) {
        const x3::Split3 b = x3::split3(dp[kb]);
#pragma unroll
        for (int o = 0; o < K; ++o) {
          const x3::bf16x8* f = fw + ((o * 4 + kb) * 3) * 64;
          x3::Split3 w;
          w.hi = f[0];
          w.mid = f[64];
          w.lo = f[128];
          acc[rt][o] = x3::mfma16_x3(w, b, acc[rt][o]);
        }
      }
    } else {
#pragma unroll
      for (int o = 0; o < K && !CG_DBG(A.dbg, 1); ++o) {
        const float* wo = s_W + o * 2048 + lane;
#pragma unroll
        for (int s = 0; s < 32; ++s)
          acc[rt][o] = __builtin_amdgcn_mfma_f32_16x16x4f32(wo[s * 64], dp[s & 3][s >> 2], acc[rt][o],
                                                            0, 0, 0);
      }
    }
  }
  CG_TS(A.ts, 2);
  // phase B: lane (row, q) holds D_o[row][16u + 4q + r] in acc[rt][o][r];
  // G_{k+1} of all rows in the LDS slot, G_{k+2} / G_{k+1} of the lane's own
  // rows in registers; one slot: gather, barrier, overwrite, barrier
  float G1[kRB][4], G2[kRB][4];
#pragma unroll
  for (int rt = 0; rt < kRB; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      G1[rt][r] = acc[rt][K - 1][r];
      G2[rt][r] = 0.f;
    }
  auto put = [&]() {
#pragma unroll
    for (int rt = 0; rt < kRB; ++rt)
      if (rows[rt] < M)
        *reinterpret_cast<float4*>(slot + rows[rt] * kBS + 4 * q) =
            make_float4(G1[rt][0], G1[rt][1], G1[rt][2], G1[rt][3]);
  };
  if (K > 1) {
    put();
    __syncthreads();
  }
#pragma unroll
  for (int k = K - 2; k >= 0 && !CG_DBG(A.dbg, 4); --k) {
    const float cc = k >= 1 ? 2.f : 1.f;
    float Gn[kRB][4];
    // tiles in pairs under ONE length switch (a padding row: rb = re = 0, sum 0)
    float4 smp[kRB];
#pragma unroll
    for (int rp = 0; rp < kRB; rp += 2)
      with_row_len(wl[rp] > wl[rp + 1] ? wl[rp] : wl[rp + 1], [&](auto lc) {
        constexpr int LL = decltype(lc)::value;
        smp[rp] = lds_row_spmm_w<LL>(slot, kBS, 4 * q, s_col, s_val, rb[rp], re[rp], M);
        smp[rp + 1] = lds_row_spmm_w<LL>(slot, kBS, 4 * q, s_col, s_val, rb[rp + 1], re[rp + 1], M);
      });
#pragma unroll
    for (int rt = 0; rt < kRB; ++rt) {
      const float4 sm = smp[rt];
      const float sv[4] = {sm.x, sm.y, sm.z, sm.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float gk = acc[rt][k][r] + cc * sv[r];
        if (k + 2 <= K - 1) gk = gk - G2[rt][r];
        Gn[rt][r] = gk;
      }
    }
#pragma unroll
    for (int rt = 0; rt < kRB; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        G2[rt][r] = G1[rt][r];
        G1[rt][r] = Gn[rt][r];
      }
    if (k > 0) {
      __syncthreads();  // every gather of G_{k+1} done
      put();
      __syncthreads();
    }
  }
  CG_TS(A.ts, 3);
#pragma unroll
  for (int rt = 0; rt < kRB; ++rt) {
    if (rows[rt] < M)
      *reinterpret_cast<float4*>(A.dh_prev + (int64_t(n) * M + rows[rt]) * kH + 16 * u + 4 * q) =
          make_float4(G1[rt][0], G1[rt][1], G1[rt][2], G1[rt][3]);
  }
  CG_TS(A.ts, 4);
}

// The x basis of every step up front (k_lstm_seq<true>'s pre-pass): each
// workgroup stages L~ once in LDS and runs the whole K-order recurrence of a
// few samples' x in LDS, writing plane 0 (= x) and planes 1..K-1.  The
// arithmetic of k_cheb_step (CSR order from +0, one rounding per product and
// per add, T_k = 2 acc - T_{k-2}), so the planes are bitwise the streaming
// steps' -- which took one launch per order, gathering 8-byte rows from L2.
constexpr int kXT = 1024;
constexpr int kXL = 16;  // CSR entries of the thread's row kept in registers
constexpr int kXS = 8;   // samples whose x a workgroup loads at once
template <int FIN, int K>
__global__ __launch_bounds__(kXT) void k_xbasis(const int* __restrict__ rowptr,
                                                const int* __restrict__ col,
                                                const float* __restrict__ val, int M, int S,
                                                int spw, const float* __restrict__ xs,
                                                float* xplanes, int64_t xpstride) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x;
  const int MF = M * FIN;
  float* s_T = sm;  // [K][M][FIN]
  // the thread's row (M <= kXT: one row each) and its CSR entries (at most kXL:
  // the host checks) in registers for every sample and order (the CSR in LDS
  // would be read with a row-length stride across the lanes: 8-way bank
  // conflicts)
  const bool live = tid < M;
  const int r = live ? tid : M - 1;  // idle lanes mirror the last row's CSR; their
                                     // global stores fall outside the descriptors'
                                     // range and they write no LDS (their x is the
                                     // out-of-range 0, not row M-1's)
  const int j0 = rowptr[r], j1 = rowptr[r + 1];
  float w[kXL];
  int c[kXL];
#pragma unroll
  for (int q = 0; q < kXL; ++q) {
    w[q] = j0 + q < j1 ? val[j0 + q] : 0.f;
    c[q] = j0 + q < j1 ? col[j0 + q] * FIN : 0;
  }
  const int voff = tid * FIN * 4;  // this lane's bytes in a sample's [M][FIN] slab
  const int s0 = blockIdx.x * spw, s1 = s0 + spw < S ? s0 + spw : S;
  // x of a sample and the planes' slabs through buffer descriptors sized to
  // the slab (an idle lane's access is dropped: no branch, so the compiler
  // counts the loads and stores exactly and the prefetched x waits only for
  // what was issued before it)
  auto slab = [&](const float* p, int smp) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p) + int64_t(smp) * MF, 0, MF * 4,
                                             0x00020000);
  };
  // the x of up to kXS samples loaded together, before any store of theirs:
  // a load consumed after stores waits for them (vmcnt counts both in order)
  for (int cb = s0; cb < s1; cb += kXS) {
    float xr[kXS][FIN];
#pragma unroll
    for (int i = 0; i < kXS; ++i) {
      const __amdgpu_buffer_rsrc_t rx = slab(xs, cb + i < s1 ? cb + i : cb);
#pragma unroll
      for (int f = 0; f < FIN; ++f)
        xr[i][f] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rx, voff + 4 * f, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < kXS; ++i) {
      const int sm_i = cb + i;
      if (sm_i >= s1) break;
      __syncthreads();  // the previous sample's last reads of s_T done
      {
        const __amdgpu_buffer_rsrc_t r0 = slab(xplanes, sm_i);
#pragma unroll
        for (int f = 0; f < FIN; ++f) {
          if (live) s_T[r * FIN + f] = xr[i][f];
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(xr[i][f]), r0, voff + 4 * f, 0, 0);
        }
      }
      __syncthreads();
#pragma unroll
      for (int k = 1; k < K; ++k) {
        const float* Tp = s_T + (k - 1) * MF;
        float acc[FIN];
#pragma unroll
        for (int f = 0; f < FIN; ++f) acc[f] = 0.f;
#pragma unroll
        for (int q = 0; q < kXL; ++q) {
          if (j0 + q < j1) {
#pragma unroll
            for (int f = 0; f < FIN; ++f) acc[f] = acc[f] + w[q] * Tp[c[q] + f];
          }
        }
        const __amdgpu_buffer_rsrc_t rk = slab(xplanes + int64_t(k) * xpstride, sm_i);
        // (T_k is a plane of its own: no barrier between the reads of T_{k-1} and
        // these writes)
#pragma unroll
        for (int f = 0; f < FIN; ++f) {
          const float o = k >= 2 ? 2.f * acc[f] - s_T[(k - 2) * MF + r * FIN + f] : acc[f];
          if (live) s_T[k * MF + r * FIN + f] = o;
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o), rk, voff + 4 * f, 0, 0);
        }
        __syncthreads();
      }
    }
  }
}

inline int round_up(int v, int m) { return (v + m - 1) / m * m; }

}  // namespace

size_t lstm_seq_lds(int M, int K, int64_t nnz, int xfin) {
  return size_t(2) * round_up(M + 1, 32) * kQ * 4 + size_t(K) * 2048 * 4 +
         (xfin > 0 ? size_t(K) * 512 * 4 : 0) + 512 + size_t(nnz) * 4 +
         align16(size_t(nnz) * 2 + kSpmmSlack) + size_t(kRT) * kST * 4;  // + the lanes' row table
}

bool lstm_seq_ok(int M, int H, int K, int64_t nnz, int xfin) {
  return H == kH && M >= 1 && M <= kRT * 8 * 32 && K >= 1 && nnz >= 1 && xfin <= 8 &&
         lstm_seq_lds(M, K, nnz, xfin) <= size_t(kLdsBytes - kSeqStaticLds);
}

size_t lstm_bstep_lds(int M, int K, int64_t nnzT, bool x3) {
  return size_t(round_up(M + 1, 16)) * kBS * 4 + size_t(K) * (x3 ? 3072 : 2048) * 4 +
         size_t(nnzT) * 4 + align16(size_t(nnzT) * 2 + kSpmmSlack);
}

bool lstm_bstep_ok(int M, int H, int K, int64_t nnzT) {
  return H == kH && M >= 1 && M <= kRB * 8 * 16 && K >= 1 && K <= 4 && nnzT >= 1 &&
         lstm_bstep_lds(M, K, nnzT, false) <= size_t(kLdsBytes);
}

int lstm_seq_pairs(int N, int device) {
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
      cus < 2)
    cus = 256;
  const int p = cus / 2;
  return N < p ? N : p;
}

hipError_t launch_lstm_seq(int gates, int T, int N, int M, int K, int64_t nnz, const int* rowptr,
                           const int* col, const float* val, const int* order, const float* xs,
                           const float* Wx, int Fin, float* xplanes, int64_t xpstride, const float* gx, const float* Wh,
                           const float* bias, const float* h0, const float* c0, float* hs,
                           float* cs, float* act, float* planes, int64_t pstride, int* flags,
                           int* status, int P, hipStream_t s, int inject_t, int max_row_nnz) {
  if (!lstm_seq_ok(M, kH, K, nnz, xs ? Fin : 0) || N < 1 || T < 1 || P < 1 || P > N ||
      (xs && (Fin < 1 || Fin > 8 || !Wx || !xplanes)) || (!xs && !gx))
    return hipErrorInvalidValue;
  // the kernel's static LDS (the abort word) counts against the same 160 KB
  // [xpre][reference gates]
  static void (*const kerns[2][2])(SeqArgs) = {{&k_lstm_seq<false, false>, &k_lstm_seq<false, true>},
                                               {&k_lstm_seq<true, false>, &k_lstm_seq<true, true>}};
  static const hipError_t attr = [] {
    for (auto& row : kerns)
      for (auto* k : row) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 kLdsBytes - kSeqStaticLds);
        if (e != hipSuccess) return e;
      }
    return hipSuccess;
  }();
  if (attr != hipSuccess) return attr;
  int dev = 0, rate_khz = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
      rate_khz <= 0)
    rate_khz = 100000;  // 100 MHz
  SeqArgs a{rowptr, col, val, order, M, round_up(M + 1, 32), K, N, T, gates, int(nnz), P,
            P % 8 == 0 ? 1 : 0, gx, xs, Wx, xplanes, xpstride, Fin, Wh, bias, h0, c0, hs, cs, act, planes, pstride, flags, status,
            // a pair hand-off that has not happened after 2 s ends the launch
            static_cast<unsigned long long>(rate_khz) * 2000ull, (debug_flags() >> 16) & 0x1ff,
            nullptr, 0, inject_t};
#ifdef CG_DEBUG
  a.ts = g_debug_ts;
#endif
  hipError_t e = hipMemsetAsync(flags, 0, sizeof(int) * size_t(2) * P, s);
  if (e != hipSuccess) return e;
  // x basis of all T steps up front (plane 0 = x, plane k = T_k(x) by the
  // streaming steps over the T*N samples: CSR order from +0, the same values
  // as the in-loop recurrence), unless CG_OPT_SEQ_XPRE = 0 (A/B runs): the loop
  // then only contracts them, and neither workgroup of a pair recomputes them
  const size_t xb_lds = size_t(K) * M * Fin * 4;
  if (xs && seq_xpre() == 1 && Fin <= 2 && K >= 2 && K <= 4 && M <= kXT && max_row_nnz <= kXL &&
      xb_lds <= size_t(kLdsBytes)) {
    // one launch: each workgroup the whole recurrence of a few samples in LDS
    // [Fin - 1][K - 2]
    static void (*const xk[2][3])(const int*, const int*, const float*, int, int, int, const float*,
                                  float*, int64_t) = {{&k_xbasis<1, 2>, &k_xbasis<1, 3>, &k_xbasis<1, 4>},
                                                      {&k_xbasis<2, 2>, &k_xbasis<2, 3>, &k_xbasis<2, 4>}};
    static const hipError_t xat = [] {
      for (auto& row : xk)
        for (auto* k : row) {
          const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
          if (e != hipSuccess) return e;
        }
      return hipSuccess;
    }();
    if (xat != hipSuccess) return xat;
    auto* xkern = xk[Fin - 1][K - 2];
    const int S = T * N;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
    int per_cu = 1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(xkern),
                                                     kXT, xb_lds) != hipSuccess || per_cu < 1)
      per_cu = 1;
    const int spw = (S + per_cu * cus - 1) / (per_cu * cus);  // every workgroup resident
    hipLaunchKernelGGL(xkern, dim3((S + spw - 1) / spw), dim3(kXT), xb_lds, s, rowptr, col, val, M,
                       S, spw, xs, xplanes, xpstride);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    a.xpre = 1;
  } else if (xs && seq_xpre()) {
    const int64_t R = int64_t(T) * N * M;
    e = hipMemcpyAsync(xplanes, xs, size_t(R) * Fin * sizeof(float), hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return e;
    for (int k = 1; k < K; ++k) {
      e = launch_cheb_step(rowptr, col, val, nullptr, xplanes + int64_t(k - 1) * xpstride,
                           k >= 2 ? xplanes + int64_t(k - 2) * xpstride : nullptr,
                           xplanes + int64_t(k) * xpstride, nullptr, nullptr, nullptr, T * N, M, Fin,
                           K, k, false, s);
      if (e != hipSuccess) return e;
    }
    a.xpre = 1;
  }
  // a pair waits for its partner, so every workgroup of the grid must be
  // resident at once: check the grid against the occupancy query (what a
  // cooperative launch would check, MI355X_MICROARCH.md §Residency; the LDS
  // footprint admits one workgroup per CU, so the grid is at most one per CU)
  // and launch plainly.  Residency on an idle chip is all this buys: kernels of
  // other streams or processes can hold CUs, which is what the hand-off
  // timeout, the NaN poisoning and the plan's fault word are for
  const size_t lds = lstm_seq_lds(M, K, nnz, xs ? Fin : 0);
  void (*const kfn)(SeqArgs) = kerns[a.xpre ? 1 : 0][gates == 0 ? 1 : 0];
  const void* kern = reinterpret_cast<const void*>(kfn);
  int per_cu = 0, cus = 0;
  e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kST, lds);
  if (e != hipSuccess) return e;
  e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return e;
  if (per_cu < 1 || 2 * P > per_cu * cus) return hipErrorCooperativeLaunchTooLarge;
  const dim3 grid(2 * P), block(kST);
  hipLaunchKernelGGL(kfn, grid, block, lds, s, a);
  return hipGetLastError();
}

hipError_t launch_lstm_bstep(int gates, int N, int M, int K, const int* trowptr, const int* tcol,
                             const float* tval, const int* order, int64_t nnzT, const float* dh, const float* dh_rec,
                             const float* dc, const float* act, int act_um, const float* c_prev,
                             const float* c_out, const float* Wh, float* dpre, float* dc_prev,
                             float* dh_prev, hipStream_t s) {
  if (!lstm_bstep_ok(M, kH, K, nnzT) || N < 1) return hipErrorInvalidValue;
  BStepArgs a{trowptr, tcol, tval, order, M, round_up(M + 1, 16), N, gates, N % 8 == 0 ? 1 : 0,
              int(nnzT), act_um ? 1 : 0, dh, dh_rec, dc, act, c_prev, c_out, Wh, dpre, dc_prev, dh_prev,
              (debug_flags() >> 16) & 0xff, nullptr};
#ifdef CG_DEBUG
  a.ts = g_debug_ts;
#endif
  // the split-bf16 D_k contraction (CG_OPT_GEMM_X3) where its larger W image fits
  const bool x3 = option(kOptGemmX3) != 0 && lstm_bstep_lds(M, K, nnzT, true) <= size_t(kLdsBytes);
  const size_t lds = lstm_bstep_lds(M, K, nnzT, x3);
#define CG_BSTEP(KK)                                                                              \
  case KK: {                                                                                      \
    static hipError_t at = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_lstm_bstep<KK, false>), \
                                               hipFuncAttributeMaxDynamicSharedMemorySize,       \
                                               kLdsBytes);                                        \
    static hipError_t atx = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_lstm_bstep<KK, true>), \
                                                hipFuncAttributeMaxDynamicSharedMemorySize,      \
                                                kLdsBytes);                                       \
    if (at != hipSuccess) return at;                                                              \
    if (atx != hipSuccess) return atx;                                                            \
    if (x3) hipLaunchKernelGGL((k_lstm_bstep<KK, true>), dim3(2 * N), dim3(kST), lds, s, a);      \
    else hipLaunchKernelGGL((k_lstm_bstep<KK, false>), dim3(2 * N), dim3(kST), lds, s, a);        \
    break;                                                                                        \
  }
  switch (K) {
    CG_BSTEP(1)
    CG_BSTEP(2)
    CG_BSTEP(3)
    CG_BSTEP(4)
    default:
      return hipErrorInvalidValue;
  }
#undef CG_BSTEP
  return hipGetLastError();
}

}  // namespace cg
