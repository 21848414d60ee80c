// Channel-group resident kernels for mid-size graphs with many input channels
// (M <= 1024, Fin a multiple of 8): the ResGNN hidden layers of the humanflow
// model (config R: M = 1024, Fin = Fout = 32, K = 20; lib/graph_conv.py:234-330)
// and the h-conv-sized filters of the gconv-LSTM.  On the streaming path each
// Chebyshev step is its own launch (K - 1 of them per filter, ~11 us each, and
// the y row GEMM re-reads the whole K-plane basis); here ONE workgroup owns one
// sample x 8 channels and runs the whole recurrence out of LDS:
//
// k_grp_fwd   T_0 = x (its 8 channels), T_{k+1} = 2 L~ T_k - T_{k-1} (CSR order
//             from +0, contraction off: the basis is bit-exact to
//             lib/graph.py::chebyshev), every T_k written ONCE as its slice of
//             basis plane k (the planes layout [K][N*M][Fin]); the contraction
//             y_g = sum_k T_k W_k over the group's 8 channels on
//             v_mfma_f32_32x32x2_f32, transposed (y^T = W^T T^T) so the B
//             operand is the lane's own T_k straight from the SpMM; the
//             per-group partial y_g leaves once per filter.
// k_grp16_fwd the same with 16-channel groups and one LDS slot (Fin % 16 == 0).
// k_grp_yred  y = act(sum_g y_g + res), groups added in a fixed order.
// k_grp_clen  the backward's reverse recurrence G_{K-1} = D_{K-1},
//             G_k = (D_k + c L~^T G_{k+1}) - G_{k+2} (c = 2; 1 at k = 0) over the
//             explicit L~^T with G in LDS, D_k streamed from the k-major dBasis
//             planes; dx (+)= G_0.  Same expressions and order as
//             cheb_stream.hip::k_clenshaw_step, so dx is bitwise the same.
//
// Geometry: 512 threads (8 waves, two per SIMD, 256 registers per lane); lane
// (row j of a 32-row tile, half hh) owns channels 4hh .. 4hh+3 of the group for
// four row tiles (rows order[(wave + 8 rt) * 32 + j], the rows dealt by
// decreasing length so each tile's unrolled gather loop -- lds_spmm.h -- is
// as long as its longest row).  LDS: two [M][8] slots (T_k /
// T_{k+1} or G_{k+1} / G_k), the CSR (16-bit columns + values), and for the
// forward the group's rows of W as MFMA A operands.  The groups of a sample sit
// on one XCD (blocks b, b + 8, .. under round-robin placement) so their 32-byte
// slices of each basis row merge in one L2.
#include "cg_internal.h"
#include "lds_spmm.h"

namespace cg {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kGT = 512;  // threads per workgroup
constexpr int kGQ = 8;    // channels per group
constexpr int kGRT = 4;   // 32-row tiles per wave (8 waves x 4 x 32 = 1024 rows)
constexpr int kGQ16 = 16; // channels per group of the one-slot kernels (Fin % 16 == 0)

// CG_OPT_SPMM_PW = 0 (ablation build only): the resident SpMMs read their CSR
// metadata one entry per LDS access (lds_row_spmm) instead of two
// (lds_row_spmm_w); it lost every A/B (profiles/r04_pw), so the release
// library carries only the paired form
#ifdef CG_DEBUG
inline bool spmm_pw() { return option(kOptSpmmPw) != 0; }
#else
constexpr bool spmm_pw() { return true; }
#endif
inline int rup(int v, int m) { return (v + m - 1) / m * m; }

// block -> (sample, group): the G groups of a sample on one XCD
__device__ __forceinline__ void grp_map(int b, int G, int& n, int& g) {
  const int per = 8 * G;  // 8 samples x G groups per block of 8*G workgroups
  const int blk = b / per, rem = b - blk * per;
  g = rem >> 3;
  n = blk * 8 + (rem & 7);
}

struct GrpFwdArgs {
  const int* rowptr;
  const int* col;
  const float* val;
  const int* order;  // rows by decreasing length (lane -> row)
  int M, Mr, Fin, K, Fout, N, nnz, G;
  const float* x;   // [N][M][Fin]
  const float* W;   // [Fin*K][Fout], row fin*K + k
  float* basis;     // planes [K][N*M][Fin]
  int64_t plane;    // N*M*Fin
  float* yp;        // [G][N*M][Fout] partial y per group, or NULL (basis only)
  unsigned long long* ts;  // ablation build: phase stamps (CG_TS), else NULL
  int dbg;                 // ablation build (k_grp16_fwd): 1 no MFMA, 2 no SpMM, 4 no plane stores
};

template <int NOT>  // 32-wide output tiles (Fout <= 32 * NOT)
__global__ __launch_bounds__(kGT) void k_grp_fwd(GrpFwdArgs A) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = lane & 31, hh = lane >> 5;
  int n, g;
  grp_map(blockIdx.x, A.G, n, g);
  if (n >= A.N) return;  // grid padded to whole XCD rounds (uniform per workgroup)
  const int M = A.M, K = A.K, Fin = A.Fin, Fout = A.Fout;
  float* slot0 = smem;
  float* slot1 = smem + A.Mr * kGQ;
  float* s_W = slot1 + A.Mr * kGQ;  // [K][s 4][hh 2][NOT][i 32]
  float* s_val = s_W + K * 256 * NOT;
  unsigned short* s_col = reinterpret_cast<unsigned short*>(s_val + A.nnz);
  const bool want_y = A.yp != nullptr;
  if (want_y) {
    stage_lds<8, kGT>(K * 256 * NOT, [&](int e) {
      const int i = e & 31, ot = (e >> 5) % NOT, h2 = (e / (32 * NOT)) & 1;
      const int s = (e / (64 * NOT)) & 3, k = e / (256 * NOT);
      const int ch = kGQ * g + 4 * h2 + s, out = ot * 32 + i;
      return out < Fout ? A.W[int64_t(ch * K + k) * Fout + out] : 0.f;
    }, [&](int e, float v) { s_W[e] = v; });
  }
  stage_csr_lds<8, kGT>(A.nnz, A.val, A.col, s_val, s_col);
  if (tid < 2 * kGQ) (tid < kGQ ? slot0 : slot1)[M * kGQ + (tid & (kGQ - 1))] = 0.f;  // zero row M
  // two lane mappings over the same 32 rows of tile (wave, rt): the MFMA's
  // (row j = lane % 32, half hh = lane / 32) reads its B operand from the slot;
  // the SpMM's (row lane / 2, half lane % 2) makes an 8-lane LDS access group
  // gather 4 whole 32-byte records
  const int js = lane >> 1, hs = lane & 1;
  int row[kGRT], rowS[kGRT], rb[kGRT], re[kGRT], wl[kGRT];
  bool rvS[kGRT];
  const int c0 = kGQ * g + 4 * hs;
#pragma unroll
  for (int rt = 0; rt < kGRT; ++rt) {
    const int idx = (wave + 8 * rt) * 32 + j;
    row[rt] = idx < M ? A.order[idx] : M;
    const int idxS = (wave + 8 * rt) * 32 + js;
    rvS[rt] = idxS < M;
    rowS[rt] = rvS[rt] ? A.order[idxS] : M;
    rb[rt] = rvS[rt] ? A.rowptr[rowS[rt]] : 0;
    re[rt] = rvS[rt] ? A.rowptr[rowS[rt] + 1] : 0;
    wl[rt] = wave_max(re[rt] - rb[rt]);
    if (rvS[rt]) {
      const int64_t o = (int64_t(n) * M + rowS[rt]) * Fin + c0;
      const float4 v = *reinterpret_cast<const float4*>(A.x + o);
      if (A.x != A.basis) *reinterpret_cast<float4*>(A.basis + o) = v;  // plane 0 = x (unless x IS it)
      *reinterpret_cast<float4*>(slot0 + rowS[rt] * kGQ + 4 * hs) = v;
    }
  }
  f32x16 acc[kGRT][NOT];
#pragma unroll
  for (int rt = 0; rt < kGRT; ++rt)
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[rt][ot][e] = 0.f;
  __syncthreads();
  for (int k = 0; k < K; ++k) {
    const float* cur = (k & 1) ? slot1 : slot0;
    if (want_y) {
      // y^T[out][row] += W_k^T[out][ch] T_k^T[ch][row], channels 4hh + s
      const float* wk = s_W + k * 256 * NOT + hh * 32 * NOT + j;
      float4 tk[kGRT];
#pragma unroll
      for (int rt = 0; rt < kGRT; ++rt)
        tk[rt] = *reinterpret_cast<const float4*>(cur + row[rt] * kGQ + 4 * hh);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int ot = 0; ot < NOT; ++ot) {
          const float a = wk[s * 64 * NOT + ot * 32];
#pragma unroll
          for (int rt = 0; rt < kGRT; ++rt)
            acc[rt][ot] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, (&tk[rt].x)[s], acc[rt][ot], 0, 0, 0);
        }
    }
    if (k + 1 < K) {
      float* nxt = (k & 1) ? slot0 : slot1;
      float* pl = A.basis + int64_t(k + 1) * A.plane;
#pragma unroll
      for (int rt = 0; rt < kGRT; ++rt) {
        if (!rvS[rt]) continue;
        float4 sm;
        with_row_len(wl[rt], [&](auto lc) {
          sm = lds_row_spmm_w<decltype(lc)::value>(cur, kGQ, 4 * hs, s_col, s_val, rb[rt], re[rt], M);
        });
        float s0 = sm.x, s1 = sm.y, s2 = sm.z, s3 = sm.w;
        float4* own = reinterpret_cast<float4*>(nxt + rowS[rt] * kGQ + 4 * hs);
        if (k >= 1) {  // T_{k-1}: the slot entry being overwritten
          const float4 p = *own;
          s0 = 2.f * s0 - p.x;
          s1 = 2.f * s1 - p.y;
          s2 = 2.f * s2 - p.z;
          s3 = 2.f * s3 - p.w;
        }
        const float4 o = make_float4(s0, s1, s2, s3);
        *own = o;
        *reinterpret_cast<float4*>(pl + (int64_t(n) * M + rowS[rt]) * Fin + c0) = o;
      }
      __syncthreads();
    }
  }
  if (!want_y) return;
  // lane (row, hh) holds outputs ot*32 + 8q + 4hh + m (q = e / 4, m = e % 4)
  float* yg = A.yp + int64_t(g) * A.N * M * Fout;
#pragma unroll
  for (int rt = 0; rt < kGRT; ++rt) {
    if (row[rt] >= M) continue;
    float* yr = yg + (int64_t(n) * M + row[rt]) * Fout;
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int o0 = ot * 32 + 8 * q + 4 * hh;
        if (o0 + 4 <= Fout && (Fout & 3) == 0) {
          *reinterpret_cast<float4*>(yr + o0) =
              make_float4(acc[rt][ot][4 * q], acc[rt][ot][4 * q + 1], acc[rt][ot][4 * q + 2],
                          acc[rt][ot][4 * q + 3]);
        } else {
#pragma unroll
          for (int m = 0; m < 4; ++m)
            if (o0 + m < Fout) yr[o0 + m] = acc[rt][ot][4 * q + m];
        }
      }
  }
}

// The same forward for 16-channel groups (Fin % 16 == 0): half the workgroups
// of the 8-channel kernel, so config R's 100 samples x 2 groups fit the 256
// CUs in ONE round (8-channel groups: 416 workgroups = two rounds, the second
// 62 % full); measured 178 vs 192 us per call (profiles/r03_grp): a workgroup
// with twice the channels takes nearly twice as long, the chip is busy either way.  ONE [M][16] slot: a step gathers T_k from it, each lane keeps
// T_{k-1} of its own rows in registers, a barrier, the lane swaps its rows'
// T_k out for T_{k+1}, a barrier.  SpMM lanes: (row lane / 4 of a 16-row half
// tile, channels 4 (lane % 4) ..); MFMA lanes: (row j, channels 8hh .. 8hh+7).
// Fout <= 32 only (NOT = 1; two output tiles spill at 256 registers).  PW: the
// rows' CSR metadata read two entries per LDS access (lds_row_spmm_w).
template <int NOT, bool PW>
__global__ __launch_bounds__(kGT) void k_grp16_fwd(GrpFwdArgs A) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = lane & 31, hh = lane >> 5;
  int n, g;
  grp_map(blockIdx.x, A.G, n, g);
  if (n >= A.N) return;  // grid padded to whole XCD rounds (uniform per workgroup)
  CG_TS(A.ts, 0);
  const int M = A.M, K = A.K, Fin = A.Fin, Fout = A.Fout;
  float* slot = smem;                     // [Mr][16]
  float* s_W = slot + A.Mr * kGQ16;       // [K][s 8][hh 2][NOT][i 32]
  float* s_val = s_W + K * 512 * NOT;
  unsigned short* s_col = reinterpret_cast<unsigned short*>(s_val + A.nnz);
  const bool want_y = A.yp != nullptr;
  if (want_y) {
    stage_lds<8, kGT>(K * 512 * NOT, [&](int e) {
      const int i = e & 31, ot = (e >> 5) % NOT, h2 = (e / (32 * NOT)) & 1;
      const int s = (e / (64 * NOT)) & 7, k = e / (512 * NOT);
      const int ch = kGQ16 * g + 8 * h2 + s, out = ot * 32 + i;
      return out < Fout ? A.W[int64_t(ch * K + k) * Fout + out] : 0.f;
    }, [&](int e, float v) { s_W[e] = v; });
  }
  stage_csr_lds<8, kGT>(A.nnz, A.val, A.col, s_val, s_col);
  if (tid < kGQ16) slot[M * kGQ16 + tid] = 0.f;  // zero row M
  const int js = lane >> 2, qs = lane & 3;
  const int c0 = kGQ16 * g + 4 * qs;
  // per (tile, half): the row, its CSR start | length << 16 (nnz < 65536 and
  // rows <= 1024 long: the LDS bound), the wave's longest row (uniform)
  int row[kGRT], rowS[kGRT][2], rbl[kGRT][2], wl[kGRT][2];
  bool rvS[kGRT][2];
  float4 tm1[kGRT][2];
#pragma unroll
  for (int rt = 0; rt < kGRT; ++rt) {
    const int idx = (wave + 8 * rt) * 32 + j;
    row[rt] = idx < M ? A.order[idx] : M;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int idxS = (wave + 8 * rt) * 32 + 16 * hf + js;
      rvS[rt][hf] = idxS < M;
      rowS[rt][hf] = rvS[rt][hf] ? A.order[idxS] : M;
      const int b0 = rvS[rt][hf] ? A.rowptr[rowS[rt][hf]] : 0;
      const int len = rvS[rt][hf] ? A.rowptr[rowS[rt][hf] + 1] - b0 : 0;
      rbl[rt][hf] = b0 | (len << 16);
      wl[rt][hf] = __builtin_amdgcn_readfirstlane(wave_max(len));
      tm1[rt][hf] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (rvS[rt][hf]) {
        const int64_t o = (int64_t(n) * M + rowS[rt][hf]) * Fin + c0;
        const float4 v = *reinterpret_cast<const float4*>(A.x + o);
        if (A.x != A.basis) *reinterpret_cast<float4*>(A.basis + o) = v;  // plane 0 = x (unless x IS it)
        *reinterpret_cast<float4*>(slot + rowS[rt][hf] * kGQ16 + 4 * qs) = v;
      }
    }
  }
  f32x16 acc[kGRT][NOT];
#pragma unroll
  for (int rt = 0; rt < kGRT; ++rt)
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[rt][ot][e] = 0.f;
  __syncthreads();
  for (int k = 0; k < K; ++k) {
    if (want_y && !CG_DBG(A.dbg, 1)) {
      // y^T[out][row] += W_k^T[out][ch] T_k^T[ch][row], channels 8hh + s
      const float* wk = s_W + k * 512 * NOT + hh * 32 * NOT + j;
      float4 ta[kGRT], tb[kGRT];
#pragma unroll
      for (int rt = 0; rt < kGRT; ++rt) {
        ta[rt] = *reinterpret_cast<const float4*>(slot + row[rt] * kGQ16 + 8 * hh);
        tb[rt] = *reinterpret_cast<const float4*>(slot + row[rt] * kGQ16 + 8 * hh + 4);
      }
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int ot = 0; ot < NOT; ++ot) {
          const float a = wk[s * 64 * NOT + ot * 32];
#pragma unroll
          for (int rt = 0; rt < kGRT; ++rt) {
            const float b = s < 4 ? (&ta[rt].x)[s] : (&tb[rt].x)[s - 4];
            acc[rt][ot] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[rt][ot], 0, 0, 0);
          }
        }
    }
    if (k + 1 < K) {
      float4 nv[kGRT][2];
#pragma unroll
      for (int rt = 0; rt < kGRT; ++rt) {
        if constexpr (PW) {
          // both halves of the tile under ONE length switch (their rows are
          // neighbours in the longest-first order, so the lengths nearly
          // agree; a padding row has length 0 and sums to 0): the two rows'
          // reads interleave in one basic block
          float4 sm[2];
          if (CG_DBG(A.dbg, 2)) {  // ablation: no gathers
            sm[0] = tm1[rt][0];
            sm[1] = tm1[rt][1];
          } else {
            const int a0 = rbl[rt][0] & 0xffff, a1 = a0 + (rbl[rt][0] >> 16);
            const int b0 = rbl[rt][1] & 0xffff, b1 = b0 + (rbl[rt][1] >> 16);
            with_row_len(wl[rt][0] > wl[rt][1] ? wl[rt][0] : wl[rt][1], [&](auto lc) {
              constexpr int LL = decltype(lc)::value;
              sm[0] = lds_row_spmm_w<LL>(slot, kGQ16, 4 * qs, s_col, s_val, a0, a1, M);
              sm[1] = lds_row_spmm_w<LL>(slot, kGQ16, 4 * qs, s_col, s_val, b0, b1, M);
            });
          }
#pragma unroll
          for (int hf = 0; hf < 2; ++hf) {
            float4 v = sm[hf];
            if (k >= 1 && !CG_DBG(A.dbg, 2)) {
              const float4 p = tm1[rt][hf];
              v = make_float4(2.f * v.x - p.x, 2.f * v.y - p.y, 2.f * v.z - p.z, 2.f * v.w - p.w);
            }
            nv[rt][hf] = v;
          }
          continue;
        }
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          if (!rvS[rt][hf]) continue;
          float4 sm;
          if (CG_DBG(A.dbg, 2)) {  // ablation: no gathers
            nv[rt][hf] = tm1[rt][hf];
            continue;
          }
          const int b0 = rbl[rt][hf] & 0xffff, b1 = b0 + (rbl[rt][hf] >> 16);
          with_row_len(wl[rt][hf], [&](auto lc) {
            sm = lds_row_spmm<decltype(lc)::value>(slot, kGQ16, 4 * qs, s_col, s_val, b0, b1, M);
          });
          if (k >= 1) {
            const float4 p = tm1[rt][hf];
            sm = make_float4(2.f * sm.x - p.x, 2.f * sm.y - p.y, 2.f * sm.z - p.z, 2.f * sm.w - p.w);
          }
          nv[rt][hf] = sm;
        }
      }
      __syncthreads();  // every gather and contraction read of T_k done
      float* pl = A.basis + int64_t(k + 1) * A.plane;
#pragma unroll
      for (int rt = 0; rt < kGRT; ++rt)
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          if (!rvS[rt][hf]) continue;
          float4* own = reinterpret_cast<float4*>(slot + rowS[rt][hf] * kGQ16 + 4 * qs);
          tm1[rt][hf] = *own;
          *own = nv[rt][hf];
          if (!CG_DBG(A.dbg, 4))
            *reinterpret_cast<float4*>(pl + (int64_t(n) * M + rowS[rt][hf]) * Fin + c0) = nv[rt][hf];
        }
      __syncthreads();
    }
  }
  CG_TS(A.ts, 2);
  if (!want_y) return;
  // lane (row, hh) holds outputs ot*32 + 8q + 4hh + m (q = e / 4, m = e % 4)
  float* yg = A.yp + int64_t(g) * A.N * M * Fout;
#pragma unroll
  for (int rt = 0; rt < kGRT; ++rt) {
    if (row[rt] >= M) continue;
    float* yr = yg + (int64_t(n) * M + row[rt]) * Fout;
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int o0 = ot * 32 + 8 * q + 4 * hh;
        if (o0 + 4 <= Fout && (Fout & 3) == 0) {
          *reinterpret_cast<float4*>(yr + o0) =
              make_float4(acc[rt][ot][4 * q], acc[rt][ot][4 * q + 1], acc[rt][ot][4 * q + 2],
                          acc[rt][ot][4 * q + 3]);
        } else {
#pragma unroll
          for (int m = 0; m < 4; ++m)
            if (o0 + m < Fout) yr[o0 + m] = acc[rt][ot][4 * q + m];
        }
      }
  }
  CG_TS(A.ts, 3);
}

// y = act(sum_g yp[g] + res), groups added in order (bitwise reproducible)
__global__ __launch_bounds__(256) void k_grp_yred(const float* __restrict__ yp, int G, int64_t n,
                                                  const float* __restrict__ res, int act,
                                                  float* __restrict__ y) {
#pragma clang fp contract(off)
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    float s = yp[i];
    for (int gg = 1; gg < G; ++gg) s = s + yp[int64_t(gg) * n + i];
    if (res) s = s + res[i];
    if (act == 1) s = s > 0.f ? s : 0.f;
    y[i] = s;
  }
}

// the same, four elements per lane (16-byte aligned operands, n % 4 == 0)
__global__ __launch_bounds__(256) void k_grp_yred4(const float4* __restrict__ yp, int G, int64_t n4,
                                                   const float4* __restrict__ res, int act,
                                                   float4* __restrict__ y) {
#pragma clang fp contract(off)
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n4; i += int64_t(gridDim.x) * 256) {
    float4 s = yp[i];
    for (int gg = 1; gg < G; ++gg) {
      const float4 p = yp[int64_t(gg) * n4 + i];
      s = make_float4(s.x + p.x, s.y + p.y, s.z + p.z, s.w + p.w);
    }
    if (res) {
      const float4 r = res[i];
      s = make_float4(s.x + r.x, s.y + r.y, s.z + r.z, s.w + r.w);
    }
    if (act == 1)
      s = make_float4(s.x > 0.f ? s.x : 0.f, s.y > 0.f ? s.y : 0.f, s.z > 0.f ? s.z : 0.f,
                      s.w > 0.f ? s.w : 0.f);
    y[i] = s;
  }
}

struct GrpClenArgs {
  const int* trowptr;  // L~^T
  const int* tcol;
  const float* tval;
  const int* order;    // rows of L~^T by decreasing length (lane -> row)
  int M, Mr, Fin, K, N, nnz, G;
  const float* D;  // k-major dBasis planes [K][N*M][Fin]
  int64_t plane;   // N*M*Fin
  float* dx;       // [N][M][Fin]
  int dx_acc;
};

// PC: the rows' columns packed in registers (lds_row_spmm_pc) for rows of at
// most 12 entries, the CSR columns read from LDS per step otherwise
template <bool PC>
__global__ __launch_bounds__(kGT) void k_grp_clen(GrpClenArgs A) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // lanes 2j, 2j+1 take the two 16-byte halves of row j's 32-byte record, so
  // an 8-lane LDS access group gathers 4 whole records (4 bank groups of 8)
  const int j = lane >> 1, hh = lane & 1;
  int n, g;
  grp_map(blockIdx.x, A.G, n, g);
  if (n >= A.N) return;
  const int M = A.M, K = A.K, Fin = A.Fin;
  float* slotA = smem;
  float* slotB = smem + A.Mr * kGQ;
  float* s_val = slotB + A.Mr * kGQ;
  unsigned short* s_col = reinterpret_cast<unsigned short*>(s_val + A.nnz);
  stage_csr_lds<8, kGT>(A.nnz, A.tval, A.tcol, s_val, s_col);
  int row[kGRT], rb[kGRT], re[kGRT], wl[kGRT];
  bool rv[kGRT];
  int64_t off[kGRT];
  if (tid < 2 * kGQ) (tid < kGQ ? slotA : slotB)[M * kGQ + (tid & (kGQ - 1))] = 0.f;  // zero row M
  const int c0 = kGQ * g + 4 * hh;
  float G1[kGRT][4], G2[kGRT][4], Dn[kGRT][4];
  auto loadD = [&](int k) {
#pragma unroll
    for (int rt = 0; rt < kGRT; ++rt) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (rv[rt]) v = *reinterpret_cast<const float4*>(A.D + int64_t(k) * A.plane + off[rt]);
      Dn[rt][0] = v.x;
      Dn[rt][1] = v.y;
      Dn[rt][2] = v.z;
      Dn[rt][3] = v.w;
    }
  };
#pragma unroll
  for (int rt = 0; rt < kGRT; ++rt) {
    const int idx = (wave + 8 * rt) * 32 + j;
    rv[rt] = idx < M;
    row[rt] = rv[rt] ? A.order[idx] : M;
    rb[rt] = rv[rt] ? A.trowptr[row[rt]] : 0;
    re[rt] = rv[rt] ? A.trowptr[row[rt] + 1] : 0;
    off[rt] = (int64_t(n) * M + (rv[rt] ? row[rt] : 0)) * Fin + c0;
    wl[rt] = wave_max(re[rt] - rb[rt]);
  }
  constexpr int NP = PC ? 6 : 1;
  unsigned pk[kGRT][NP];
  if (PC) {
    __syncthreads();  // s_col staged
#pragma unroll
    for (int rt = 0; rt < kGRT; ++rt) pack_row_cols<NP>(pk[rt], s_col, rb[rt], re[rt], M);
  }
  loadD(K - 1);
  // G_{K-1} = D_{K-1} + c * (+0)  (k_clenshaw_step's expression with no G_K)
  const float cl = (K - 1 >= 1) ? 2.f : 1.f;
#pragma unroll
  for (int rt = 0; rt < kGRT; ++rt)
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      G1[rt][m] = Dn[rt][m] + cl * 0.f;
      G2[rt][m] = 0.f;
    }
  if (K > 1) {
#pragma unroll
    for (int rt = 0; rt < kGRT; ++rt)
      if (rv[rt])
        *reinterpret_cast<float4*>(slotA + row[rt] * kGQ + 4 * hh) =
            make_float4(G1[rt][0], G1[rt][1], G1[rt][2], G1[rt][3]);
    loadD(K - 2);
  }
  __syncthreads();
  for (int k = K - 2; k >= 0; --k) {
    const float* cur = ((K - 2 - k) & 1) ? slotB : slotA;
    float* nxt = ((K - 2 - k) & 1) ? slotA : slotB;
    const float c = k >= 1 ? 2.f : 1.f;
    float Dk[kGRT][4];
#pragma unroll
    for (int rt = 0; rt < kGRT; ++rt)
#pragma unroll
      for (int m = 0; m < 4; ++m) Dk[rt][m] = Dn[rt][m];
    if (k >= 1) loadD(k - 1);  // in flight during this step's gathers
#pragma unroll
    for (int rt = 0; rt < kGRT; ++rt) {
      float4 sm = make_float4(0.f, 0.f, 0.f, 0.f);
      if (rv[rt]) {
        if constexpr (PC) {
          with_row_len(wl[rt], [&](auto lc) {
            constexpr int LL = decltype(lc)::value;
            if constexpr (LL > 0 && LL <= 2 * NP)
              sm = lds_row_spmm_pc<LL, NP, 3>(cur, 4 * hh, pk[rt], s_val, rb[rt], re[rt]);
            else
              sm = lds_row_spmm_w<LL>(cur, kGQ, 4 * hh, s_col, s_val, rb[rt], re[rt], M);
          });
        } else {
          with_row_len(wl[rt], [&](auto lc) {
            sm = lds_row_spmm_w<decltype(lc)::value>(cur, kGQ, 4 * hh, s_col, s_val, rb[rt], re[rt], M);
          });
        }
      }
      const float sv[4] = {sm.x, sm.y, sm.z, sm.w};
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        float o = Dk[rt][m] + c * sv[m];
        if (k + 2 <= K - 1) o = o - G2[rt][m];
        G2[rt][m] = G1[rt][m];
        G1[rt][m] = o;
      }
      if (k > 0 && rv[rt])
        *reinterpret_cast<float4*>(nxt + row[rt] * kGQ + 4 * hh) =
            make_float4(G1[rt][0], G1[rt][1], G1[rt][2], G1[rt][3]);
    }
    if (k > 0) __syncthreads();
  }
#pragma unroll
  for (int rt = 0; rt < kGRT; ++rt) {
    if (!rv[rt]) continue;
    float4* d = reinterpret_cast<float4*>(A.dx + off[rt]);
    float4 o = make_float4(G1[rt][0], G1[rt][1], G1[rt][2], G1[rt][3]);
    if (A.dx_acc) {
      const float4 p = *d;
      o = make_float4(p.x + o.x, p.y + o.y, p.z + o.z, p.w + o.w);
    }
    *d = o;
  }
}

// k_grp_clen_dy: k_grp_clen with dBasis computed in the kernel instead of read
// from the k-major planes a separate row GEMM wrote (config R: 237 MB written
// and 262 MB read back per hidden-layer backward).  For each group of four
// Chebyshev orders kg .. kg+3 a wave computes, per 32-row tile,
//   D_k[r][c] = sum_f dy[r][f] W[(c0 + c) K + k][f]
// as ONE transposed 32x32 MFMA tile (rows (order, channel) = 8 ko + c, columns
// the tile's graph rows) on v_mfma_f32_32x32x2_f32 with the inner index split
// exactly as k_rowgemm splits it (lane half h feeds f = h KC2 + s at step s,
// s ascending from a zero accumulator), so every D value is the same sequence
// of MFMA operations as the row GEMM's and dx stays bitwise the streaming
// path's.  The MFMA leaves lane (row n, half h) channels 4h .. 4h+3 of the
// four orders; ds_bpermute hands them to the recurrence's lane (2n + h).
// The group's W rows sit in LDS (row stride Fout + 4: the 32 (order, channel)
// rows of an operand read spread over the banks).  The first order group is
// formed up front; each later one tile per recurrence step of the group
// before it, so its MFMAs run under the LDS-bound steps: waves 0-3 issue them
// before the step's gathers, waves 4-7 (the other wave of each SIMD) after,
// and the tile's result is handed over at the start of the next step.
struct GrpClenDyArgs {
  const int* trowptr;
  const int* tcol;
  const float* tval;
  const int* order;
  int M, Mr, Fin, K, N, nnz, G, Fout, KC2;
  const float* dy;  // [N][M][Fout]
  const float* W;   // [Fin*K][Fout], row fin*K + k
  float* dx;        // [N][M][Fin]
  int dx_acc;
  int pipe;  // 1: the next group's tiles during this group's steps; 0: each group's up front
  unsigned long long* ts;  // ablation build: phase stamps (CG_TS), else NULL
  int dbg;  // ablation build: 1 no D-tile MFMAs, 2 no SpMM, 4 no dy loads, 8 no hand-over
};

template <int KC2>  // Fout / 2: the row GEMM's inner half (16 or 32)
__global__ __launch_bounds__(kGT) void k_grp_clen_dy(GrpClenDyArgs A) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = lane >> 1, hh = lane & 1;   // recurrence lanes: row j, channels 4hh..
  const int mi = lane & 31, mh = lane >> 5;  // MFMA lanes: tile row / column mi, half mh
  int n, g;
  grp_map(blockIdx.x, A.G, n, g);
  if (n >= A.N) return;
  CG_TS(A.ts, 0);
  const int M = A.M, K = A.K, Fin = A.Fin;
  constexpr int Fout = 2 * KC2;
  constexpr int WS = Fout + 4;  // LDS row stride of the staged W rows
  float* slotA = smem;
  float* slotB = smem + A.Mr * kGQ;
  float* s_w = slotB + A.Mr * kGQ;  // [K][8][WS]: W row (c0 + ch) K + k
  float* s_val = s_w + K * kGQ * WS;
  unsigned short* s_col = reinterpret_cast<unsigned short*>(s_val + A.nnz);
  const int c0 = kGQ * g;
  stage_csr_lds<8, kGT>(A.nnz, A.tval, A.tcol, s_val, s_col);
  stage_lds<8, kGT>(K * kGQ * Fout, [&](int e) {
    const int f = e % Fout, kc = e / Fout, ch = kc % kGQ, k = kc / kGQ;
    return A.W[(int64_t(c0 + ch) * K + k) * Fout + f];
  }, [&](int e, float v) { s_w[(e / Fout) * WS + e % Fout] = v; });
  int row[kGRT], rb[kGRT], re[kGRT], wl[kGRT];
  bool rv[kGRT];
  int drow[kGRT];  // the MFMA lane's tile row (graph row of column mi), -1 past M
#pragma unroll
  for (int rt = 0; rt < kGRT; ++rt) {
    const int idx = (wave + 8 * rt) * 32 + j;
    rv[rt] = idx < M;
    row[rt] = rv[rt] ? A.order[idx] : M;
    rb[rt] = rv[rt] ? A.trowptr[row[rt]] : 0;
    re[rt] = rv[rt] ? A.trowptr[row[rt] + 1] : 0;
    wl[rt] = wave_max(re[rt] - rb[rt]);
    const int midx = (wave + 8 * rt) * 32 + mi;
    drow[rt] = midx < M ? A.order[midx] : -1;
  }
  if (tid < 2 * kGQ) (tid < kGQ ? slotA : slotB)[M * kGQ + (tid & (kGQ - 1))] = 0.f;  // zero row M
  __syncthreads();
  CG_TS(A.ts, 1);
  const int bsrc = ((lane >> 1) + 32 * (lane & 1)) * 4;  // ds_bpermute source of lane 2n + h
  const bool mfma_first = wave < 4;
  // dy operand of tile rt (the MFMA lane's half row: KC2 floats), loaded ahead
  // of its MFMAs (global / L2: the sample's dy is read by every group)
  auto dload = [&](int rt, float (&b)[KC2]) {
    if (CG_DBG(A.dbg, 4)) {  // ablation: no dy loads
#pragma unroll
      for (int q = 0; q < KC2; ++q) b[q] = float(q);
      return;
    }
    const float* dr = A.dy + (int64_t(n) * M + (drow[rt] >= 0 ? drow[rt] : 0)) * Fout + mh * KC2;
    if constexpr (KC2 % 4 == 0) {
#pragma unroll
      for (int q = 0; q < KC2 / 4; ++q) {
        const float4 v = drow[rt] >= 0 ? *reinterpret_cast<const float4*>(dr + 4 * q)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
        b[4 * q] = v.x; b[4 * q + 1] = v.y; b[4 * q + 2] = v.z; b[4 * q + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < KC2; ++q) b[q] = drow[rt] >= 0 ? dr[q] : 0.f;
    }
  };
  // one D tile: orders kg .. kg+3 of a 32-row tile on the MFMA (acc), W from LDS
  auto dtile = [&](int kg, const float (&b)[KC2], f32x16& acc) {
    const int kk = kg + (mi >> 3);
    const float* wr = s_w + ((kk < K ? kk : 0) * kGQ + (mi & 7)) * WS + mh * KC2;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    if (CG_DBG(A.dbg, 1)) {  // ablation: no D-tile MFMAs
      acc[0] = b[0];
      return;
    }
#pragma unroll
    for (int q = 0; q < KC2; ++q) {
      const float a = kk < K ? wr[q] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b[q], acc, 0, 0, 0);
    }
  };
  // D of the current order group in ONE register array, whose layout
  // alternates between groups: even groups Dg[rt][ko], odd groups Dg[ko][rt].
  // Step ko of an even group consumes column [*][ko] and the next (odd)
  // group's tile rt' = ko lands in that same column ([ko'][rt' = ko]); odd
  // groups consume and refill rows the same way -- so the next group's tiles
  // fill exactly the registers the current group has finished with.
  float Dg[4][4][4];
  // acc[4 ko + m] at lane (n, h): order kg + ko, channel 4h + m of row n
  auto handover = [&](const f32x16& acc, int rt, bool odd) {
#pragma unroll
    for (int ko = 0; ko < 4; ++ko)
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const float v = CG_DBG(A.dbg, 8)  // ablation: no hand-over
                            ? acc[4 * ko + m]
                            : __int_as_float(__builtin_amdgcn_ds_bpermute(bsrc, __float_as_int(acc[4 * ko + m])));
        if (odd) Dg[ko][rt][m] = v;
        else Dg[rt][ko][m] = v;
      }
  };
  // G_{k+2} is read back from the slot G_k overwrites (same lane, same row),
  // so only the latest G lives in registers (G_0 at the end)
  float G0[kGRT][4];
  const int ktop = ((K - 1) / 4) * 4;
  const bool pipe = A.pipe != 0;
  auto run_group = [&](int kg, auto odd_c) {
    constexpr bool odd = decltype(odd_c)::value;
    if (kg == ktop || !pipe) {
      constexpr int NL = KC2 <= 16 ? kGRT : 1;  // tiles' dy loads in flight together
      float b[NL][KC2];
#pragma unroll
      for (int rt = 0; rt < NL; ++rt) dload(rt, b[rt]);
#pragma unroll
      for (int rt = 0; rt < kGRT; ++rt) {
        if (NL == 1 && rt > 0) dload(rt, b[0]);
        f32x16 a0;
        dtile(kg, b[NL == 1 ? 0 : rt], a0);
        handover(a0, rt, odd);
      }
    }
    const bool more = pipe && kg >= 4;  // form the next (lower) order group meanwhile
    f32x16 acc;
    float pb[KC2];  // dy of the next tile, loaded one step ahead
    if (more) dload(3, pb);
#pragma unroll
    for (int ko = 3; ko >= 0; --ko) {
      const int k = kg + ko;
      // the next group's tile formed during the previous step (its registers
      // held orders of this group that are consumed by now)
      if (more && ko < 3) handover(acc, ko + 1, !odd);
      const bool step = k < K - 1;  // a recurrence step (k == K-1: the start)
      if (more && (mfma_first || !step)) {
        dtile(kg - 4, pb, acc);
        if (ko > 0) dload(ko - 1, pb);
      }
      if (k == K - 1) {
        // G_{K-1} = D_{K-1} + c * (+0)  (k_clenshaw_step's expression with no G_K)
        const float cl = (K - 1 >= 1) ? 2.f : 1.f;
#pragma unroll
        for (int rt = 0; rt < kGRT; ++rt) {
#pragma unroll
          for (int m = 0; m < 4; ++m) G0[rt][m] = (odd ? Dg[ko][rt][m] : Dg[rt][ko][m]) + cl * 0.f;
          if (K > 1 && rv[rt])
            *reinterpret_cast<float4*>(slotA + row[rt] * kGQ + 4 * hh) =
                make_float4(G0[rt][0], G0[rt][1], G0[rt][2], G0[rt][3]);
        }
        __syncthreads();
      } else if (step) {
        const float* cur = ((K - 2 - k) & 1) ? slotB : slotA;
        float* nxt = ((K - 2 - k) & 1) ? slotA : slotB;
        const float c = k >= 1 ? 2.f : 1.f;
        // tiles in pairs under ONE length switch (the longer row's bound; a
        // padding row has rb = re = 0 and sums to 0): the two rows' reads
        // interleave in one basic block
        float4 smp[kGRT];
#pragma unroll
        for (int rp = 0; rp < kGRT; rp += 2)
          if (CG_DBG(A.dbg, 2)) {  // ablation: no SpMM
            smp[rp] = smp[rp + 1] = make_float4(1.f, 1.f, 1.f, 1.f);
          } else
          with_row_len(wl[rp] > wl[rp + 1] ? wl[rp] : wl[rp + 1], [&](auto lc) {
            constexpr int LL = decltype(lc)::value;
            smp[rp] = lds_row_spmm_w<LL>(cur, kGQ, 4 * hh, s_col, s_val, rb[rp], re[rp], M);
            smp[rp + 1] = lds_row_spmm_w<LL>(cur, kGQ, 4 * hh, s_col, s_val, rb[rp + 1], re[rp + 1], M);
          });
#pragma unroll
        for (int rt = 0; rt < kGRT; ++rt) {
          const float4 sm = smp[rt];
          const float sv[4] = {sm.x, sm.y, sm.z, sm.w};
          float4* own = reinterpret_cast<float4*>(nxt + row[rt] * kGQ + 4 * hh);
          float g2[4] = {0.f, 0.f, 0.f, 0.f};
          if (k + 2 <= K - 1 && rv[rt]) {  // G_{k+2}: this slot, written two steps ago
            const float4 p = *own;
            g2[0] = p.x; g2[1] = p.y; g2[2] = p.z; g2[3] = p.w;
          }
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            float o = (odd ? Dg[ko][rt][m] : Dg[rt][ko][m]) + c * sv[m];
            if (k + 2 <= K - 1) o = o - g2[m];
            G0[rt][m] = o;
          }
          if (k > 0 && rv[rt]) *own = make_float4(G0[rt][0], G0[rt][1], G0[rt][2], G0[rt][3]);
        }
        if (more && !mfma_first) {
          dtile(kg - 4, pb, acc);
          if (ko > 0) dload(ko - 1, pb);
        }
        if (k > 0) __syncthreads();
      }
    }
    if (more) handover(acc, 0, !odd);
  };
  int gi = 0;  // order groups done (phase stamps 2.. of the ablation build)
  for (int kg = ktop;;) {
    run_group(kg, IntC<0>{});
    if (gi < 5) CG_TS(A.ts, 2 + gi);
    ++gi;
    if (kg < 4) break;
    kg -= 4;
    run_group(kg, IntC<1>{});
    if (gi < 5) CG_TS(A.ts, 2 + gi);
    ++gi;
    if (kg < 4) break;
    kg -= 4;
  }
  (void)gi;
#pragma unroll
  for (int rt = 0; rt < kGRT; ++rt) {
    if (!rv[rt]) continue;
    float4* d = reinterpret_cast<float4*>(A.dx + (int64_t(n) * M + row[rt]) * Fin + c0 + 4 * hh);
    float4 o = make_float4(G0[rt][0], G0[rt][1], G0[rt][2], G0[rt][3]);
    if (A.dx_acc) {
      const float4 p = *d;
      o = make_float4(p.x + o.x, p.y + o.y, p.z + o.z, p.w + o.w);
    }
    *d = o;
  }
  CG_TS(A.ts, 7);
}

}  // namespace

size_t grp_fwd_lds(int M, int K, int Fout, int64_t nnz) {
  const int NOT = Fout <= 32 ? 1 : 2;
  return size_t(2) * rup(M + 1, 32) * kGQ * 4 + size_t(K) * 256 * NOT * 4 + size_t(nnz) * 4 +
         align16(size_t(nnz) * 2 + kSpmmSlack);
}

size_t grp16_fwd_lds(int M, int K, int Fout, int64_t nnz) {
  const int NOT = Fout <= 32 ? 1 : 2;
  return size_t(rup(M + 1, 32)) * kGQ16 * 4 + size_t(K) * 512 * NOT * 4 + size_t(nnz) * 4 +
         align16(size_t(nnz) * 2 + kSpmmSlack);
}

// the 16-channel forward serves Fin % 16 == 0, Fout <= 32 when its LDS fits
// (CG_OPT_GRP16 = 0 keeps the 8-channel one, for A/B runs).  A 16-channel
// one-slot Clenshaw kernel (dx bitwise the same) was measured slower than the
// 8-channel one on config R (160 vs 148 us) and dropped.
static bool grp16_enabled() { return option(kOptGrp16) != 0; }

size_t grp_clen_lds(int M, int64_t nnzT) {
  return size_t(2) * rup(M + 1, 32) * kGQ * 4 + size_t(nnzT) * 4 + align16(size_t(nnzT) * 2 + kSpmmSlack);
}

bool grp_ok(int M, int64_t nnz, int Fin, int K, int Fout) {
  return M >= 1 && M <= kGRT * 8 * 32 && nnz >= 1 && Fin % kGQ == 0 && Fin >= kGQ && K >= 2 &&
         Fout >= 1 && Fout <= 64 && grp_fwd_lds(M, K, Fout, nnz) <= size_t(kLdsBytes) &&
         grp_clen_lds(M, nnz) <= size_t(kLdsBytes);
}

size_t grp_partial_bytes(int N, int M, int Fin, int Fout) {
  return size_t(Fin / kGQ) * size_t(N) * size_t(M) * size_t(Fout) * 4;
}

static int grp_grid(int N, int G) { return rup(N, 8) * G; }

hipError_t launch_grp_fwd(const int* rowptr, const int* col, const float* val, const int* order,
                          int64_t nnz, int N,
                          int M, int Fin, int K, int Fout, const float* x, const float* W,
                          float* basis, float* yp, const float* res, int act, float* y,
                          hipStream_t s) {
  if (!grp_ok(M, nnz, Fin, K, Fout)) return hipErrorInvalidValue;
  const bool g16 = grp16_enabled() && Fin % kGQ16 == 0 && Fout <= 32 && nnz < 65536 &&
                   grp16_fwd_lds(M, K, Fout, nnz) <= size_t(kLdsBytes);
  const int G = Fin / (g16 ? kGQ16 : kGQ);
  GrpFwdArgs a{rowptr, col, val, order, M, rup(M + 1, 32), Fin, K, Fout, N, int(nnz), G, x, W, basis,
               int64_t(N) * M * Fin, y ? yp : nullptr, nullptr};
#ifdef CG_DEBUG
  a.ts = g_debug_ts;
  a.dbg = (debug_flags() >> 24) & 0xff;
#endif
  const size_t lds = g16 ? grp16_fwd_lds(M, K, Fout, nnz) : grp_fwd_lds(M, K, Fout, nnz);
  if (g16 && Fout <= 32) {
    static hipError_t at = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_grp16_fwd<1, true>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
    if (at != hipSuccess) return at;
#ifdef CG_DEBUG
    static hipError_t at0 = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_grp16_fwd<1, false>),
                                                hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
    if (at0 != hipSuccess) return at0;
    if (!spmm_pw()) hipLaunchKernelGGL((k_grp16_fwd<1, false>), dim3(grp_grid(N, G)), dim3(kGT), lds, s, a);
    else
#endif
    hipLaunchKernelGGL((k_grp16_fwd<1, true>), dim3(grp_grid(N, G)), dim3(kGT), lds, s, a);
  } else if (Fout <= 32) {
    static hipError_t at = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_grp_fwd<1>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
    if (at != hipSuccess) return at;
    hipLaunchKernelGGL(k_grp_fwd<1>, dim3(grp_grid(N, G)), dim3(kGT), lds, s, a);
  } else {
    static hipError_t at = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_grp_fwd<2>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
    if (at != hipSuccess) return at;
    hipLaunchKernelGGL(k_grp_fwd<2>, dim3(grp_grid(N, G)), dim3(kGT), lds, s, a);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !y) return e;
  const int64_t n = int64_t(N) * M * Fout;
  const bool a16 = ((reinterpret_cast<uintptr_t>(yp) | reinterpret_cast<uintptr_t>(res) |
                     reinterpret_cast<uintptr_t>(y)) & 15) == 0;
  if (a16 && n % 4 == 0) {
    int64_t blocks = (n / 4 + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_grp_yred4, dim3(unsigned(blocks)), dim3(256), 0, s,
                       reinterpret_cast<const float4*>(yp), G, n / 4,
                       reinterpret_cast<const float4*>(res), act, reinterpret_cast<float4*>(y));
    return hipGetLastError();
  }
  int64_t blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(k_grp_yred, dim3(unsigned(blocks)), dim3(256), 0, s, yp, G, n, res, act, y);
  return hipGetLastError();
}

hipError_t launch_grp_clen(const int* trowptr, const int* tcol, const float* tval, const int* order,
                           int64_t nnzT,
                           int N, int M, int Fin, int K, const float* D, float* dx, int dx_acc,
                           hipStream_t s) {
  if (M > kGRT * 8 * 32 || Fin % kGQ || K < 1 || grp_clen_lds(M, nnzT) > size_t(kLdsBytes))
    return hipErrorInvalidValue;
  const int G = Fin / kGQ;
  GrpClenArgs a{trowptr, tcol, tval, order, M, rup(M + 1, 32), Fin, K, N, int(nnzT), G, D,
                int64_t(N) * M * Fin, dx, dx_acc};
  static hipError_t at1 = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_grp_clen<true>),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
  if (at1 != hipSuccess) return at1;
#ifdef CG_DEBUG
  // CG_OPT_GRP_PC = 0 (ablation build only): columns read from LDS every step
  // (dx bitwise the same; lost its A/B, profiles/r04_r)
  static hipError_t at0 = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_grp_clen<false>),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
  if (at0 != hipSuccess) return at0;
  if (option(kOptGrpPc) == 0) {
    hipLaunchKernelGGL(k_grp_clen<false>, dim3(grp_grid(N, G)), dim3(kGT), grp_clen_lds(M, nnzT), s, a);
    return hipGetLastError();
  }
#endif
  hipLaunchKernelGGL(k_grp_clen<true>, dim3(grp_grid(N, G)), dim3(kGT), grp_clen_lds(M, nnzT), s, a);
  return hipGetLastError();
}

// the fused variant serves Fout 2, 32 and 64 (the row GEMM's inner split
// KC2 = Fout / 2: 1, 16, 32 -- the ResGNN's output layer and hidden layers);
// CG_OPT_CLEN_DY = 0 keeps the row GEMM + k_grp_clen pair (A/B runs)

size_t grp_clen_dy_lds(int M, int64_t nnzT, int K, int Fout) {
  return grp_clen_lds(M, nnzT) + size_t(K) * kGQ * (Fout + 4) * 4;
}

bool grp_clen_dy_ok(int M, int64_t nnzT, int K, int Fout) {
  return option(kOptClenDy) != 0 && (Fout == 2 || Fout == 32 || Fout == 64) && M <= kGRT * 8 * 32 &&
         grp_clen_dy_lds(M, nnzT, K, Fout) <= size_t(kLdsBytes);
}

hipError_t launch_grp_clen_dy(const int* trowptr, const int* tcol, const float* tval,
                              const int* order, int64_t nnzT, int N, int M, int Fin, int K,
                              int Fout, const float* dy, const float* W, float* dx, int dx_acc,
                              hipStream_t s) {
  if (Fin % kGQ || K < 1 || !grp_clen_dy_ok(M, nnzT, K, Fout))
    return hipErrorInvalidValue;
  const int G = Fin / kGQ;
  // 2 (ablation build only): each group's tiles up front
  const int pipe = option(kOptClenDy) == 2 ? 0 : 1;
  GrpClenDyArgs a{trowptr, tcol, tval, order, M, rup(M + 1, 32), Fin, K, N, int(nnzT), G, Fout,
                  Fout / 2, dy, W, dx, dx_acc, pipe, nullptr};
#ifdef CG_DEBUG
  a.ts = g_debug_ts;
  a.dbg = (debug_flags() >> 24) & 0xff;
#endif
  static hipError_t at16 = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_grp_clen_dy<16>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
  static hipError_t at32 = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_grp_clen_dy<32>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
  const size_t lds = grp_clen_dy_lds(M, nnzT, K, Fout);
  static hipError_t at1 = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_grp_clen_dy<1>),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
  if (Fout == 2) {
    if (at1 != hipSuccess) return at1;
    hipLaunchKernelGGL(k_grp_clen_dy<1>, dim3(grp_grid(N, G)), dim3(kGT), lds, s, a);
  } else if (Fout == 32) {
    if (at16 != hipSuccess) return at16;
    hipLaunchKernelGGL(k_grp_clen_dy<16>, dim3(grp_grid(N, G)), dim3(kGT), lds, s, a);
  } else {
    if (at32 != hipSuccess) return at32;
    hipLaunchKernelGGL(k_grp_clen_dy<32>, dim3(grp_grid(N, G)), dim3(kGT), lds, s, a);
  }
  return hipGetLastError();
}

}  // namespace cg
