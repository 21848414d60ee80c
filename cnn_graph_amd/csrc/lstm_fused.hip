// One gconv-LSTM time step's h path in ONE launch (lib/gconv_lstm.py:77-221,
// the four h-gate convolutions of GConvLSTMCell.__call__ plus its pointwise
// update), H = 32 hidden units, M <= 1024 vertices:
//
//   T_0 = h, T_1 = L~ h, T_k = 2 L~ T_{k-1} - T_{k-2}        (cheby_conv, :183-207)
//   a   = (gx + sum_k T_k Wh_k) + b      gx = the x-conv of this step (precomputed
//                                        for every step at once)
//   z = tan(a_z), i = sigmoid(a_i), f = sigmoid(a_f), o = tanh(a_o)  (reference)
//   c' = f c + i z ;  h' = o tanh(c')                           (:215, :218)
//
// Two 1024-thread workgroups per sample (units [0,16) and [16,32): each owns
// 64 of the 128 gate columns), so a batch of 128 samples fills the 256 CUs;
// the two workgroups of a sample are placed on one XCD (blocks b and b + 8)
// so their half-row stores of c', h' and the gate activations merge in its L2.
// Both compute the whole Chebyshev recurrence of h (cheap: 8 332 nnz for
// config E) in LDS, one 8-channel quarter of h at a time:
//   LDS  two [M][12]-float slots (T_{k-1}, T_k of the quarter; 12-float rows:
//        the MFMA operand reads are bank-conflict-free) + this workgroup's
//        Wh columns [K*32][64]
//   per quarter and order k: the contraction acc += T_k Wh_k on
//        v_mfma_f32_32x32x2_f32 (each wave: 2 row tiles x 2 column tiles), and
//        the SpMM of the next order (thread = CSR row, sequential CSR-order
//        accumulation with contraction off -- the basis is the same as
//        lib/graph.py::chebyshev's), one barrier per order
//   epilogue  the gate pre-activations never leave registers: lanes j and
//        j^16 swap (z, i) / (f, o), each lane updates 8 (row, unit) cells
//        per row tile without divergence
// Saved for the backward: the gate activations, c', and the h basis planes
// T_1 .. T_{K-1} ([K-1][N][M][32], written half by each workgroup).
//
// Bound: the fp32 contraction, 2*M*(K*32)*128 FLOP per sample and step, on
// MFMA (157 TF/s peak) -- with config E's K = 3, 25 MFLOP per sample.
#include "cg_internal.h"
#include "lstm_gates.h"

namespace cg {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kHT = 1024;  // threads per workgroup
constexpr int kH = 32;     // hidden units
constexpr int kQ = 8;      // channels per SpMM pass (quarter of H)
constexpr int kSR = 12;    // LDS slot row stride (floats)
constexpr int kWC = 64;    // gate columns per workgroup

__device__ __forceinline__ float sigm(float a) { return gate_sigmoid(a); }

struct HStepArgs {
  const int* rowptr;
  const int* col;
  const float* val;
  int M, K, N, gates, pair_xcd;
  const float* h_prev;  // [N][M][32]
  const float* c_prev;  // [N][M][32] or NULL (zero state)
  const float* gx;      // [N][M][128] x-conv gate pre-activations
  const float* Wh;      // [K*32][128], row c*K + k
  const float* bias;    // [128] or NULL
  float* c_out;
  float* h_out;
  float* act;     // [N][M][128] gate activations or NULL
  float* planes;  // T_1..T_{K-1}: plane k-1 at (k-1)*plane, [N][M][32]; NULL: not kept
  int64_t plane;
};

__global__ __launch_bounds__(kHT) void k_lstm_hstep(HStepArgs A) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, hh = lane >> 5;
  const int M = A.M, K = A.K;
  int n, u;
  if (A.pair_xcd) {
    const int b = blockIdx.x;
    n = (b >> 4) * 8 + (b & 7);
    u = (b >> 3) & 1;
  } else {
    n = blockIdx.x >> 1;
    u = blockIdx.x & 1;
  }
  float* slot0 = smem;
  float* slot1 = smem + M * kSR;
  float* s_W = smem + 2 * M * kSR;  // [K*32][64]
  // this workgroup's columns: wc -> gate (wc/16), unit 16u + wc%16
  for (int e = tid; e < K * kH * kWC; e += kHT) {
    const int wr = e / kWC, wc = e - wr * kWC;
    s_W[e] = A.Wh[int64_t(wr) * 128 + (wc >> 4) * 32 + 16 * u + (wc & 15)];
  }
  const int ntiles = (M + 31) >> 5;
  f32x16 acc[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[t][c][e] = 0.f;
  // CSR row of this thread
  const int row = tid;
  const bool rv = row < M;
  const int j0 = rv ? A.rowptr[row] : 0, j1 = rv ? A.rowptr[row + 1] : 0;
  const float* hn = A.h_prev + int64_t(n) * M * kH;

  for (int q = 0; q < kH / kQ; ++q) {
    // T_0 quarter into slot 0
    if (rv) {
      const float4* src = reinterpret_cast<const float4*>(hn + int64_t(row) * kH + q * kQ);
      float4* dst = reinterpret_cast<float4*>(slot0 + row * kSR);
      dst[0] = src[0];
      dst[1] = src[1];
    }
    __syncthreads();
    for (int k = 0; k < K; ++k) {
      float* cur = (k & 1) ? slot1 : slot0;
      float* nxt = (k & 1) ? slot0 : slot1;
      // contraction with T_k: channels q*8 + 4*hh + s, s < 4
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int tile = wave + 16 * t;
        if (tile < ntiles) {
          const int r = tile * 32 + li;
          const float4 a4 = (r < M) ? *reinterpret_cast<const float4*>(cur + r * kSR + 4 * hh)
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
          const float av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const float* wrow = s_W + ((q * kQ + 4 * hh + s) * K + k) * kWC;
#pragma unroll
            for (int c = 0; c < 2; ++c)
              acc[t][c] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s], wrow[c * 32 + li], acc[t][c],
                                                               0, 0, 0);
          }
        }
      }
      // next order of this quarter: thread = CSR row, CSR order from +0
      if (k + 1 < K && rv) {
        float s8[kQ];
#pragma unroll
        for (int c = 0; c < kQ; ++c) s8[c] = 0.f;
        // 8 entries at a time: their col/val loads are issued together
        // (unpredicated: past the row end they re-read its last entry), then the
        // LDS gathers and the CSR-order accumulation (per-entry predicated loads
        // serialised one L2 round trip per entry: r02m-p 150-176 us/step)
        for (int jb = j0; jb < j1; jb += 8) {
          int cc[8];
          float ww[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int jj = (jb + e < j1) ? jb + e : j1 - 1;
            cc[e] = A.col[jj];
            ww[e] = A.val[jj];
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float4* g = reinterpret_cast<const float4*>(cur + cc[e] * kSR);
            const float4 g0 = g[0], g1 = g[1];
            if (jb + e < j1) {
              const float w = ww[e];
              s8[0] = s8[0] + w * g0.x;
              s8[1] = s8[1] + w * g0.y;
              s8[2] = s8[2] + w * g0.z;
              s8[3] = s8[3] + w * g0.w;
              s8[4] = s8[4] + w * g1.x;
              s8[5] = s8[5] + w * g1.y;
              s8[6] = s8[6] + w * g1.z;
              s8[7] = s8[7] + w * g1.w;
            }
          }
        }
        float4* own = reinterpret_cast<float4*>(nxt + row * kSR);  // T_{k-1} (k >= 1)
        if (k >= 1) {
          const float4 p0 = own[0], p1 = own[1];
          s8[0] = 2.f * s8[0] - p0.x;
          s8[1] = 2.f * s8[1] - p0.y;
          s8[2] = 2.f * s8[2] - p0.z;
          s8[3] = 2.f * s8[3] - p0.w;
          s8[4] = 2.f * s8[4] - p1.x;
          s8[5] = 2.f * s8[5] - p1.y;
          s8[6] = 2.f * s8[6] - p1.z;
          s8[7] = 2.f * s8[7] - p1.w;
        }
        const float4 o0 = make_float4(s8[0], s8[1], s8[2], s8[3]);
        const float4 o1 = make_float4(s8[4], s8[5], s8[6], s8[7]);
        own[0] = o0;
        own[1] = o1;
        if (A.planes && (q & 1) == u) {  // basis plane T_{k+1}, this workgroup's quarters
          float4* p = reinterpret_cast<float4*>(A.planes + int64_t(k) * A.plane +
                                                (int64_t(n) * M + row) * kH + q * kQ);
          p[0] = o0;
          p[1] = o1;
        }
      }
      __syncthreads();
    }
  }

  // epilogue: a = (gx + gh) + b, gates, c', h'
  const int64_t rbase = int64_t(n) * M;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int tile = wave + 16 * t;
    if (tile >= ntiles) continue;
    // lanes < 16 take accumulator rows e, lanes >= 16 rows e + 8 (no divergence:
    // each lane sends the partner the element the partner needs)
#pragma unroll
    for (int e0 = 0; e0 < 8; ++e0) {
      const bool lo = li < 16;
      const int e = lo ? e0 : e0 + 8;
      const float v0 = lo ? acc[t][0][e0] : acc[t][0][e0 + 8];
      const float v1 = lo ? acc[t][1][e0] : acc[t][1][e0 + 8];
      const float x0 = __shfl_xor(lo ? acc[t][0][e0 + 8] : acc[t][0][e0], 16);
      const float x1 = __shfl_xor(lo ? acc[t][1][e0 + 8] : acc[t][1][e0], 16);
      const int r = tile * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh;
      if (r >= M) continue;
      const float hz = li < 16 ? v0 : x0, hi = li < 16 ? x0 : v0;
      const float hf = li < 16 ? v1 : x1, ho = li < 16 ? x1 : v1;
      const int j = 16 * u + (li & 15);
      const int64_t rr = rbase + r;
      const float* g = A.gx + rr * 128 + j;
      float az = g[0] + hz, ai = g[32] + hi, af = g[64] + hf, ao = g[96] + ho;
      if (A.bias) {
        az = az + A.bias[j];
        ai = ai + A.bias[32 + j];
        af = af + A.bias[64 + j];
        ao = ao + A.bias[96 + j];
      }
      const float z = A.gates == 0 ? gate_tan(az) : gate_tanh(az);
      const float ig = sigm(ai), fg = sigm(af);
      const float o = A.gates == 0 ? gate_tanh(ao) : sigm(ao);
      const float cp = A.c_prev ? A.c_prev[rr * kH + j] : 0.f;
      const float cn = fg * cp + ig * z;
      A.c_out[rr * kH + j] = cn;
      A.h_out[rr * kH + j] = o * gate_tanh(cn);
      if (A.act) {
        float* a = A.act + rr * 128 + j;
        a[0] = z;
        a[32] = ig;
        a[64] = fg;
        a[96] = o;
      }
    }
  }
}

}  // namespace

size_t lstm_hstep_lds(int M, int K) {
  return (size_t(2) * M * kSR + size_t(K) * kH * kWC) * sizeof(float);
}

bool lstm_hstep_ok(int M, int H, int K) {
  return H == kH && M >= 1 && M <= kHT && K >= 1 && lstm_hstep_lds(M, K) <= size_t(kLdsBytes);
}

hipError_t launch_lstm_hstep(int gates, int N, int M, int K, const int* rowptr, const int* col,
                             const float* val, const float* h_prev, const float* c_prev,
                             const float* gx, const float* Wh, const float* bias, float* c_out,
                             float* h_out, float* act, float* planes, int64_t plane,
                             hipStream_t s) {
  if (!lstm_hstep_ok(M, kH, K) || N < 1) return hipErrorInvalidValue;
  static hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_lstm_hstep),
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               kLdsBytes);
  if (attr != hipSuccess) return attr;
  HStepArgs a{rowptr, col, val, M, K, N, gates, N % 8 == 0 ? 1 : 0, h_prev, c_prev, gx, Wh, bias,
              c_out, h_out, act, planes, plane};
  hipLaunchKernelGGL(k_lstm_hstep, dim3(2 * N), dim3(kHT), lstm_hstep_lds(M, K), s, a);
  return hipGetLastError();
}

}  // namespace cg
