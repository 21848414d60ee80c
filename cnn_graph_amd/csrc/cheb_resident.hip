// Resident (LDS) path of the Chebyshev graph convolution for gfx950.
//
// One 1024-thread workgroup (16 waves, 4 per SIMD) per sample n.  The whole
// K-step recurrence
//   T_0 = X, T_1 = L~X, T_k = 2 L~ T_{k-1} - T_{k-2}      (lib/graph_conv.py:163-169)
// runs on chip:
//   * each thread owns RPT rows of L~ and keeps their entries in REGISTERS for
//     the whole launch.  The host lays the sparse operand out as a padded ELL
//     image in "thread-slot" order (cheb_abi.cpp::build_slots): rows sorted by
//     degree so the rows of one wave have (nearly) equal length, column-major
//     so the prologue loads are coalesced, and a per-wave max length that lets
//     whole gather instructions be skipped;
//   * the 3-slot ring T_{k-2}, T_{k-1}, T_k lives in LDS as [vertex][slot]
//     (12-byte stride: consecutive vertices hit consecutive banks), and the k
//     loop is unrolled by 6 so the ring slot of every gather is an immediate
//     offset of the ds_read (no address arithmetic per step).
// A step is one burst of independent LDS gathers per row, a sequential fp32
// accumulation, one LDS store and one barrier.
//
// The weight contraction y = basis @ W (lib/graph_conv.py:175) is folded into
// the recurrence: every two steps each wave feeds the pair (T_{2s}, T_{2s+1})
// of its 32-vertex tiles to v_mfma_f32_32x32x2_f32, whose K=2 is exactly one
// Chebyshev pair, accumulating y in registers.  The same A-operand values are
// the basis entries: they are staged in LDS in the HBM layout of
// lib/graph_conv.py:172 ([m][fin*K+k], one contiguous block per sample) and
// leave with coalesced 16-byte stores at the end (a row of that layout is only
// complete after the last step, so streaming it earlier writes partial lines:
// measured 28 us of scattered 4-byte stores on config B).
//
// The backward kernel does, per sample:
//   A. dBasis = dy W^T on MFMA into LDS (D[j][m], j = fin*K + k);
//   B. the reverse (Clenshaw) recurrence over L~^T with the same register /
//      ring machinery
//        G_{K-1} = D_{K-1};  G_k = D_k + 2 L~^T G_{k+1} - G_{k+2};  G_0 = D_0 + L~^T G_1 - G_2
//      writing dx = G_0 straight to HBM.
// dW = basis^T dy is HBM-streaming work done by k_dw_slabs (cheb_stream.hip).
//
// Numerics: each row accumulates sequentially from +0 in CSR order with one
// rounding per product and per add (fp contraction OFF) -- the order of scipy
// csr_matvecs / TF SparseTensorDenseMatMul -- so the basis is bit-exact to
// lib/graph.py::chebyshev.  Padding entries gather a word kept at 0 with
// weight 0 and add an exact +0 (the running sum is never -0).  MFMA f32 is an
// exact fp32 fma chain.
#include <type_traits>

#include "cg_internal.h"

namespace cg {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kT = kResidentThreads;  // 1024
constexpr int kWaves = kT / 64;       // 16
template <int V>
using I = std::integral_constant<int, V>;

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int imin(int a, int b) { return a < b ? a : b; }
__device__ __forceinline__ float lds_f(const char* p) { return *reinterpret_cast<const float*>(p); }
__device__ __forceinline__ void lds_st(char* p, float v) { *reinterpret_cast<float*>(p) = v; }

// Registers of the rows a thread owns (thread slot t = q*kT + tid).
template <int RPT, int MAXNNZ>
struct RowRegs {
  int row[RPT];    // vertex, or -1 for an idle slot
  int rb[RPT];     // row * 12: byte offset of the vertex in a [Mp][3] ring block
  int beg[RPT];    // CSR offset of the row (tail loop for rows longer than MAXNNZ)
  int len[RPT];
  int wl[RPT];     // wave-uniform max row length of the slot group
  int ca[RPT][MAXNNZ];  // gather byte offsets (column * 12); padding -> zero word
  float v[RPT][MAXNNZ];

  __device__ __forceinline__ void load(const SlotLayout& E, int tid, int wave) {
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const int t = q * kT + tid;
      row[q] = E.row[t];
      len[q] = E.len[t];
      beg[q] = E.beg[t];
      wl[q] = E.wlen[q * kWaves + wave];  // uniform index: scalar load
      rb[q] = row[q] * 12;
#pragma unroll
      for (int j = 0; j < MAXNNZ; ++j) {
        ca[q][j] = E.col[j * E.S + t] * 12;
        v[q][j] = E.val[j * E.S + t];
      }
    }
  }

  // sum_{j in row, CSR order} v_j * T[c_j][SLOT]   (sequential, no contraction)
  template <int SLOT>
  __device__ __forceinline__ float dot(int q, const char* __restrict__ Tb,
                                       const int* __restrict__ col,
                                       const float* __restrict__ val) const {
#pragma clang fp contract(off)
    const char* base = Tb + SLOT * 4;
    float g[MAXNNZ];
#pragma unroll
    for (int j = 0; j < MAXNNZ; ++j) g[j] = (j < wl[q]) ? lds_f(base + ca[q][j]) : 0.f;
    float a = 0.f;
#pragma unroll
    for (int j = 0; j < MAXNNZ; ++j)
      if (j < wl[q]) a = a + v[q][j] * g[j];
    if (wl[q] > MAXNNZ)  // rows longer than MAXNNZ (rare): CSR tail from L2
      for (int j = MAXNNZ; j < len[q]; ++j)
        a = a + val[beg[q] + j] * lds_f(base + col[beg[q] + j] * 12);
    return a;
  }
};

// ---------------------------------------------------------------------------
// Forward
// ---------------------------------------------------------------------------
template <int RPT, int MAXNNZ, int NT, bool FIN1>
__global__ __launch_bounds__(kT) void cheb_fwd_resident(ResidentFwdArgs A) {
#pragma clang fp contract(off)
  constexpr int MT = 2 * RPT;  // 32-vertex tiles per wave: ceil(M/32)/16 <= 2*RPT
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int M = A.M, K = A.K, Fout = A.Fout, Mp = A.Mp, dbg = A.dbg;
  (void)dbg;  // only read by the debug build's ablation switches
  const int Fin = FIN1 ? 1 : A.Fin;
  const int n = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, li = lane & 31;
  const int FinK = Fin * K;
  const int slab = Mp * 12;  // bytes of one [Mp][3] ring block (one fin)

  float* s_W = reinterpret_cast<float*>(smem);
  size_t off = align16(size_t(FinK) * Fout * 4);
  char* s_T = smem + off;  // [Fin][Mp][3] floats
  off = align16(off + size_t(Fin) * slab);
  float* s_B = reinterpret_cast<float*>(smem + off);  // [M][FinK]

  RowRegs<RPT, MAXNNZ> rows;
  rows.load(A.E, tid, wave);
  for (int i = tid; i < FinK * Fout; i += kT) s_W[i] = A.W ? A.W[i] : 0.f;
  const float* xn = A.x + size_t(n) * M * Fin;
  for (int i = tid; i < M * Fin; i += kT) {
    const int m = i / Fin, fin = i - m * Fin;
    lds_st(s_T + fin * slab + m * 12, xn[i]);  // slot 0 = T_0
  }
  for (int i = tid; i < 3 * Fin; i += kT)  // zero words gathered by padding entries
    lds_st(s_T + (i / 3) * slab + M * 12 + (i % 3) * 4, 0.f);
  __syncthreads();
  if (CG_DBG(dbg, 16)) return;

  const int ntiles = (M + 31) >> 5;
  f32x16 acc[MT][NT];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int q = 0; q < NT; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][q][r] = 0.f;
  const bool keep_basis = A.basis && !CG_DBG(dbg, 2);

  // Contraction of the pair (T_{2s}, T_{2s+1}) on MFMA; stage the basis.
  auto mfma_pair = [&](int s) {
    const int kk = 2 * s + h;
    const bool kv = kk < K;
    const int soff = (kk % 3) * 4;
    for (int fin = 0; fin < Fin; ++fin) {
      float b[NT];
#pragma unroll
      for (int q = 0; q < NT; ++q) {
        const int f = q * 32 + li;
        b[q] = (kv && f < Fout) ? s_W[(fin * K + kk) * Fout + f] : 0.f;
      }
      const char* Tb = s_T + fin * slab + soff;
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int tile = wave + t * kWaves;
        if (tile < ntiles) {
          const int m = tile * 32 + li;
          float a = 0.f;
          if (kv && m < M) {
            a = lds_f(Tb + m * 12);
            if (keep_basis) s_B[m * FinK + fin * K + kk] = a;  // banks (FinK*li+kk) mod 32
          }
          if (!CG_DBG(dbg, 4)) {
#pragma unroll
            for (int q = 0; q < NT; ++q) acc[t][q] = mfma32(a, b[q], acc[t][q]);
          }
        }
      }
    }
  };

  // One recurrence step k with compile-time ring slots (slot(k) = k mod 3).
  auto step = [&](auto cur_c, auto prv_c, auto prv2_c, int k) {
    constexpr int CUR = decltype(cur_c)::value, PRV = decltype(prv_c)::value,
                  PRV2 = decltype(prv2_c)::value;
    for (int fin = 0; fin < Fin; ++fin) {
      char* Tb = s_T + (FIN1 ? 0 : fin * slab);
#pragma unroll
      for (int q = 0; q < RPT; ++q) {
        if (rows.row[q] >= 0) {
          char* rp = Tb + rows.rb[q];
          const float a = CG_DBG(dbg, 1) ? lds_f(rp + PRV * 4)
                                    : rows.template dot<PRV>(q, Tb, A.col, A.val);
          const float o = (k == 1) ? a : (2.f * a - lds_f(rp + PRV2 * 4));
          lds_st(rp + CUR * 4, o);
        }
      }
    }
    __syncthreads();
  };

  for (int k = 1; k < K; k += 6) {  // k = 1 (mod 6): slots cur/prv/prv2 = 1/0/2
    step(I<1>(), I<0>(), I<2>(), k);
    if (k + 1 < K) { mfma_pair((k - 1) >> 1); step(I<2>(), I<1>(), I<0>(), k + 1); }
    if (k + 2 < K) step(I<0>(), I<2>(), I<1>(), k + 2);
    if (k + 3 < K) { mfma_pair((k + 1) >> 1); step(I<1>(), I<0>(), I<2>(), k + 3); }
    if (k + 4 < K) step(I<2>(), I<1>(), I<0>(), k + 4);
    if (k + 5 < K) { mfma_pair((k + 3) >> 1); step(I<0>(), I<2>(), I<1>(), k + 5); }
  }
  mfma_pair((K - 1) >> 1);  // the last (possibly half-empty) pair

  if (keep_basis) {
    __syncthreads();
    float* basis_n = A.basis + size_t(n) * M * FinK;
    const int total = M * FinK;
    if ((reinterpret_cast<uintptr_t>(basis_n) & 15) == 0) {
      const int n4 = total >> 2;
      const float4* src = reinterpret_cast<const float4*>(s_B);
      float4* dst = reinterpret_cast<float4*>(basis_n);
      for (int i = tid; i < n4; i += kT) dst[i] = src[i];
      for (int i = (n4 << 2) + tid; i < total; i += kT) basis_n[i] = s_B[i];
    } else {
      for (int i = tid; i < total; i += kT) basis_n[i] = s_B[i];
    }
  }

  if (A.y && !CG_DBG(dbg, 8)) {
    float* yn = A.y + size_t(n) * M * Fout;
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int tile = wave + t * kWaves;
      if (tile < ntiles) {
#pragma unroll
        for (int q = 0; q < NT; ++q) {
          const int f = q * 32 + li;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = tile * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (m < M && f < Fout) {
              float v = acc[t][q][r];
              if (A.res) v = v + A.res[size_t(n) * M * Fout + size_t(m) * Fout + f];
              if (A.act) v = v > 0.f ? v : 0.f;
              yn[size_t(m) * Fout + f] = v;
            }
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Backward (dx)
// ---------------------------------------------------------------------------
template <int RPT, int MAXNNZ, bool FIN1>
__global__ __launch_bounds__(kT) void cheb_bwd_resident(ResidentBwdArgs A) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int M = A.M, K = A.K, Fout = A.Fout, Mp = A.Mp, dbg = A.dbg;
  (void)dbg;
  const int Fin = FIN1 ? 1 : A.Fin;
  const int n = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, li = lane & 31;
  const int FinK = Fin * K;
  const int slab = Mp * 12;
  const int ws = Fout + 1;  // padded W row stride: the transposed B-operand read is conflict-free

  float* s_D = reinterpret_cast<float*>(smem);  // [FinK][Mp]
  size_t off = align16(size_t(FinK) * Mp * 4);
  char* s_G = smem + off;  // [Fin][Mp][3]
  off = align16(off + size_t(Fin) * slab);
  float* s_W = reinterpret_cast<float*>(smem + off);  // [FinK][Fout+1]

  const float* dyn = A.dy + size_t(n) * M * Fout;
  const int mtiles = (M + 31) >> 5, jtiles = (FinK + 31) >> 5;
  const int ns = (Fout + 1) >> 1;  // lane half h owns f in [h*ns, h*ns + ns)
  // Fast Phase-A operand path (config B/E shapes): each wave's <= 2 dy tiles
  // are loaded as float4 at kernel entry, so their HBM latency overlaps the
  // register / W prologue.
  const bool fastA =
      RPT == 1 && mtiles <= 2 * kWaves && jtiles == 1 && Fout <= 32 && (Fout & 7) == 0;
  float4 av[2][4];
  if constexpr (RPT == 1) {
    if (fastA) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int m = imin((wave + t * kWaves) * 32 + li, M - 1);
        const float4* rowp = reinterpret_cast<const float4*>(dyn + size_t(m) * Fout + h * ns);
#pragma unroll
        for (int c = 0; c < 4; ++c) av[t][c] = rowp[imin(c, (ns >> 2) - 1)];
      }
    }
  }

  RowRegs<RPT, MAXNNZ> rows;
  rows.load(A.E, tid, wave);
  for (int i = tid; i < FinK * Fout; i += kT) s_W[(i / Fout) * ws + (i % Fout)] = A.W[i];
  for (int i = tid; i < 3 * Fin; i += kT)
    lds_st(s_G + (i / 3) * slab + M * 12 + (i % 3) * 4, 0.f);
  __syncthreads();
  if (CG_DBG(dbg, 16)) return;

  // A. dBasis = dy W^T  (rows m, cols j = fin*K + k, inner f) on MFMA into LDS
  auto store_D = [&](const f32x16& acc, int mt, int j) {
    if (j < FinK) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mm = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (mm < M) s_D[j * Mp + mm] = acc[r];
      }
    }
  };
  if (!CG_DBG(dbg, 1)) {
    if (RPT == 1 && fastA) {
      const int j = li;
      const bool jv = j < FinK;
      const float* wrow = s_W + imin(j, FinK - 1) * ws + h * ns;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int mt = wave + t * kWaves;
        if (mt < mtiles) {
          const bool mv = mt * 32 + li < M;
          f32x16 acc;
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
          for (int s = 0; s < 16; ++s) {
            if (s < ns) acc = mfma32(mv ? av[t][s >> 2][s & 3] : 0.f, jv ? wrow[s] : 0.f, acc);
          }
          store_D(acc, mt, j);
        }
      }
    } else {
      for (int task = wave; task < mtiles * jtiles; task += kWaves) {
        const int mt = task / jtiles, jt = task - mt * jtiles;
        const int m = mt * 32 + li, j = jt * 32 + li;
        const bool mv = m < M, jv = j < FinK;
        const float* dyrow = dyn + size_t(imin(m, M - 1)) * Fout;
        const float* wrow = s_W + imin(j, FinK - 1) * ws;
        f32x16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
        for (int s0 = 0; s0 < ns; s0 += 8) {
          float a[8], b[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {  // 8 independent loads in flight
            const int fc = imin(h * ns + s0 + u, Fout - 1);
            a[u] = dyrow[fc];
            b[u] = wrow[fc];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const bool fv = (s0 + u) < ns && (h * ns + s0 + u) < Fout;
            acc = mfma32((mv && fv) ? a[u] : 0.f, (jv && fv) ? b[u] : 0.f, acc);
          }
        }
        store_D(acc, mt, j);
      }
    }
  }
  __syncthreads();

  // B. reverse recurrence over L~^T; step i = K-1-k writes ring slot i mod 3.
  auto step = [&](auto cur_c, auto nx1_c, auto nx2_c, int i) {
    constexpr int CUR = decltype(cur_c)::value, NX1 = decltype(nx1_c)::value,
                  NX2 = decltype(nx2_c)::value;
    const int k = K - 1 - i;
    const float c = (k >= 1) ? 2.f : 1.f;
    for (int fin = 0; fin < Fin; ++fin) {
      char* Gb = s_G + (FIN1 ? 0 : fin * slab);
      const float* Dk = s_D + (fin * K + k) * Mp;
#pragma unroll
      for (int q = 0; q < RPT; ++q) {
        const int r = rows.row[q];
        if (r >= 0) {
          char* rp = Gb + rows.rb[q];
          const float a = (i >= 1) ? (CG_DBG(dbg, 2) ? lds_f(rp + NX1 * 4)
                                                : rows.template dot<NX1>(q, Gb, A.col, A.val))
                                   : 0.f;
          float g = Dk[r] + c * a;
          if (i >= 2) g = g - lds_f(rp + NX2 * 4);
          if (k == 0) {
            if (A.dx) {
              float* d = A.dx + (size_t(n) * M + r) * Fin + fin;
              *d = A.dx_acc ? *d + g : g;
            }
          } else {
            lds_st(rp + CUR * 4, g);
          }
        }
      }
    }
    if (k > 0) __syncthreads();
  };
  for (int i = 0; i < K; i += 3) {
    step(I<0>(), I<2>(), I<1>(), i);
    if (i + 1 < K) step(I<1>(), I<0>(), I<2>(), i + 1);
    if (i + 2 < K) step(I<2>(), I<1>(), I<0>(), i + 2);
  }
}

template <typename Kern>
hipError_t allow_big_lds(Kern k) {
  return hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                             hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
}

template <int RPT, int MAXNNZ, int NT, bool FIN1>
hipError_t launch_fwd_t(const ResidentGeom& g, int N, const ResidentFwdArgs& a, hipStream_t s) {
  static hipError_t attr = allow_big_lds(&cheb_fwd_resident<RPT, MAXNNZ, NT, FIN1>);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL((cheb_fwd_resident<RPT, MAXNNZ, NT, FIN1>), dim3(N), dim3(kT), g.fwd_lds, s,
                     a);
  return hipGetLastError();
}

template <int RPT, int MAXNNZ, bool FIN1>
hipError_t launch_bwd_t(const ResidentGeom& g, int N, const ResidentBwdArgs& a, hipStream_t s) {
  static hipError_t attr = allow_big_lds(&cheb_bwd_resident<RPT, MAXNNZ, FIN1>);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL((cheb_bwd_resident<RPT, MAXNNZ, FIN1>), dim3(N), dim3(kT), g.bwd_lds, s, a);
  return hipGetLastError();
}

}  // namespace

int resident_slot_width(int M, int max_row_nnz) {
  const int rpt = (M + kT - 1) / kT;
  if (max_row_nnz <= 16) return 16;
  return rpt == 1 ? 32 : 16;  // longer rows take the (rare) CSR tail loop
}

ResidentGeom resident_geometry(int M, int nnz, int max_row_nnz, int max_row_nnzT, int Fin, int K,
                               int Fout) {
  ResidentGeom g{};
  g.nnz = nnz;
  const int Mp = lds_vertex_stride(M);
  g.rpt = (M + kT - 1) / kT;
  g.nt = (Fout + 31) / 32;
  g.maxnnz = resident_slot_width(M, max_row_nnz);
  g.maxnnzT = resident_slot_width(M, max_row_nnzT);
  const size_t FinK = size_t(Fin) * K;
  const size_t ring = align16(size_t(Fin) * Mp * 12);
  // The forward always stages the sample's basis in LDS (coalesced store at
  // the end); a shape whose basis block does not fit takes the streaming path.
  g.fwd_lds = align16(FinK * Fout * 4) + ring + size_t(M) * FinK * 4;
  g.stage = true;
  g.bwd_lds = align16(FinK * Mp * 4) + ring + FinK * (Fout + 1) * 4;
  const bool shape_ok = M >= 1 && nnz >= 1 && Fin >= 1 && K >= 1 && Fout >= 1 && g.rpt <= 2;
  // RPT=2 with two Fout tiles spills hundreds of VGPRs: leave it to the streaming path
  g.fwd_ok = shape_ok && g.nt <= 2 && !(g.rpt == 2 && g.nt == 2) &&
             !(g.rpt == 2 && g.maxnnz == 32) && g.fwd_lds <= size_t(kLdsBytes);
  g.bwd_ok = shape_ok && !(g.rpt == 2 && g.maxnnzT == 32) && g.bwd_lds <= size_t(kLdsBytes);
  return g;
}

hipError_t launch_resident_forward(const ResidentGeom& g, int N, const ResidentFwdArgs& a,
                                   hipStream_t s) {
  const bool f1 = a.Fin == 1;
#define CG_FWD(R_, Z_, NT_)                                 \
  if (g.rpt == R_ && g.maxnnz == Z_ && g.nt == NT_)         \
    return f1 ? launch_fwd_t<R_, Z_, NT_, true>(g, N, a, s) \
              : launch_fwd_t<R_, Z_, NT_, false>(g, N, a, s);
  CG_FWD(1, 16, 1) CG_FWD(1, 32, 1) CG_FWD(2, 16, 1) CG_FWD(1, 16, 2) CG_FWD(1, 32, 2)
#undef CG_FWD
  return hipErrorInvalidValue;
}

hipError_t launch_resident_backward(const ResidentGeom& g, int N, const ResidentBwdArgs& a,
                                    hipStream_t s) {
  const bool f1 = a.Fin == 1;
#define CG_BWD(R_, Z_)                  \
  if (g.rpt == R_ && g.maxnnzT == Z_)   \
    return f1 ? launch_bwd_t<R_, Z_, true>(g, N, a, s) : launch_bwd_t<R_, Z_, false>(g, N, a, s);
  CG_BWD(1, 16) CG_BWD(1, 32) CG_BWD(2, 16)
#undef CG_BWD
  return hipErrorInvalidValue;
}

}  // namespace cg
