// Wide-column streaming path of the Chebyshev graph convolution for gfx950:
// graphs too large for one CU's LDS (M > 1024) with few input features
// (Fin < 8), e.g. config C's first layer (M = 10 000, Fin = 1, N = 128).
//
// In the sample-major layout of cheb_stream.hip a Fin = 1 gather reads 4
// bytes and each lane walks its own CSR row (uncoalesced index loads).  Here
// the dense operand uses the reference's own layout X0 = [M][B], B = Fin*N,
// column b = fin*N + n (lib/graph_conv.py:155-157), so a gather of vertex c
// reads a contiguous run of B*4 bytes and a row's CSR entries are shared by
// the lanes that cover its columns:
//
//   k_sm_to_vm / k_vm_to_sm   [P][N][M*Fin] <-> [P][M*Fin][N] LDS-tiled
//                             transposes (x -> T_0, dBasis planes -> D_k,
//                             G_0 -> dx with optional accumulation)
//   k_wide_step               one Chebyshev step over all rows:
//                               forward   T_k = 2 L~ T_{k-1} - T_{k-2} (T_1 = L~ T_0)
//                               backward  G_k = D_k + c L~^T G_{k+1} - G_{k+2}
//                             LPR lanes per row (a power of 2 <= 64), PL floats per lane
//   k_wide_assemble           basis[n][m][fin*K + k] = T_k[m][fin*N + n]
//                             (lib/graph_conv.py:170-172), staged in LDS so
//                             each sample's run of rows leaves contiguously
//   k_wide_dypass             the backward's dense pass, ONE read of dy:
//                             D_k = (dy W^T) planes written directly in the
//                             [M][Fin*N] layout, and the dW = basis^T dy
//                             partial of every block, both on MFMA
//
// XCD-aware columns: the columns are cut into G <= 8 groups of CB >= 32 and
// block i works on group i mod G (blocks i and i + 8 share an XCD under
// round-robin placement -- speed only, never correctness), so each XCD
// gathers only its share of every row and its working set (C1: M * 128 B =
// 1.3 MB) stays in its own 4 MB L2: 84 % L2 hits on the C1 steps (r02g PMC).
//
// Numerics are those of cheb_stream.hip: each row accumulates sequentially in
// CSR order from +0 with fp contraction off (bit-exact basis), and the
// Clenshaw step applies its terms in the same order, so both streaming
// layouts give identical results.
#include "cg_internal.h"

namespace cg {
namespace {

template <int PL>
struct WV;
template <>
struct WV<1> {
  typedef float T;
  static __device__ __forceinline__ T ld(const float* p) { return *p; }
  static __device__ __forceinline__ void st(float* p, T v) { *p = v; }
  static __device__ __forceinline__ T zero() { return 0.f; }
  static __device__ __forceinline__ T fma_seq(T a, float w, T t) {
#pragma clang fp contract(off)
    return a + w * t;
  }
  static __device__ __forceinline__ T two_minus(T a, T p) {
#pragma clang fp contract(off)
    return 2.f * a - p;
  }
  static __device__ __forceinline__ T add_c(T d, float c, T a) {
#pragma clang fp contract(off)
    return d + c * a;
  }
  static __device__ __forceinline__ T sub(T a, T b) {
#pragma clang fp contract(off)
    return a - b;
  }
};
template <>
struct WV<2> {
  typedef float2 T;
  static __device__ __forceinline__ T ld(const float* p) { return *reinterpret_cast<const float2*>(p); }
  static __device__ __forceinline__ void st(float* p, T v) { *reinterpret_cast<float2*>(p) = v; }
  static __device__ __forceinline__ T zero() { return make_float2(0.f, 0.f); }
  static __device__ __forceinline__ T fma_seq(T a, float w, T t) {
#pragma clang fp contract(off)
    return make_float2(a.x + w * t.x, a.y + w * t.y);
  }
  static __device__ __forceinline__ T two_minus(T a, T p) {
#pragma clang fp contract(off)
    return make_float2(2.f * a.x - p.x, 2.f * a.y - p.y);
  }
  static __device__ __forceinline__ T add_c(T d, float c, T a) {
#pragma clang fp contract(off)
    return make_float2(d.x + c * a.x, d.y + c * a.y);
  }
  static __device__ __forceinline__ T sub(T a, T b) {
#pragma clang fp contract(off)
    return make_float2(a.x - b.x, a.y - b.y);
  }
};
template <>
struct WV<4> {
  typedef float4 T;
  static __device__ __forceinline__ T ld(const float* p) { return *reinterpret_cast<const float4*>(p); }
  static __device__ __forceinline__ void st(float* p, T v) { *reinterpret_cast<float4*>(p) = v; }
  static __device__ __forceinline__ T zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
  static __device__ __forceinline__ T fma_seq(T a, float w, T t) {
#pragma clang fp contract(off)
    return make_float4(a.x + w * t.x, a.y + w * t.y, a.z + w * t.z, a.w + w * t.w);
  }
  static __device__ __forceinline__ T two_minus(T a, T p) {
#pragma clang fp contract(off)
    return make_float4(2.f * a.x - p.x, 2.f * a.y - p.y, 2.f * a.z - p.z, 2.f * a.w - p.w);
  }
  static __device__ __forceinline__ T add_c(T d, float c, T a) {
#pragma clang fp contract(off)
    return make_float4(d.x + c * a.x, d.y + c * a.y, d.z + c * a.z, d.w + c * a.w);
  }
  static __device__ __forceinline__ T sub(T a, T b) {
#pragma clang fp contract(off)
    return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w);
  }
};

struct WideArgs {
  const int* rowptr;
  const int* col;
  const float* val;
  const int* rperm;  // row visiting order (degree-sorted) or NULL
  const float* Tp;   // gathered plane: T_{k-1} / G_{k+1} (NULL: the sum is +0)
  const float* Tpp;  // own-row plane T_{k-2} / G_{k+2} (NULL: none)
  const float* Dk;   // backward: own-row plane D_k
  float* out;        // T_k / G_k (may be Dk: same lane reads then writes)
  int M, B, CB, G;
  float c;   // backward coefficient (2 for k >= 1, 1 for k = 0)
  int mode;  // 0: T_1 = acc; 1: T_k = 2 acc - T_{k-2}; 2: G_k = D_k + c acc [- G_{k+2}]
};

// sum_{j in row r, CSR order} val[j] * Tp[col[j]][cb .. cb+PL), sequential
// from +0 with one rounding per product and per add (Tp NULL: +0)
template <int PL>
__device__ __forceinline__ typename WV<PL>::T wide_gather(const WideArgs& a, int r, int64_t cb) {
#pragma clang fp contract(off)
  typedef WV<PL> V;
  typename V::T acc = V::zero();
  if (a.Tp) {
    const int j0 = a.rowptr[r], j1 = a.rowptr[r + 1];
    const float* S = a.Tp + cb;
    int j = j0;
    // eight gathers in flight per lane (the rows average ~18 entries: a
    // step is bound by the gather latency, not by bandwidth), accumulated
    // strictly in CSR order
    for (; j + 8 <= j1; j += 8) {
      int c[8];
      float w[8];
      typename V::T t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        c[u] = a.col[j + u];
        w[u] = a.val[j + u];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = V::ld(S + int64_t(c[u]) * a.B);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = V::fma_seq(acc, w[u], t[u]);
    }
    if (j + 4 <= j1) {
      int c[4];
      float w[4];
      typename V::T t[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        c[u] = a.col[j + u];
        w[u] = a.val[j + u];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) t[u] = V::ld(S + int64_t(c[u]) * a.B);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc = V::fma_seq(acc, w[u], t[u]);
      j += 4;
    }
    for (; j < j1; ++j) acc = V::fma_seq(acc, a.val[j], V::ld(S + int64_t(a.col[j]) * a.B));
  }
  return acc;
}

// 256 threads = 4 waves; a wave holds 64/LPR rows, LPR = CB/PL lanes per row.
template <int PL>
__global__ __launch_bounds__(256) void k_wide_step(WideArgs a) {
#pragma clang fp contract(off)
  typedef WV<PL> V;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = blockIdx.x % a.G;
  const int rbk = blockIdx.x / a.G;
  const int lpr = a.CB / PL, rpw = 64 / lpr;
  const int sub = lane / lpr, lc = lane - sub * lpr;
  const int ri = (rbk * 4 + wave) * rpw + sub;
  if (ri >= a.M) return;
  const int r = a.rperm ? a.rperm[ri] : ri;
  const int64_t cb = int64_t(g) * a.CB + lc * PL;
  const int64_t own = int64_t(r) * a.B + cb;
  typename V::T acc = wide_gather<PL>(a, r, cb);
  typename V::T o;
  if (a.mode == 0) {
    o = acc;
  } else if (a.mode == 1) {
    o = V::two_minus(acc, V::ld(a.Tpp + own));
  } else {
    o = V::add_c(V::ld(a.Dk + own), a.c, acc);
    if (a.Tpp) o = V::sub(o, V::ld(a.Tpp + own));
  }
  V::st(a.out + own, o);
}

// The last forward step fused with the basis assembly (Fin == 1, natural row
// order): T_{K-1} of the block's rows x group columns (= samples) is computed
// as in k_wide_step, the own rows' T_0 .. T_{K-2} are read from their planes,
// and the [sample][row][k] block leaves through LDS as one contiguous run of
// rows*K floats per sample (lib/graph_conv.py:170-172); T_{K-1} itself is
// never stored.
template <int PL>
__global__ __launch_bounds__(256) void k_wide_last(WideArgs a, const float* __restrict__ planes,
                                                   int64_t plane, int K, float* __restrict__ basis) {
#pragma clang fp contract(off)
  typedef WV<PL> V;
  extern __shared__ float st[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = blockIdx.x % a.G;
  const int rbk = blockIdx.x / a.G;
  const int lpr = a.CB / PL, rpw = 64 / lpr, rows_b = 4 * rpw;
  const int sub = lane / lpr, lc = lane - sub * lpr;
  const int r0 = rbk * rows_b;
  const int rl = wave * rpw + sub;
  const int r = r0 + rl;
  const int SR = rows_b * K + 1;  // odd sample stride in LDS
  if (r < a.M) {
    const int64_t cb = int64_t(g) * a.CB + lc * PL;
    const int64_t own = int64_t(r) * a.B + cb;
    const typename V::T acc = wide_gather<PL>(a, r, cb);
    const typename V::T o = (a.mode == 0) ? acc : V::two_minus(acc, V::ld(a.Tpp + own));
    const float* ov = reinterpret_cast<const float*>(&o);
#pragma unroll
    for (int v = 0; v < PL; ++v) st[(lc * PL + v) * SR + rl * K + (K - 1)] = ov[v];
    for (int k = 0; k < K - 1; ++k) {
      const typename V::T t = V::ld(planes + k * plane + own);
      const float* tv = reinterpret_cast<const float*>(&t);
#pragma unroll
      for (int v = 0; v < PL; ++v) st[(lc * PL + v) * SR + rl * K + k] = tv[v];
    }
  }
  __syncthreads();
  const int nr = (a.M - r0 < rows_b) ? a.M - r0 : rows_b;
  if (nr <= 0) return;
  const int span = nr * K;
  for (int sidx = 0; sidx < a.CB; ++sidx) {
    const int n = g * a.CB + sidx;  // Fin == 1: column = sample
    float* dst = basis + (int64_t(n) * a.M + r0) * K;
    for (int e = threadIdx.x; e < span; e += 256) dst[e] = st[sidx * SR + e];
  }
}

// dst[p][q][n] = src[p][n][q], q < Q (= M*Fin), n < N: 32x32 tiles, +1 padding.
__global__ __launch_bounds__(256) void k_sm_to_vm(const float* __restrict__ src, int N, int64_t Q,
                                                  float* __restrict__ dst) {
  __shared__ float tile[32][33];
  const int64_t p = blockIdx.z;
  const int n0 = blockIdx.y * 32;
  const int64_t q0 = int64_t(blockIdx.x) * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const float* s = src + p * int64_t(N) * Q;
  float* d = dst + p * int64_t(N) * Q;
#pragma unroll
  for (int j = 0; j < 32; j += 8) {
    const int n = n0 + ty + j;
    const int64_t q = q0 + tx;
    tile[ty + j][tx] = (n < N && q < Q) ? s[int64_t(n) * Q + q] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 32; j += 8) {
    const int64_t q = q0 + ty + j;
    const int n = n0 + tx;
    if (n < N && q < Q) d[q * N + n] = tile[tx][ty + j];
  }
}

// dst[n][q] (+)= src[q][n]: the reverse re-layout (G_0 -> dx).
__global__ __launch_bounds__(256) void k_vm_to_sm(const float* __restrict__ src, int N, int64_t Q,
                                                  float* __restrict__ dst, int accumulate) {
#pragma clang fp contract(off)
  __shared__ float tile[32][33];
  const int n0 = blockIdx.y * 32;
  const int64_t q0 = int64_t(blockIdx.x) * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
  for (int j = 0; j < 32; j += 8) {
    const int64_t q = q0 + ty + j;
    const int n = n0 + tx;
    tile[ty + j][tx] = (n < N && q < Q) ? src[q * N + n] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 32; j += 8) {
    const int n = n0 + ty + j;
    const int64_t q = q0 + tx;
    if (n < N && q < Q) {
      float* o = dst + int64_t(n) * Q + q;
      const float v = tile[tx][ty + j];
      *o = accumulate ? *o + v : v;
    }
  }
}

// basis[n][m][fin*K + k] = T[k][m][fin*N + n] for a tile of TM rows x 32
// samples: gathered from the K planes with 32-lane (128-B) row reads into
// LDS [32 n][TM][FinK] (sample stride padded to an odd count), then each sample's TM*FinK contiguous floats leave
// with consecutive-lane stores.
__global__ __launch_bounds__(256) void k_wide_assemble(const float* __restrict__ T, int64_t plane,
                                                       int N, int M, int Fin, int K, int TM,
                                                       float* __restrict__ basis) {
  extern __shared__ float st[];
  const int FinK = Fin * K;
  const int n0 = blockIdx.x * 32;
  const int m0 = blockIdx.y * TM;
  const int B = Fin * N;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int rows = (M - m0 < TM) ? M - m0 : TM;
  const int nn = (N - n0 < 32) ? N - n0 : 32;
  const int SS = TM * FinK + 1;  // odd sample stride: the 32 lanes' writes hit 32 banks
  // read: (k, row, fin) triples over 8 thread rows, 32 samples per lane row
#pragma unroll 4
  for (int t = ty; t < K * rows * Fin; t += 8) {
    const int k = t / (rows * Fin);
    const int rem = t - k * rows * Fin;
    const int mm = rem / Fin, fin = rem - mm * Fin;
    if (tx < nn)
      st[tx * SS + mm * FinK + fin * K + k] =
          T[k * plane + int64_t(m0 + mm) * B + int64_t(fin) * N + n0 + tx];
  }
  __syncthreads();
  const int span = rows * FinK;
  for (int s = 0; s < nn; ++s) {
    float* dst = basis + (int64_t(n0 + s) * M + m0) * FinK;
    const float* src = st + s * SS;
    for (int e = threadIdx.x; e < span; e += 256) dst[e] = src[e];
  }
}

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void wave_sync_lds() {
  // LDS written by other lanes of this wave, read next: order + wait
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One wave-tile = 32 samples n0 + i of one vertex m (rows r = n*M + m).
// Lane (i, h) loads dy[n0+i][m][h*ns .. h*ns+ns) (ns = Fout/2, float4s):
//   D:  C[i][j] = sum_f dy[i][f] W[j][f]   (A = the loaded dy, B = W rows in
//       registers) -> LDS [j][i] -> plane k = j % K, columns fin*N + n0 + i
//       (j = fin*K + k): 128 contiguous bytes per (j, m)
//   dW: C[j][f] += sum_i basis[i][j] dy[i][f]   (A = basis from HBM, B = the
//       dy tile re-read from LDS in the lane = f layout)
// Persistent blocks of 4 waves; each block's dW partial (fixed-order sum of
// its waves) is one [FinK][Fout] slab.
__global__ __launch_bounds__(256) void k_wide_dypass(const float* __restrict__ dy,
                                                     const float* __restrict__ basis,
                                                     const float* __restrict__ W, int N, int M,
                                                     int Fin, int K, int Fout,
                                                     float* __restrict__ D, int64_t plane,
                                                     float* __restrict__ slab) {
  __shared__ float s_dy[4][32][33];
  __shared__ float s_d[4][32][33];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 31, h = lane >> 5;
  const int FinK = Fin * K, ns = Fout >> 1, B = Fin * N;
  // W rows for the D tile's B operand: lane (j, h) holds W[j][h*ns + s]
  float wr[16];
#pragma unroll
  for (int s = 0; s < 16; ++s)
    wr[s] = (li < FinK && s < ns) ? W[int64_t(li) * Fout + h * ns + s] : 0.f;
  f32x16 dacc;
#pragma unroll
  for (int e = 0; e < 16; ++e) dacc[e] = 0.f;
  const int ntn = (N + 31) >> 5;
  const int64_t ntiles = int64_t(M) * ntn;
  for (int64_t tile = int64_t(blockIdx.x) * 4 + wave; tile < ntiles; tile += int64_t(gridDim.x) * 4) {
    // consecutive tiles (a block's 4 waves, and neighbouring blocks) take
    // consecutive vertices of the same 32 samples: contiguous dy / basis runs
    const int nb = int(tile / M);
    const int m = int(tile - int64_t(nb) * M);
    const int n0 = nb * 32;
    const int ni = n0 + li;
    const bool nv = ni < N;
    // dy row (ni, m), this lane's half
    float a[16];
    {
      const float4* rowp = reinterpret_cast<const float4*>(
          dy + (int64_t(nv ? ni : N - 1) * M + m) * Fout + h * ns);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = (q * 4 < ns) ? rowp[q] : make_float4(0.f, 0.f, 0.f, 0.f);
        a[4 * q] = v.x;
        a[4 * q + 1] = v.y;
        a[4 * q + 2] = v.z;
        a[4 * q + 3] = v.w;
      }
    }
    // basis operands of the dW MFMAs: lane (j, h) takes rows 2u + h
    float bv[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int n = n0 + 2 * u + h;
      // basis == NULL: a dx-only call (no dW), the dW MFMAs run on zeros
      bv[u] = (basis && li < FinK && n < N) ? basis[(int64_t(n) * M + m) * FinK + li] : 0.f;
    }
    // the dy tile into LDS, [row][f]
#pragma unroll
    for (int s = 0; s < 16; ++s)
      if (s < ns) s_dy[wave][li][h * ns + s] = nv ? a[s] : 0.f;
    // D tile
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
    for (int s = 0; s < 16; ++s)
      if (s < ns) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(nv ? a[s] : 0.f, wr[s], acc, 0, 0, 0);
    wave_sync_lds();
    // dW: B operand lane (f, h) = dy[2u + h][f]
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const float b = (li < Fout) ? s_dy[wave][2 * u + h][li] : 0.f;
      dacc = __builtin_amdgcn_mfma_f32_32x32x2f32(bv[u], b, dacc, 0, 0, 0);
    }
    // D tile -> LDS [j][row] -> 128-B runs of plane k
#pragma unroll
    for (int e = 0; e < 16; ++e) s_d[wave][li][(e & 3) + 8 * (e >> 2) + 4 * h] = acc[e];
    wave_sync_lds();
    for (int j = h; j < FinK; j += 2) {
      const int fin = j / K, k = j - fin * K;
      if (nv) D[k * plane + int64_t(m) * B + int64_t(fin) * N + ni] = s_d[wave][j][li];
    }
    wave_sync_lds();  // s_dy / s_d are rewritten by the next tile
  }
  // block partial: waves added in a fixed order
  __syncthreads();
  float* part = &s_dy[0][0][0];  // [4][32][33] reused as [wave][j][f]
#pragma unroll
  for (int e = 0; e < 16; ++e) part[(wave * 32 + (e & 3) + 8 * (e >> 2) + 4 * h) * 33 + li] = dacc[e];
  __syncthreads();
  for (int idx = threadIdx.x; slab && idx < FinK * Fout; idx += 256) {
    const int j = idx / Fout, f = idx - j * Fout;
    float sum = part[(0 * 32 + j) * 33 + f];
    sum = sum + part[(1 * 32 + j) * 33 + f];
    sum = sum + part[(2 * 32 + j) * 33 + f];
    sum = sum + part[(3 * 32 + j) * 33 + f];
    slab[int64_t(blockIdx.x) * FinK * Fout + idx] = sum;
  }
}

// k_wide_dypass for FinK <= 8 (config C1: FinK = 5) on the VALU (the 32x32
// MFMA tiles of k_wide_dypass would be 84 % padding).  Same tiles (32 samples
// of one vertex) and data flow; the next tile's dy and basis loads are issued
// before the current tile is processed, W lives in registers and the basis
// tile is read back as 16-byte LDS broadcasts (per-element LDS reads of W and
// the basis made it LDS-instruction bound: r02i-k 89-98 us).  Per lane:
//   D:  lane (i, h) sums its half of f, the two halves are added across
//       lanes (xor 32), and lanes store j = h, h+2, ..
//   dW: lane (f, h) accumulates rows 2u + h: acc[j] += basis[row][j] dy[row][f];
//       halves, then waves, added in a fixed order.
struct DyTile {
  float a[16];
  float b[4];
};

__device__ __forceinline__ void dypass_load(const float* __restrict__ dy,
                                            const float* __restrict__ basis, int N, int M,
                                            int FinK, int Fout, int64_t tile, int li, int h,
                                            DyTile& t) {
  const int ns = Fout >> 1;
  const int nb = int(tile / M);
  const int m = int(tile - int64_t(nb) * M);
  const int ni = nb * 32 + li;
  const bool nv = ni < N;
  const float4* rowp =
      reinterpret_cast<const float4*>(dy + (int64_t(nv ? ni : N - 1) * M + m) * Fout + h * ns);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 v = (q * 4 < ns && nv) ? rowp[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    t.a[4 * q] = v.x;
    t.a[4 * q + 1] = v.y;
    t.a[4 * q + 2] = v.z;
    t.a[4 * q + 3] = v.w;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int j = 4 * h + q;
    t.b[q] = (basis && nv && j < FinK) ? basis[(int64_t(ni) * M + m) * FinK + j] : 0.f;
  }
}

template <int FJ>  // FJ = FinK (1..8), compile-time: W rows in FJ*16 registers
__global__ __launch_bounds__(256) void k_wide_dypass_small(const float* __restrict__ dy,
                                                           const float* __restrict__ basis,
                                                           const float* __restrict__ W, int N,
                                                           int M, int Fin, int K, int Fout,
                                                           float* __restrict__ D, int64_t plane,
                                                           float* __restrict__ slab) {
#pragma clang fp contract(off)
  __shared__ float s_dy[4][32][33];
  __shared__ __attribute__((aligned(16))) float s_b[4][32][8];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 31, h = lane >> 5;
  constexpr int FinK = FJ;
  const int ns = Fout >> 1, B = Fin * N;
  // W[j][h*ns + s] in registers (FinK <= 8, ns <= 16)
  float wr[FJ][16];
#pragma unroll
  for (int j = 0; j < FJ; ++j)
#pragma unroll
    for (int s = 0; s < 16; ++s)
      wr[j][s] = (s < ns) ? W[int64_t(j) * Fout + h * ns + s] : 0.f;
  float acc[FJ];
#pragma unroll
  for (int j = 0; j < FJ; ++j) acc[j] = 0.f;
  const int ntn = (N + 31) >> 5;
  const int64_t ntiles = int64_t(M) * ntn;
  const int64_t stride = int64_t(gridDim.x) * 4;
  int64_t tile = int64_t(blockIdx.x) * 4 + wave;
  DyTile cur, nxt;
  if (tile < ntiles) dypass_load(dy, basis, N, M, FinK, Fout, tile, li, h, cur);
  for (; tile < ntiles; tile += stride) {
    if (tile + stride < ntiles) dypass_load(dy, basis, N, M, FinK, Fout, tile + stride, li, h, nxt);
    const int nb = int(tile / M);
    const int m = int(tile - int64_t(nb) * M);
    const int ni = nb * 32 + li;
    const bool nv = ni < N;
#pragma unroll
    for (int s = 0; s < 16; ++s)
      if (s < ns) s_dy[wave][li][h * ns + s] = cur.a[s];
    *reinterpret_cast<float4*>(&s_b[wave][li][4 * h]) = make_float4(cur.b[0], cur.b[1], cur.b[2], cur.b[3]);
    // D: this lane's half of the f sum, then the other half's partial
    float d[FJ];
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      float t = 0.f;
#pragma unroll
      for (int s = 0; s < 16; ++s)
        if (s < ns) t = t + cur.a[s] * wr[j][s];
      d[j] = t;
    }
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const float o = __shfl_xor(d[j], 32);
      d[j] = h == 0 ? d[j] + o : o + d[j];  // the same sum on both halves
    }
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      if ((j & 1) == h && nv) {
        const int fin = j / K, k = j - fin * K;
        D[k * plane + int64_t(m) * B + int64_t(fin) * N + ni] = d[j];
      }
    }
    wave_sync_lds();
    // dW: lane (f, h), rows 2u + h of the tile
    if (li < Fout) {
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int row = 2 * u + h;
        const float g = s_dy[wave][row][li];
        const float4 b0 = *reinterpret_cast<const float4*>(&s_b[wave][row][0]);
        const float4 b1 = FinK > 4 ? *reinterpret_cast<const float4*>(&s_b[wave][row][4])
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
        const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[j] = acc[j] + bb[j] * g;
      }
    }
    wave_sync_lds();  // the tile buffers are rewritten next
    cur = nxt;
  }
  // halves (xor 32), then the 4 waves in a fixed order
#pragma unroll
  for (int j = 0; j < FJ; ++j) {
    const float o = __shfl_xor(acc[j], 32);
    acc[j] = h == 0 ? acc[j] + o : o + acc[j];
  }
  __syncthreads();
  float* part = &s_dy[0][0][0];  // [wave][j][f]
  if (h == 0) {
#pragma unroll
    for (int j = 0; j < FJ; ++j) part[(wave * 8 + j) * 32 + li] = acc[j];
  }
  __syncthreads();
  for (int idx = threadIdx.x; slab && idx < FinK * Fout; idx += 256) {
    const int j = idx / Fout, f = idx - j * Fout;
    float sum = part[(0 * 8 + j) * 32 + f];
    sum = sum + part[(1 * 8 + j) * 32 + f];
    sum = sum + part[(2 * 8 + j) * 32 + f];
    sum = sum + part[(3 * 8 + j) * 32 + f];
    slab[int64_t(blockIdx.x) * FinK * Fout + idx] = sum;
  }
}

inline int wide_tm(int FinK) {
  int tm = 8192 / (32 * FinK);  // <= 32 KB of LDS staging, <= 256 items per 8 thread rows
  if (tm > 32) tm = 32;
  return tm < 1 ? 1 : tm;
}

}  // namespace

WideGeom wide_geometry(int N, int Fin, int M) {
  WideGeom g{};
  const int64_t B = int64_t(N) * Fin;
  // column groups of >= 32 columns (a whole 128-B line per row-gather), at
  // most 8 (one per XCD): measured on C1 (r02g, B = 128) 4 groups x 32
  // columns beat 8 x 16 by 14 % (full-line requests; each XCD's slice is
  // still ~1.3 MB of its L2), and equal 2 x 64 / 1 x 128
  g.G = 1;
  for (int G = 8; G > 1; G >>= 1)
    if (B % (32 * G) == 0) {
      g.G = G;
      break;
    }
  const int Gd = debug_param(0, -1);  // ablation build: column groups override
  if (Gd > 0 && B % Gd == 0) g.G = Gd;
  g.CB = int(B / g.G);
  // widest per-lane vector whose lanes-per-row is a power of two <= 64: few
  // lanes per row = many rows (and their gathers) in flight per wave -- the
  // steps are bound by gather latency (C1: 16 columns per group -> 4 lanes x
  // float4, 16 rows per wave; r02e measured 17.7 us per step with 16 lanes x 1)
  g.pl = 0;
  for (int pl = debug_param(1, 4); pl >= 1; pl >>= 1) {  // (ablation build: widest pl override)
    if (g.CB % pl) continue;
    const int lpr = g.CB / pl;
    if (lpr >= 1 && lpr <= 64 && (lpr & (lpr - 1)) == 0) {
      g.pl = pl;
      break;
    }
  }
  g.ok = Fin >= 1 && Fin < 8 && M > 0 && B <= (int64_t(1) << 30) && g.pl > 0;
  g.rpb = g.ok ? 4 * (64 / (g.CB / g.pl)) : 0;
  return g;
}

hipError_t launch_wide_step(const WideGeom& g, const int* rowptr, const int* col, const float* val,
                            const int* rperm, const float* Tp, const float* Tpp, const float* Dk,
                            float* out, int M, int B, int mode, float c, hipStream_t s) {
  WideArgs a{rowptr, col, val, rperm, Tp, Tpp, Dk, out, M, B, g.CB, g.G, c, mode};
  const int64_t blocks = int64_t((M + g.rpb - 1) / g.rpb) * g.G;
  if (blocks > (int64_t(1) << 31) - 1) return hipErrorInvalidValue;
  const dim3 grid{unsigned(blocks)}, block{256};
  if (g.pl == 4) hipLaunchKernelGGL(k_wide_step<4>, grid, block, 0, s, a);
  else if (g.pl == 2) hipLaunchKernelGGL(k_wide_step<2>, grid, block, 0, s, a);
  else hipLaunchKernelGGL(k_wide_step<1>, grid, block, 0, s, a);
  return hipGetLastError();
}

bool wide_last_ok(const WideGeom& g, int Fin, int K, bool rperm) {
  const int rows_b = 4 * (64 / (g.CB / g.pl));
  return g.ok && Fin == 1 && !rperm && K >= 2 &&
         (size_t(g.CB) * (rows_b * K + 1)) * sizeof(float) <= size_t(64) * 1024;
}

hipError_t launch_wide_last(const WideGeom& g, const int* rowptr, const int* col, const float* val,
                            const float* planes, int64_t plane, float* basis, int M, int N, int K,
                            hipStream_t s) {
  if (!wide_last_ok(g, 1, K, false)) return hipErrorInvalidValue;
  const int k = K - 1;
  WideArgs a{rowptr, col, val, nullptr, planes + (k - 1) * plane,
             k >= 2 ? planes + (k - 2) * plane : nullptr, nullptr, nullptr, M, N, g.CB, g.G, 2.f,
             k == 1 ? 0 : 1};
  const int rows_b = 4 * (64 / (g.CB / g.pl));
  const size_t lds = size_t(g.CB) * (rows_b * K + 1) * sizeof(float);
  const int64_t blocks = int64_t((M + g.rpb - 1) / g.rpb) * g.G;
  const dim3 grid{unsigned(blocks)}, block{256};
  if (g.pl == 4) hipLaunchKernelGGL(k_wide_last<4>, grid, block, lds, s, a, planes, plane, K, basis);
  else if (g.pl == 2) hipLaunchKernelGGL(k_wide_last<2>, grid, block, lds, s, a, planes, plane, K, basis);
  else hipLaunchKernelGGL(k_wide_last<1>, grid, block, lds, s, a, planes, plane, K, basis);
  return hipGetLastError();
}

hipError_t launch_sm_to_vm(const float* src, int P, int N, int64_t Q, float* dst, hipStream_t s) {
  if ((Q + 31) / 32 > (int64_t(1) << 31) - 1 || P > 65535 || (N + 31) / 32 > 65535)
    return hipErrorInvalidValue;
  const dim3 grid(unsigned((Q + 31) / 32), unsigned((N + 31) / 32), unsigned(P));
  hipLaunchKernelGGL(k_sm_to_vm, grid, dim3(256), 0, s, src, N, Q, dst);
  return hipGetLastError();
}

hipError_t launch_vm_to_sm(const float* src, int N, int64_t Q, float* dst, int accumulate,
                           hipStream_t s) {
  if ((Q + 31) / 32 > (int64_t(1) << 31) - 1 || (N + 31) / 32 > 65535) return hipErrorInvalidValue;
  const dim3 grid(unsigned((Q + 31) / 32), unsigned((N + 31) / 32));
  hipLaunchKernelGGL(k_vm_to_sm, grid, dim3(256), 0, s, src, N, Q, dst, accumulate);
  return hipGetLastError();
}

bool wide_dypass_ok(int FinK, int Fout) {
  return FinK >= 1 && FinK <= 32 && Fout >= 8 && Fout <= 32 && Fout % 8 == 0;
}

int wide_dypass_blocks(int N, int M) {
  const int64_t tiles = int64_t(M) * ((N + 31) / 32);
  int64_t b = (tiles + 15) / 16;  // >= 4 wave-tiles per wave
  if (b > 2048) b = 2048;         // 8 blocks (32 waves) per CU
  return int(b < 1 ? 1 : b);
}

hipError_t launch_wide_dypass(const float* dy, const float* basis, const float* W, int N, int M,
                              int Fin, int K, int Fout, float* D, int64_t plane, float* slab,
                              hipStream_t s) {
  if (!wide_dypass_ok(Fin * K, Fout)) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(dy) & 15) != 0) return hipErrorInvalidValue;
  const dim3 grid(wide_dypass_blocks(N, M));
  switch (Fin * K) {
#define CG_DP(FJ_)                                                                              \
  case FJ_:                                                                                     \
    hipLaunchKernelGGL(k_wide_dypass_small<FJ_>, grid, dim3(256), 0, s, dy, basis, W, N, M, Fin, K, \
                       Fout, D, plane, slab);                                                    \
    return hipGetLastError();
    CG_DP(1) CG_DP(2) CG_DP(3) CG_DP(4) CG_DP(5) CG_DP(6) CG_DP(7) CG_DP(8)
#undef CG_DP
    default:
      break;
  }
  hipLaunchKernelGGL(k_wide_dypass, grid, dim3(256), 0, s, dy, basis, W, N, M, Fin, K, Fout, D, plane,
                     slab);
  return hipGetLastError();
}

hipError_t launch_wide_assemble(const float* T, int64_t plane, int N, int M, int Fin, int K,
                                float* basis, hipStream_t s) {
  const int tm = wide_tm(Fin * K);
  const size_t lds = (size_t(32) * tm * Fin * K + 32) * sizeof(float);
  if (lds > size_t(64) * 1024 || (M + tm - 1) / tm > 65535) return hipErrorInvalidValue;
  const dim3 grid(unsigned((N + 31) / 32), unsigned((M + tm - 1) / tm));
  hipLaunchKernelGGL(k_wide_assemble, grid, dim3(256), lds, s, T, plane, N, M, Fin, K, tm, basis);
  return hipGetLastError();
}

}  // namespace cg
