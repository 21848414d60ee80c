// C ABI of libcheb_mi355.so (see include/cheb_mi355.h): plan management,
// argument validation, workspace layout and kernel-path dispatch.
#include "../../include/cheb_mi355.h"
#include "../../include/cheb_mi355_testing.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "cg_internal.h"

#ifdef CG_DEBUG
namespace cg {
int g_debug_flags = 0;
int g_debug_params[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
unsigned long long* g_debug_ts = nullptr;
}
#endif

struct cg_plan {
  int device = 0;
  int M = 0;
  int64_t nnz = 0, nnzT = 0;
  int max_row_nnz = 0, max_row_nnzT = 0;
  int path = CG_PATH_AUTO;
  int variant = CG_VARIANT_AUTO;
  int* rowptr = nullptr;
  int* col = nullptr;
  float* val = nullptr;
  int* trowptr = nullptr;
  int* tcol = nullptr;
  float* tval = nullptr;
  // degree-sorted row orders of L~ / L~^T (longest rows first), used by the
  // streaming steps on skewed (power-law) graphs so a wave's rows have similar
  // lengths; null when the row lengths are near-uniform
  int* rperm = nullptr;
  int* trperm = nullptr;
  // rows of L~ / L~^T by decreasing length, always present: the LDS-resident
  // kernels deal rows to lanes in this order so a wave's rows have (nearly)
  // equal lengths and its unrolled gather loop has no idle entries
  int* lorder = nullptr;
  int* tlorder = nullptr;
  // thread-slot images of L~ and L~^T for the resident kernels (M <= 2048)
  struct Slots {
    int* buf = nullptr;  // one allocation: row | len | beg | col | val | wlen
    cg::SlotLayout view{};
  } slots, tslots;
  // images of L~ and L~^T for the fast resident kernels (cheb_fast.hip)
  struct Fast {
    void* buf = nullptr;
    cg::FastImage view{};
    bool ok = false;  // max row length <= cg::kFastWidth and M <= 1024
    long gather_cycles = 0, gather_ideal = 0;  // modelled LDS cycles per step
  } fast, tfast;
  // the gconv-LSTM sequence launches' sticky fault word: host-mapped pinned
  // memory the kernel writes (system scope) when a pair hand-off times out,
  // read by cg_lstm_seq_fault without a device copy once seq_event (recorded
  // behind every sequence launch) has completed
  int* seq_fault = nullptr;      // host pointer
  int* seq_fault_dev = nullptr;  // its device alias
  hipEvent_t seq_event = nullptr;
  bool seq_launched = false;
  // test hook (cg_plan_set_seq_fault_test): >= 0 makes workgroup 0 of pair 0
  // of this plan's sequence launches stop publishing its step counter from
  // that step on; -1 (default) off
  int seq_fault_test = -1;
};

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int ok() {
  g_err.clear();
  return CG_OK;
}

#define CG_HIP(call)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (call);                                                                 \
    if (e_ != hipSuccess) return fail(CG_ERR_HIP, "%s: %s", #call, hipGetErrorString(e_)); \
  } while (0)

// Validates a host CSR: rowptr[0] = 0, non-decreasing, rowptr[M] = nnz,
// columns in [0, M) strictly increasing inside each row (canonical order,
// what tf.sparse_reorder produces at lib/graph_conv.py:153).
int check_csr(const char* what, int32_t M, int64_t nnz, const int32_t* rowptr, const int32_t* col,
              const float* val) {
  if (!rowptr || (nnz > 0 && (!col || !val))) return fail(CG_ERR_ARG, "%s: null CSR array", what);
  if (rowptr[0] != 0 || rowptr[M] != nnz)
    return fail(CG_ERR_ARG, "%s: rowptr[0]=%d rowptr[M]=%d nnz=%lld", what, rowptr[0], rowptr[M],
                (long long)nnz);
  for (int32_t r = 0; r < M; ++r) {
    if (rowptr[r + 1] < rowptr[r]) return fail(CG_ERR_ARG, "%s: rowptr decreases at row %d", what, r);
    for (int32_t j = rowptr[r]; j < rowptr[r + 1]; ++j) {
      if (col[j] < 0 || col[j] >= M)
        return fail(CG_ERR_ARG, "%s: column %d out of range at nnz %d", what, col[j], j);
      if (j > rowptr[r] && col[j] <= col[j - 1])
        return fail(CG_ERR_ARG, "%s: columns not strictly increasing in row %d", what, r);
    }
  }
  return CG_OK;
}

// Exact transpose (counting sort by column; rows come out in increasing order,
// so columns of the transpose are sorted).
void transpose_csr(int32_t M, int64_t nnz, const int32_t* rp, const int32_t* ci, const float* v,
                   std::vector<int32_t>& trp, std::vector<int32_t>& tci, std::vector<float>& tv) {
  trp.assign(size_t(M) + 1, 0);
  tci.resize(size_t(nnz));
  tv.resize(size_t(nnz));
  for (int64_t j = 0; j < nnz; ++j) trp[size_t(ci[j]) + 1]++;
  for (int32_t r = 0; r < M; ++r) trp[size_t(r) + 1] += trp[size_t(r)];
  std::vector<int32_t> fill(trp.begin(), trp.end() - 1);
  for (int32_t r = 0; r < M; ++r)
    for (int32_t j = rp[r]; j < rp[r + 1]; ++j) {
      const int32_t dst = fill[size_t(ci[j])]++;
      tci[size_t(dst)] = r;
      tv[size_t(dst)] = v[j];
    }
}

// Thread-slot ELL image of a CSR operand for the resident kernels
// (cg_internal.h::SlotLayout).  Rows are dealt to thread slots in order of
// decreasing length (stable), so the 64 rows of a wave have nearly equal
// length and the kernel can skip whole gather instructions past the wave's
// maximum; the ELL arrays are column-major so each prologue load is one
// coalesced 256-byte wave access.
int build_slots(cg_plan::Slots* out, int32_t M, const int32_t* rp, const int32_t* ci,
                const float* v) {
  constexpr int kT = cg::kResidentThreads, kW = kT / 64;
  const int rpt = (M + kT - 1) / kT;
  if (rpt > 2) return CG_OK;  // resident path not available: no image
  int maxlen = 0;
  for (int32_t r = 0; r < M; ++r) maxlen = std::max(maxlen, rp[r + 1] - rp[r]);
  const int width = cg::resident_slot_width(M, maxlen);
  const int S = rpt * kT;
  std::vector<int32_t> order(static_cast<size_t>(M));
  for (int32_t r = 0; r < M; ++r) order[size_t(r)] = r;
  std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
    return (rp[a + 1] - rp[a]) > (rp[b + 1] - rp[b]);
  });
  // slot t = q*kT + tid: deal sorted rows tid-major inside each slot group
  std::vector<int32_t> row(size_t(S), -1), len(size_t(S), 0), beg(size_t(S), 0);
  std::vector<int32_t> col(size_t(width) * S, M), wlen(size_t(rpt) * kW, 0);
  std::vector<float> val(size_t(width) * S, 0.f);
  for (int32_t i = 0; i < M; ++i) {
    const int32_t r = order[size_t(i)];
    const int t = i;  // group q = i / kT, tid = i % kT
    row[size_t(t)] = r;
    len[size_t(t)] = rp[r + 1] - rp[r];
    beg[size_t(t)] = rp[r];
    for (int j = 0; j < std::min(width, len[size_t(t)]); ++j) {
      col[size_t(j) * S + t] = ci[rp[r] + j];
      val[size_t(j) * S + t] = v[rp[r] + j];
    }
    const int w = (t / kT) * kW + (t % kT) / 64;
    wlen[size_t(w)] = std::max(wlen[size_t(w)], len[size_t(t)]);
  }
  const size_t n_int = 3 * size_t(S) + size_t(width) * S + size_t(width) * S + wlen.size();
  int* d = nullptr;
  CG_HIP(hipMalloc(reinterpret_cast<void**>(&d), n_int * 4));
  size_t o = 0;
  auto put = [&](const void* src, size_t count) -> int {
    CG_HIP(hipMemcpy(d + o, src, count * 4, hipMemcpyHostToDevice));
    o += count;
    return CG_OK;
  };
  int rc = put(row.data(), row.size());
  if (!rc) rc = put(len.data(), len.size());
  if (!rc) rc = put(beg.data(), beg.size());
  if (!rc) rc = put(col.data(), col.size());
  if (!rc) rc = put(val.data(), val.size());
  if (!rc) rc = put(wlen.data(), wlen.size());
  if (rc) {
    (void)hipFree(d);
    return rc;
  }
  out->buf = d;
  cg::SlotLayout& e = out->view;
  e.S = S;
  e.width = width;
  e.row = d;
  e.len = d + S;
  e.beg = d + 2 * size_t(S);
  e.col = d + 3 * size_t(S);
  e.val = reinterpret_cast<const float*>(d + 3 * size_t(S) + size_t(width) * S);
  e.wlen = d + 3 * size_t(S) + 2 * size_t(width) * S;
  return CG_OK;
}

// Image of a CSR operand for the fast resident kernels (cg_internal.h::
// FastImage): thread->row assignment and bank-aware record layout from
// lds_layout.cpp, uploaded as one device allocation.
int build_fast_image(cg_plan::Fast* out, int32_t M, const int32_t* rp, const int32_t* ci,
                     const float* v, cg::FastLayout* keep = nullptr, const cg::FastLayout* reuse = nullptr) {
  constexpr int kT = 1024, kWd = cg::kFastWidth;
  if (M > kT) return CG_OK;
  int maxlen = 0;
  for (int32_t r = 0; r < M; ++r) maxlen = std::max(maxlen, rp[r + 1] - rp[r]);
  if (maxlen > kWd) return CG_OK;
  cg::FastLayout lay;
  if (reuse) lay = *reuse;  // the same sparsity pattern: the same layout
  else cg::plan_fast_layout(M, rp, ci, &lay);
  if (keep) *keep = lay;
  std::vector<float> val(size_t(kWd) * kT, 0.f);
  for (int t = 0; t < kT; ++t) {
    const int r = lay.row[size_t(t)];
    if (r < 0) continue;
    for (int j = 0; j < rp[r + 1] - rp[r]; ++j) val[size_t(j) * kT + t] = v[rp[r] + j];
  }
  // gather records packed two per word (record indices < 2^16): the per-thread
  // image the fast kernels load in their prologue is 8 words smaller
  if (lay.P >= 65536) return CG_OK;  // (never for M <= 1024: P ~ 2M + 66)
  std::vector<int> cpos2(size_t(kWd / 2) * kT);
  for (int j2 = 0; j2 < kWd / 2; ++j2)
    for (int t = 0; t < kT; ++t)
      cpos2[size_t(j2) * kT + t] = int(uint32_t(lay.cpos[size_t(2 * j2) * kT + t]) |
                                       (uint32_t(lay.cpos[size_t(2 * j2 + 1) * kT + t]) << 16));
  const std::vector<int>* ints[] = {&lay.row, &lay.rpos0, &lay.rpos1, &lay.rposr, &cpos2,
                                    &lay.wlen, &lay.mpos, &lay.pos0, &lay.pos1};
  size_t bytes = val.size() * 4;
  for (const auto* a : ints) bytes += a->size() * 4;
  char* d = nullptr;
  CG_HIP(hipMalloc(reinterpret_cast<void**>(&d), bytes));
  out->buf = d;
  size_t o = 0;
  bool okc = true;
  auto put = [&](const void* src, size_t count) -> const void* {
    const void* at = d + o;
    if (hipMemcpy(d + o, src, count * 4, hipMemcpyHostToDevice) != hipSuccess) okc = false;
    o += count * 4;
    return at;
  };
  cg::FastImage& e = out->view;
  e.row = static_cast<const int*>(put(lay.row.data(), lay.row.size()));
  e.rpos = static_cast<const int*>(put(lay.rpos0.data(), lay.rpos0.size()));
  e.rpos1 = static_cast<const int*>(put(lay.rpos1.data(), lay.rpos1.size()));
  e.rposr = static_cast<const int*>(put(lay.rposr.data(), lay.rposr.size()));
  e.cpos = static_cast<const int*>(put(cpos2.data(), cpos2.size()));
  e.val = static_cast<const float*>(put(val.data(), val.size()));
  e.wlen = static_cast<const int*>(put(lay.wlen.data(), lay.wlen.size()));
  e.mpos = static_cast<const int*>(put(lay.mpos.data(), lay.mpos.size()));
  e.pos0 = static_cast<const int*>(put(lay.pos0.data(), lay.pos0.size()));
  e.pos1 = static_cast<const int*>(put(lay.pos1.data(), lay.pos1.size()));
  e.zpos = lay.zero_base;
  e.P = lay.P;
  if (!okc) return fail(CG_ERR_HIP, "build_fast_image: hipMemcpy failed");
  out->gather_cycles = lay.gather_cycles;
  out->gather_ideal = lay.gather_ideal;
  out->ok = true;
  return CG_OK;
}

template <typename T>
int upload(T** dst, const T* src, size_t count) {
  *dst = nullptr;
  const size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
  CG_HIP(hipMalloc(reinterpret_cast<void**>(dst), bytes));
  if (count) CG_HIP(hipMemcpy(*dst, src, count * sizeof(T), hipMemcpyHostToDevice));
  return CG_OK;
}

void free_plan(cg_plan* p) {
  if (!p) return;
  void* ptrs[] = {p->rowptr, p->col, p->val, p->trowptr, p->tcol, p->tval, p->rperm, p->trperm,
                  p->lorder, p->tlorder};
  for (void* q : ptrs)
    if (q) (void)hipFree(q);
  if (p->slots.buf) (void)hipFree(p->slots.buf);
  if (p->tslots.buf) (void)hipFree(p->tslots.buf);
  if (p->fast.buf) (void)hipFree(p->fast.buf);
  if (p->tfast.buf) (void)hipFree(p->tfast.buf);
  if (p->seq_event) (void)hipEventDestroy(p->seq_event);
  if (p->seq_fault) (void)hipHostFree(p->seq_fault);
  delete p;
}

int check_device(const cg_plan* p) {
  int d = -1;
  CG_HIP(hipGetDevice(&d));
  if (d != p->device)
    return fail(CG_ERR_ARG, "current HIP device %d differs from the plan's device %d", d,
                p->device);
  return CG_OK;
}

int check_shape(const cg_plan* p, int32_t N, int32_t Fin, int32_t K, int32_t Fout) {
  if (!p) return fail(CG_ERR_ARG, "null plan");
  if (N < 1 || Fin < 1 || K < 1 || Fout < 1)
    return fail(CG_ERR_ARG, "bad shape N=%d Fin=%d K=%d Fout=%d", N, Fin, K, Fout);
  if (int64_t(N) * p->M >= (int64_t(1) << 31) || int64_t(N) * Fin >= (int64_t(1) << 31))
    return fail(CG_ERR_ARG, "N*M or N*Fin exceeds 2^31");
  return CG_OK;
}

// CG_VARIANT_CLASSIC runs the classic resident kernels (cheb_resident.hip)
// where the fast ones (cheb_fast.hip) would; CG_VARIANT_UNFUSED_DW keeps the
// fast kernels but computes dW with the separate streaming GEMM.
cg::FastGeom fast_geom(const cg_plan* p, int32_t Fin, int32_t K, int32_t Fout) {
  return cg::fast_geometry(p->M, p->fast.view.P, p->max_row_nnz, p->max_row_nnzT, Fin, K, Fout);
}

bool use_fast(const cg_plan* p, int32_t Fin, int32_t K, int32_t Fout, bool backward) {
  if (p->variant == CG_VARIANT_CLASSIC) return false;
  if (!(backward ? p->tfast.ok : p->fast.ok)) return false;
  const cg::FastGeom g = fast_geom(p, Fin, K, Fout);
  return backward ? g.bwd_ok : g.fwd_ok;
}

bool fused_dw(const cg_plan* p, int32_t Fin, int32_t K, int32_t Fout) {
  return use_fast(p, Fin, K, Fout, true) && fast_geom(p, Fin, K, Fout).dw_fused &&
         p->variant != CG_VARIANT_UNFUSED_DW;
}

int choose_path(const cg_plan* p, int32_t Fin, int32_t K, int32_t Fout, bool backward,
                int* path) {
  const cg::ResidentGeom g = cg::resident_geometry(p->M, int(p->nnz), p->max_row_nnz, p->max_row_nnzT, Fin, K, Fout);
  const bool fits = use_fast(p, Fin, K, Fout, backward) || (backward ? g.bwd_ok : g.fwd_ok);
  if (p->path == CG_PATH_STREAM) {
    *path = CG_PATH_STREAM;
  } else if (p->path == CG_PATH_RESIDENT) {
    if (!fits)
      return fail(CG_ERR_UNSUPPORTED,
                  "resident path does not fit: M=%d nnz=%lld Fin=%d K=%d Fout=%d (lds fwd %zu / "
                  "bwd %zu bytes)",
                  p->M, (long long)p->nnz, Fin, K, Fout, g.fwd_lds, g.bwd_lds);
    *path = CG_PATH_RESIDENT;
  } else {
    *path = fits ? CG_PATH_RESIDENT : CG_PATH_STREAM;
  }
  return CG_OK;
}

inline size_t al256(size_t b) { return (b + 255) & ~size_t(255); }

// Basis layouts (cheb_mi355.h): CG_BASIS_ROWS [N*M][Fin*K] (lib/graph_conv.py:172)
// on every path; CG_BASIS_ORDERS [N][Fin*K][Mb] (Mb = M rounded up to 32) where
// the fast forward stores it during the recurrence and the fused-dW fast
// backward reads it back.
inline int32_t basis_mb(int32_t M) { return (M + 31) & ~31; }

int check_layout(const cg_plan* p, int32_t Fin, int32_t K, int32_t Fout, int layout) {
  if (layout == CG_BASIS_ROWS) return CG_OK;
  if (layout == CG_BASIS_PLANES) {
    // the sample-major streaming path both ways (Fin >= 16 never takes the
    // wide-column layout), planes whose 16-float chunks the row GEMM loads
    int pf = 0, pb = 0;
    const bool ok = Fin % 16 == 0 && K >= 2 && !choose_path(p, Fin, K, Fout, false, &pf) &&
                    !choose_path(p, Fin, K, Fout, true, &pb) && pf == CG_PATH_STREAM &&
                    pb == CG_PATH_STREAM && cg::rowgemm_ok(Fin * K, Fin * K, Fout);
    if (!ok)
      return fail(CG_ERR_UNSUPPORTED,
                  "planes basis layout needs the sample-major streaming path forward and "
                  "backward, Fin a multiple of 16 and K >= 2 (M=%d Fin=%d K=%d Fout=%d)",
                  p->M, Fin, K, Fout);
    return CG_OK;
  }
  if (layout != CG_BASIS_ORDERS) return fail(CG_ERR_ARG, "unknown basis layout %d", layout);
  // the fast forward without the basis staging (so it also serves shapes whose
  // staged basis would not fit in LDS) and the fused-dW fast backward
  if (Fin > 2 || p->path == CG_PATH_STREAM || p->variant == CG_VARIANT_CLASSIC || !p->fast.ok ||
      !fast_geom(p, Fin, K, Fout).fwd_ok_ob || !fused_dw(p, Fin, K, Fout))
    return fail(CG_ERR_UNSUPPORTED,
                "orders basis layout needs Fin <= 2, the fast resident forward and the "
                "fused-dW fast backward (M=%d Fin=%d K=%d Fout=%d)",
                p->M, Fin, K, Fout);
  return CG_OK;
}

struct StreamWs {
  bool wide;     // wide-column layout (cheb_wide.hip) for small Fin
  size_t slots;  // forward: T_1 .. T_{K-2} (sample-major), or the K planes T_0 .. T_{K-1} ([M][B], wide)
  size_t dA;     // backward: dBasis, N*M*FinK floats (k-major); G_k overwrites plane k
                 // (wide: + the same again for the [K][M][B] planes D_k / G_k)
};

// The wide-column path serves the streaming path when Fin < 8 (sample-major
// gathers of Fin*4 < 32 bytes) and its column split fits (cheb_wide.hip).
bool use_wide(const cg_plan* p, int32_t N, int32_t Fin, int32_t K) {
  return p->variant != CG_VARIANT_NARROW && int64_t(Fin) * K <= 256 &&
         cg::wide_geometry(N, Fin, p->M).ok;
}

StreamWs stream_ws(const cg_plan* p, int32_t N, int32_t Fin, int32_t K, int32_t Fout) {
  StreamWs w{};
  const int64_t B = int64_t(N) * Fin;
  const int64_t FinK = int64_t(Fin) * K;
  const int64_t NM = int64_t(N) * p->M;
  w.wide = use_wide(p, N, Fin, K);
  const size_t plane = size_t(p->M) * size_t(B) * 4;
  w.slots = al256(w.wide ? size_t(K) * plane : size_t(K > 2 ? K - 2 : 0) * plane);
  w.dA = al256(size_t(NM) * size_t(FinK) * 4);
  // wide: the [K][M][B] planes D_k / G_k (+ the sample-major dBasis when the
  // fused dy pass does not apply)
  if (w.wide) w.dA = al256(size_t(K) * plane) + (cg::wide_dypass_ok(int(FinK), Fout) ? 0 : w.dA);
  (void)Fout;
  return w;
}

// dW partial slabs: dw_chunks(R) of them from k_dw_slabs, or one per sample
// from the fused backward.
// M > 0: the wide path's fused dy pass writes the slabs (one per block)
size_t dw_slab_bytes(int64_t R, int32_t N, int FinK, int Fout, int32_t M = 0) {
  size_t n = std::max<size_t>(size_t(cg::dw_chunks(R)), size_t(N));
  if (M > 0) n = std::max<size_t>(n, size_t(cg::wide_dypass_blocks(N, M)));
  return al256(n * size_t(FinK) * size_t(Fout) * 4);
}

// Channel-group resident kernels (cheb_group.hip) serve the sample-major
// streaming path for M <= 1024, Fin % 8 == 0 (forward: planes layout only).
bool use_group(const cg_plan* p, int32_t Fin, int32_t K, int32_t Fout) {
  return p->variant != CG_VARIANT_STEPS && p->variant != CG_VARIANT_NARROW &&
         cg::grp_ok(p->M, std::max(p->nnz, p->nnzT), Fin, K, Fout);
}

// Workspace layout.  forward: [T_1 .. T_{K-2}] (streaming path only).
// backward: [dW slabs][dBasis] (dBasis for the streaming path only; the
// reverse recurrence writes G_k over plane k of it, so it needs no ring).
// The forward's workspace is dead once the forward has returned, so one
// buffer of max(fwd, bwd) bytes may serve both.
int workspace_bytes(const cg_plan* p, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                    size_t* fwd, size_t* bwd) {
  int pf = 0, pb = 0, rc;
  if ((rc = choose_path(p, Fin, K, Fout, false, &pf))) return rc;
  if ((rc = choose_path(p, Fin, K, Fout, true, &pb))) return rc;
  const StreamWs w = stream_ws(p, N, Fin, K, Fout);
  const bool dypass = pb != CG_PATH_RESIDENT && stream_ws(p, N, Fin, K, Fout).wide &&
                      cg::wide_dypass_ok(Fin * K, Fout);
  const size_t slabs = dw_slab_bytes(int64_t(N) * p->M, N, Fin * K, Fout, dypass ? p->M : 0);
  *fwd = (pf == CG_PATH_RESIDENT) ? 0 : w.slots;
  if (pf != CG_PATH_RESIDENT && use_group(p, Fin, K, Fout))  // per-group partial y (planes layout)
    *fwd = std::max(*fwd, al256(cg::grp_partial_bytes(N, p->M, Fin, Fout)));
  *bwd = slabs + ((pb == CG_PATH_RESIDENT) ? 0 : w.dA);
  return CG_OK;
}

}  // namespace

namespace cg {
namespace {
// CG_OPT_* values (defaults: the measured-faster kernels) and their ranges
std::atomic<int> g_opts[kOptCount] = {{1}, {1}, {8}, {1}, {1}, {1}, {1}, {1}, {1}, {1}};
// The release library accepts only the values a user would choose between;
// the alternatives that lost every A/B exist in the ablation
// build only (`make debug`): CG_OPT_DW_DIRECT 2 / 3 (forced direct dW), CG_OPT_DW_W2
// 0 (one-wave dW builds), CG_OPT_SPMM_PW 0, CG_OPT_GRP_PC 0, CG_OPT_CLEN_DY 0 / 2.
bool option_valid(int o, int v) {
#ifndef CG_DEBUG
  switch (o) {
    case kOptDwDirect: return v == 0 || v == 1;
    case kOptDwW2:
    case kOptSpmmPw:
    case kOptGrpPc:
    case kOptClenDy: return v == 1;
    default: break;
  }
#endif
  switch (o) {
    case kOptDwDirect: return v >= 0 && v <= 3;
    case kOptDwWaves: return v == 4 || v == 8;
    case kOptClenDy: return v >= 0 && v <= 2;
    case kOptSeqXpre: return v >= 0 && v <= 2;
    default: return v == 0 || v == 1;
  }
}
}  // namespace
int option(Opt o) { return g_opts[o].load(std::memory_order_relaxed); }
}  // namespace cg

extern "C" {

int cg_version(void) { return 301; }


int cg_set_option(int32_t option, int32_t value) {
  if (option < 0 || option >= cg::kOptCount) return fail(CG_ERR_ARG, "unknown option %d", option);
  if (!cg::option_valid(option, value))
    return fail(CG_ERR_ARG, "value %d out of range for option %d", value, option);
  cg::g_opts[option].store(value, std::memory_order_relaxed);
  return ok();
}

int cg_get_option(int32_t option, int32_t* value) {
  if (option < 0 || option >= cg::kOptCount || !value)
    return fail(CG_ERR_ARG, "unknown option %d or null value", option);
  *value = cg::g_opts[option].load(std::memory_order_relaxed);
  return ok();
}

#ifdef CG_DEBUG
// Timing-ablation hook of the debug build only (`make debug`; not in the
// public header, not in the release library; outputs are WRONG when set).
int cg_debug_set_flags(int flags) {
  cg::g_debug_flags = flags;
  return ok();
}
// Tuning override (ablation build only): launch code reads key k < 8 with
// cg::debug_param(k, default); value -1 restores the default.
// Phase timestamps of the fast kernels (ablation build only): a device buffer
// of N * 8 uint64 or NULL.
int cg_debug_set_ts(void* dev_buf) {
  cg::g_debug_ts = static_cast<unsigned long long*>(dev_buf);
  return ok();
}
int cg_debug_set_param(int key, int value) {
  if (key < 0 || key >= 8) return fail(CG_ERR_ARG, "bad debug param %d", key);
  cg::g_debug_params[key] = value;
  return ok();
}
#endif

// Not in the public header: lets comm.cpp report through cg_last_error().
int cg_internal_set_error(int code, const char* msg) {
  if (code == CG_OK) return ok();
  return fail(code, "%s", msg ? msg : "");
}

const char* cg_last_error(void) { return g_err.c_str(); }

// Not in the public header (tests / diagnostics): plan the fast-path LDS layout
// of a host CSR operand without a GPU, check its invariants, and report the
// modelled LDS cycles of one step's gathers (with the layout and conflict-free).
int cg_debug_layout_stats(int32_t M, const int32_t* rowptr, const int32_t* col,
                          long* gather_cycles, long* gather_ideal, int* records) {
  if (M < 1 || M > 1024 || !rowptr || !col) return fail(CG_ERR_ARG, "layout_stats: bad args");
  for (int r = 0; r < M; ++r)
    if (rowptr[r + 1] - rowptr[r] > cg::kFastWidth)
      return fail(CG_ERR_UNSUPPORTED, "layout_stats: row %d longer than %d", r, cg::kFastWidth);
  cg::FastLayout lay;
  cg::plan_fast_layout(M, rowptr, col, &lay);
  std::vector<int> seen(size_t(lay.P), 0);
  for (int v = 0; v < M; ++v) {
    for (int p : {lay.pos0[size_t(v)], lay.pos1[size_t(v)]}) {
      if (p < 64 || p >= lay.P || seen[size_t(p)]++)
        return fail(CG_ERR_ARG, "layout: bad/duplicate record %d of vertex %d", p, v);
    }
  }
  for (int t = 0; t < 1024; ++t) {
    const int r = lay.row[size_t(t)];
    for (int j = 0; j < cg::kFastWidth; ++j) {
      const int p = lay.cpos[size_t(j) * 1024 + t];
      if (r >= 0 && j < rowptr[r + 1] - rowptr[r]) {
        const int c = col[rowptr[r] + j];
        if (p != lay.pos0[size_t(c)] && p != lay.pos1[size_t(c)])
          return fail(CG_ERR_ARG, "layout: thread %d slot %d reads record %d, not vertex %d", t, j, p, c);
      } else if (p >= 32) {
        return fail(CG_ERR_ARG, "layout: padding of thread %d slot %d is not a zero record", t, j);
      }
    }
    if (r >= 0 && (lay.rpos0[size_t(t)] != lay.pos0[size_t(r)] || lay.rpos1[size_t(t)] != lay.pos1[size_t(r)] ||
                   (lay.rposr[size_t(t)] != lay.pos0[size_t(r)] && lay.rposr[size_t(t)] != lay.pos1[size_t(r)])))
      return fail(CG_ERR_ARG, "layout: own records of thread %d", t);
    if (r < 0 && (lay.rpos0[size_t(t)] < 32 || lay.rpos0[size_t(t)] >= 64))
      return fail(CG_ERR_ARG, "layout: idle thread %d does not write a dummy record", t);
  }
  for (int m = 0; m < M; ++m)
    if (lay.mpos[size_t(m)] != lay.pos0[size_t(m)] && lay.mpos[size_t(m)] != lay.pos1[size_t(m)])
      return fail(CG_ERR_ARG, "layout: tile read of vertex %d", m);
  if (gather_cycles) *gather_cycles = lay.gather_cycles;
  if (gather_ideal) *gather_ideal = lay.gather_ideal;
  if (records) *records = lay.P;
  return ok();
}

int cg_plan_create(cg_plan** plan, int device, int32_t M, int64_t nnz, const int32_t* rowptr,
                   const int32_t* col, const float* val, const int32_t* t_rowptr,
                   const int32_t* t_col, const float* t_val) {
  if (!plan) return fail(CG_ERR_ARG, "null plan out-pointer");
  *plan = nullptr;
  if (M < 1 || nnz < 0 || nnz >= (int64_t(1) << 31))
    return fail(CG_ERR_ARG, "bad M=%d nnz=%lld", M, (long long)nnz);
  int rc = check_csr("L", M, nnz, rowptr, col, val);
  if (rc) return rc;
  std::vector<int32_t> trp, tci;
  std::vector<float> tv;
  if (t_rowptr) {
    const int64_t nnzT = t_rowptr[M];
    if (nnzT != nnz) return fail(CG_ERR_ARG, "transpose nnz %lld != nnz %lld", (long long)nnzT,
                                 (long long)nnz);
    if ((rc = check_csr("L^T", M, nnz, t_rowptr, t_col, t_val))) return rc;
    trp.assign(t_rowptr, t_rowptr + M + 1);
    tci.assign(t_col, t_col + nnz);
    tv.assign(t_val, t_val + nnz);
  } else {
    transpose_csr(M, nnz, rowptr, col, val, trp, tci, tv);
  }

  int prev = 0;
  CG_HIP(hipGetDevice(&prev));
  CG_HIP(hipSetDevice(device));
  cg_plan* p = new (std::nothrow) cg_plan();
  if (!p) return fail(CG_ERR_ALLOC, "out of host memory");
  p->device = device;
  p->M = M;
  p->nnz = nnz;
  p->nnzT = nnz;
  for (int32_t r = 0; r < M; ++r) {
    p->max_row_nnz = std::max(p->max_row_nnz, rowptr[r + 1] - rowptr[r]);
    p->max_row_nnzT = std::max(p->max_row_nnzT, trp[size_t(r) + 1] - trp[size_t(r)]);
  }
  rc = upload(&p->rowptr, rowptr, size_t(M) + 1);
  if (!rc) rc = upload(&p->col, col, size_t(nnz));
  if (!rc) rc = upload(&p->val, val, size_t(nnz));
  if (!rc) rc = upload(&p->trowptr, trp.data(), trp.size());
  if (!rc) rc = upload(&p->tcol, tci.data(), tci.size());
  if (!rc) rc = upload(&p->tval, tv.data(), tv.size());
  auto order = [M](const int32_t* rp) {
    std::vector<int32_t> o(size_t(M), 0);
    for (int32_t r = 0; r < M; ++r) o[size_t(r)] = r;
    std::stable_sort(o.begin(), o.end(), [rp](int32_t a, int32_t b) {
      return rp[a + 1] - rp[a] > rp[b + 1] - rp[b];
    });
    return o;
  };
  if (!rc && M > 0) {
    const std::vector<int32_t> o = order(rowptr), ot = order(trp.data());
    rc = upload(&p->lorder, o.data(), o.size());
    if (!rc) rc = upload(&p->tlorder, ot.data(), ot.size());
    if (!rc && nnz > 0 && p->max_row_nnz > 2 * (nnz / M) + 8) {
      rc = upload(&p->rperm, o.data(), o.size());
      if (!rc) rc = upload(&p->trperm, ot.data(), ot.size());
    }
  }
  if (!rc && nnz > 0) rc = build_slots(&p->slots, M, rowptr, col, val);
  if (!rc && nnz > 0) rc = build_slots(&p->tslots, M, trp.data(), tci.data(), tv.data());
  // a symmetric pattern (every Laplacian here) shares one layout between L~
  // and L~^T: the annealing (lds_layout.cpp) runs once
  const bool sym = nnz > 0 && std::equal(rowptr, rowptr + M + 1, trp.begin()) &&
                   std::equal(col, col + nnz, tci.begin());
  cg::FastLayout lay;
  if (!rc && nnz > 0) rc = build_fast_image(&p->fast, M, rowptr, col, val, sym ? &lay : nullptr);
  if (!rc && nnz > 0)
    rc = build_fast_image(&p->tfast, M, trp.data(), tci.data(), tv.data(), nullptr,
                          sym && p->fast.ok ? &lay : nullptr);
  (void)hipSetDevice(prev);
  if (rc) {
    free_plan(p);
    return rc;
  }
  *plan = p;
  return ok();
}

int cg_plan_destroy(cg_plan* plan) {
  free_plan(plan);
  return ok();
}

int cg_plan_set_path(cg_plan* plan, int path) {
  if (!plan) return fail(CG_ERR_ARG, "null plan");
  if (path != CG_PATH_AUTO && path != CG_PATH_RESIDENT && path != CG_PATH_STREAM)
    return fail(CG_ERR_ARG, "bad path %d", path);
  plan->path = path;
  return ok();
}

int cg_plan_set_variant(cg_plan* plan, int variant) {
  if (!plan) return fail(CG_ERR_ARG, "null plan");
  if (variant != CG_VARIANT_AUTO && variant != CG_VARIANT_CLASSIC &&
      variant != CG_VARIANT_UNFUSED_DW && variant != CG_VARIANT_NARROW && variant != CG_VARIANT_STEPS)
    return fail(CG_ERR_ARG, "bad kernel variant %d", variant);
  plan->variant = variant;
  return ok();
}

int cg_plan_query_path(const cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                       int* path) {
  int rc = check_shape(plan, N, Fin, K, Fout);
  if (rc) return rc;
  if (!path) return fail(CG_ERR_ARG, "null path out-pointer");
  if ((rc = choose_path(plan, Fin, K, Fout, false, path))) return rc;
  return ok();
}

int cg_cheb_workspace_bytes(const cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                            size_t* fwd_bytes, size_t* bwd_bytes) {
  int rc = check_shape(plan, N, Fin, K, Fout);
  if (rc) return rc;
  size_t f = 0, b = 0;
  if ((rc = workspace_bytes(plan, N, Fin, K, Fout, &f, &b))) return rc;
  if (fwd_bytes) *fwd_bytes = f;
  if (bwd_bytes) *bwd_bytes = b;
  return ok();
}

}  // extern "C"

namespace {
// Adam applied to W by the forward that consumes it (cg_cheb_forward_adam)
struct FwdAdam {
  const float* grad;
  const float* m;
  const float* v;
  float* W_out;
  float* m_out;
  float* v_out;
  float lr_t, beta1, beta2, eps, grad_scale;
};

// forward with the residual / activation epilogue y = act(basis W + res)
int forward_impl(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout, const float* x,
                 const float* W, const float* res, int act, float* basis, float* y, void* workspace,
                 size_t ws_bytes, void* stream, int layout = CG_BASIS_ROWS,
                 const FwdAdam* fa = nullptr) {
  int rc = check_shape(plan, N, Fin, K, Fout);
  if (rc) return rc;
  if ((rc = check_layout(plan, Fin, K, Fout, layout))) return rc;
  if (!x) return fail(CG_ERR_ARG, "null x");
  if (act != CG_ACT_NONE && act != CG_ACT_RELU) return fail(CG_ERR_ARG, "unknown activation %d", act);
  if (!y && (res || act)) return fail(CG_ERR_ARG, "an epilogue needs y");
  if (y && !W) return fail(CG_ERR_ARG, "null W with non-null y");
  if (!y && !basis) return fail(CG_ERR_ARG, "nothing to compute (basis and y both null)");
  if ((rc = check_device(plan))) return rc;
  int path = 0;
  if ((rc = choose_path(plan, Fin, K, Fout, false, &path))) return rc;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int M = plan->M;
  const bool fast_fwd =
      layout == CG_BASIS_ORDERS || (path == CG_PATH_RESIDENT && use_fast(plan, Fin, K, Fout, false));
  if (fa && !fast_fwd) {
    // other kernels: the same update out of place by k_adam, then the forward on W'
    const size_t nb = size_t(Fin) * K * Fout * sizeof(float);
    CG_HIP(hipMemcpyAsync(fa->W_out, W, nb, hipMemcpyDeviceToDevice, s));
    CG_HIP(hipMemcpyAsync(fa->m_out, fa->m, nb, hipMemcpyDeviceToDevice, s));
    CG_HIP(hipMemcpyAsync(fa->v_out, fa->v, nb, hipMemcpyDeviceToDevice, s));
    CG_HIP(cg::launch_adam(fa->W_out, fa->grad, fa->m_out, fa->v_out, int64_t(Fin) * K * Fout,
                           fa->lr_t, fa->beta1, fa->beta2, fa->eps, fa->grad_scale, s));
    W = fa->W_out;
    fa = nullptr;
  }

  if (fast_fwd) {
    cg::FastFwdArgs a{};
    a.M = M;
    a.Fin = Fin;
    a.K = K;
    a.Fout = Fout;
    a.dbg = cg::debug_flags() & 0xff;
    a.E = plan->fast.view;
    a.x = x;
    a.W = y ? W : nullptr;
    a.basis = basis;
    a.y = y;
    a.res = res;
    a.act = act;
    a.bord = layout == CG_BASIS_ORDERS ? basis_mb(M) : 0;
#ifdef CG_DEBUG
    a.ts = cg::g_debug_ts;
#endif
    if (fa) {
      a.W = W;
      a.ad_grad = fa->grad;
      a.ad_m = fa->m;
      a.ad_v = fa->v;
      a.ad_W = fa->W_out;
      a.ad_mo = fa->m_out;
      a.ad_vo = fa->v_out;
      a.ad_lr_t = fa->lr_t;
      a.ad_b1 = fa->beta1;
      a.ad_b2 = fa->beta2;
      a.ad_eps = fa->eps;
      a.ad_scale = fa->grad_scale;
    }
    CG_HIP(cg::launch_fast_forward(fast_geom(plan, Fin, K, Fout), N, a, s));
    return ok();
  }
  if (path == CG_PATH_RESIDENT) {
    const cg::ResidentGeom g = cg::resident_geometry(M, int(plan->nnz), plan->max_row_nnz, plan->max_row_nnzT, Fin, K, Fout);
    cg::ResidentFwdArgs a{};
    a.M = M;
    a.Fin = Fin;
    a.K = K;
    a.Fout = Fout;
    a.Mp = cg::lds_vertex_stride(M);
    a.dbg = cg::debug_flags() & 0xff;
    a.E = plan->slots.view;
    a.col = plan->col;
    a.val = plan->val;
    a.x = x;
    a.W = y ? W : nullptr;
    a.basis = basis;
    a.y = y;
    a.res = res;
    a.act = act;
    CG_HIP(cg::launch_resident_forward(g, N, a, s));
    return ok();
  }
  // streaming path
  if (!basis) return fail(CG_ERR_ARG, "streaming path needs a basis buffer (the GEMM reads it)");
  const StreamWs w = stream_ws(plan, N, Fin, K, Fout);
  if (w.slots && (!workspace || ws_bytes < w.slots))
    return fail(CG_ERR_ARG, "forward workspace too small: %zu < %zu", ws_bytes, w.slots);
  float* slots = static_cast<float*>(workspace);
  const size_t slot = size_t(M) * size_t(N) * size_t(Fin);
  if (K == 1) {
    if (x != basis) CG_HIP(hipMemcpyAsync(basis, x, slot * sizeof(float), hipMemcpyDeviceToDevice, s));
  } else if (w.wide) {
    // wide columns: T_0 = x re-laid [M][Fin*N] into plane 0, the K-1 steps
    // plane to plane, then the basis (lib/graph_conv.py:155-172)
    const cg::WideGeom g = cg::wide_geometry(N, Fin, M);
    const int B = N * Fin;
    const int* rperm = plan->rperm;
    const bool fused_last = cg::wide_last_ok(g, Fin, K, rperm != nullptr);
    CG_HIP(cg::launch_sm_to_vm(x, 1, N, int64_t(M) * Fin, slots, s));
    for (int k = 1; k < (fused_last ? K - 1 : K); ++k)
      CG_HIP(cg::launch_wide_step(g, plan->rowptr, plan->col, plan->val, rperm,
                                  slots + size_t(k - 1) * slot,
                                  k >= 2 ? slots + size_t(k - 2) * slot : nullptr, nullptr,
                                  slots + size_t(k) * slot, M, B, k == 1 ? 0 : 1, 2.f, s));
    if (fused_last)  // T_{K-1} and the basis assembly in one launch
      CG_HIP(cg::launch_wide_last(g, plan->rowptr, plan->col, plan->val, slots, int64_t(slot), basis,
                                  M, N, K, s));
    else
      CG_HIP(cg::launch_wide_assemble(slots, int64_t(slot), N, M, Fin, K, basis, s));
  } else if (layout == CG_BASIS_PLANES && use_group(plan, Fin, K, Fout)) {
    // channel-group resident kernel: the whole recurrence in LDS per (sample,
    // 8 channels), planes written once, y from per-group MFMA partials
    if (y && (!workspace || ws_bytes < cg::grp_partial_bytes(N, M, Fin, Fout)))
      return fail(CG_ERR_ARG, "forward workspace too small for the group partials");
    CG_HIP(cg::launch_grp_fwd(plan->rowptr, plan->col, plan->val, plan->lorder, plan->nnz, N, M, Fin, K,
                              Fout, x,
                              W, basis, static_cast<float*>(workspace), res, act, y, s));
    return ok();
  } else if (layout == CG_BASIS_PLANES) {
    // planes layout: T_k IS plane k of the basis (plane 0 = x: copied unless
    // the caller placed x there), every step writes its own plane, no assembly
    // step (lib/graph_conv.py:159-169)
    const int* rperm = (Fin >= 16) ? plan->rperm : nullptr;
    auto P = [&](int k) { return basis + size_t(k) * slot; };
    if (x != basis) CG_HIP(hipMemcpyAsync(basis, x, slot * sizeof(float), hipMemcpyDeviceToDevice, s));
    for (int k = 1; k < K; ++k)
      CG_HIP(cg::launch_cheb_step(plan->rowptr, plan->col, plan->val, rperm, k == 1 ? x : P(k - 1),
                                  k == 2 ? x : (k > 2 ? P(k - 2) : nullptr), P(k), x, nullptr,
                                  nullptr, N, M, Fin, K, k, false, s));
  } else {
    // sample-major steps: T_0 = x, T_j (1 <= j <= K-2) in slots[j-1], the last
    // step writes the whole basis (lib/graph_conv.py:159-172)
    const int* rperm = (Fin >= 16) ? plan->rperm : nullptr;
    auto T = [&](int k) -> const float* { return k == 0 ? x : slots + size_t(k - 1) * slot; };
    for (int k = 1; k < K; ++k) {
      const bool last = (k == K - 1);
      CG_HIP(cg::launch_cheb_step(plan->rowptr, plan->col, plan->val, rperm, T(k - 1),
                                  k >= 2 ? T(k - 2) : nullptr,
                                  last ? nullptr : slots + size_t(k - 1) * slot, x, slots, basis, N,
                                  M, Fin, K, k, last, s));
    }
  }
  if (y && layout == CG_BASIS_PLANES) {
    // y = sum_k T_k W_k straight from the planes (row GEMM, A addressed per plane)
    const int FinK = Fin * K;
    CG_HIP(cg::launch_rowgemm(basis, int64_t(N) * M, FinK, FinK, W, Fout, 1, 0, 1, Fout, y, Fout, 0,
                              s, res, act, 0, Fin, int64_t(slot), K));
  } else if (y) {
    const int FinK = Fin * K;
    if (cg::rowgemm_ok(FinK, FinK, Fout)) {
      CG_HIP(cg::launch_rowgemm(basis, int64_t(N) * M, FinK, FinK, W, Fout, 1, 0, 1, Fout, y, Fout,
                                0, s, res, act));
    } else {
      CG_HIP(cg::launch_gemm_f32(false, false, N * M, Fout, FinK, basis, FinK, W, Fout, y, Fout, 1,
                                 s));
      if (res || act) CG_HIP(cg::launch_act_fwd(y, res, act, int64_t(N) * M * Fout, s));
    }
  }
  return ok();
}

int backward_impl(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout, const float* dy,
                  const float* basis, const float* W, float* dx, int dx_acc, float* dW,
                  void* workspace, size_t ws_bytes, void* stream,
                  const cg::AdamStep* adam = nullptr, int layout = CG_BASIS_ROWS) {
  int rc = check_shape(plan, N, Fin, K, Fout);
  if (rc) return rc;
  if ((rc = check_layout(plan, Fin, K, Fout, layout))) return rc;
  if (layout == CG_BASIS_ORDERS && dW && !dx)
    return fail(CG_ERR_UNSUPPORTED, "orders basis layout: dW is fused into the dx pass (dx needed)");
  if (!dy || !W) return fail(CG_ERR_ARG, "null dy/W");
  if (!basis && dW) return fail(CG_ERR_ARG, "null basis: dW needs the forward's basis");
  if (!dx && !dW) return fail(CG_ERR_ARG, "dx and dW are both NULL: nothing to compute");
  if ((rc = check_device(plan))) return rc;
  int path = 0;
  if ((rc = choose_path(plan, Fin, K, Fout, true, &path))) return rc;
  size_t need_f = 0, need_b = 0;
  if ((rc = workspace_bytes(plan, N, Fin, K, Fout, &need_f, &need_b))) return rc;
  if (!workspace || ws_bytes < need_b)
    return fail(CG_ERR_ARG, "backward workspace too small: %zu < %zu", ws_bytes, need_b);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int M = plan->M;
  const int FinK = Fin * K;
  const int64_t R = int64_t(N) * M;
  const int chunks = cg::dw_chunks(R);

  // Everything runs on the caller's stream.  (Forking the streaming dW GEMM onto a side stream to
  // overlap the dx recurrence was measured on MI355X in round 1: the event
  // fork + join costs ~20 us per call, more than the overlap gains there.)
  char* base = static_cast<char*>(workspace);
  float* slabs = reinterpret_cast<float*>(base);
  const bool dypass = path != CG_PATH_RESIDENT && stream_ws(plan, N, Fin, K, Fout).wide &&
                      cg::wide_dypass_ok(FinK, Fout);
  char* rest = base + dw_slab_bytes(R, N, FinK, Fout, dypass ? M : 0);
  const bool fused =
      dx != nullptr && dW != nullptr && path == CG_PATH_RESIDENT && fused_dw(plan, Fin, K, Fout);
  int nslab_ready = 0;  // dW slabs a kernel of the dx pass already wrote
  auto launch_dw = [&](hipStream_t st) -> hipError_t {
    if (cg::debug_flags() & (1 << 22)) return hipSuccess;  // ablation hook (debug build): skip dW
    return cg::launch_dw_slabs(basis, dy, R, FinK, Fout, slabs, st,
                               layout == CG_BASIS_PLANES ? Fin : 0,
                               layout == CG_BASIS_PLANES ? int64_t(R) * Fin : 0, K);
  };
  if (dx) {
    if (path == CG_PATH_RESIDENT && use_fast(plan, Fin, K, Fout, true)) {
      const cg::FastGeom g = fast_geom(plan, Fin, K, Fout);
      cg::FastBwdArgs a{};
      a.M = M;
      a.Fin = Fin;
      a.K = K;
      a.Fout = Fout;
      a.Mp = cg::lds_vertex_stride(M);
      a.dbg = (cg::debug_flags() >> 8) & 0xff;
      a.dscratch_bytes = g.dscratch;
      a.E = plan->tfast.view;
      a.dy = dy;
      a.basis = basis;
      a.W = W;
      a.dx = dx;
      a.dx_acc = dx_acc;
      a.dw_slab = fused ? slabs : nullptr;
      a.bord = layout == CG_BASIS_ORDERS ? basis_mb(M) : 0;
      a.x3 = cg::option(cg::kOptGemmX3) != 0 ? 1 : 0;
#ifdef CG_DEBUG
      a.ts = cg::g_debug_ts;
#endif
      CG_HIP(cg::launch_fast_backward(g, N, a, s));
    } else if (path == CG_PATH_RESIDENT) {
      const cg::ResidentGeom g = cg::resident_geometry(M, int(plan->nnz), plan->max_row_nnz,
                                                       plan->max_row_nnzT, Fin, K, Fout);
      cg::ResidentBwdArgs a{};
      a.M = M;
      a.Fin = Fin;
      a.K = K;
      a.Fout = Fout;
      a.Mp = cg::lds_vertex_stride(M);
      a.dbg = (cg::debug_flags() >> 8) & 0xff;
      a.E = plan->tslots.view;
      a.col = plan->tcol;
      a.val = plan->tval;
      a.dy = dy;
      a.W = W;
      a.dx = dx;
      a.dx_acc = dx_acc;
      CG_HIP(cg::launch_resident_backward(g, N, a, s));
    } else if (dypass) {
      // wide columns: ONE pass over dy writes the D_k planes straight in the
      // [M][Fin*N] layout and the dW slabs; then G_k in place of D_k, one
      // launch per step, and G_0 re-laid into dx (dx += when accumulating)
      const cg::WideGeom g = cg::wide_geometry(N, Fin, M);
      const int B = N * Fin;
      const size_t slot = size_t(M) * size_t(B);
      float* D = reinterpret_cast<float*>(rest);
      CG_HIP(cg::launch_wide_dypass(dy, basis, W, N, M, Fin, K, Fout, D, int64_t(slot),
                                    dW ? slabs : nullptr, s));
      if (dW) nslab_ready = cg::wide_dypass_blocks(N, M);
      auto G = [&](int k) { return D + size_t(k) * slot; };
      // (G_{K-1} = D_{K-1}: the last order's step would rewrite its plane in place)
      for (int k = K - 2; k >= 0; --k)
        CG_HIP(cg::launch_wide_step(g, plan->trowptr, plan->tcol, plan->tval, plan->trperm,
                                    (k + 1 <= K - 1) ? G(k + 1) : nullptr,
                                    (k + 2 <= K - 1) ? G(k + 2) : nullptr, G(k), G(k), M, B, 2,
                                    k >= 1 ? 2.f : 1.f, s));
      CG_HIP(cg::launch_vm_to_sm(G(0), N, int64_t(M) * Fin, dx, dx_acc, s));
    } else if (!stream_ws(plan, N, Fin, K, Fout).wide && use_group(plan, Fin, K, Fout) &&
               cg::grp_clen_dy_ok(M, plan->nnzT, K, Fout)) {
      // the whole reverse recurrence in LDS per (sample, 8 channels), dBasis
      // formed in the kernel from dy and W (no dBasis planes)
      CG_HIP(cg::launch_grp_clen_dy(plan->trowptr, plan->tcol, plan->tval, plan->tlorder, plan->nnzT,
                                    N, M, Fin, K, Fout, dy, W, dx, dx_acc, s));
    } else {
      float* dA = reinterpret_cast<float*>(rest);
      const int NM = N * M;
      // dBasis = dy W^T written k-major ([K][N*M][Fin]), then the reverse
      // recurrence one launch per step in the sample-major layout.  Step k
      // reads D_k[r] and writes G_k[r] at the same address (same lane), and
      // the steps below k gather G_{k+1} / read G_{k+2} from planes k+1 / k+2,
      // so G lives in place of dBasis: no separate ring (for config D at
      // N = 256 that is 3 x 17.2 GB less workspace).
      const size_t slot = size_t(M) * size_t(N) * size_t(Fin);
      // plane k: dA_k[r][fin] = sum_f dy[r][f] W[fin*K+k][f]; all K planes in
      // one pass over dy when the FinK columns fit one row-GEMM block
      if (cg::rowgemm_ok(Fout, Fout, FinK))
        CG_HIP(cg::launch_rowgemm(dy, NM, Fout, Fout, W, 1, int64_t(K) * Fout, Fout, 1, FinK, dA, Fin,
                                  int64_t(slot), s, nullptr, 0, Fin));
      else if (cg::rowgemm_ok(Fout, Fout, Fin))
        CG_HIP(cg::launch_rowgemm(dy, NM, Fout, Fout, W, 1, int64_t(K) * Fout, Fout, K, Fin, dA, Fin,
                                  int64_t(slot), s));
      else
        CG_HIP(cg::launch_gemm_f32(false, true, NM, FinK, Fout, dy, Fout, W, Fout, dA, FinK, 1, s, K));
      const StreamWs w = stream_ws(plan, N, Fin, K, Fout);
      if (w.wide) {
        // wide columns: the k-planes re-laid [M][Fin*N], then G_k in place of
        // D_k one launch per step, G_0 re-laid into dx (dx += when accumulating)
        const cg::WideGeom g = cg::wide_geometry(N, Fin, M);
        const int B = N * Fin;
        float* D = reinterpret_cast<float*>(rest + al256(size_t(R) * size_t(FinK) * 4));
        CG_HIP(cg::launch_sm_to_vm(dA, K, N, int64_t(M) * Fin, D, s));
        auto G = [&](int k) { return D + size_t(k) * slot; };
        for (int k = K - 2; k >= 0; --k)  // (G_{K-1} = D_{K-1} in place: no step)
          CG_HIP(cg::launch_wide_step(g, plan->trowptr, plan->tcol, plan->tval, plan->trperm,
                                      (k + 1 <= K - 1) ? G(k + 1) : nullptr,
                                      (k + 2 <= K - 1) ? G(k + 2) : nullptr, G(k), G(k), M, B, 2,
                                      k >= 1 ? 2.f : 1.f, s));
        CG_HIP(cg::launch_vm_to_sm(G(0), N, int64_t(M) * Fin, dx, dx_acc, s));
      } else if (use_group(plan, Fin, K, Fout)) {
        // the whole reverse recurrence in LDS per (sample, 8 channels)
        CG_HIP(cg::launch_grp_clen(plan->trowptr, plan->tcol, plan->tval, plan->tlorder, plan->nnzT, N,
                                   M, Fin, K,
                                   dA, dx, dx_acc, s));
      } else {
        const int* rperm = (Fin >= 16) ? plan->trperm : nullptr;
        auto G = [&](int k) { return dA + size_t(k) * slot; };
        // G_{K-1} = D_{K-1} already sits in its plane (G lives in place of D):
        // the last order's step would only rewrite it (D's 17 GB at N = 256);
        // with K = 1 the one step is dx = D_0
        for (int k = K >= 2 ? K - 2 : 0; k >= 0; --k)
          CG_HIP(cg::launch_clenshaw(plan->trowptr, plan->tcol, plan->tval, rperm,
                                     (k + 1 <= K - 1) ? G(k + 1) : nullptr,
                                     (k + 2 <= K - 1) ? G(k + 2) : nullptr, k == 0 ? dx : G(k),
                                     G(k), N, M, Fin, K, k, dx_acc, s));
      }
    }
  }
  if (!dW) return ok();
  if (fused) nslab_ready = N;
  // small problems (config A): dW in one block, no slabs and no reduction
  // launch (with Adam: the one result is the single slab of the fused reduction)
  if (!nslab_ready && layout == CG_BASIS_ROWS && cg::dw_small_ok(R, FinK, Fout) &&
      cg::dw_small_aligned(basis, dy) && !(cg::debug_flags() & (1 << 22))) {
    CG_HIP(cg::launch_dw_small(basis, dy, R, FinK, Fout, adam ? slabs : dW, s));
    if (!adam) return ok();
    nslab_ready = 1;
  }
  if (!nslab_ready) CG_HIP(launch_dw(s));
  const int nslab = nslab_ready ? nslab_ready : chunks;
  if (adam)  // reduction + optimizer step in one launch (no exchange in between)
    CG_HIP(cg::launch_reduce_slabs_adam(slabs, nslab, int64_t(FinK) * Fout, dW, *adam, s));
  else if (!(cg::debug_flags() & (1 << 23)))  // ablation hook (debug build): skip the reduction
    CG_HIP(cg::launch_reduce_slabs(slabs, nslab, int64_t(FinK) * Fout, dW, s));
  return ok();
}

}  // namespace

extern "C" {

int cg_cheb_forward(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                    const float* x, const float* W, float* basis, float* y, void* workspace,
                    size_t ws_bytes, void* stream) {
  return forward_impl(plan, N, Fin, K, Fout, x, W, nullptr, CG_ACT_NONE, basis, y, workspace,
                      ws_bytes, stream);
}

int cg_cheb_forward_ex(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                       const float* x, const float* W, const float* residual, int32_t act,
                       float* basis, float* y, void* workspace, size_t ws_bytes, void* stream) {
  return forward_impl(plan, N, Fin, K, Fout, x, W, residual, act, basis, y, workspace, ws_bytes,
                      stream);
}

int cg_cheb_backward(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                     const float* dy, const float* basis, const float* W, float* dx, float* dW,
                     void* workspace, size_t ws_bytes, void* stream) {
  return backward_impl(plan, N, Fin, K, Fout, dy, basis, W, dx, 0, dW, workspace, ws_bytes, stream);
}

namespace {
int backward_adam_impl(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                       int layout, const float* dy, const float* basis, float* W, float* dx,
                       float* dW, float* m, float* v, float lr, float beta1, float beta2,
                       float eps, int32_t step, float grad_scale, void* workspace,
                       size_t ws_bytes, void* stream) {
  if (!dW || !W || !m || !v || step < 1)
    return fail(CG_ERR_ARG, "cheb_backward_adam: dW, W, m, v required and step >= 1");
  // the reduction stores grad[i] and then updates param/m/v[i] in place:
  // any two of them sharing memory would corrupt the update
  const void* bufs[4] = {dW, W, m, v};
  for (int i = 0; i < 4; ++i)
    for (int j = i + 1; j < 4; ++j)
      if (bufs[i] == bufs[j])
        return fail(CG_ERR_ARG, "cheb_backward_adam: dW, W, m and v must be distinct buffers");
  if (cg::debug_flags() & ((1 << 22) | (1 << 23)))
    return fail(CG_ERR_UNSUPPORTED, "cheb_backward_adam: dW ablation bits would corrupt W");
  cg::AdamStep a{};
  a.param = W;
  a.m = m;
  a.v = v;
  a.lr_t = float(double(lr) * std::sqrt(1.0 - std::pow(double(beta2), step)) /
                 (1.0 - std::pow(double(beta1), step)));
  a.beta1 = beta1;
  a.beta2 = beta2;
  a.eps = eps;
  a.grad_scale = grad_scale;
  return backward_impl(plan, N, Fin, K, Fout, dy, basis, W, dx, 0, dW, workspace, ws_bytes, stream,
                       &a, layout);
}

int backward_ex_impl(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                     const float* dy, const float* y, int32_t act, int layout, const float* basis,
                     const float* W, float* dx, int32_t dx_accumulate, float* dW, float* dz,
                     void* workspace, size_t ws_bytes, void* stream) {
  if (act != CG_ACT_NONE && act != CG_ACT_RELU) return fail(CG_ERR_ARG, "unknown activation %d", act);
  if (!plan || !dy) return fail(CG_ERR_ARG, "null plan / dy");
  int rc = check_shape(plan, N, Fin, K, Fout);
  if (rc) return rc;
  if ((rc = check_layout(plan, Fin, K, Fout, layout))) return rc;
  const float* dy_eff = dy;
  if (act == CG_ACT_RELU) {
    if (!y || !dz) return fail(CG_ERR_ARG, "ReLU backward needs y (its output) and dz");
    CG_HIP(cg::launch_relu_bwd(dy, y, dz, int64_t(N) * plan->M * Fout,
                               reinterpret_cast<hipStream_t>(stream)));
    dy_eff = dz;
  } else if (dz) {
    CG_HIP(hipMemcpyAsync(dz, dy, size_t(N) * plan->M * Fout * sizeof(float),
                          hipMemcpyDeviceToDevice, reinterpret_cast<hipStream_t>(stream)));
  }
  if (!dx && !dW) return ok();
  return backward_impl(plan, N, Fin, K, Fout, dy_eff, basis, W, dx, dx_accumulate != 0, dW,
                       workspace, ws_bytes, stream, nullptr, layout);
}
}  // namespace

int cg_cheb_backward_adam(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                          const float* dy, const float* basis, float* W, float* dx, float* dW,
                          float* m, float* v, float lr, float beta1, float beta2, float eps,
                          int32_t step, float grad_scale, void* workspace, size_t ws_bytes,
                          void* stream) {
  return backward_adam_impl(plan, N, Fin, K, Fout, CG_BASIS_ROWS, dy, basis, W, dx, dW, m, v, lr,
                            beta1, beta2, eps, step, grad_scale, workspace, ws_bytes, stream);
}

int cg_cheb_backward_ex(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                        const float* dy, const float* y, int32_t act, const float* basis,
                        const float* W, float* dx, int32_t dx_accumulate, float* dW, float* dz,
                        void* workspace, size_t ws_bytes, void* stream) {
  return backward_ex_impl(plan, N, Fin, K, Fout, dy, y, act, CG_BASIS_ROWS, basis, W, dx,
                          dx_accumulate, dW, dz, workspace, ws_bytes, stream);
}

int cg_cheb_basis_elems(const cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                        int32_t layout, int64_t* elems) {
  int rc = check_shape(plan, N, Fin, K, Fout);
  if (rc) return rc;
  if (!elems) return fail(CG_ERR_ARG, "null elems out-pointer");
  if ((rc = check_layout(plan, Fin, K, Fout, layout))) return rc;
  const int64_t rows = layout == CG_BASIS_ORDERS ? basis_mb(plan->M) : plan->M;
  *elems = int64_t(N) * rows * Fin * K;
  return ok();
}

int cg_cheb_forward_layout(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                           const float* x, const float* W, const float* residual, int32_t act,
                           int32_t layout, float* basis, float* y, void* workspace,
                           size_t ws_bytes, void* stream) {
  return forward_impl(plan, N, Fin, K, Fout, x, W, residual, act, basis, y, workspace, ws_bytes,
                      stream, layout);
}

int cg_cheb_forward_adam(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                         const float* x, const float* W, const float* grad, const float* m,
                         const float* v, float lr, float beta1, float beta2, float eps,
                         int32_t step, float grad_scale, float* W_out, float* m_out, float* v_out,
                         int32_t layout, float* basis, float* y, void* workspace,
                         size_t ws_bytes, void* stream) {
  if (!W || !grad || !m || !v || !W_out || !m_out || !v_out || step < 1 || !y)
    return fail(CG_ERR_ARG, "cheb_forward_adam: W, grad, m, v, W_out, m_out, v_out, y required "
                            "and step >= 1");
  // every workgroup reads W, m, v while workgroup 0 writes W', m', v': the
  // outputs must not alias any input
  const void* outs[3] = {W_out, m_out, v_out};
  const void* ins[4] = {W, grad, m, v};
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 4; ++j)
      if (outs[i] == ins[j])
        return fail(CG_ERR_ARG, "cheb_forward_adam: W_out, m_out, v_out must not alias the inputs");
    for (int j = i + 1; j < 3; ++j)
      if (outs[i] == outs[j])
        return fail(CG_ERR_ARG, "cheb_forward_adam: W_out, m_out, v_out must be distinct");
  }
  FwdAdam fa{grad, m, v, W_out, m_out, v_out,
             float(double(lr) * std::sqrt(1.0 - std::pow(double(beta2), step)) /
                   (1.0 - std::pow(double(beta1), step))),
             beta1, beta2, eps, grad_scale};
  return forward_impl(plan, N, Fin, K, Fout, x, W, nullptr, CG_ACT_NONE, basis, y, workspace,
                      ws_bytes, stream, layout, &fa);
}

int cg_cheb_backward_layout(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                            const float* dy, const float* y, int32_t act, int32_t layout,
                            const float* basis, const float* W, float* dx, int32_t dx_accumulate,
                            float* dW, float* dz, void* workspace, size_t ws_bytes, void* stream) {
  return backward_ex_impl(plan, N, Fin, K, Fout, dy, y, act, layout, basis, W, dx, dx_accumulate,
                          dW, dz, workspace, ws_bytes, stream);
}

int cg_cheb_backward_adam_layout(cg_plan* plan, int32_t N, int32_t Fin, int32_t K, int32_t Fout,
                                 int32_t layout, const float* dy, const float* basis, float* W,
                                 float* dx, float* dW, float* m, float* v, float lr, float beta1,
                                 float beta2, float eps, int32_t step, float grad_scale,
                                 void* workspace, size_t ws_bytes, void* stream) {
  return backward_adam_impl(plan, N, Fin, K, Fout, layout, dy, basis, W, dx, dW, m, v, lr, beta1,
                            beta2, eps, step, grad_scale, workspace, ws_bytes, stream);
}

int cg_mse_loss_workspace_bytes(int64_t n, size_t* bytes) {
  if (!bytes || n < 1) return fail(CG_ERR_ARG, "mse_loss: bad arguments");
  *bytes = al256(size_t(cg::mse_chunks(n)) * 4);
  return ok();
}

int cg_mse_loss(const float* pred, const float* labels, int64_t n, float* loss, float* dpred,
                void* workspace, size_t ws_bytes, void* stream) {
  if (!pred || !labels || !loss || n < 1) return fail(CG_ERR_ARG, "mse_loss: bad arguments");
  const size_t need = al256(size_t(cg::mse_chunks(n)) * 4);
  if (!workspace || ws_bytes < need)
    return fail(CG_ERR_ARG, "mse_loss workspace too small: %zu < %zu", ws_bytes, need);
  CG_HIP(cg::launch_mse(pred, labels, n, static_cast<float*>(workspace), loss, dpred,
                        reinterpret_cast<hipStream_t>(stream)));
  return ok();
}

int cg_mse_loss_ema(const float* pred, const float* labels, int64_t n, float* loss, float* dpred,
                    float* ema, float decay, void* workspace, size_t ws_bytes, void* stream) {
  if (!pred || !labels || !loss || !ema || n < 1 || !(decay >= 0.f && decay <= 1.f))
    return fail(CG_ERR_ARG, "mse_loss_ema: bad arguments");
  const size_t need = al256(size_t(cg::mse_chunks(n)) * 4);
  if (!workspace || ws_bytes < need)
    return fail(CG_ERR_ARG, "mse_loss_ema workspace too small: %zu < %zu", ws_bytes, need);
  CG_HIP(cg::launch_mse(pred, labels, n, static_cast<float*>(workspace), loss, dpred,
                        reinterpret_cast<hipStream_t>(stream), ema, decay));
  return ok();
}

int cg_dropout_forward(const float* x, int64_t n, float keep_prob, uint64_t seed, float* y,
                       void* stream) {
  if (!x || !y || n < 1 || !(keep_prob > 0.f && keep_prob <= 1.f))
    return fail(CG_ERR_ARG, "dropout_forward: bad arguments (keep_prob=%g)", keep_prob);
  CG_HIP(cg::launch_dropout(x, y, n, keep_prob, seed, 0, reinterpret_cast<hipStream_t>(stream)));
  return ok();
}

int cg_dropout_backward(const float* dy, int64_t n, float keep_prob, uint64_t seed, float* dx,
                        void* stream) {
  if (!dy || !dx || n < 1 || !(keep_prob > 0.f && keep_prob <= 1.f))
    return fail(CG_ERR_ARG, "dropout_backward: bad arguments (keep_prob=%g)", keep_prob);
  CG_HIP(cg::launch_dropout(dy, dx, n, keep_prob, seed, 1, reinterpret_cast<hipStream_t>(stream)));
  return ok();
}

int cg_clip_by_norm(float* t, int64_t n, float clip_norm, int32_t* nonfinite, void* stream) {
  if (!t || n < 1 || !(clip_norm > 0.f))
    return fail(CG_ERR_ARG, "clip_by_norm: bad arguments (n=%lld, clip_norm=%g)", (long long)n,
                clip_norm);
  CG_HIP(cg::launch_clip_norm(t, n, clip_norm, nonfinite, reinterpret_cast<hipStream_t>(stream)));
  return ok();
}

int cg_slice_channels(const float* x, int64_t rows, int32_t C, int32_t c0, int32_t c1, float* out,
                      void* stream) {
  if (!x || !out || rows < 1 || C < 1 || c0 < 0 || c1 <= c0 || c1 > C)
    return fail(CG_ERR_ARG, "slice_channels: bad arguments (C=%d, [%d, %d))", C, c0, c1);
  CG_HIP(cg::launch_slice_channels(x, rows, C, c0, c1, out, reinterpret_cast<hipStream_t>(stream)));
  return ok();
}

int cg_stack_merge_forward(int32_t N, int32_t M, int32_t F, const float* out_i, const float* w_i,
                           int32_t accumulate, float* y, void* stream) {
  if (N < 1 || M < 1 || F < 1 || !out_i || !w_i || !y)
    return fail(CG_ERR_ARG, "stack_merge_forward: bad arguments");
  if (out_i == y) return fail(CG_ERR_ARG, "stack_merge_forward: y must not alias out_i");
  CG_HIP(cg::launch_stack_merge_fwd(out_i, w_i, N, int64_t(M) * F, accumulate, y,
                                    reinterpret_cast<hipStream_t>(stream)));
  return ok();
}

int cg_stack_merge_backward(int32_t N, int32_t M, int32_t F, const float* dy, const float* out_i,
                            const float* w_i, float* dout_i, float* dw_i, void* stream) {
  if (N < 1 || M < 1 || F < 1 || !dy || !out_i || !w_i || (!dout_i && !dw_i))
    return fail(CG_ERR_ARG, "stack_merge_backward: bad arguments");
  if (dout_i && (dout_i == out_i || dout_i == dy))
    return fail(CG_ERR_ARG, "stack_merge_backward: dout_i must not alias dy / out_i");
  CG_HIP(cg::launch_stack_merge_bwd(dy, out_i, w_i, N, int64_t(M) * F, dout_i, dw_i,
                                    reinterpret_cast<hipStream_t>(stream)));
  return ok();
}

int cg_weight_grad_workspace_bytes(int64_t R, int32_t FinK, int32_t Fout, size_t* bytes) {
  if (!bytes || R < 1 || FinK < 1 || Fout < 1) return fail(CG_ERR_ARG, "weight_grad: bad arguments");
  *bytes = dw_slab_bytes(R, 0, FinK, Fout);
  return ok();
}

int cg_weight_grad(int64_t R, int32_t FinK, int32_t Fout, const float* basis, const float* dy,
                   float* dW, int32_t accumulate, void* workspace, size_t ws_bytes, void* stream) {
  if (!basis || !dy || !dW || R < 1 || FinK < 1 || Fout < 1)
    return fail(CG_ERR_ARG, "weight_grad: bad arguments");
  const size_t need = dw_slab_bytes(R, 0, FinK, Fout);
  if (!workspace || ws_bytes < need)
    return fail(CG_ERR_ARG, "weight_grad workspace too small: %zu < %zu", ws_bytes, need);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* slabs = static_cast<float*>(workspace);
  CG_HIP(cg::launch_dw_slabs(basis, dy, R, FinK, Fout, slabs, s));
  CG_HIP(cg::launch_reduce_slabs_acc(slabs, cg::dw_chunks(R), int64_t(FinK) * Fout, dW,
                                     accumulate != 0, s));
  return ok();
}

int cg_weight_grad_planes(int64_t R, int32_t Fin, int32_t K, int32_t Fout, const float* planes,
                          int64_t plane_stride, const float* dy, float* dW, int32_t accumulate,
                          void* workspace, size_t ws_bytes, void* stream) {
  if (!planes || !dy || !dW || R < 1 || Fin < 1 || K < 1 || Fout < 1 || plane_stride < R * Fin)
    return fail(CG_ERR_ARG, "weight_grad_planes: bad arguments");
  const int FinK = Fin * K;
  const size_t need = dw_slab_bytes(R, 0, FinK, Fout);
  if (!workspace || ws_bytes < need)
    return fail(CG_ERR_ARG, "weight_grad_planes workspace too small: %zu < %zu", ws_bytes, need);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* slabs = static_cast<float*>(workspace);
  CG_HIP(cg::launch_dw_slabs(planes, dy, R, FinK, Fout, slabs, s, Fin, plane_stride, K));
  CG_HIP(cg::launch_reduce_slabs_acc(slabs, cg::dw_chunks(R), int64_t(FinK) * Fout, dW,
                                     accumulate != 0, s));
  return ok();
}

static size_t lstm_wgrad_rows(int32_t H, int32_t Fin, int32_t K) {
  return size_t(H + Fin) * size_t(K) + 1;
}

int cg_lstm_weight_grads_workspace_bytes(int64_t R, int32_t H, int32_t Fin, int32_t K,
                                         size_t* bytes) {
  if (!bytes || R < 1 || H < 1 || Fin < 1 || K < 1)
    return fail(CG_ERR_ARG, "lstm_weight_grads: bad arguments");
  const size_t rows = lstm_wgrad_rows(H, Fin, K);
  *bytes = dw_slab_bytes(R, 0, int(rows), 4 * H) + al256(rows * size_t(4 * H) * 4);
  return ok();
}

int cg_lstm_weight_grads(int64_t R, int32_t H, int32_t Fin, int32_t K, const float* h_planes,
                         int64_t h_plane_stride, const float* x_planes, int64_t x_plane_stride,
                         const float* dpre, float* dWh, float* dWx, float* db, void* workspace,
                         size_t ws_bytes, void* stream) {
  if (!h_planes || !x_planes || !dpre || !dWh || !dWx || !db || R < 1 || H < 1 || Fin < 1 ||
      K < 1 || h_plane_stride < R * H || x_plane_stride < R * Fin)
    return fail(CG_ERR_ARG, "lstm_weight_grads: bad arguments");
  if (4 * H > 256 || Fin * K + 1 > 64)
    return fail(CG_ERR_UNSUPPORTED, "lstm_weight_grads: needs 4H <= 256, Fin*K < 64 (H=%d Fin=%d K=%d)",
                H, Fin, K);
  size_t need = 0;
  int rc = cg_lstm_weight_grads_workspace_bytes(R, H, Fin, K, &need);
  if (rc) return rc;
  if (!workspace || ws_bytes < need)
    return fail(CG_ERR_ARG, "lstm_weight_grads workspace too small: %zu < %zu", ws_bytes, need);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int rows = int(lstm_wgrad_rows(H, Fin, K)), C = 4 * H;
  const size_t slab_bytes = dw_slab_bytes(R, 0, rows, C);
  float* slabs = static_cast<float*>(workspace);
  float* comb = reinterpret_cast<float*>(static_cast<char*>(workspace) + slab_bytes);
  CG_HIP(cg::launch_dw_slabs(h_planes, dpre, R, H * K, C, slabs, s, H, h_plane_stride, K, x_planes,
                             Fin, x_plane_stride));
  (void)comb;
  // the fixed-order slab sums straight into dWh | dWx | db (one launch, no copies)
  CG_HIP(cg::launch_reduce_slabs3(slabs, cg::dw_chunks(R), int64_t(rows) * C, dWh,
                                  int64_t(H) * K * C, dWx, int64_t(H + Fin) * K * C, db, s));
  return ok();
}

int cg_bias_grad_workspace_bytes(int64_t R, int32_t C, size_t* bytes) {
  if (!bytes || R < 1 || C < 1) return fail(CG_ERR_ARG, "bias_grad: bad arguments");
  *bytes = al256(size_t(cg::colsum_chunks(R)) * size_t(C) * 4);
  return ok();
}

int cg_bias_grad(int64_t R, int32_t C, const float* dy, float* db, int32_t accumulate,
                 void* workspace, size_t ws_bytes, void* stream) {
  if (!dy || !db || R < 1 || C < 1) return fail(CG_ERR_ARG, "bias_grad: bad arguments");
  const size_t need = al256(size_t(cg::colsum_chunks(R)) * size_t(C) * 4);
  if (!workspace || ws_bytes < need)
    return fail(CG_ERR_ARG, "bias_grad workspace too small: %zu < %zu", ws_bytes, need);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* slabs = static_cast<float*>(workspace);
  CG_HIP(cg::launch_colsum_slabs(dy, R, C, slabs, s));
  CG_HIP(cg::launch_reduce_slabs_acc(slabs, cg::colsum_chunks(R), C, db, accumulate != 0, s));
  return ok();
}

// ---- bias + activation (b1relu / b1tanh / b2relu) and fc GEMM -----------------
int cg_bias_act_forward(int64_t n, int32_t bias_len, const float* x, const float* bias,
                        int32_t act, float* y, void* stream) {
  if (!x || !y || n < 1) return fail(CG_ERR_ARG, "bias_act_forward: bad arguments");
  if (act < CG_ACT_NONE || act > CG_ACT_TANH) return fail(CG_ERR_ARG, "unknown activation %d", act);
  if (bias && (bias_len < 1 || n % bias_len))
    return fail(CG_ERR_ARG, "bias_act_forward: n=%lld is not a multiple of bias_len=%d",
                (long long)n, bias_len);
  CG_HIP(cg::launch_bias_act_fwd(x, bias, bias ? bias_len : 1, act, n, y,
                                 reinterpret_cast<hipStream_t>(stream)));
  return ok();
}

int cg_bias_act_workspace_bytes(int64_t n, int32_t bias_len, size_t* bytes) {
  if (!bytes || n < 1 || bias_len < 1 || n % bias_len)
    return fail(CG_ERR_ARG, "bias_act_workspace_bytes: bad arguments");
  *bytes = al256(size_t(cg::colsum_chunks(n / bias_len)) * size_t(bias_len) * 4);
  return ok();
}

int cg_bias_act_backward(int64_t n, int32_t bias_len, const float* dy, const float* y, int32_t act,
                         float* dz, float* db, int32_t accumulate, void* workspace,
                         size_t ws_bytes, void* stream) {
  if (!dy || !dz || n < 1) return fail(CG_ERR_ARG, "bias_act_backward: bad arguments");
  if (act < CG_ACT_NONE || act > CG_ACT_TANH) return fail(CG_ERR_ARG, "unknown activation %d", act);
  if (act != CG_ACT_NONE && !y) return fail(CG_ERR_ARG, "bias_act_backward: activation needs y");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  CG_HIP(cg::launch_bias_act_bwd(dy, y, act, n, dz, s));
  if (!db) return ok();
  if (bias_len < 1 || n % bias_len)
    return fail(CG_ERR_ARG, "bias_act_backward: n=%lld is not a multiple of bias_len=%d",
                (long long)n, bias_len);
  const int64_t R = n / bias_len;
  const size_t need = al256(size_t(cg::colsum_chunks(R)) * size_t(bias_len) * 4);
  if (!workspace || ws_bytes < need)
    return fail(CG_ERR_ARG, "bias_act workspace too small: %zu < %zu", ws_bytes, need);
  float* slabs = static_cast<float*>(workspace);
  CG_HIP(cg::launch_colsum_slabs(dz, R, bias_len, slabs, s));
  CG_HIP(cg::launch_reduce_slabs_acc(slabs, cg::colsum_chunks(R), bias_len, db, accumulate != 0, s));
  return ok();
}

int cg_gemm_f32(int32_t trans_a, int32_t trans_b, int32_t M, int32_t N, int32_t K, const float* A,
                int32_t lda, const float* B, int32_t ldb, float* C, int32_t ldc, void* stream) {
  if (!A || !B || !C || M < 1 || N < 1 || K < 1) return fail(CG_ERR_ARG, "gemm_f32: bad arguments");
  if (lda < (trans_a ? M : K) || ldb < (trans_b ? K : N) || ldc < N)
    return fail(CG_ERR_ARG, "gemm_f32: leading dimension too small (lda=%d ldb=%d ldc=%d)", lda, ldb,
                ldc);
  if ((M + 63) / 64 > 2147483647 / 2 || (N + 63) / 64 > 65535)
    return fail(CG_ERR_ARG, "gemm_f32: N=%d too large for the grid", N);
  CG_HIP(cg::launch_gemm_f32(trans_a != 0, trans_b != 0, M, N, K, A, lda, B, ldb, C, ldc, 1,
                             reinterpret_cast<hipStream_t>(stream)));
  return ok();
}

// ---- Fourier filter (lib/graph_conv.py:83-111) ----------------------------------
static bool fourier_shape_ok(int32_t N, int32_t M, int32_t Fin, int32_t Fout) {
  if (N < 1 || M < 1 || Fin < 1 || Fout < 1 || N > 65535) return false;
  const int64_t big = int64_t(N) * (Fin > Fout ? Fin : Fout) * M;
  return big < (int64_t(1) << 31) && M <= 65535 * 32;
}

static void fourier_ws(int32_t N, int32_t M, int32_t Fin, int32_t Fout, size_t* fwd, size_t* bwd) {
  const size_t xin = size_t(N) * Fin * M * 4, yout = size_t(N) * Fout * M * 4;
  if (fwd) *fwd = (Fin > 1 ? al256(xin) : 0) + al256(yout) + (Fout > 1 ? al256(yout) : 0);
  if (bwd) *bwd = (Fout > 1 ? al256(yout) : 0) + al256(yout) + al256(xin) + (Fin > 1 ? al256(xin) : 0);
}

int cg_fourier_workspace_bytes(int32_t N, int32_t M, int32_t Fin, int32_t Fout, size_t* fwd_bytes,
                               size_t* bwd_bytes) {
  if (!fourier_shape_ok(N, M, Fin, Fout)) return fail(CG_ERR_ARG, "fourier: bad shape");
  fourier_ws(N, M, Fin, Fout, fwd_bytes, bwd_bytes);
  return ok();
}

int cg_fourier_forward(int32_t N, int32_t M, int32_t Fin, int32_t Fout, const float* U,
                       const float* W, const float* x, float* xhat, float* y, void* workspace,
                       size_t ws_bytes, void* stream) {
  if (!U || !W || !x || !xhat || !y) return fail(CG_ERR_ARG, "fourier_forward: null pointer");
  if (!fourier_shape_ok(N, M, Fin, Fout)) return fail(CG_ERR_ARG, "fourier_forward: bad shape");
  size_t need;
  fourier_ws(N, M, Fin, Fout, &need, nullptr);
  if (ws_bytes < need || (need && !workspace))
    return fail(CG_ERR_ARG, "fourier_forward workspace too small: %zu < %zu", ws_bytes, need);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  char* w = static_cast<char*>(workspace);
  const size_t xin = size_t(N) * Fin * M * 4, yout = size_t(N) * Fout * M * 4;
  const float* xs = x;
  if (Fin > 1) {  // [N][M][Fin] -> [N][Fin][M]
    float* xt = reinterpret_cast<float*>(w);
    w += al256(xin);
    CG_HIP(cg::launch_transpose_batched(x, N, M, Fin, xt, s));
    xs = xt;
  }
  float* Yh = reinterpret_cast<float*>(w);
  w += al256(yout);
  // Xh = x U  (every signal row against the eigenvector matrix: U^T x of :90)
  CG_HIP(cg::launch_gemm_f32(false, false, N * Fin, M, M, xs, M, U, M, xhat, M, 1, s));
  CG_HIP(cg::launch_fourier_mix(xhat, W, N, M, Fin, Fout, Yh, s));
  // y = Yh U^T (inverse transform, :97)
  float* yt = Fout > 1 ? reinterpret_cast<float*>(w) : y;
  CG_HIP(cg::launch_gemm_f32(false, true, N * Fout, M, M, Yh, M, U, M, yt, M, 1, s));
  if (Fout > 1) CG_HIP(cg::launch_transpose_batched(yt, N, Fout, M, y, s));
  return ok();
}

int cg_fourier_backward(int32_t N, int32_t M, int32_t Fin, int32_t Fout, const float* U,
                        const float* W, const float* xhat, const float* dy, float* dx, float* dW,
                        void* workspace, size_t ws_bytes, void* stream) {
  if (!U || !W || !xhat || !dy) return fail(CG_ERR_ARG, "fourier_backward: null pointer");
  if (!fourier_shape_ok(N, M, Fin, Fout)) return fail(CG_ERR_ARG, "fourier_backward: bad shape");
  size_t need;
  fourier_ws(N, M, Fin, Fout, nullptr, &need);
  if (!workspace || ws_bytes < need)
    return fail(CG_ERR_ARG, "fourier_backward workspace too small: %zu < %zu", ws_bytes, need);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  char* w = static_cast<char*>(workspace);
  const size_t xin = size_t(N) * Fin * M * 4, yout = size_t(N) * Fout * M * 4;
  const float* dys = dy;
  if (Fout > 1) {
    float* dyt = reinterpret_cast<float*>(w);
    w += al256(yout);
    CG_HIP(cg::launch_transpose_batched(dy, N, M, Fout, dyt, s));
    dys = dyt;
  }
  float* dYh = reinterpret_cast<float*>(w);
  w += al256(yout);
  float* dXh = reinterpret_cast<float*>(w);
  w += al256(xin);
  CG_HIP(cg::launch_gemm_f32(false, false, N * Fout, M, M, dys, M, U, M, dYh, M, 1, s));
  if (dW) CG_HIP(cg::launch_fourier_dw(dYh, xhat, N, M, Fin, Fout, dW, s));
  if (dx) {
    CG_HIP(cg::launch_fourier_mix_t(dYh, W, N, M, Fin, Fout, dXh, s));
    float* dxt = Fin > 1 ? reinterpret_cast<float*>(w) : dx;
    CG_HIP(cg::launch_gemm_f32(false, true, N * Fin, M, M, dXh, M, U, M, dxt, M, 1, s));
    if (Fin > 1) CG_HIP(cg::launch_transpose_batched(dxt, N, Fin, M, dx, s));
  }
  return ok();
}

static int check_lstm(int64_t R, int32_t H, int32_t gates) {
  if (R < 1 || H < 1) return fail(CG_ERR_ARG, "lstm: bad shape R=%lld H=%d", (long long)R, H);
  if (R * int64_t(H) * 4 >= (int64_t(1) << 31))
    return fail(CG_ERR_ARG, "lstm: R*4H = %lld exceeds 2^31", (long long)(R * H * 4));
  if (gates != CG_LSTM_GATES_REFERENCE && gates != CG_LSTM_GATES_STANDARD)
    return fail(CG_ERR_ARG, "lstm: unknown gate set %d", gates);
  return CG_OK;
}

int cg_lstm_cell_forward(int64_t R, int32_t H, int32_t gates, const float* gx, const float* gh,
                         const float* bias, const float* c, float* c_out, float* h_out, float* act,
                         void* stream) {
  int rc = check_lstm(R, H, gates);
  if (rc) return rc;
  if (!gx || !c_out || !h_out) return fail(CG_ERR_ARG, "lstm_cell_forward: null gx/c_out/h_out");
  CG_HIP(cg::launch_lstm_fwd(gates, R, H, gx, gh, bias, c, c_out, h_out, act,
                             reinterpret_cast<hipStream_t>(stream)));
  return ok();
}

int cg_lstm_cell_backward(int64_t R, int32_t H, int32_t gates, const float* dh,
                          const float* dh_rec, const float* dc,
                          const float* act, const float* c, const float* c_out, float* dpre,
                          float* dc_prev, void* stream) {
  int rc = check_lstm(R, H, gates);
  if (rc) return rc;
  if (!act || !c_out || !dpre) return fail(CG_ERR_ARG, "lstm_cell_backward: null act/c_out/dpre");
  CG_HIP(cg::launch_lstm_bwd(gates, R, H, dh, dh_rec, dc, act, c, c_out, dpre, dc_prev,
                             reinterpret_cast<hipStream_t>(stream)));
  return ok();
}

int cg_lstm_hconv_supported(const cg_plan* plan, int32_t H, int32_t K, int32_t* supported) {
  if (!plan || !supported) return fail(CG_ERR_ARG, "lstm_hconv_supported: null argument");
  *supported = cg::lstm_hstep_ok(plan->M, H, K) ? 1 : 0;
  return ok();
}

int cg_lstm_hconv_step(cg_plan* plan, int32_t N, int32_t H, int32_t K, int32_t gates,
                       const float* h_prev, const float* c_prev, const float* gx, const float* Wh,
                       const float* bias, float* c_out, float* h_out, float* act, float* planes,
                       int64_t plane_stride, void* stream) {
  int rc = check_lstm(int64_t(N) * (plan ? plan->M : 1), H, gates);
  if (rc) return rc;
  if (!plan || N < 1 || K < 1) return fail(CG_ERR_ARG, "lstm_hconv_step: bad plan / N / K");
  if (!h_prev || !gx || !Wh || !c_out || !h_out)
    return fail(CG_ERR_ARG, "lstm_hconv_step: null h_prev / gx / Wh / c_out / h_out");
  if (!cg::lstm_hstep_ok(plan->M, H, K))
    return fail(CG_ERR_UNSUPPORTED, "lstm_hconv_step: needs H = 32, M <= 1024 and the LDS for K "
                                    "(M=%d H=%d K=%d)", plan->M, H, K);
  if (planes && K > 1 && plane_stride < int64_t(N) * plan->M * H)
    return fail(CG_ERR_ARG, "lstm_hconv_step: plane stride %lld < N*M*H", (long long)plane_stride);
  // the kernel moves h_prev and the planes as float4
  if ((reinterpret_cast<uintptr_t>(h_prev) & 15) || (planes && (reinterpret_cast<uintptr_t>(planes) & 15)) ||
      (planes && K > 1 && (plane_stride & 3)))
    return fail(CG_ERR_ARG, "lstm_hconv_step: h_prev / planes must be 16-byte aligned and the "
                            "plane stride a multiple of 4 floats");
  const void* outs[] = {c_out, h_out, act, planes};
  const void* ins[] = {h_prev, c_prev, gx};
  for (const void* o : outs)
    for (const void* i : ins)
      if (o && o == i) return fail(CG_ERR_ARG, "lstm_hconv_step: outputs must not alias inputs");
  if ((rc = check_device(plan))) return rc;
  CG_HIP(cg::launch_lstm_hstep(gates, N, plan->M, K, plan->rowptr, plan->col, plan->val, h_prev,
                               c_prev, gx, Wh, bias, c_out, h_out, act, planes, plane_stride,
                               reinterpret_cast<hipStream_t>(stream)));
  return ok();
}

static bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

int cg_lstm_seq_supported(const cg_plan* plan, int32_t H, int32_t K, int32_t* supported) {
  if (!plan || !supported) return fail(CG_ERR_ARG, "lstm_seq_supported: null argument");
  *supported =
      (cg::lstm_seq_ok(plan->M, H, K, plan->nnz) && cg::lstm_bstep_ok(plan->M, H, K, plan->nnzT)) ? 1 : 0;
  return ok();
}

int cg_lstm_seq_x_supported(const cg_plan* plan, int32_t Fin, int32_t H, int32_t K, int32_t* supported) {
  if (!plan || !supported) return fail(CG_ERR_ARG, "lstm_seq_x_supported: null argument");
  *supported = (Fin >= 1 && Fin <= 8 && cg::lstm_seq_ok(plan->M, H, K, plan->nnz, Fin) &&
                cg::lstm_bstep_ok(plan->M, H, K, plan->nnzT)) ? 1 : 0;
  return ok();
}

int cg_lstm_seq_workspace_bytes(const cg_plan* plan, int32_t N, size_t* bytes) {
  if (!plan || !bytes || N < 1) return fail(CG_ERR_ARG, "lstm_seq_workspace_bytes: bad arguments");
  *bytes = al256(sizeof(int) * size_t(2) * cg::lstm_seq_pairs(N, plan->device));
  return ok();
}

static int lstm_seq_impl(cg_plan* plan, int32_t T, int32_t N, int32_t H, int32_t K, int32_t gates,
                         const float* gx, const float* xs, const float* Wx, int32_t Fin,
                         float* xplanes, int64_t xplane_stride, const float* Wh, const float* bias,
                         const float* h0, const float* c0, float* hs, float* cs, float* act,
                         float* planes, int64_t plane_stride, void* workspace, size_t ws_bytes,
                         void* stream) {
  int rc = check_lstm(int64_t(T) * N * (plan ? plan->M : 1), H, gates);
  if (rc) return rc;
  if (!plan || T < 1 || N < 1 || K < 1) return fail(CG_ERR_ARG, "lstm_seq_forward: bad plan / T / N / K");
  if ((!gx && !xs) || !Wh || !hs || !cs) return fail(CG_ERR_ARG, "lstm_seq_forward: null gx|xs / Wh / hs / cs");
  if (xs && (Fin < 1 || Fin > 8 || !Wx || !xplanes))
    return fail(CG_ERR_ARG, "lstm_seq_forward_x: needs 1 <= feat_in <= 8, Wx and the x planes");
  if (!cg::lstm_seq_ok(plan->M, H, K, plan->nnz, xs ? Fin : 0))
    return fail(CG_ERR_UNSUPPORTED, "lstm_seq_forward: needs H = 32, M <= 1024 and L~ plus the "
                                    "weights in LDS (M=%d nnz=%lld H=%d K=%d)",
                plan->M, (long long)plan->nnz, H, K);
  const int64_t R = int64_t(T) * N * plan->M;
  if (!planes && K > 1)
    return fail(CG_ERR_ARG, "lstm_seq_forward: planes are required for K > 1 (the pair hands "
                            "its quarters' Chebyshev orders to the partner through them)");
  if (planes && K > 1 && plane_stride < R * H)
    return fail(CG_ERR_ARG, "lstm_seq_forward: plane stride %lld < T*N*M*H", (long long)plane_stride);
  if (xs && xplane_stride < R * Fin)
    return fail(CG_ERR_ARG, "lstm_seq_forward_x: x plane stride %lld < T*N*M*feat_in",
                (long long)xplane_stride);
  if ((gx && !al16(gx)) || !al16(hs) || !al16(cs) || (act && !al16(act)) || (planes && !al16(planes)) ||
      (h0 && !al16(h0)) || (c0 && !al16(c0)) || (bias && !al16(bias)) ||
      (planes && K > 1 && (plane_stride & 3)))
    return fail(CG_ERR_ARG, "lstm_seq_forward: tensors must be 16-byte aligned (float4 access), "
                            "plane stride a multiple of 4");
  const void* outs[] = {hs, cs, act, planes, xplanes};
  const void* ins[] = {gx, xs, Wx, Wh, bias, h0, c0};
  for (const void* o : outs)
    for (const void* i : ins)
      if (o && o == i) return fail(CG_ERR_ARG, "lstm_seq_forward: outputs must not alias inputs");
  size_t need = 0;
  if ((rc = cg_lstm_seq_workspace_bytes(plan, N, &need))) return rc;
  if (!workspace || ws_bytes < need)
    return fail(CG_ERR_ARG, "lstm_seq_forward: workspace %zu < %zu bytes", ws_bytes, need);
  if ((rc = check_device(plan))) return rc;
  const int P = cg::lstm_seq_pairs(N, plan->device);
  int* flags = static_cast<int*>(workspace);
  if (!plan->seq_fault) {
    void* hp = nullptr;
    CG_HIP(hipHostMalloc(&hp, 64, hipHostMallocMapped | hipHostMallocCoherent));
    plan->seq_fault = static_cast<int*>(hp);
    *plan->seq_fault = 0;
    void* dp = nullptr;
    CG_HIP(hipHostGetDevicePointer(&dp, hp, 0));
    plan->seq_fault_dev = static_cast<int*>(dp);
    CG_HIP(hipEventCreateWithFlags(&plan->seq_event, hipEventDisableTiming));
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  CG_HIP(cg::launch_lstm_seq(gates, T, N, plan->M, K, plan->nnz, plan->rowptr, plan->col, plan->val,
                             plan->lorder, xs, Wx, Fin, xplanes, xplane_stride, gx, Wh, bias, h0,
                             c0, hs, cs, act, planes, plane_stride, flags, plan->seq_fault_dev, P, s,
                             plan->seq_fault_test, plan->max_row_nnz));
  CG_HIP(hipEventRecord(plan->seq_event, s));
  plan->seq_launched = true;
  return ok();
}

int cg_lstm_seq_forward(cg_plan* plan, int32_t T, int32_t N, int32_t H, int32_t K, int32_t gates,
                        const float* gx, const float* Wh, const float* bias, const float* h0,
                        const float* c0, float* hs, float* cs, float* act, float* planes,
                        int64_t plane_stride, void* workspace, size_t ws_bytes, void* stream) {
  return lstm_seq_impl(plan, T, N, H, K, gates, gx, nullptr, nullptr, 0, nullptr, 0, Wh, bias, h0,
                       c0, hs, cs, act, planes, plane_stride, workspace, ws_bytes, stream);
}

int cg_lstm_seq_forward_x(cg_plan* plan, int32_t T, int32_t N, int32_t Fin, int32_t H, int32_t K,
                          int32_t gates, const float* xs, const float* Wx, float* xplanes,
                          int64_t xplane_stride, const float* Wh, const float* bias,
                          const float* h0, const float* c0, float* hs, float* cs, float* act,
                          float* planes, int64_t plane_stride, void* workspace, size_t ws_bytes,
                          void* stream) {
  if (!xs) return fail(CG_ERR_ARG, "lstm_seq_forward_x: null xs");
  return lstm_seq_impl(plan, T, N, H, K, gates, nullptr, xs, Wx, Fin, xplanes, xplane_stride, Wh,
                       bias, h0, c0, hs, cs, act, planes, plane_stride, workspace, ws_bytes, stream);
}

int cg_lstm_seq_fault(cg_plan* plan, int32_t wait, int32_t clear, int32_t* fault) {
  if (!plan || !fault) return fail(CG_ERR_ARG, "lstm_seq_fault: null argument");
  *fault = 0;
  if (!plan->seq_launched) return ok();
  if (wait) {
    CG_HIP(hipEventSynchronize(plan->seq_event));
  } else {
    const hipError_t q = hipEventQuery(plan->seq_event);
    if (q == hipErrorNotReady) {
      *fault = -1;  // the last sequence launch is still in flight
      return ok();
    }
    if (q != hipSuccess) return fail(CG_ERR_HIP, "lstm_seq_fault: %s", hipGetErrorString(q));
  }
  const int v = __atomic_load_n(plan->seq_fault, __ATOMIC_ACQUIRE);
  if (!v) return ok();
  *fault = 1;
  if (clear) __atomic_store_n(plan->seq_fault, 0, __ATOMIC_RELEASE);
  return fail(CG_ERR_HIP, "lstm_seq_forward: a workgroup pair hand-off timed out (a partner "
                          "workgroup was not co-resident); the launch's hs / cs / act hold NaN "
                          "from the lost step on");
}

int cg_lstm_seq_status(const cg_plan* plan, int32_t N, const void* workspace, int32_t* status,
                       void* stream) {
  if (!plan || !status || N < 1) return fail(CG_ERR_ARG, "lstm_seq_status: bad arguments");
  (void)workspace;  // the fault word lives in the plan (sticky), not in the workspace
  CG_HIP(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));
  return cg_lstm_seq_fault(const_cast<cg_plan*>(plan), 1, 0, status);
}

int cg_plan_set_seq_fault_test(cg_plan* plan, int32_t step) {
  if (!plan || step < -1) return fail(CG_ERR_ARG, "plan_set_seq_fault_test: bad arguments");
  plan->seq_fault_test = step;
  return ok();
}

int cg_lstm_bwd_step(cg_plan* plan, int32_t N, int32_t H, int32_t K, int32_t gates, const float* dh,
                     const float* dh_rec, const float* dc, const float* act,
                     int32_t act_unit_major, const float* c_prev, const float* c_out,
                     const float* Wh, float* dpre, float* dc_prev, float* dh_prev, void* stream) {
  int rc = check_lstm(int64_t(N) * (plan ? plan->M : 1), H, gates);
  if (rc) return rc;
  if (!plan || N < 1 || K < 1) return fail(CG_ERR_ARG, "lstm_bwd_step: bad plan / N / K");
  if (!act || !c_out || !Wh || !dpre)
    return fail(CG_ERR_ARG, "lstm_bwd_step: null act / c_out / Wh / dpre");
  if (!cg::lstm_bstep_ok(plan->M, H, K, plan->nnzT))
    return fail(CG_ERR_UNSUPPORTED, "lstm_bwd_step: needs H = 32, M <= 1024, K <= 4 (M=%d H=%d K=%d)",
                plan->M, H, K);
  const void* all[] = {dh, dh_rec, dc, act, c_prev, c_out, dpre, dc_prev, dh_prev};
  for (const void* p : all)
    if (p && !al16(p)) return fail(CG_ERR_ARG, "lstm_bwd_step: tensors must be 16-byte aligned");
  const void* outs[] = {dpre, dc_prev, dh_prev};
  const void* ins[] = {dh, dh_rec, dc, act, c_prev, c_out, Wh};
  for (const void* o : outs)
    for (const void* i : ins)
      if (o && o == i) return fail(CG_ERR_ARG, "lstm_bwd_step: outputs must not alias inputs");
  if ((rc = check_device(plan))) return rc;
  if (!dh_prev) {  // no h-conv at this step (a zero-state layer's step 0): the pointwise part
    CG_HIP(cg::launch_lstm_bwd(gates, int64_t(N) * plan->M, H, dh, dh_rec, dc, act, c_prev, c_out,
                               dpre, dc_prev, reinterpret_cast<hipStream_t>(stream),
                               act_unit_major));
    return ok();
  }
  CG_HIP(cg::launch_lstm_bstep(gates, N, plan->M, K, plan->trowptr, plan->tcol, plan->tval,
                               plan->tlorder, plan->nnzT, dh, dh_rec,
                               dc, act, act_unit_major, c_prev, c_out, Wh, dpre, dc_prev, dh_prev,
                               reinterpret_cast<hipStream_t>(stream)));
  return ok();
}

int cg_perm_gather(const float* x, const int32_t* perm, int32_t N, int32_t M_in, int32_t M_out,
                   int32_t F, float* out, void* stream) {
  if (!x || !perm || !out || N < 1 || M_in < 1 || M_out < 1 || F < 1)
    return fail(CG_ERR_ARG, "perm_gather: bad arguments");
  CG_HIP(cg::launch_perm_gather(x, perm, N, M_in, M_out, F, out,
                                reinterpret_cast<hipStream_t>(stream)));
  return ok();
}

int cg_maxpool_forward(const float* x, int32_t N, int32_t M, int32_t F, int32_t p, float* y,
                       int32_t* argmax, void* stream) {
  if (!x || !y || N < 1 || M < 1 || F < 1 || p < 1 || M % p)
    return fail(CG_ERR_ARG, "maxpool_forward: bad arguments (M=%d p=%d)", M, p);
  CG_HIP(cg::launch_maxpool_fwd(x, N, M, F, p, y, argmax, reinterpret_cast<hipStream_t>(stream)));
  return ok();
}

int cg_maxpool_backward(const float* dy, const int32_t* argmax, int32_t N, int32_t M, int32_t F,
                        int32_t p, float* dx, void* stream) {
  if (!dy || !argmax || !dx || N < 1 || M < 1 || F < 1 || p < 1 || M % p)
    return fail(CG_ERR_ARG, "maxpool_backward: bad arguments (M=%d p=%d)", M, p);
  CG_HIP(cg::launch_maxpool_bwd(dy, argmax, N, M, F, p, dx, reinterpret_cast<hipStream_t>(stream)));
  return ok();
}

int cg_avgpool_forward(const float* x, int32_t N, int32_t M, int32_t F, int32_t p, float* y,
                       void* stream) {
  if (!x || !y || N < 1 || M < 1 || F < 1 || p < 1 || M % p)
    return fail(CG_ERR_ARG, "avgpool_forward: bad arguments (M=%d p=%d)", M, p);
  CG_HIP(cg::launch_avgpool_fwd(x, N, M, F, p, y, reinterpret_cast<hipStream_t>(stream)));
  return ok();
}

int cg_avgpool_backward(const float* dy, int32_t N, int32_t M, int32_t F, int32_t p, float* dx,
                        void* stream) {
  if (!dy || !dx || N < 1 || M < 1 || F < 1 || p < 1 || M % p)
    return fail(CG_ERR_ARG, "avgpool_backward: bad arguments (M=%d p=%d)", M, p);
  CG_HIP(cg::launch_avgpool_bwd(dy, N, M, F, p, dx, reinterpret_cast<hipStream_t>(stream)));
  return ok();
}

int cg_adam_update(float* param, const float* grad, float* m, float* v, int64_t n, float lr,
                   float beta1, float beta2, float eps, int32_t step, float grad_scale,
                   void* stream) {
  if (!param || !grad || !m || !v || n < 0 || step < 1)
    return fail(CG_ERR_ARG, "adam_update: bad arguments");
  if (n == 0) return ok();
  const double lr_t =
      double(lr) * std::sqrt(1.0 - std::pow(double(beta2), step)) / (1.0 - std::pow(double(beta1), step));
  CG_HIP(cg::launch_adam(param, grad, m, v, n, float(lr_t), beta1, beta2, eps, grad_scale,
                         reinterpret_cast<hipStream_t>(stream)));
  return ok();
}

int cg_sgd_update(float* param, const float* grad, int64_t n, float lr, float grad_scale,
                  void* stream) {
  if (!param || !grad || n < 0) return fail(CG_ERR_ARG, "sgd_update: bad arguments");
  if (n == 0) return ok();
  CG_HIP(cg::launch_sgd(param, grad, n, lr, grad_scale, reinterpret_cast<hipStream_t>(stream)));
  return ok();
}

int cg_rmsprop_update(float* param, const float* grad, float* ms, float* mom, int64_t n, float lr,
                      float rho, float momentum, float eps, float grad_scale, void* stream) {
  if (!param || !grad || !ms || !mom || n < 0 || !(eps > 0.f))
    return fail(CG_ERR_ARG, "rmsprop_update: bad arguments");
  if (n == 0) return ok();
  CG_HIP(cg::launch_rmsprop(param, grad, ms, mom, n, lr, rho, momentum, eps, grad_scale,
                            reinterpret_cast<hipStream_t>(stream)));
  return ok();
}

}  // extern "C"
