// Host-side graph coarsening for the pooling hierarchy (lib/coarsening.py).
//
// The reference runs these as pure-Python loops (seconds per graph at MNIST
// size, minutes at 10^5 vertices); they are restated here as plain C++ with
// the reference's exact visiting order and arithmetic, so the pooling
// indices that drive the device perm/max-pool kernels are identical.
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "../../include/cheb_mi355.h"

extern "C" int cg_internal_set_error(int code, const char* msg);

namespace {

int set_error(int code, const char* fmt, ...) {
  char buf[256];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return cg_internal_set_error(code, buf);
}

// lib/coarsening.py:119-165.  Note the reference's quirks, kept on purpose:
//  * rowlength[count] is incremented BEFORE the row-change test (:128-132),
//    so the first entry of a row is credited to the previous row's length;
//  * rowstart/rowlength are indexed by the ordinal of the distinct row, which
//    equals the vertex id only when no row is empty;
//  * a marked neighbour scores 0 and only a strictly larger score replaces the
//    current best (first maximum in stored order wins).
template <typename T>
int graclus_match(int64_t nnz, const int32_t* rr, const int32_t* cc, const T* vv, int32_t n_visit,
                  const int64_t* rid, const T* weights, int32_t* cluster_id, int32_t* n_clusters) {
#pragma clang fp contract(off)
  if (nnz < 1 || !rr || !cc || !vv || !rid || !weights || !cluster_id || !n_clusters)
    return set_error(CG_ERR_ARG, "graclus_match: empty graph or null argument");
  const int64_t N = int64_t(rr[nnz - 1]) + 1;
  if (N < 1) return set_error(CG_ERR_ARG, "graclus_match: negative row index");
  std::vector<char> marked(size_t(N), 0);
  std::vector<int64_t> rowstart(size_t(N), 0), rowlength(size_t(N), 0);
  for (int64_t i = 0; i < N; ++i) cluster_id[i] = 0;
  int64_t oldval = rr[0], count = 0;
  for (int64_t ii = 0; ii < nnz; ++ii) {
    if (count >= N) return set_error(CG_ERR_ARG, "graclus_match: rows not ascending");
    rowlength[size_t(count)] += 1;
    if (rr[ii] > oldval) {
      oldval = rr[ii];
      if (count + 1 >= N) return set_error(CG_ERR_ARG, "graclus_match: rows not ascending");
      rowstart[size_t(count + 1)] = ii;
      count += 1;
    }
  }
  int32_t clustercount = 0;
  for (int64_t ii = 0; ii < N; ++ii) {
    if (ii >= n_visit) return set_error(CG_ERR_ARG, "graclus_match: visit order too short");
    const int64_t tid = rid[ii];
    if (tid < 0 || tid >= N)
      return set_error(CG_ERR_ARG, "graclus_match: visit order entry %lld out of range",
                           static_cast<long long>(tid));
    if (marked[size_t(tid)]) continue;
    T wmax = T(0);
    const int64_t rs = rowstart[size_t(tid)];
    marked[size_t(tid)] = 1;
    int64_t best = -1;
    for (int64_t jj = 0; jj < rowlength[size_t(tid)]; ++jj) {
      if (rs + jj >= nnz) break;  // the reference would raise IndexError here
      const int64_t nid = cc[rs + jj];
      if (nid < 0 || nid >= N) return set_error(CG_ERR_ARG, "graclus_match: column out of range");
      T tval;
      if (marked[size_t(nid)]) {
        tval = T(0);
      } else {
        const T a = T(1) / weights[tid];
        const T b = T(1) / weights[nid];
        const T s = a + b;
        tval = vv[rs + jj] * s;
      }
      if (tval > wmax) {
        wmax = tval;
        best = nid;
      }
    }
    cluster_id[tid] = clustercount;
    if (best > -1) {
      cluster_id[best] = clustercount;
      marked[size_t(best)] = 1;
    }
    clustercount += 1;
  }
  *n_clusters = clustercount;
  return cg_internal_set_error(CG_OK, nullptr);
}

}  // namespace

extern "C" {

int cg_graclus_match_f32(int64_t nnz, const int32_t* rr, const int32_t* cc, const float* vv,
                         int32_t n_visit, const int64_t* rid, const float* weights,
                         int32_t* cluster_id, int32_t* n_clusters) {
  return graclus_match<float>(nnz, rr, cc, vv, n_visit, rid, weights, cluster_id, n_clusters);
}

int cg_graclus_match_f64(int64_t nnz, const int32_t* rr, const int32_t* cc, const double* vv,
                         int32_t n_visit, const int64_t* rid, const double* weights,
                         int32_t* cluster_id, int32_t* n_clusters) {
  return graclus_match<double>(nnz, rr, cc, vv, n_visit, rid, weights, cluster_id, n_clusters);
}

// lib/coarsening.py:167-214: walk from the coarsest level down; a real coarse
// vertex expands to its children in ascending id order (plus one new fake
// vertex if it is a singleton), a fake coarse vertex to two new fakes.  Fake
// ids continue after the level's real vertices in creation order.
int cg_compute_perm(int32_t levels, const int32_t* sizes, const int32_t* parents,
                    int32_t* perm_out, int64_t perm_cap, int32_t* sizes_out) {
  if (levels < 1 || !sizes || !parents || !perm_out || !sizes_out)
    return set_error(CG_ERR_ARG, "compute_perm: levels < 1 or null argument");
  std::vector<int64_t> off(size_t(levels) + 1, 0);
  for (int l = 0; l < levels; ++l) {
    if (sizes[l] < 1) return set_error(CG_ERR_ARG, "compute_perm: empty level %d", l);
    off[size_t(l) + 1] = off[size_t(l)] + sizes[l];
  }
  const int64_t n_last = sizes[levels];
  if (n_last < 1) return set_error(CG_ERR_ARG, "compute_perm: no coarsest vertices");
  // output offsets: level l holds n_last * 2^(levels-l) entries
  std::vector<int64_t> out_off(size_t(levels) + 2, 0);
  for (int l = 0; l <= levels; ++l) {
    const int64_t len = n_last << (levels - l);
    sizes_out[l] = static_cast<int32_t>(len);
    out_off[size_t(l) + 1] = out_off[size_t(l)] + len;
  }
  if (out_off[size_t(levels) + 1] > perm_cap)
    return set_error(CG_ERR_ARG, "compute_perm: perm_out capacity %lld < %lld",
                         static_cast<long long>(perm_cap),
                         static_cast<long long>(out_off[size_t(levels) + 1]));
  int32_t* coarse = perm_out + out_off[size_t(levels)];
  for (int64_t i = 0; i < n_last; ++i) coarse[i] = static_cast<int32_t>(i);
  for (int l = levels - 1; l >= 0; --l) {
    const int32_t* par = parents + off[size_t(l)];
    const int64_t n_fine = sizes[l];
    int64_t n_coarse = 0;  // max(parent) + 1, as np.where(parent == i) sees it
    for (int64_t v = 0; v < n_fine; ++v) n_coarse = par[v] + 1 > n_coarse ? par[v] + 1 : n_coarse;
    // children of each real coarse vertex, ascending (at most two)
    std::vector<int32_t> ch(size_t(n_coarse) * 2, -1);
    std::vector<uint8_t> nch(size_t(n_coarse), 0);
    for (int64_t v = 0; v < n_fine; ++v) {
      const int64_t p = par[v];
      if (p < 0)
        return set_error(CG_ERR_ARG, "compute_perm: parent %lld of level %d out of range",
                             static_cast<long long>(p), l);
      if (nch[size_t(p)] >= 2)
        return set_error(CG_ERR_ARG, "compute_perm: vertex %lld of level %d has > 2 children",
                             static_cast<long long>(p), l + 1);
      ch[size_t(p) * 2 + nch[size_t(p)]++] = static_cast<int32_t>(v);
    }
    const int32_t* up = perm_out + out_off[size_t(l) + 1];
    const int64_t n_up = sizes_out[l + 1];
    int32_t* dst = perm_out + out_off[size_t(l)];
    int64_t w = 0, fake = n_fine;
    for (int64_t t = 0; t < n_up; ++t) {
      const int64_t i = up[t];
      const int k = (i < n_coarse) ? nch[size_t(i)] : 0;
      for (int c = 0; c < k; ++c) dst[w++] = ch[size_t(i) * 2 + c];
      for (int c = k; c < 2; ++c) dst[w++] = static_cast<int32_t>(fake++);
    }
  }
  return cg_internal_set_error(CG_OK, nullptr);
}

}  // extern "C"
