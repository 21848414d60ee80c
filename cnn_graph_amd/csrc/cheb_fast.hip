// Geometry and dispatch of the fast resident kernels (cheb_fast_kern.h; the
// instantiations are compiled separately from cheb_fast_inst.hip).
#include <algorithm>

#include "cg_internal.h"

namespace cg {
namespace fastk {
template <int FV, int NT, bool OB>
hipError_t launch_fwd_fast_t(size_t lds, int N, const FastFwdArgs& a, hipStream_t s);
template <int FV, int DW>
hipError_t launch_bwd_fast_t(size_t lds, int N, const FastBwdArgs& a, hipStream_t s);
}  // namespace fastk

FastGeom fast_geometry(int M, int P, int max_row_nnz, int max_row_nnzT, int Fin, int K, int Fout) {
  FastGeom g{};
  const bool fin_ok = Fin == 1 || Fin == 2 || Fin == 4;
  const size_t FinK = size_t(Fin) * K;
  const size_t rec = 12 * size_t(Fin);
  const size_t ring = align16(size_t(P) * rec);
  g.nt = (Fout + 31) / 32;
  g.fwd_lds_ob = ring + align16(FinK * Fout * 4);  // orders layout: no basis staging
  g.fwd_lds = g.fwd_lds_ob + size_t(M) * FinK * 4;
  g.dw_fused = FinK <= 32 && Fout <= 32 && Fout % 8 == 0;  // (the phase-A tile loads of cheb_bwd_fast)
  const size_t d_bytes = FinK * size_t(lds_vertex_stride(M)) * 4;
  g.dscratch = g.dw_fused ? std::max<size_t>(d_bytes, 16 * 32 * 32 * 4) : d_bytes;
  g.bwd_lds = ring + align16(g.dscratch) + FinK * (Fout + 1) * 4;
  const bool shape_ok = M >= 1 && M <= 1024 && K >= 1 && Fout >= 1 && fin_ok && P >= 1;
  g.fwd_ok_ob = shape_ok && max_row_nnz <= kFastWidth && g.nt <= 2 && g.fwd_lds_ob <= size_t(kLdsBytes);
  g.fwd_ok = g.fwd_ok_ob && g.fwd_lds <= size_t(kLdsBytes);
  g.bwd_ok = shape_ok && max_row_nnzT <= kFastWidth && g.bwd_lds <= size_t(kLdsBytes);
  return g;
}

hipError_t launch_fast_forward(const FastGeom& g, int N, const FastFwdArgs& a, hipStream_t s) {
  // orders-layout basis: Fin <= 2 (cheb_abi.cpp::check_layout)
#define CG_F(FV_, NT_)                                                                   \
  if (a.Fin == FV_ && g.nt == NT_)                                                       \
    return a.bord ? fastk::launch_fwd_fast_t<FV_, NT_, true>(g.fwd_lds_ob, N, a, s)      \
                  : fastk::launch_fwd_fast_t<FV_, NT_, false>(g.fwd_lds, N, a, s);
  CG_F(1, 1) CG_F(1, 2) CG_F(2, 1) CG_F(2, 2)
#undef CG_F
  if (a.Fin == 4 && !a.bord && g.nt == 1) return fastk::launch_fwd_fast_t<4, 1, false>(g.fwd_lds, N, a, s);
  if (a.Fin == 4 && !a.bord && g.nt == 2) return fastk::launch_fwd_fast_t<4, 2, false>(g.fwd_lds, N, a, s);
  return hipErrorInvalidValue;
}

hipError_t launch_fast_backward(const FastGeom& g, int N, const FastBwdArgs& a, hipStream_t s) {
  // orders-layout basis: the fused dW on the split-bf16 matrix pipe with CG_OPT_GEMM_X3
  const int dw = a.dw_slab == nullptr ? 0 : (a.bord ? (a.x3 ? 3 : 2) : 1);
#define CG_B(FV_)                                                                      \
  if (a.Fin == FV_)                                                                    \
    return dw == 3 ? fastk::launch_bwd_fast_t<FV_, 3>(g.bwd_lds, N, a, s)              \
           : dw == 2 ? fastk::launch_bwd_fast_t<FV_, 2>(g.bwd_lds, N, a, s)            \
           : dw == 1 ? fastk::launch_bwd_fast_t<FV_, 1>(g.bwd_lds, N, a, s)            \
                     : fastk::launch_bwd_fast_t<FV_, 0>(g.bwd_lds, N, a, s);
  CG_B(1) CG_B(2)
#undef CG_B
  if (a.Fin == 4 && dw == 1) return fastk::launch_bwd_fast_t<4, 1>(g.bwd_lds, N, a, s);
  if (a.Fin == 4 && dw == 0) return fastk::launch_bwd_fast_t<4, 0>(g.bwd_lds, N, a, s);
  return hipErrorInvalidValue;
}

}  // namespace cg
