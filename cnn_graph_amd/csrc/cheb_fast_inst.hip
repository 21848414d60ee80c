// One instantiation of the fast resident kernels (cheb_fast_kern.h), chosen
// by the Makefile through -DCG_FAST_FWD/-DCG_FAST_BWD, -DCG_FV and
// -DCG_NT (forward: 32-wide Fout tiles) -DCG_OB (forward: orders-layout basis) or -DCG_DW (backward: 0 no fused dW, 1 fused dW, 2 fused dW from the orders-layout basis, 3 the
// same on the split-bf16 matrix pipe).
#include "cheb_fast_kern.h"

namespace cg {
namespace fastk {
#if defined(CG_FAST_FWD)
template hipError_t launch_fwd_fast_t<CG_FV, CG_NT, (CG_OB != 0)>(size_t, int, const FastFwdArgs&,
                                                                 hipStream_t);
#elif defined(CG_FAST_BWD)
template hipError_t launch_bwd_fast_t<CG_FV, CG_DW>(size_t, int, const FastBwdArgs&, hipStream_t);
#else
#error "cheb_fast_inst.hip: define CG_FAST_FWD or CG_FAST_BWD"
#endif
}  // namespace fastk
}  // namespace cg
