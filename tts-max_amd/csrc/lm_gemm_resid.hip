// lm_gemm_resid.hip — wgemm instantiations for the EPI_RESID epilogue (see lm_gemm_kernel.h).
#include "lm_gemm_kernel.h"

namespace tts {

void launch_wgemm_resid(const WgemmArgs& a, const WgemmPlan& p, bool norm, hipStream_t s) {
  if (!p.a_lds) launch_cfg<1, A_GLOBAL, false, EPI_RESID>(a, p.cfg, p.grid, s);
  else launch_cfg<1, A_LDS, false, EPI_RESID>(a, p.cfg, p.grid, s);
}

}  // namespace tts
