// lm_gemm_swiglu.hip — wgemm instantiations for the EPI_SWIGLU epilogue (see lm_gemm_kernel.h).
#include "lm_gemm_kernel.h"

namespace tts {

void launch_wgemm_swiglu(const WgemmArgs& a, const WgemmPlan& p, bool norm, hipStream_t s) {
  if (!p.a_lds) launch_cfg<2, A_GLOBAL, false, EPI_SWIGLU>(a, p.cfg, p.grid, s);
  else if (norm) launch_cfg<2, A_LDS, true, EPI_SWIGLU>(a, p.cfg, p.grid, s);
  else launch_cfg<2, A_LDS, false, EPI_SWIGLU>(a, p.cfg, p.grid, s);
}

}  // namespace tts
