// lm_gemm_store.hip — wgemm instantiations for the EPI_STORE epilogue (see lm_gemm_kernel.h).
#include "lm_gemm_kernel.h"

namespace tts {

void launch_wgemm_store(const WgemmArgs& a, const WgemmPlan& p, bool norm, hipStream_t s) {
  if (!p.a_lds) launch_cfg<1, A_GLOBAL, false, EPI_STORE>(a, p.cfg, p.grid, s);
  else if (norm) launch_cfg<1, A_LDS, true, EPI_STORE>(a, p.cfg, p.grid, s);
  else launch_cfg<1, A_LDS, false, EPI_STORE>(a, p.cfg, p.grid, s);
}

}  // namespace tts
