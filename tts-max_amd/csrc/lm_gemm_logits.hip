// lm_gemm_logits.hip — wgemm instantiations for the EPI_LOGITS epilogue (see lm_gemm_kernel.h).
#include "lm_gemm_kernel.h"

namespace tts {

void launch_wgemm_logits(const WgemmArgs& a, const WgemmPlan& p, bool norm, hipStream_t s) {
  if (!p.a_lds) launch_cfg<1, A_GLOBAL, false, EPI_LOGITS>(a, p.cfg, p.grid, s);
  else if (norm) launch_cfg<1, A_LDS, true, EPI_LOGITS>(a, p.cfg, p.grid, s);
  else launch_cfg<1, A_LDS, false, EPI_LOGITS>(a, p.cfg, p.grid, s);
}

}  // namespace tts
