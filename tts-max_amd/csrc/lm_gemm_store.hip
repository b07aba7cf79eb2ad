// lm_gemm_store.hip — wgemm instantiations for the EPI_STORE epilogue (see lm_gemm_kernel.h).
#include "lm_gemm_kernel.h"

namespace tts {

void launch_wgemm_store(const WgemmArgs& a, const WgemmPlan& p, bool norm, hipStream_t s) {
  if (!p.a_lds) launch_cfg<1, A_GLOBAL, false, EPI_STORE>(a, p.cfg, p.grid, s);
  else if (norm) launch_cfg<1, A_LDS, true, EPI_STORE>(a, p.cfg, p.grid, s);
  else launch_cfg<1, A_LDS, false, EPI_STORE>(a, p.cfg, p.grid, s);
}

void launch_wgemm_kslice(const WgemmArgs& a_in, int units, hipStream_t s) {
  WgemmArgs a = a_in;
  if (dry_record(wgemm_inst_name(8, 2, 2, 1, 16, A_LDS, false, EPI_STORE, 2, false, 4, false))) return;
  if (a.M < 1 || a.M > 32 || a.K % 512 != 0 || a.kc != 1 || !a.part_out)
    throw std::runtime_error("wgemm kslice: 1..32 rows, K / 4 a multiple of 512, kc 1, partial workspace");
  a.sliced = 0;
  a.csplit = 1;
  const size_t lds = (((size_t)a.M * (a.K + 8) * 2 + 15) & ~(size_t)15) +
                     (size_t)wgemm_red_floats(8, 4, 1, 2, a.M, a.K) * sizeof(float);
  hipLaunchKernelGGL((wgemm_kernel<8, 2, 2, 1, 16, A_LDS, false, EPI_STORE, 2, false, 4>), dim3((units + 1) / 2, 4),
                     dim3(512), lds, s, a);
}

}  // namespace tts
