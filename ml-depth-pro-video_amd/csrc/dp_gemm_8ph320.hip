// dp_gemm_8ph320.hip: the 8-phase 320 x 256 engine.
#include "dp_gemm_impl.h"

namespace dpg {
int launch_part_8ph320(const GemmP& p, bool conv, bool bf16, hipStream_t s) {
  if (conv) return DP_ERR_ARG;
  return bf16 ? launch_8ph320<KBF16>(p, s) : launch_8ph320<KF16>(p, s);
}
}  // namespace dpg
