// dp_gemm_splitk.hip: split-K for small grids (the 256 x 256 big engine over K ranges + a reduce launch).
#include "dp_gemm_impl.h"

namespace dpg {
int launch_part_splitk(const GemmP& p, bool conv, bool bf16, hipStream_t s) {
  return (bf16 ? launch_splitk<KBF16>(p, conv, s) : launch_splitk<KF16>(p, conv, s));
}
}  // namespace dpg
