// dp_gemm_sk.hip: the stream-K engine.
#include "dp_gemm_impl.h"

namespace dpg {
int launch_part_sk(const GemmP& p, bool conv, void* ws, bool bf16, hipStream_t s) {
  return (bf16 ? launch_sk<KBF16>(p, conv, ws, s) : launch_sk<KF16>(p, conv, ws, s));
}
}  // namespace dpg
