// dp_gemm_8ph.hip: the 8-phase 256 x 256 engine.
#include "dp_gemm_impl.h"

namespace dpg {
int launch_part_8ph(const GemmP& p, int tile, bool conv, bool bf16, hipStream_t s) {
  if (tile == DP_TILE_P8PH_256x256) {
    if (conv) return DP_ERR_ARG;
    return bf16 ? launch_p8ph<KBF16>(p, s) : launch_p8ph<KF16>(p, s);
  }
  return (bf16 ? launch_8ph<KBF16>(p, conv, s) : launch_8ph<KF16>(p, conv, s));
}
}  // namespace dpg

#ifdef DP_STAMPS
// timing-only builds: the persistent 8-phase engine's per-tile stamps of its last launch
// (tools/p8ph_stamps.py); this translation unit instantiates that engine
extern "C" int dp_p8_stamps(void* host_dst, int n_wg) {
  return (int)hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(g_p8_stamps), (size_t)n_wg * P8_STAMP_W * 8, 0,
                                  hipMemcpyDeviceToHost);
}
#endif
