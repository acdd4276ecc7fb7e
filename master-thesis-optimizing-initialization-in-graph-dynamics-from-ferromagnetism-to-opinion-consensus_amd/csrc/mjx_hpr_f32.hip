// float instantiations of the HPR message update (templates in mjx_hpr_impl.h).
#include "mjx_hpr_impl.h"

namespace mjx {
namespace hpr {
int update_f32(const void* ci, void* co, const void* b, const int32_t* nb, const int32_t* ir, const int32_t* orr,
               int64_t n, int d, int p, int c, int ap, double wp, double wm, double dp, hipStream_t st) {
    return dispatch_tp<float>(p, c, d, ci, co, b, nb, ir, orr, n, ap, wp, wm, dp, st);
}
}  // namespace hpr
}  // namespace mjx

#ifdef MJX_HPR_PROF
// profiling build only (-DMJX_HPR_PROF): per-phase cycle sums of k_hpr_update
extern "C" int mjx_hpr_prof_read(unsigned long long* host8, int reset) {
    if (hipMemcpyFromSymbol(host8, HIP_SYMBOL(mjx::hpr::mjx_hpr_prof), 8 * sizeof(unsigned long long)) != hipSuccess)
        return MJX_EHIP;
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(mjx::hpr::mjx_hpr_prof), z, sizeof(z)) != hipSuccess) return MJX_EHIP;
    }
    return MJX_OK;
}
#endif
