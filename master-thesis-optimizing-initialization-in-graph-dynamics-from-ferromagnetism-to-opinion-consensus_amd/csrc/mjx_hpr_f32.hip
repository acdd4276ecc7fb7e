// float instantiations of the HPR message update (templates in mjx_hpr_impl.h).
#include "mjx_hpr_impl.h"

namespace mjx {
namespace hpr {
int update_f32(const void* ci, void* co, const void* b, const int32_t* nb, const int32_t* ir, const int32_t* orr,
               int64_t n, int d, int p, int c, int ap, double wp, double wm, double dp, hipStream_t st) {
    return dispatch_tp<float>(p, c, d, ci, co, b, nb, ir, orr, n, ap, wp, wm, dp, st);
}
int update_q_f32(const void* ci, void* co, const void* b, const int32_t* nb, const int32_t* ir, const int32_t* orr,
                 int64_t n, int d, int p, int c, int ap, double wp, double wm, double dp, const float* sc,
                 hipStream_t st) {
    if (!q_supported(d, p, c)) return MJX_ERANGE;
#define MJX_Q(PP, DD) \
    if (p == PP && d == DD) return launch_update_q<4, PP, DD>(ci, co, b, nb, ir, orr, n, ap, wp, wm, dp, sc, st);
    MJX_Q(1, 2) MJX_Q(1, 3) MJX_Q(1, 4) MJX_Q(2, 2) MJX_Q(2, 3) MJX_Q(2, 4) MJX_Q(3, 2) MJX_Q(3, 3) MJX_Q(3, 4)
#undef MJX_Q
    return MJX_ERANGE;
}
}  // namespace hpr
}  // namespace mjx

#ifdef MJX_HPR_PROF
// profiling build only (-DMJX_HPR_PROF): per-phase cycle sums of k_hpr_update
extern "C" int mjx_hpr_prof_read(unsigned long long* host32, int reset) {
    if (hipMemcpyFromSymbol(host32, HIP_SYMBOL(mjx::hpr::mjx_hpr_prof), 32 * sizeof(unsigned long long)) != hipSuccess)
        return MJX_EHIP;
    if (reset) {
        unsigned long long z[32] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(mjx::hpr::mjx_hpr_prof), z, sizeof(z)) != hipSuccess) return MJX_EHIP;
    }
    return MJX_OK;
}
#endif
