// double instantiations of the HPR message update (templates in mjx_hpr_impl.h).
#include "mjx_hpr_impl.h"

namespace mjx {
namespace hpr {
int update_f64(const void* ci, void* co, const void* b, const int32_t* nb, const int32_t* ir, const int32_t* orr,
               int64_t n, int d, int p, int c, int ap, double wp, double wm, double dp, hipStream_t st) {
    return dispatch_tp<double>(p, c, d, ci, co, b, nb, ir, orr, n, ap, wp, wm, dp, st);
}
}  // namespace hpr
}  // namespace mjx
