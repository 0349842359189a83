// split.hip -- host-side exact splitting of the distributed sort (no
// kernels): the C-ABI entries over dr_plan::split_windows / split_exact
// (include/dr/details/split_plan.hpp, where the algorithm is described).
#include "common.hpp"

#include "../include/dr/details/split_plan.hpp"

extern "C" int drhip_split_windows(int p, const uint64_t *n, const uint64_t *stride, const uint64_t *nsamples,
                                   const uint64_t *samples, int nb, const uint64_t *g, uint64_t *lo,
                                   uint64_t *hi, uint64_t *win) {
  if (const char *e = dr_plan::split_windows(p, n, stride, nsamples, samples, nb, g, lo, hi, win))
    return drhip::set_error(DRHIP_ERR_BAD_ARG, e);
  return DRHIP_OK;
}

extern "C" int drhip_split_exact(int p, const uint64_t *n, int nb, const uint64_t *g, const uint64_t *lo,
                                 const uint64_t *hi, const uint64_t *win, const uint64_t *wkeys,
                                 uint64_t *split) {
  if (const char *e = dr_plan::split_exact(p, n, nb, g, lo, hi, win, wkeys, split))
    return drhip::set_error(DRHIP_ERR_BAD_ARG, e);
  return DRHIP_OK;
}
