// sort.hip -- placeholder until the LSD radix sort lands.
#include "common.hpp"

using namespace drhip;

extern "C" int drhip_sort_workspace(int seg, int dtype, size_t n, size_t *bytes) {
  return set_error(DRHIP_ERR_UNSUPPORTED, "drhip_sort: not implemented yet");
}
extern "C" int drhip_sort(int seg, int dtype, void *keys, size_t n, void *tmp, size_t tmp_bytes) {
  return set_error(DRHIP_ERR_UNSUPPORTED, "drhip_sort: not implemented yet");
}
extern "C" int drhip_sort_sample(int seg, int dtype, const void *sorted, size_t n, size_t count,
                                 void *samples) {
  return set_error(DRHIP_ERR_UNSUPPORTED, "drhip_sort_sample: not implemented yet");
}
extern "C" int drhip_sort_bucket_counts(int seg, int dtype, const void *sorted, size_t n,
                                        const void *splitters, int nsplit, uint64_t *counts) {
  return set_error(DRHIP_ERR_UNSUPPORTED, "drhip_sort_bucket_counts: not implemented yet");
}
