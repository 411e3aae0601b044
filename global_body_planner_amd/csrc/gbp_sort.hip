// gbp_sort.hip — the device radix sort behind the planner trees' nearest-
// neighbour index (gbp_plan.hip, nn_index_build): (32-bit Morton key, vertex
// index) pairs sorted by key, stable, so equal keys keep index order and an
// index build is deterministic.  rocPRIM's onesweep radix sort, kept in a
// translation unit of its own (its templates are heavy to compile).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <rocprim/device/device_radix_sort.hpp>

#include "gbp_internal.h"

// temp == nullptr: *temp_bytes receives the scratch size for n pairs
// (the TU is compiled -fvisibility=hidden: nothing here is exported)
int gbp_internal_sort_pairs_u32(void *temp, size_t *temp_bytes, const uint32_t *keys_in,
                                uint32_t *keys_out, const int32_t *vals_in, int32_t *vals_out,
                                int64_t n, hipStream_t s) {
  size_t bytes = temp ? *temp_bytes : 0;
  const hipError_t e = rocprim::radix_sort_pairs(temp, bytes, keys_in, keys_out, vals_in, vals_out,
                                                 (size_t)n, 0u, 32u, s);
  if (!temp) *temp_bytes = bytes;
  return e == hipSuccess ? GBP_OK : GBP_E_HIP;
}
