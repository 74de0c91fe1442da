// check.hpp — launch interface of the device invariant checks (check.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "../../include/accord_deps.h"
#include "common.hpp"

namespace adx {

int device_cu_count();
// out_dev: {u64 n_violations, u64 first failing item}, initialised by the caller to {0, ~0}
hipError_t run_check_result(const ad_deps_result& r, uint64_t n_dict, void* out_dev, hipStream_t st);
hipError_t run_check_snapshot(const DevSnapshot& s, void* out_dev, hipStream_t st);

}  // namespace adx
