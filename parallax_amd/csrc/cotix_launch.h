// cotix_launch.h -- entry points of the fused step kernel's translation units.
//
// cotix_step_kernel.hip is compiled once per envs-per-wave tiling EW
// (-DCOTIX_EW=1/2/4/8, in parallel) and each object defines launch_step_ewN:
// the step_kernel<EW, FNSET, MODE> instantiation for the scene's contact
// function set `fs` and `mode` (0 step, 1 rollout forward, 2 backward re-play)
// launched on `st` with `lds` bytes of dynamic LDS per workgroup; `spec`
// (cxk::spec_of of the header) selects a scene specialization where one is
// compiled (EW = 4), else the generic kernel runs.
#pragma once
#include <hip/hip_runtime.h>

#include "cotix_kernel.h"

namespace cxl {
// waves per workgroup: WPB (one per SIMD of a CU) -- or, for a scene whose
// tiles do not fit the LDS four at a time, 2 or 1 (wpb: the launch's count;
// each wave still owns its own tile, so the bits do not depend on it)
constexpr int WPB = 4;
hipError_t launch_step_ew1(const cxk::KArgs& ka, int fs, int mode, size_t lds, hipStream_t st, int spec, int wpb);
hipError_t launch_step_ew2(const cxk::KArgs& ka, int fs, int mode, size_t lds, hipStream_t st, int spec, int wpb);
hipError_t launch_step_ew4(const cxk::KArgs& ka, int fs, int mode, size_t lds, hipStream_t st, int spec, int wpb);
hipError_t launch_step_ew8(const cxk::KArgs& ka, int fs, int mode, size_t lds, hipStream_t st, int spec, int wpb);
}  // namespace cxl
