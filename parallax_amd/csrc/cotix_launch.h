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
// the tape backward at two waves per env group (EW = 4, analytic scenes of 5
// or 7 bodies; cxk::run_backward_split), workgroups of 2 * WPB waves with
// `lds` = cxk::lds_bytes(header, 2 * WPB, 4): 0 launched, 1 not compiled for
// this scene (the caller launches MODE 4)
int launch_bwd_split(const cxk::KArgs& ka, int spec, size_t lds, hipStream_t st);
// the step program (mode 0) with a key-window helper wave per env group
// (EW = 4, RoboCup's specialization; cxk::KeyHelper), workgroups of 2 * WPB
// waves with `lds` = cxk::help_lds_bytes<4>(header, WPB): 0 launched, 1 not
// compiled for this scene (the caller launches step_kernel)
int launch_step_help(const cxk::KArgs& ka, int spec, size_t lds, hipStream_t st);
}  // namespace cxl
