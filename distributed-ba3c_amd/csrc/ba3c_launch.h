// ba3c_launch.h — host launchers of kernels that live in their own translation units.
#pragma once
#include <hip/hip_runtime.h>

namespace ba3c {

struct Conv0SArgs;
struct Conv0WArgs;
struct Wg6Args;

// conv0 forward (persistent bands, ba3c_split.h); returns hipGetLastError() of the launch
hipError_t launch_conv0s_fwd(dim3 grid, hipStream_t s, const Conv0SArgs& a);
// conv0 weight gradient partial slabs (ba3c_split.h)
hipError_t launch_conv0s_wgrad(dim3 grid, hipStream_t s, const Conv0WArgs& a);
// conv1 whole-channel weight gradient (g1 workgroups) + conv0 weight gradient (g0), one launch
hipError_t launch_wgrad01_pair(hipStream_t s, const Wg6Args& a1, int g1, const Conv0WArgs& a0, int g0);

}  // namespace ba3c
