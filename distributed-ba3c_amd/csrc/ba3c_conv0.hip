// ba3c_conv0.hip — the conv0 forward / weight-gradient kernels (ba3c_split.h) in a translation
// unit of their own, compiled with MFMA results in architectural VGPRs (-mllvm
// --amdgpu-mfma-vgpr-form, Makefile): their pool / un-pool epilogues read every accumulator
// with VALU instructions, which costs a v_accvgpr_read per value when the compiler places the
// accumulators in AGPRs.  ba3c_capi.hip launches them through these host functions.
#include <hip/hip_runtime.h>

#define BA3C_SHARED_KERNELS 0

#include "ba3c_launch.h"
#include "ba3c_split.h"

namespace ba3c {

hipError_t launch_conv0s_fwd(int ns, int lay, dim3 grid, hipStream_t s, const Conv0SArgs& a) {
  if (ns == 2 && lay == 3) hipLaunchKernelGGL((conv0s_fwd_kernel<2, 3>), grid, dim3(256), 0, s, a);
  else if (ns == 2) hipLaunchKernelGGL((conv0s_fwd_kernel<2, 2>), grid, dim3(256), 0, s, a);
  else if (lay == 3) hipLaunchKernelGGL((conv0s_fwd_kernel<3, 3>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((conv0s_fwd_kernel<3, 2>), grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_conv0s_wgrad(int ns, dim3 grid, hipStream_t s, const Conv0WArgs& a) {
  if (ns == 2) hipLaunchKernelGGL(conv0s_wgrad_kernel<2>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(conv0s_wgrad_kernel<3>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace ba3c
