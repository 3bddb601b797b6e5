// ba3c_conv0.hip — the conv0 forward / weight-gradient kernels (ba3c_split.h) in a translation
// unit of their own, compiled with MFMA results in architectural VGPRs (-mllvm
// --amdgpu-mfma-vgpr-form, Makefile): their pool / un-pool epilogues read every accumulator
// with VALU instructions, which costs a v_accvgpr_read per value when the compiler places the
// accumulators in AGPRs.  ba3c_capi.hip launches them through these host functions.
#include <hip/hip_runtime.h>

#define BA3C_SHARED_KERNELS 0

#include "ba3c_launch.h"
#include "ba3c_split.h"
#include "ba3c_wgrad6.h"

namespace ba3c {

hipError_t launch_conv0s_fwd(dim3 grid, hipStream_t s, const Conv0SArgs& a) {
  hipLaunchKernelGGL(conv0s_fwd_kernel, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

// conv1's whole-channel weight gradient (wgrad6w_body, MFMA-bound) beside conv0's weight
// gradient (VALU-bound un-pooling) in one launch: blocks [0, g1) walk conv1's images, blocks
// [g1, g1 + g0) conv0's bands, one workgroup of each per CU.  Both read only the finished
// output gradients dP1 / dP0 and write their own partial slabs; each body runs exactly as in
// its plain kernel with (bx, gx) = (block - first block of its job, job grid).
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
wgrad01_pair_kernel(const Wg6Args a1, const Conv0WArgs a0, int g1, int g0) {
  constexpr int B1 = wgrad6w_lds_bytes<Conv1W6W>(), B0 = Conv0W<2>::ALLOC_U4 * 16;
  __shared__ uint4 lds[(B1 > B0 ? B1 : B0) / 16];
  __shared__ uint32_t red4[4];
  const int b = blockIdx.x;
#ifndef BA3C_DIAG_PAIR
#define BA3C_DIAG_PAIR 0      // diagnostics only (A/B timing): 1 = conv1 job skipped, 2 = conv0 job skipped
#endif
  if (b < g1) {
    if (BA3C_DIAG_PAIR != 1) wgrad6w_body<Conv1W6W>(a1, b, g1, reinterpret_cast<char*>(lds), red4);
  } else if (BA3C_DIAG_PAIR != 2) {
    conv0s_wgrad_body<2>(a0, b - g1, g0, lds, red4);
  }
}

hipError_t launch_wgrad01_pair(hipStream_t s, const Wg6Args& a1, int g1, const Conv0WArgs& a0, int g0) {
  hipLaunchKernelGGL(wgrad01_pair_kernel, dim3(g1 + g0), dim3(256), 0, s, a1, a0, g1, g0);
  return hipGetLastError();
}

hipError_t launch_conv0s_wgrad(dim3 grid, hipStream_t s, const Conv0WArgs& a) {
  hipLaunchKernelGGL(conv0s_wgrad_kernel<2>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace ba3c
