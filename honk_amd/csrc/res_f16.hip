// The f16x2 pair / last-layer kernels (res15's headline path) in a translation unit of
// their own, so they alone are compiled with `-mllvm -amdgpu-mfma-vgpr-form`
// (honk_amd/build.py: FLAGS): the MFMAs then take their accumulators in VGPRs, and the
// epilogue reads them directly instead of copying each m-tile's 12 results out of
// AGPRs first (12 v_accvgpr_read + 12 v_mov_b64 per step fewer: 1.87 -> 1.82 ms per
// res15 pair launch, 1.00 -> 0.99 ms for the last layer, same box).
// The flag is per compilation, and under it the two-stream bf16 pair kernel
// (<3,1,4,4,2,0>) splits a spill reload, which the spill guard refuses -- so the
// other kernels stay in res.hip.
//
// This file includes res.hip with HONK_RES_F16_TU defined: the device templates and
// their argument structs only (no host code, no non-template kernels), and defines
// the two launchers res.hip's forward_bf16 calls for FM == 2.
#define HONK_RES_F16_TU 1
#include "res.hip"

namespace honk {
namespace res {

// the pair (layers i, i + 1; dilations dA, dB) -- res.hip:forward_bf16.  imm: the
// tap-step instances (plan_pair with pad columns, pair_imm); returns false when no
// instance matches (the caller reports HONK_ERR_UNSUPPORTED).
bool launch_pair_f16(bool imm, int ppr, int dA, int dB, dim3 gd, dim3 bd, hipStream_t st, const Block16PArgs& pa) {
  if (imm) {
#define HONK_PI(a_, b_)                                                                              \
  if (dA == a_ && dB == b_) {                                                                        \
    hipLaunchKernelGGL((block16p_kernel<3, 1, 4, 4, 1, 2, a_, b_>), gd, bd, 0, st, pa);             \
    return true;                                                                                     \
  }
    HONK_PI(1, 1) HONK_PI(1, 2) HONK_PI(2, 2) HONK_PI(4, 4) HONK_PI(4, 8) HONK_PI(8, 8)
#undef HONK_PI
    return false;
  }
  if (ppr == 4) hipLaunchKernelGGL((block16p_kernel<3, 1, 4, 4, 1, 2>), gd, bd, 0, st, pa);
  else hipLaunchKernelGGL((block16p_kernel<3, 1, 2, 5, 1, 2>), gd, bd, 0, st, pa);
  return true;
}

// the last (odd) layer with its channel sums (dilation d)
void launch_last_f16(int d, dim3 gd, dim3 bd, hipStream_t st, const Block16PArgs& pa) {
  if (d == 16) hipLaunchKernelGGL((block16l_kernel<3, 1, 4, 4, 2, 2, 16>), gd, bd, 0, st, pa);
  else hipLaunchKernelGGL((block16l_kernel<3, 1, 4, 4, 2, 2>), gd, bd, 0, st, pa);
}

}  // namespace res
}  // namespace honk
