// The pair / last-layer kernels (block16p / block16l: res15's headline path) in a
// translation unit of their own, compiled with `-mllvm -amdgpu-mfma-vgpr-form`
// (honk_amd/build.py: FLAGS): the MFMAs then take their accumulators in VGPRs, and the
// epilogue reads them directly instead of copying each m-tile's results out of AGPRs
// first (f16x2: 12 v_accvgpr_read + 12 v_mov_b64 per step fewer, 1.87 -> 1.82 ms per
// res15 pair launch, 1.00 -> 0.99 ms for the last layer, same box).
// The flag is per compilation (the walk-based two-stream bf16 pair kernel split a spill
// reload under it -- round 6 replaced that kernel by the row-table one below, which
// does not spill); every other kernel stays in res.hip.
//
// This file includes res.hip with HONK_RES_VF_TU defined: the device templates and
// their argument structs only (no host code, no non-template kernels), and defines
// the two launchers res.hip's forward_bf16 calls.
#define HONK_RES_VF_TU 1
#include "res.hip"

namespace honk {
namespace res {

// the pair (layers i, i + 1; dilations dA, dB) -- res.hip:forward_bf16, which has
// planned it (PairPlan pp: ppr, padb, ns).  FM 2 with pad columns: the tap-step
// instances (pair_imm).  Returns false when no instance matches (the caller reports
// HONK_ERR_UNSUPPORTED); the two-stream bf16 instance (ns == 2) is not here.
bool launch_pair_vf(int FM, int ppr, bool imm, int dA, int dB, dim3 gd, dim3 bd, hipStream_t st,
                    const Block16PArgs& pa) {
  if ((FM == 2 || FM == 0) && imm) {
#define HONK_PI(a_, b_)                                                                              \
  if (dA == a_ && dB == b_) {                                                                        \
    if (FM == 2) hipLaunchKernelGGL((block16p_kernel<3, 1, 4, 4, 1, 2, a_, b_>), gd, bd, 0, st, pa); \
    else hipLaunchKernelGGL((block16p_kernel<3, 1, 4, 4, 1, 0, a_, b_>), gd, bd, 0, st, pa);        \
    return true;                                                                                     \
  }
    HONK_PI(1, 1) HONK_PI(1, 2) HONK_PI(2, 2) HONK_PI(4, 4) HONK_PI(4, 8) HONK_PI(8, 8)
#undef HONK_PI
    return false;
  }
  if (FM == 1 && ppr == 9) hipLaunchKernelGGL((block16p_kernel<3, 2, 9, 9, 1>), gd, bd, 0, st, pa);
  else if (FM == 1 && ppr == 5) hipLaunchKernelGGL((block16p_kernel<3, 2, 5, 10, 1>), gd, bd, 0, st, pa);
  else if (FM == 1) hipLaunchKernelGGL((block16p_kernel<3, 2, 3, 9, 1>), gd, bd, 0, st, pa);
  else if (FM == 2 && ppr == 4) hipLaunchKernelGGL((block16p_kernel<3, 1, 4, 4, 1, 2>), gd, bd, 0, st, pa);
  else if (FM == 2) hipLaunchKernelGGL((block16p_kernel<3, 1, 2, 5, 1, 2>), gd, bd, 0, st, pa);
  else if (ppr == 4) hipLaunchKernelGGL((block16p_kernel<3, 1, 4, 4, 1>), gd, bd, 0, st, pa);
  else hipLaunchKernelGGL((block16p_kernel<3, 1, 2, 5, 1>), gd, bd, 0, st, pa);
  return true;
}

// bf16, two streams per workgroup on the row-table walk (SCA = -1: no tap-step
// immediates -- the two streams' rings leave no room for pad columns); ppr 4: 40-pixel
// rows (res15), 2: 13..21-pixel rows (res8, res26); lin: their linear A-in DMA
void launch_pair2t_vf(int ppr, bool lin, dim3 gd, dim3 bd, hipStream_t st, const Block16PArgs& pa) {
  if (lin) hipLaunchKernelGGL((block16p_kernel<3, 1, 2, 4, 2, 0, -1, -1, true>), gd, bd, 0, st, pa);
  else if (ppr == 4) hipLaunchKernelGGL((block16p_kernel<3, 1, 4, 4, 2, 0, -1, -1>), gd, bd, 0, st, pa);
  else hipLaunchKernelGGL((block16p_kernel<3, 1, 2, 5, 2, 0, -1, -1>), gd, bd, 0, st, pa);
}

// bf16, two streams on the compile-time tap-step instances (rings with zero pad columns,
// where those fit two streams: res15's (1,1) (1,2) (2,2) (4,4) pairs, (8,8) with shared pads;
// (4,8) needs 17 ring slots, 4.6 KiB past half the LDS, and stays on the row table)
bool launch_pair2i_vf(int dA, int dB, dim3 gd, dim3 bd, hipStream_t st, const Block16PArgs& pa) {
#define HONK_P2I(a_, b_)                                                              \
  if (dA == a_ && dB == b_) {                                                         \
    hipLaunchKernelGGL((block16p_kernel<3, 1, 4, 4, 2, 0, a_, b_>), gd, bd, 0, st, pa); \
    return true;                                                                      \
  }
  HONK_P2I(1, 1) HONK_P2I(1, 2) HONK_P2I(2, 2) HONK_P2I(4, 4) HONK_P2I(8, 8)
#undef HONK_P2I
  return false;
}

// f16x2 with the contraction split over two waves per SIMD (res_bf16k.inc)
bool launch_pairk_vf(int dA, int dB, dim3 gd, dim3 bd, hipStream_t st, const Block16PArgs& pa) {
#define HONK_PK(a_, b_)                                                       \
  if (dA == a_ && dB == b_) {                                                 \
    hipLaunchKernelGGL((block16k_kernel<a_, b_>), gd, bd, 0, st, pa);        \
    return true;                                                              \
  }
  HONK_PK(1, 1) HONK_PK(1, 2) HONK_PK(2, 2) HONK_PK(4, 4) HONK_PK(4, 8) HONK_PK(8, 8)
#undef HONK_PK
  return false;
}

// the last (odd) layer with its channel sums (dilation d)
void launch_last_vf(int FM, int d, dim3 gd, dim3 bd, hipStream_t st, const Block16PArgs& pa) {
  if (FM == 1) hipLaunchKernelGGL((block16l_kernel<3, 2, 9, 9, 2>), gd, bd, 0, st, pa);
  else if (FM == 2 && d == 16) hipLaunchKernelGGL((block16l_kernel<3, 1, 4, 4, 2, 2, 16>), gd, bd, 0, st, pa);
  // bf16, res15's last layer: the row table with pad columns and the compile-time tap step
  else if (FM == 0 && d == 16 && pa.padb > 0) hipLaunchKernelGGL((block16l_kernel<3, 1, 4, 4, 2, 0, 16>), gd, bd, 0, st, pa);
  else if (FM == 2) hipLaunchKernelGGL((block16l_kernel<3, 1, 4, 4, 2, 2>), gd, bd, 0, st, pa);
  else hipLaunchKernelGGL((block16l_kernel<3, 1, 4, 4, 2>), gd, bd, 0, st, pa);
}

}  // namespace res
}  // namespace honk
