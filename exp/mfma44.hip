// Probe of v_mfma_f32_4x4x1_16b_f32 on gfx950: operand / result lane layout, the
// CBSZ/ABID A-broadcast, and issue throughput against v_mfma_f32_16x16x4_f32.
//   hipcc --offload-arch=gfx950 -O3 exp/mfma44.hip -o exp/_var/mfma44 && exp/_var/mfma44
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int ABID, int CBSZ>
__global__ void layout_kernel(f4* o, const float* a, const float* b) {
  const int l = threadIdx.x;
  f4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a[l], b[l], acc, CBSZ, ABID, 0);
  o[l] = acc;
}

// 4x4 transpose of 16-lane rows across 4 registers: on exit row g of x[q] = row q of x[g]
__global__ void tr_kernel(float* o, const float* a) {
  const int l = threadIdx.x;
  unsigned x0 = __float_as_uint(a[l]), x1 = __float_as_uint(a[64 + l]), x2 = __float_as_uint(a[128 + l]),
           x3 = __float_as_uint(a[192 + l]);
  auto p = __builtin_amdgcn_permlane32_swap(x0, x2, false, false);
  auto q = __builtin_amdgcn_permlane32_swap(x1, x3, false, false);
  auto r = __builtin_amdgcn_permlane16_swap(p[0], q[0], false, false);
  auto s = __builtin_amdgcn_permlane16_swap(p[1], q[1], false, false);
  o[l] = __uint_as_float(r[0]); o[64 + l] = __uint_as_float(r[1]);
  o[128 + l] = __uint_as_float(s[0]); o[192 + l] = __uint_as_float(s[1]);
}

template <int NACC, bool BIG>
__global__ void tput_kernel(float* o, int iters) {
  const int l = threadIdx.x;
  f4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = f4{0, 0, 0, 0};
  float a = l * 0.001f, b = 1.0f - l * 0.0005f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
      if (BIG)
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
      else
        acc[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[i], 4, 3, 0);
    }
  }
  float s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  o[blockIdx.x * blockDim.x + l] = s;
}

int main() {
  std::vector<float> ha(64), hb(64);
  for (int i = 0; i < 64; ++i) { ha[i] = 1 + i; hb[i] = 1000 * (1 + i); }
  float *da, *db; f4* dout;
  hipMalloc(&da, 256); hipMalloc(&db, 256); hipMalloc(&dout, 64 * 16);
  hipMemcpy(da, ha.data(), 256, hipMemcpyHostToDevice);
  hipMemcpy(db, hb.data(), 256, hipMemcpyHostToDevice);
  std::vector<f4> ho(64);
  // no broadcast: expect lane l, reg i = A[block l/4][row i] * B[block l/4][col l%4]
  //  with A lane = 4*block + row, B lane = 4*block + col
  hipLaunchKernelGGL((layout_kernel<0, 0>), dim3(1), dim3(64), 0, 0, dout, da, db);
  hipMemcpy(ho.data(), dout, 64 * 16, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 4; ++i) {
      const int blk = l / 4, col = l % 4;
      const float want = ha[4 * blk + i] * hb[4 * blk + col];
      if (ho[l][i] != want) ++bad;
    }
  printf("layout (row = reg, col = lane%%4, block = lane/4): %s (%d bad)\n", bad ? "NO" : "yes", bad);
  if (bad) for (int l = 0; l < 8; ++l) printf("  lane %d: %g %g %g %g\n", l, ho[l][0], ho[l][1], ho[l][2], ho[l][3]);
  hipLaunchKernelGGL((layout_kernel<5, 4>), dim3(1), dim3(64), 0, 0, dout, da, db);
  hipMemcpy(ho.data(), dout, 64 * 16, hipMemcpyDeviceToHost);
  bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 4; ++i) {
      const int blk = l / 4, col = l % 4;
      const float want = ha[4 * 5 + i] * hb[4 * blk + col];
      if (ho[l][i] != want) ++bad;
    }
  printf("CBSZ=4 ABID=5 broadcasts block 5's A to all 16 blocks: %s (%d bad)\n", bad ? "NO" : "yes", bad);
  if (bad) for (int l = 0; l < 8; ++l) printf("  lane %d: %g %g %g %g\n", l, ho[l][0], ho[l][1], ho[l][2], ho[l][3]);

  {
    std::vector<float> hx(256), hy(256);
    for (int i = 0; i < 256; ++i) hx[i] = i;
    float *dx, *dy; hipMalloc(&dx, 1024); hipMalloc(&dy, 1024);
    hipMemcpy(dx, hx.data(), 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(tr_kernel, dim3(1), dim3(64), 0, 0, dy, dx);
    hipMemcpy(hy.data(), dy, 1024, hipMemcpyDeviceToHost);
    int tb = 0;
    for (int q = 0; q < 4; ++q)
      for (int l = 0; l < 64; ++l) {
        const int g = l / 16, i = l % 16;
        if (hy[64 * q + l] != hx[64 * g + 16 * q + i]) ++tb;
      }
    printf("permlane32/16 swap 4x4 row transpose: %s (%d bad)\n", tb ? "NO" : "yes", tb);
    if (tb) for (int q = 0; q < 4; ++q) printf("  x%d rows: %g %g %g %g\n", q, hy[64*q], hy[64*q+16], hy[64*q+32], hy[64*q+48]);
  }
  float* dt; hipMalloc(&dt, 256 * 1024 * 4 * 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 20000, grid = 256 * 4;
  auto run = [&](auto kern, const char* name, double macs_per_instr, int nacc) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, 0, dt, 10);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, 0, dt, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double instr = (double)grid * iters * nacc;
    printf("%-28s %8.3f ms  %7.1f TF  %.2f ns/instr/SIMD\n", name, ms, instr * macs_per_instr * 2 / (ms * 1e-3) / 1e12,
           ms * 1e6 / (instr / 1024));
  };
  run(tput_kernel<8, true>, "16x16x4 f32, 8 chains", 1024, 8);
  run(tput_kernel<8, false>, "4x4x1_16b f32, 8 chains", 256, 8);
  run(tput_kernel<16, false>, "4x4x1_16b f32, 16 chains", 256, 16);
  return 0;
}
