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

// the conv3x3d inner loop's instruction mix per k-step: 4 16x16x4 (4 chains) + 4 4x4x1
// (one chain); PERM: + the 16-lane row transpose of the operands; LDS: operands read from
// LDS a step ahead.  512 threads per workgroup (2 waves per SIMD), as conv3x3d_kernel.
template <bool PERM, bool LDS>
__global__ __launch_bounds__(512, 1) void mix_kernel(float* o, int iters) {
  __shared__ float lds[16384];
  const int l = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 16384; i += 512) lds[i] = i * 1e-4f;
  __syncthreads();
  f4 acc[4], acc4 = {0, 0, 0, 0};
  for (int i = 0; i < 4; ++i) acc[i] = f4{0, 0, 0, 0};
  float w = l * 0.001f, wt = 1.0f - l * 0.0005f;
  float xv[4] = {l * 1e-3f, l * 2e-3f, l * 3e-3f, l * 4e-3f};
  int base = (threadIdx.x >> 6) * 64 + l;
  for (int it = 0; it < iters; ++it) {
    float xn[4];
    if (LDS) {
#pragma unroll
      for (int g = 0; g < 4; ++g) xn[g] = lds[(base + g * 16 + (it & 7) * 1024) & 16383];
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(w, xv[g], acc[g], 0, 0, 0);
    float t0 = xv[0], t1 = xv[1], t2 = xv[2], t3 = xv[3];
    if (PERM) {
      auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(t0), __float_as_uint(t2), false, false);
      auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(t1), __float_as_uint(t3), false, false);
      auto r = __builtin_amdgcn_permlane16_swap(p[0], q[0], false, false);
      auto u = __builtin_amdgcn_permlane16_swap(p[1], q[1], false, false);
      t0 = __uint_as_float(r[0]); t1 = __uint_as_float(r[1]); t2 = __uint_as_float(u[0]); t3 = __uint_as_float(u[1]);
    }
    acc4 = __builtin_amdgcn_mfma_f32_4x4x1f32(wt, t0, acc4, 4, 0, 0);
    acc4 = __builtin_amdgcn_mfma_f32_4x4x1f32(wt, t1, acc4, 4, 1, 0);
    acc4 = __builtin_amdgcn_mfma_f32_4x4x1f32(wt, t2, acc4, 4, 2, 0);
    acc4 = __builtin_amdgcn_mfma_f32_4x4x1f32(wt, t3, acc4, 4, 3, 0);
    if (LDS) {
#pragma unroll
      for (int g = 0; g < 4; ++g) xv[g] = xn[g];
    }
  }
  float s = acc4[0] + acc4[1] + acc4[2] + acc4[3];
  for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  o[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// variants without the transpose: LDS8 = the 16x16x4 operands and the 4x4 operands both
// read from LDS (8 reads per k-step); ALL4 = 20 rows as 5 4x4x1 chains (4 reads)
template <int MODE>
__global__ __launch_bounds__(512, 1) void mix2_kernel(float* o, int iters) {
  __shared__ float lds[16384];
  const int l = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 16384; i += 512) lds[i] = i * 1e-4f;
  __syncthreads();
  f4 acc[5];
  for (int i = 0; i < 5; ++i) acc[i] = f4{0, 0, 0, 0};
  float w = l * 0.001f, wt = 1.0f - l * 0.0005f;
  float xv[8];
  for (int g = 0; g < 8; ++g) xv[g] = l * 1e-3f * g;
  int base = (threadIdx.x >> 6) * 64 + l;
  for (int it = 0; it < iters; ++it) {
    float xn[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) xn[g] = lds[(base + g * 16 + (it & 7) * 1024) & 16383];
    if (MODE == 0) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(w, xv[g], acc[g], 0, 0, 0);
      }
      acc[4] = __builtin_amdgcn_mfma_f32_4x4x1f32(wt, xv[4], acc[4], 4, 0, 0);
      acc[4] = __builtin_amdgcn_mfma_f32_4x4x1f32(wt, xv[5], acc[4], 4, 1, 0);
      acc[4] = __builtin_amdgcn_mfma_f32_4x4x1f32(wt, xv[6], acc[4], 4, 2, 0);
      acc[4] = __builtin_amdgcn_mfma_f32_4x4x1f32(wt, xv[7], acc[4], 4, 3, 0);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int c = 0; c < 5; ++c) acc[c] = __builtin_amdgcn_mfma_f32_4x4x1f32(wt + c, xv[q], acc[c], 4, 3, 0);
    }
#pragma unroll
    for (int g = 0; g < 8; ++g) xv[g] = xn[g];
  }
  float s = 0;
  for (int i = 0; i < 5; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  o[blockIdx.x * blockDim.x + threadIdx.x] = s;
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
  auto runmix = [&](auto kern, const char* name) {
    const int it2 = 4000;
    hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, dt, 10);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, dt, it2);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%-34s %8.3f ms  %.1f ns per k-step per SIMD (2 waves)\n", name, ms, ms * 1e6 / it2 / 2);
  };
  runmix(mix_kernel<false, false>, "mix 4x16x16x4 + 4x4x4x1");
  runmix(mix_kernel<true, false>, "mix + permlane transpose");
  runmix(mix_kernel<true, true>, "mix + permlane + LDS operands");
  runmix(mix2_kernel<0>, "mix, 8 LDS reads, no permlane");
  runmix(mix2_kernel<1>, "20 rows as 5 4x4 chains, LDS");
  return 0;
}
