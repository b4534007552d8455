// MFMA shape probe (MI355X_MICROARCH.md 'DVFS give-back' item 7): the same
// fp16 FLOP on v_mfma_f32_32x32x16_f16 vs v_mfma_f32_16x16x32_f16, one wave
// per SIMD on every CU, operands from registers that change every MFMA (8 A
// and 4 B fragments cycled, random data), 128 accumulator registers either
// way.  Prints TF/s per shape over interleaved rounds (rule 24).
//   hipcc -O3 --offload-arch=gfx950 scripts/mfma_shape_probe.hip -o /tmp/mfma_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));

template <int SHAPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void probe(
    const h8* __restrict__ src, int iters, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  h8 a[8], b[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = src[(blockIdx.x * 12 + i) * 64 + lane];
#pragma unroll
  for (int i = 0; i < 4; ++i) b[i] = src[(blockIdx.x * 12 + 8 + i) * 64 + lane];
  if constexpr (SHAPE == 32) {
    f16v acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = f16v{};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i)
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[(i + j) & 7], b[j], acc[i], 0, 0, 0);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) s += acc[i][e];
    out[blockIdx.x * 256 + threadIdx.x] = s;
  } else {
    f4v acc[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) acc[i] = f4v{};
    for (int it = 0; it < iters; ++it) {
      // two 16x16x32 MFMAs per 32x32x16 one (same FLOP): 64 per iteration
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 32; ++i)
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[(i + j) & 7], b[(2 * j + (i >> 4)) & 3],
                                                          acc[i], 0, 0, 0);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) s += acc[i][e];
    out[blockIdx.x * 256 + threadIdx.x] = s;
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = ncu;
  const size_t nsrc = (size_t)blocks * 12 * 64;
  std::vector<_Float16> hs(nsrc * 8);
  srand(1);
  for (auto& v : hs) v = (_Float16)((rand() / (float)RAND_MAX) * 2.f - 1.f);
  h8* src;
  float* out;
  hipMalloc(&src, nsrc * sizeof(h8));
  hipMalloc(&out, (size_t)blocks * 256 * 4);
  hipMemcpy(src, hs.data(), nsrc * sizeof(h8), hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  // flop per launch: blocks x 4 waves x iters x 32 (32x32x16 equivalents) x 32768
  const double flop = (double)blocks * 4 * iters * 32 * 32768.0;
  for (int w = 0; w < 3; ++w) {  // warm the clock
    hipLaunchKernelGGL(probe<32>, dim3(blocks), dim3(256), 0, 0, src, iters, out);
    hipLaunchKernelGGL(probe<16>, dim3(blocks), dim3(256), 0, 0, src, iters, out);
  }
  hipDeviceSynchronize();
  for (int round = 0; round < 5; ++round) {
    for (int shape : {32, 16}) {
      hipEventRecord(e0);
      for (int k = 0; k < 4; ++k) {
        if (shape == 32)
          hipLaunchKernelGGL(probe<32>, dim3(blocks), dim3(256), 0, 0, src, iters, out);
        else
          hipLaunchKernelGGL(probe<16>, dim3(blocks), dim3(256), 0, 0, src, iters, out);
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      printf("round %d shape %dx%d: %.3f ms per launch, %.1f TF/s\n", round, shape, shape,
             ms / 4, 4 * flop / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
