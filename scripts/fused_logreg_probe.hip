// Skeleton of a fused logreg score tile, to price the
// design before building it: per 128-particle block, one wave per SIMD
// (wave w: particles 32 w .. +31, its 32 x 256 W rows as FmtH2 fragments in
// 128 VGPRs), the data streamed in chunks of 32 rows through a 2 x 64 KiB
// LDS-DMA ring: per chunk the Z-phase (zT = Xd_chunk . W^T, K = 256, 48
// MFMAs), the sigmoid + 2-part split of z into the G-phase's B fragments,
// the G-phase (accT += XdT_chunk . G, 8 column blocks x K = 32, 48 MFMAs).
// Same MFMA count, LDS traffic, DMA and conversion VALU as the real tile;
// the images hold random fp16 (the numbers are not a score).  Prints the
// time per launch at n = 65536 particles, N = 16384 data rows, p = 256,
// next to the two-kernel scores stage measured in the bench (3.2-3.3 ms).
//   hipcc -O3 --offload-arch=gfx950 scripts/fused_logreg_probe.hip -o build_probe/fused_logreg_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int kQ = 32;                        // data rows per chunk
constexpr int kChunkBytes = 2 * 32 * 1024;    // A_Z (2 parts x 16 K-steps x 32 q x 32 B) + A_G
constexpr int kAG = 32 * 1024;                // A_G: 2 parts x 2 K-steps x 256 c x 32 B

__device__ __forceinline__ int x3_off(int x, int h) { return x * 32 + ((h ^ ((x >> 3) & 1)) << 4); }

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void fused_probe(
    const _Float16* __restrict__ img, int nchunks, const h8* __restrict__ wimg,
    float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kChunkBytes];
  const int t = threadIdx.x, lane = t & 63, r = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  // W fragments of the wave's 32 particles: [K-step][part]
  h8 wb[16][2];
#pragma unroll
  for (int ks = 0; ks < 16; ++ks)
#pragma unroll
    for (int p = 0; p < 2; ++p)
      wb[ks][p] = wimg[(((int64_t)blockIdx.x * 4 + w) * 32 + ks * 2 + p) * 64 + lane];
  f16v acc[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) acc[c] = f16v{};
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)img, (short)0, 0x7fffffff, 0x00020000);
  auto dma = [&](int chunk, char* st) {
    // 64 KiB: 16 x 1 KiB per wave
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int off = (w * 16 + u) * 1024;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(st + off), 16, off + lane * 16,
          chunk * kChunkBytes, 0, 0);
    }
  };
  dma(0, smem);
  const float c1 = -1.4426950408889634f;
  for (int ch = 0; ch < nchunks; ++ch) {
    char* st = smem + (ch & 1) * kChunkBytes;
    if (ch + 1 < nchunks) {
      dma(ch + 1, smem + ((ch + 1) & 1) * kChunkBytes);
      asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
    // Z-phase: zT[q][i] over K = 256
    f16v z = f16v{};
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const h8 a0 = *reinterpret_cast<const h8*>(st + ks * 1024 + x3_off(r, h));
      const h8 a1 = *reinterpret_cast<const h8*>(st + 16 * 1024 + ks * 1024 + x3_off(r, h));
      z = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, wb[ks][0], z, 0, 0, 0);
      z = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, wb[ks][1], z, 0, 0, 0);
      z = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, wb[ks][0], z, 0, 0, 0);
    }
    // G' = 2^15 sigma(-z), split into two fp16 parts: the G-phase's B
    // fragments (lane's 16 values = q 4h + 8g + e: K-steps g >> 1)
    h8 g[2][2];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float ex = __builtin_amdgcn_exp2f(z[e] * c1);
      const float gv = 32768.f * __builtin_amdgcn_rcpf(1.f + ex);
      const _Float16 g0 = (_Float16)gv;
      g[e >> 3][0][e & 7] = g0;
      g[e >> 3][1][e & 7] = (_Float16)(gv - (float)g0);
    }
    // G-phase: accT[c][i] over the chunk's 32 q
    const char* ag = st + kAG;
#pragma unroll
    for (int kg = 0; kg < 2; ++kg)
#pragma unroll
      for (int cb = 0; cb < 8; ++cb) {
        const h8 a0 = *reinterpret_cast<const h8*>(ag + kg * 8192 + x3_off(32 * cb + r, h));
        const h8 a1 = *reinterpret_cast<const h8*>(ag + 16384 + kg * 8192 + x3_off(32 * cb + r, h));
        acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, g[kg][0], acc[cb], 0, 0, 0);
        acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, g[kg][1], acc[cb], 0, 0, 0);
        acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, g[kg][0], acc[cb], 0, 0, 0);
      }
    // every wave is past its reads of this stage before it is refilled
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 8; ++c)
#pragma unroll
    for (int e = 0; e < 16; ++e) s += acc[c][e];
  out[blockIdx.x * 256 + t] = s;
}

int main(int argc, char** argv) {
  const int n = 65536, N = 16384;
  const int blocks = n / 128, nchunks = N / kQ;
  const size_t img_bytes = (size_t)nchunks * kChunkBytes;
  const size_t w_elems = (size_t)blocks * 4 * 32 * 64 * 8;
  std::vector<_Float16> hi(img_bytes / 2), hw(w_elems);
  srand(3);
  for (auto& v : hi) v = (_Float16)((rand() / (float)RAND_MAX) - 0.5f);
  for (auto& v : hw) v = (_Float16)(((rand() / (float)RAND_MAX) - 0.5f) * 0.1f);
  _Float16* img;
  h8* wimg;
  float* out;
  hipMalloc(&img, img_bytes);
  hipMalloc(&wimg, w_elems * 2);
  hipMalloc(&out, (size_t)blocks * 256 * 4);
  hipMemcpy(img, hi.data(), img_bytes, hipMemcpyHostToDevice);
  hipMemcpy(wimg, hw.data(), w_elems * 2, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i)
    hipLaunchKernelGGL(fused_probe, dim3(blocks), dim3(256), 0, 0, img, nchunks, wimg, out);
  hipDeviceSynchronize();
  const double flop = 4.0 * n * (double)N * 256;  // algorithmic fp32 products x2
  for (int round = 0; round < 5; ++round) {
    hipEventRecord(e0);
    for (int k = 0; k < 10; ++k)
      hipLaunchKernelGGL(fused_probe, dim3(blocks), dim3(256), 0, 0, img, nchunks, wimg, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    printf("round %d: fused skeleton %.3f ms per launch = %.1f TF/s of fp32 products (FmtH2)\n",
           round, ms / 10, flop / (ms / 10 * 1e-3) / 1e12);
  }
  return 0;
}
