// bf16 MFMA shape vs the clock the chip holds (dev tool; MI355X_MICROARCH.md 'DVFS give-back'
// item 7, cdna_hip_programming.md §5.4 rule 28): the same register-resident MFMA stream on
// v_mfma_f32_16x16x32_bf16 and v_mfma_f32_32x32x16_bf16, random operands rotated every MFMA, one
// 256-thread workgroup per CU slot (4 waves, one per SIMD) x 1 or 2 per CU (argv[2]). After ~2 s of back-to-back
// launches it reports TFLOP/s (HIP events), the in-kernel clock (s_memtime / s_memrealtime x
// 100 MHz, median over workgroups) and the MFMA issue efficiency per clock.
//   hipcc --offload-arch=gfx950 -O3 -o lifelong-clip_amd/lcclip/ab/mfma_shape_clock tools/mfma_shape_clock.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

constexpr int NOP = 4;  // operand pairs rotated through

// SHAPE 16: 8 16x16x32 MFMAs per round on 4 accumulators; SHAPE 32: 4 32x32x16 ones on 4 (the
// same work per round: 16x16x32 = 16 Kflop, 32x32x16 = 32 Kflop, one 32x32 MFMA = two 16x16).
template <int SHAPE>
__global__ void __launch_bounds__(256) mfma_loop(const bf16x8* __restrict__ src, float* __restrict__ dst,
                                                 int iters, unsigned long long* __restrict__ clk) {
  const int tid = threadIdx.x;
  bf16x8 a[NOP], b[NOP];
#pragma unroll
  for (int i = 0; i < NOP; ++i) {
    a[i] = src[(blockIdx.x * 256 + tid) * 2 * NOP + 2 * i];
    b[i] = src[(blockIdx.x * 256 + tid) * 2 * NOP + 2 * i + 1];
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  if constexpr (SHAPE == 16) {
    // 4 accumulators, each taking two MFMAs per round (8 per round as the 32x32 form's 4), issued
    // in place by inline asm: through the builtin hipcc rotated them through AGPR copies (24
    // v_accvgpr_* per 32 MFMAs)
    f32x4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < iters; it += NOP) {
#pragma unroll
      for (int u = 0; u < NOP; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                       : "+a"(acc[j & 3])
                       : "v"(a[(j + u) % NOP]), "v"(b[(j + 3 * u) % NOP]));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  } else {
    f32x16 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
    for (int it = 0; it < iters; it += NOP) {
#pragma unroll
      for (int u = 0; u < NOP; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[(j + u) % NOP], b[(j + 3 * u) % NOP],
                                                           acc[j], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) s += acc[j][e];
  }
  dst[blockIdx.x * 256 + tid] = s;
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

int main(int argc, char** argv) {
  const bool zero = argc > 1 && argv[1][0] == 'z';
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int per_cu = argc > 2 ? atoi(argv[2]) : 2;  // workgroups (= waves per SIMD) per CU
  const int wgs = per_cu * cus, iters = 4096;
  const size_t nsrc = (size_t)wgs * 256 * 2 * NOP;
  std::vector<uint16_t> h(nsrc * 8);
  unsigned x = 12345;
  for (auto& v : h) {
    x = x * 1664525u + 1013904223u;
    // bf16 of a value in [-2, 2): sign, exponent 126..128, random mantissa
    v = zero ? 0 : (uint16_t)(((x >> 31) << 15) | ((126 + (x >> 8) % 3) << 7) | ((x >> 12) & 0x7F));
  }
  bf16x8* src;
  float* dst;
  unsigned long long* clk;
  CHECK(hipMalloc(&src, nsrc * 16));
  CHECK(hipMalloc(&dst, wgs * 256 * 4));
  CHECK(hipMalloc(&clk, wgs * 16));
  CHECK(hipMemcpy(src, h.data(), nsrc * 16, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  printf("data=%s wgs=%d (%d per CU, 4 waves each) iters=%d\n", zero ? "zeros" : "random", wgs, per_cu,
         iters);
  for (int shape : {16, 32, 16, 32}) {
    auto launch = [&]() {
      if (shape == 16)
        hipLaunchKernelGGL(mfma_loop<16>, dim3(wgs), dim3(256), 0, 0, src, dst, iters, clk);
      else
        hipLaunchKernelGGL(mfma_loop<32>, dim3(wgs), dim3(256), 0, 0, src, dst, iters, clk);
    };
    const auto end = std::chrono::steady_clock::now() + std::chrono::seconds(2);
    while (std::chrono::steady_clock::now() < end) {
      for (int i = 0; i < 10; ++i) launch();
      CHECK(hipDeviceSynchronize());
    }
    CHECK(hipEventRecord(e0));
    const int reps = 20;
    for (int i = 0; i < reps; ++i) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipGetLastError());
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    std::vector<unsigned long long> c(2 * wgs);
    CHECK(hipMemcpy(c.data(), clk, wgs * 16, hipMemcpyDeviceToHost));
    std::vector<double> ghz;
    double cyc = 0;
    for (int w = 0; w < wgs; ++w) {
      ghz.push_back((double)c[2 * w] / (double)c[2 * w + 1] * 0.1);
      cyc = std::max(cyc, (double)c[2 * w]);
    }
    std::sort(ghz.begin(), ghz.end());
    // flops per launch: wgs x 4 waves x iters x (8 x 16x16x32 | 4 x 32x32x16) = 4 x 32 Kflop per iter
    const double flops = (double)wgs * 4 * iters * 4 * 32768.0;
    const double tf = flops / (ms * 1e-3) / 1e12;
    // per-clock: the dense bf16 rate is 2.5 PF at 2.4 GHz = 1024 flop / SIMD / clock
    const double need = (double)iters * 4 * 32768.0 * per_cu / 1024.0;  // cycles per SIMD
    printf("shape %dx%d: %.3f ms  %.0f TF (%.3f of 2.5 PF)  clock %.3f GHz (median, min %.3f max %.3f)"
           "  issue eff %.3f  (TF / (clock x 1024 flop x 1024 SIMDs) %.3f)\n",
           shape, shape, ms, tf, tf / 2500.0, ghz[wgs / 2], ghz[0], ghz[wgs - 1], need / cyc,
           tf * 1e12 / (ghz[wgs / 2] * 1e9 * 1024.0 * 4 * cus));
  }
  return 0;
}
