// Block-scaled fp8 quantisation (the operand format of the fp8 GEMMs, lc_common.h): e4m3 values
// plus one E8M0 scale per 32 consecutive k of a row, scales stored [K/128][rows_pad][4].
// Used for MaPLe's frozen-backbone GEMMs (BASELINE config 5: models/maple_clip/model.py:749-772
// casts the backbone to half; here the frozen weights and the activations / gradients feeding
// the QKV / c_fc / c_proj GEMMs are fp8) — weights once per checkpoint, activations per call.
// One lane quantises 8 consecutive k (4 lanes = one scale block), a wave 512 k of one row.
#include "lc_common.h"

namespace {

__global__ void __launch_bounds__(256)
quant_fp8_kernel(long rows, int K, const void* __restrict__ src, int src_f32, long sr, long sk,
                 uint8_t* __restrict__ dst, long ldd, uint8_t* __restrict__ scales, long rows_pad) {
  const int lane = threadIdx.x & 63;
  const int chunks = (K + 511) / 512;
  const long items = rows * chunks;
  const long wave0 = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
  for (long it = wave0; it < items; it += nwaves) {
    const long r = it / chunks;
    const int k0 = (int)(it % chunks) * 512 + lane * 8;
    const bool on = k0 < K;  // K % 128 == 0: whole scale blocks are on or off together
    float v[8];
    if (on) {
      if (!src_f32 && sk == 1) {
        const uint4 u = *reinterpret_cast<const uint4*>(static_cast<const bf16_t*>(src) + r * sr + k0);
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[2 * i] = bf2f(w[i] & 0xffff);
          v[2 * i + 1] = bf2f(w[i] >> 16);
        }
      } else if (src_f32) {
        const float* p = static_cast<const float*>(src) + r * sr + (long)k0 * sk;
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = p[i * sk];
      } else {
        const bf16_t* p = static_cast<const bf16_t*>(src) + r * sr + (long)k0 * sk;
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = bf2f(p[i * sk]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = 0.f;
    }
    uint32_t amax = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) amax = lc_amax_bits(amax, v[i]);
    amax = max(amax, (uint32_t)__shfl_xor((int)amax, 1));
    amax = max(amax, (uint32_t)__shfl_xor((int)amax, 2));
    const uint32_t byte = e8m0_of_bits(amax);
    const float inv = e8m0_inv(byte);
    if (on) {
      uint2 q;
      q.x = pack4_fp8(v[0] * inv, v[1] * inv, v[2] * inv, v[3] * inv);
      q.y = pack4_fp8(v[4] * inv, v[5] * inv, v[6] * inv, v[7] * inv);
      *reinterpret_cast<uint2*>(dst + r * ldd + k0) = q;
      if ((lane & 3) == 0) scales[fp8_scale_index(r, k0 >> 5, rows_pad)] = (uint8_t)byte;
    }
  }
}

}  // namespace

extern "C" {

int lc_quant_fp8(hipStream_t st, long rows, int K, const void* src, int src_f32, long sr, long sk,
                 void* dst, long ldd, void* scales, long rows_pad) {
  LC_CHECK_ARG(rows >= 0 && K > 0 && K % 128 == 0 && ldd >= K && ldd % 8 == 0);
  LC_CHECK_ARG(rows_pad >= rows && rows_pad % 256 == 0 && src && dst && scales);
  LC_CHECK_ARG(sk >= 1 && (sk > 1 || src_f32 || sr % 8 == 0));
  if (rows == 0) return LC_OK;
  const long waves = rows * ((K + 511) / 512);
  long blocks = (waves + 3) / 4;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(quant_fp8_kernel, dim3((unsigned)blocks), dim3(256), 0, st, rows, K, src,
                     src_f32, sr, sk, static_cast<uint8_t*>(dst), ldd,
                     static_cast<uint8_t*>(scales), rows_pad);
  LC_LAUNCH_RET();
}

}  // extern "C"
