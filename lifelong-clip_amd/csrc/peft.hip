// PEFT residual kernels and the optimizer step.
//  LoRA  (models/clip/lora.py:419-452, 837-839, 1072-1074; lora.Linear :100-173): the rank-r
//        update is merged into the frozen weight once per optimizer step,
//        W_eff = W + scaling * B @ A (bf16, both [out,in] and [in,out] layouts), so the
//        forward/dX GEMMs run at full MFMA width; dA/dB come from one fused reduction pass
//        over the saved activations.
//  Adapter (models/clip/adapter.py:53-72, used twice per block, model.py:440-441): fused
//        down(64)+ReLU+dropout+up+scale+residual forward and the matching row-local backward;
//        the weight gradients go through lc_gemm_tn.
//  AdamW (torch.optim.AdamW as selected by utils/train_utils.py:27-28) over one flat fp32
//        buffer holding every trainable tensor, with the GradScaler-style non-finite skip.
#include "lc_common.h"

namespace {

// ---------------------------------------------------------------------------- casts / merge
__global__ void cast_bf16_kernel(long n, const float* __restrict__ src, bf16_t* __restrict__ dst) {
  for (long i = (blockIdx.x * (long)blockDim.x + threadIdx.x) * 4; i < n;
       i += (long)gridDim.x * blockDim.x * 4) {
    if (i + 3 < n) {
      const float4 v = *reinterpret_cast<const float4*>(src + i);
      *reinterpret_cast<uint2*>(dst + i) = uint2{pack2bf(v.x, v.y), pack2bf(v.z, v.w)};
    } else {
      for (long j = i; j < n; ++j) dst[j] = f2bf(src[j]);
    }
  }
}

// dst (+)= bf16 of W[N,K] + s*B[N,r]@A[r,K] in [N,K] layout and optionally [K,N].
// 64x64 tiles through LDS so the transposed write is coalesced.
__global__ void merge_kernel(int N, int K, int r, const float* __restrict__ W,
                             const float* __restrict__ A, const float* __restrict__ B, float s,
                             bf16_t* __restrict__ out, bf16_t* __restrict__ outT) {
  __shared__ float tile[64][65];
  const int n0 = blockIdx.y * 64, k0 = blockIdx.x * 64;
  for (int i = threadIdx.x; i < 64 * 64; i += blockDim.x) {
    const int nn = i / 64, kk = i % 64;
    const int n = n0 + nn, k = k0 + kk;
    float v = 0.f;
    if (n < N && k < K) {
      v = W[(long)n * K + k];
      for (int j = 0; j < r; ++j) v += s * B[n * r + j] * A[(long)j * K + k];
      out[(long)n * K + k] = f2bf(v);
    }
    tile[nn][kk] = v;
  }
  if (!outT) return;
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += blockDim.x) {
    const int kk = i / 64, nn = i % 64;
    const int n = n0 + nn, k = k0 + kk;
    if (n < N && k < K) outT[(long)k * N + n] = f2bf(tile[nn][kk]);
  }
}

// ---------------------------------------------------------------------------- LoRA gradients
// For rows m of a chunk: U[m][j] = X[m]·A[j], G[m][j] = dY[m]·B[:,j]
//   dB[n][j] += s * sum_m dY[m][n] U[m][j]      dA[j][k] += s * sum_m G[m][j] X[m][k]
// One workgroup = 256 threads, a strided set of 16-row groups; partial dA/dB kept in registers
// (each thread owns columns tid, tid+256, ...), flushed with one f32 atomic per element.
template <int R, int NMAX, int KMAX>
__global__ void __launch_bounds__(256)
lora_grad_kernel(int M, int N, int K, const bf16_t* __restrict__ dY, long ldy,
                 const bf16_t* __restrict__ X, long ldx, const float* __restrict__ A,
                 const float* __restrict__ B, float s, float* __restrict__ dA,
                 float* __restrict__ dB) {
  constexpr int RB = 16;  // rows per group
  __shared__ float uS[RB][R], gS[RB][R];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  float accB[NMAX / 256][R], accA[KMAX / 256][R];
#pragma unroll
  for (int i = 0; i < NMAX / 256; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) accB[i][j] = 0.f;
#pragma unroll
  for (int i = 0; i < KMAX / 256; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) accA[i][j] = 0.f;

  const int ngroups = (M + RB - 1) / RB;
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int m0 = grp * RB;
    // each wave computes U, G for 4 rows
    for (int rr = 0; rr < RB / 4; ++rr) {
      const int lr = w * (RB / 4) + rr;
      const int m = m0 + lr;
      float u[R], gg[R];
#pragma unroll
      for (int j = 0; j < R; ++j) u[j] = gg[j] = 0.f;
      if (m < M) {
        for (int k = lane; k < K; k += 64) {
          const float x = bf2f(X[(long)m * ldx + k]);
#pragma unroll
          for (int j = 0; j < R; ++j) u[j] += x * A[(long)j * K + k];
        }
        for (int n = lane; n < N; n += 64) {
          const float d = bf2f(dY[(long)m * ldy + n]);
#pragma unroll
          for (int j = 0; j < R; ++j) gg[j] += d * B[(long)n * R + j];
        }
      }
#pragma unroll
      for (int j = 0; j < R; ++j) {
        u[j] = wave_sum(u[j]);
        gg[j] = wave_sum(gg[j]);
      }
      if (lane == 0) {
#pragma unroll
        for (int j = 0; j < R; ++j) {
          uS[lr][j] = u[j];
          gS[lr][j] = gg[j];
        }
      }
    }
    __syncthreads();
    const int rows = min(RB, M - m0);
    for (int lr = 0; lr < rows; ++lr) {
      const int m = m0 + lr;
#pragma unroll
      for (int i = 0; i < NMAX / 256; ++i) {
        const int n = tid + i * 256;
        if (n < N) {
          const float d = bf2f(dY[(long)m * ldy + n]);
#pragma unroll
          for (int j = 0; j < R; ++j) accB[i][j] += d * uS[lr][j];
        }
      }
#pragma unroll
      for (int i = 0; i < KMAX / 256; ++i) {
        const int k = tid + i * 256;
        if (k < K) {
          const float x = bf2f(X[(long)m * ldx + k]);
#pragma unroll
          for (int j = 0; j < R; ++j) accA[i][j] += gS[lr][j] * x;
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < NMAX / 256; ++i) {
    const int n = tid + i * 256;
    if (n < N)
#pragma unroll
      for (int j = 0; j < R; ++j) atomicAdd(dB + (long)n * R + j, s * accB[i][j]);
  }
#pragma unroll
  for (int i = 0; i < KMAX / 256; ++i) {
    const int k = tid + i * 256;
    if (k < K)
#pragma unroll
      for (int j = 0; j < R; ++j) atomicAdd(dA + (long)j * K + k, s * accA[i][j]);
  }
}

// ---------------------------------------------------------------------------- adapter
// 64 rows per workgroup, 4 waves x 16 rows, everything in registers:
//   down  D^T[j][m] = sum_k Wd[j][k] z[m][k]      (A = Wd rows, B = z rows; K = width)
//   h = dropout(relu(D + bd))                      (lane holds 4 consecutive j of one row m)
//   up    U^T[n][m] = sum_j Wu[n][j] h[m][j]       (B = h straight from the accumulators; the
//                                                    A fragment reads Wu in the same j order)
//   x_out = resid + z + scale*(U + bu)             (adapter.py:59-72, model.py:440-441)
constexpr int AD_H = 64;  // adapter.py:38 hard-codes the down width (Q7)

// k-order used when an accumulator pair (tiles 2s, 2s+1) becomes a B operand:
// slot j<4 -> 32s + 4g + j ; j>=4 -> 32s + 16 + 4g + (j-4)
LC_DEV bf16x8 load_perm(const bf16_t* row, int s, int g) {
  const uint2 lo = *reinterpret_cast<const uint2*>(row + 32 * s + 4 * g);
  const uint2 hi = *reinterpret_cast<const uint2*>(row + 32 * s + 16 + 4 * g);
  bf16x8 r;
  r[0] = (short)(lo.x & 0xffff); r[1] = (short)(lo.x >> 16);
  r[2] = (short)(lo.y & 0xffff); r[3] = (short)(lo.y >> 16);
  r[4] = (short)(hi.x & 0xffff); r[5] = (short)(hi.x >> 16);
  r[6] = (short)(hi.y & 0xffff); r[7] = (short)(hi.y >> 16);
  return r;
}
LC_DEV bf16x8 pack8(const f32x4& a, const f32x4& b) {
  uint32_t w0 = pack2bf(a[0], a[1]), w1 = pack2bf(a[2], a[3]);
  uint32_t w2 = pack2bf(b[0], b[1]), w3 = pack2bf(b[2], b[3]);
  bf16x8 r;
  r[0] = (short)(w0 & 0xffff); r[1] = (short)(w0 >> 16);
  r[2] = (short)(w1 & 0xffff); r[3] = (short)(w1 >> 16);
  r[4] = (short)(w2 & 0xffff); r[5] = (short)(w2 >> 16);
  r[6] = (short)(w3 & 0xffff); r[7] = (short)(w3 >> 16);
  return r;
}

LC_DEV float drop_mul(uint64_t seed, long m, int j, float keep) {
  if (keep >= 1.0f) return 1.0f;
  const uint32_t hsh = lc_hash(seed, (uint64_t)m * AD_H + j);
  const float u = (hsh >> 8) * (1.0f / 16777216.0f);
  return u < keep ? 1.0f / keep : 0.0f;
}

__global__ void __launch_bounds__(256)
adapter_fwd_kernel(int M, int Dw, const bf16_t* __restrict__ z, long ldz,
                   const bf16_t* __restrict__ Wd, const float* __restrict__ bd,
                   const bf16_t* __restrict__ Wu, const float* __restrict__ bu, float scale,
                   float keep, uint64_t seed, const float* __restrict__ resid,
                   float* __restrict__ xout, long ldx, bf16_t* __restrict__ hout) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, t = lane & 15;
  const int m = blockIdx.x * 64 + w * 16 + t;
  const bool ok = m < M;
  const long mr = ok ? m : (M - 1);
  const bf16_t* zr = z + mr * ldz;

  f32x4 dn[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) dn[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < Dw; k0 += 32) {
    const bf16x8 zb = *reinterpret_cast<const bf16x8*>(zr + k0 + 8 * g);
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) {
      const bf16x8 wa = *reinterpret_cast<const bf16x8*>(Wd + (long)(jt * 16 + t) * Dw + k0 + 8 * g);
      dn[jt] = mfma16(wa, zb, dn[jt]);
    }
  }
  // lane holds D[j = jt*16 + 4g + r][m]
#pragma unroll
  for (int jt = 0; jt < 4; ++jt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = jt * 16 + 4 * g + r;
      const float v = fmaxf(dn[jt][r] + bd[j], 0.f) * drop_mul(seed, m, j, keep);
      dn[jt][r] = __uint_as_float((uint32_t)f2bf(v) << 16);  // round to the stored bf16 value
    }
  if (ok) {
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
      *reinterpret_cast<uint2*>(hout + (long)m * AD_H + jt * 16 + 4 * g) =
          uint2{pack2bf(dn[jt][0], dn[jt][1]), pack2bf(dn[jt][2], dn[jt][3])};
  }
  const bf16x8 hb0 = pack8(dn[0], dn[1]);  // k-step 0 (j 0..31)
  const bf16x8 hb1 = pack8(dn[2], dn[3]);  // k-step 1 (j 32..63)
  for (int nt = 0; nt < Dw / 16; ++nt) {
    const bf16_t* wrow = Wu + (long)(nt * 16 + t) * AD_H;
    f32x4 u = f32x4{0.f, 0.f, 0.f, 0.f};
    u = mfma16(load_perm(wrow, 0, g), hb0, u);
    u = mfma16(load_perm(wrow, 1, g), hb1, u);
    if (ok) {
      const int n = nt * 16 + 4 * g;
      const float4 rs = *reinterpret_cast<const float4*>(resid + (long)m * ldx + n);
      const uint2 zz = *reinterpret_cast<const uint2*>(zr + n);
      const float4 bb = *reinterpret_cast<const float4*>(bu + n);
      float4 o;
      o.x = rs.x + bf2f(zz.x & 0xffff) + scale * (u[0] + bb.x);
      o.y = rs.y + bf2f(zz.x >> 16) + scale * (u[1] + bb.y);
      o.z = rs.z + bf2f(zz.y & 0xffff) + scale * (u[2] + bb.z);
      o.w = rs.w + bf2f(zz.y >> 16) + scale * (u[3] + bb.w);
      *reinterpret_cast<float4*>(xout + (long)m * ldx + n) = o;
    }
  }
}

// Backward of out = z + scale*(h Wu^T + bu), h = drop(relu(z Wd^T + bd)), given gout:
//   dh^T[j][m] = scale * sum_n WuT[j][n] gout[m][n]
//   dpre = dh * (h > 0) / keep            -> dpre_out (bf16), dbd += sum_m dpre
//   dz^T[n][m] = sum_j WdT[n][j] dpre[m][j]; dz = gout + dz   -> dz_out (bf16)
//   dbu += scale * sum_m gout
// (dWu = scale * gout^T h and dWd = dpre^T z are done by lc_gemm_tn.)
__global__ void __launch_bounds__(256)
adapter_bwd_kernel(int M, int Dw, const bf16_t* __restrict__ gout, long ldg,
                   const bf16_t* __restrict__ h, const bf16_t* __restrict__ WuT,
                   const bf16_t* __restrict__ WdT, float scale, float keep,
                   bf16_t* __restrict__ dpre_out, bf16_t* __restrict__ dz_out, long ldz,
                   float* __restrict__ dbd, float* __restrict__ dbu) {
  __shared__ float colsum[1024];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, t = lane & 15;
  const int m = blockIdx.x * 64 + w * 16 + t;
  const bool ok = m < M;
  const long mr = ok ? m : (M - 1);
  const bf16_t* gr = gout + mr * ldg;
  for (int i = tid; i < Dw; i += 256) colsum[i] = 0.f;

  f32x4 dh[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) dh[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < Dw; k0 += 32) {
    const bf16x8 gb = *reinterpret_cast<const bf16x8*>(gr + k0 + 8 * g);
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) {
      const bf16x8 wa = *reinterpret_cast<const bf16x8*>(WuT + (long)(jt * 16 + t) * Dw + k0 + 8 * g);
      dh[jt] = mfma16(wa, gb, dh[jt]);
    }
  }
  float dbd_loc[4][4];
#pragma unroll
  for (int jt = 0; jt < 4; ++jt) {
    const uint2 hv = *reinterpret_cast<const uint2*>(h + mr * AD_H + jt * 16 + 4 * g);
    const float hh[4] = {bf2f(hv.x & 0xffff), bf2f(hv.x >> 16), bf2f(hv.y & 0xffff), bf2f(hv.y >> 16)};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = (ok && hh[r] > 0.f) ? dh[jt][r] * scale / keep : 0.f;
      v = __uint_as_float((uint32_t)f2bf(v) << 16);
      dh[jt][r] = v;
      dbd_loc[jt][r] = v;
    }
    if (ok)
      *reinterpret_cast<uint2*>(dpre_out + (long)m * AD_H + jt * 16 + 4 * g) =
          uint2{pack2bf(dh[jt][0], dh[jt][1]), pack2bf(dh[jt][2], dh[jt][3])};
  }
  // dbd: reduce over the 16 rows (lanes t) of this wave, then atomics
#pragma unroll
  for (int jt = 0; jt < 4; ++jt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = dbd_loc[jt][r];
      v += __shfl_xor(v, 1); v += __shfl_xor(v, 2); v += __shfl_xor(v, 4); v += __shfl_xor(v, 8);
      if (t == 0) atomicAdd(dbd + jt * 16 + 4 * g + r, v);
    }
  __syncthreads();  // colsum zeroed
  const bf16x8 pb0 = pack8(dh[0], dh[1]);
  const bf16x8 pb1 = pack8(dh[2], dh[3]);
  for (int nt = 0; nt < Dw / 16; ++nt) {
    const bf16_t* wrow = WdT + (long)(nt * 16 + t) * AD_H;
    f32x4 u = f32x4{0.f, 0.f, 0.f, 0.f};
    u = mfma16(load_perm(wrow, 0, g), pb0, u);
    u = mfma16(load_perm(wrow, 1, g), pb1, u);
    const int n = nt * 16 + 4 * g;
    const uint2 gg = *reinterpret_cast<const uint2*>(gr + n);
    const float g4[4] = {bf2f(gg.x & 0xffff), bf2f(gg.x >> 16), bf2f(gg.y & 0xffff), bf2f(gg.y >> 16)};
    if (ok)
      *reinterpret_cast<uint2*>(dz_out + (long)m * ldz + n) =
          uint2{pack2bf(g4[0] + u[0], g4[1] + u[1]), pack2bf(g4[2] + u[2], g4[3] + u[3])};
    // column sums of gout over this wave's 16 rows
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = ok ? g4[r] : 0.f;
      v += __shfl_xor(v, 1); v += __shfl_xor(v, 2); v += __shfl_xor(v, 4); v += __shfl_xor(v, 8);
      if (t == 0) atomicAdd(&colsum[n + r], v);
    }
  }
  __syncthreads();
  for (int i = tid; i < Dw; i += 256) atomicAdd(dbu + i, scale * colsum[i]);
}

// ---------------------------------------------------------------------------- AdamW
__global__ void finite_kernel(long n, const float* __restrict__ g, int* __restrict__ flag) {
  int bad = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    bad |= !isfinite(g[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

__global__ void adamw_kernel(long n, float* __restrict__ p, const float* __restrict__ g,
                             float* __restrict__ m, float* __restrict__ v, float lr, float b1,
                             float b2, float eps, float wd, float bc1, float bc2,
                             const int* __restrict__ skip) {
  if (skip && *skip) return;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float gi = g[i];
    float pi = p[i] * (1.0f - lr * wd);
    const float mi = b1 * m[i] + (1.0f - b1) * gi;
    const float vi = b2 * v[i] + (1.0f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi / bc2) + eps;
    p[i] = pi - (lr / bc1) * mi / denom;
  }
}

int grid_for(long work, int block) {
  long gsz = (work + block - 1) / block;
  if (gsz > 4096) gsz = 4096;
  return (int)(gsz < 1 ? 1 : gsz);
}

}  // namespace

extern "C" {

int lc_cast_bf16(hipStream_t st, long n, const float* src, void* dst) {
  LC_CHECK_ARG(n >= 0);
  if (n == 0) return LC_OK;
  hipLaunchKernelGGL(cast_bf16_kernel, dim3(grid_for(n / 4 + 1, 256)), dim3(256), 0, st, n, src,
                     (bf16_t*)dst);
  LC_LAUNCH_RET();
}

int lc_merge_weight(hipStream_t st, int N, int K, int r, const float* W, const float* A,
                    const float* B, float scaling, void* out, void* outT) {
  LC_CHECK_ARG(N > 0 && K > 0 && r >= 0 && (r == 0 || (A && B)));
  dim3 grid((K + 63) / 64, (N + 63) / 64);
  hipLaunchKernelGGL(merge_kernel, grid, dim3(256), 0, st, N, K, r, W, A, B, scaling,
                     (bf16_t*)out, (bf16_t*)outT);
  LC_LAUNCH_RET();
}

int lc_lora_grad(hipStream_t st, int M, int N, int K, int r, const void* dY, long ldy,
                 const void* X, long ldx, const float* A, const float* B, float scaling,
                 float* dA, float* dB) {
  LC_CHECK_ARG(M > 0 && r == 4 && N <= 3072 && K <= 1024 && N > 0 && K > 0);
  const int groups = (M + 15) / 16;
  const int grid = groups < 512 ? groups : 512;
  if (N <= 1024)
    hipLaunchKernelGGL((lora_grad_kernel<4, 1024, 1024>), dim3(grid), dim3(256), 0, st, M, N, K,
                       (const bf16_t*)dY, ldy, (const bf16_t*)X, ldx, A, B, scaling, dA, dB);
  else
    hipLaunchKernelGGL((lora_grad_kernel<4, 3072, 1024>), dim3(grid), dim3(256), 0, st, M, N, K,
                       (const bf16_t*)dY, ldy, (const bf16_t*)X, ldx, A, B, scaling, dA, dB);
  LC_LAUNCH_RET();
}

int lc_adapter_fwd(hipStream_t st, int M, int D, const void* z, long ldz, const void* Wd,
                   const float* bd, const void* Wu, const float* bu, float scale, float keep,
                   unsigned long long seed, const float* resid, float* xout, long ldx, void* hout) {
  LC_CHECK_ARG(M > 0 && D % 32 == 0 && D % 16 == 0 && ldz % 8 == 0 && ldx % 4 == 0);
  LC_CHECK_ARG(keep > 0.f && keep <= 1.f);
  hipLaunchKernelGGL(adapter_fwd_kernel, dim3((M + 63) / 64), dim3(256), 0, st, M, D,
                     (const bf16_t*)z, ldz, (const bf16_t*)Wd, bd, (const bf16_t*)Wu, bu, scale,
                     keep, (uint64_t)seed, resid, xout, ldx, (bf16_t*)hout);
  LC_LAUNCH_RET();
}

int lc_adapter_bwd(hipStream_t st, int M, int D, const void* gout, long ldg, const void* h,
                   const void* WuT, const void* WdT, float scale, float keep, void* dpre,
                   void* dz, long ldz, float* dbd, float* dbu) {
  LC_CHECK_ARG(M > 0 && D % 32 == 0 && D <= 1024 && ldg % 8 == 0 && ldz % 4 == 0);
  LC_CHECK_ARG(keep > 0.f && keep <= 1.f);
  hipLaunchKernelGGL(adapter_bwd_kernel, dim3((M + 63) / 64), dim3(256), 0, st, M, D,
                     (const bf16_t*)gout, ldg, (const bf16_t*)h, (const bf16_t*)WuT,
                     (const bf16_t*)WdT, scale, keep, (bf16_t*)dpre, (bf16_t*)dz, ldz, dbd, dbu);
  LC_LAUNCH_RET();
}

int lc_check_finite(hipStream_t st, long n, const float* g, int* flag) {
  LC_CHECK_ARG(n >= 0);
  if (n == 0) return LC_OK;
  hipLaunchKernelGGL(finite_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, n, g, flag);
  LC_LAUNCH_RET();
}

int lc_adamw(hipStream_t st, long n, float* p, const float* g, float* m, float* v, float lr,
             float b1, float b2, float eps, float wd, int step, const int* skip) {
  LC_CHECK_ARG(n >= 0 && step >= 1);
  if (n == 0) return LC_OK;
  const float bc1 = 1.0f - powf(b1, (float)step), bc2 = 1.0f - powf(b2, (float)step);
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, n, p, g, m, v, lr, b1,
                     b2, eps, wd, bc1, bc2, skip);
  LC_LAUNCH_RET();
}

}  // extern "C"
