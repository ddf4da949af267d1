// Row-local kernels: LayerNorm fwd/bwd (models/clip/model.py:194-200, fp32 statistics,
// eps 1e-5), ViT patch im2col + token assembly (model.py:756-764), text token embedding
// (model.py:943-946) and EOT row selection (model.py:953-954).
// One wave per row; rows are independent, so the grid is rows/4 workgroups of 4 waves. All
// global traffic is 16 B per lane where the row width allows (D % 256 == 0: 768, 512, 1024).
#include "lc_common.h"

namespace {

template <int V>  // V = D / 64 elements per lane
struct RowBuf {
  float v[V];
};

// Load a row of D = 64*V floats: lane holds elements {lane*4 + 256*i + j} when V % 4 == 0,
// else {lane + 64*i}. Both layouts are used consistently for params and outputs.
template <int V>
LC_DEV void load_row_f32(const float* __restrict__ p, int lane, float (&v)[V]) {
  if constexpr (V % 4 == 0) {
#pragma unroll
    for (int i = 0; i < V / 4; ++i) {
      float4 t = *reinterpret_cast<const float4*>(p + i * 256 + lane * 4);
      v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = p[i * 64 + lane];
  }
}
template <int V>
LC_DEV void load_row_bf16(const bf16_t* __restrict__ p, int lane, float (&v)[V]) {
  if constexpr (V % 4 == 0) {
#pragma unroll
    for (int i = 0; i < V / 4; ++i) {
      uint2 t = *reinterpret_cast<const uint2*>(p + i * 256 + lane * 4);
      v[4 * i] = bf2f(t.x & 0xffff); v[4 * i + 1] = bf2f(t.x >> 16);
      v[4 * i + 2] = bf2f(t.y & 0xffff); v[4 * i + 3] = bf2f(t.y >> 16);
    }
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = bf2f(p[i * 64 + lane]);
  }
}
template <int V>
LC_DEV void store_row_f32(float* __restrict__ p, int lane, const float (&v)[V]) {
  if constexpr (V % 4 == 0) {
#pragma unroll
    for (int i = 0; i < V / 4; ++i)
      *reinterpret_cast<float4*>(p + i * 256 + lane * 4) =
          make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) p[i * 64 + lane] = v[i];
  }
}
template <int V>
LC_DEV void store_row_bf16(bf16_t* __restrict__ p, int lane, const float (&v)[V]) {
  if constexpr (V % 4 == 0) {
#pragma unroll
    for (int i = 0; i < V / 4; ++i)
      *reinterpret_cast<uint2*>(p + i * 256 + lane * 4) =
          uint2{pack2bf(v[4 * i], v[4 * i + 1]), pack2bf(v[4 * i + 2], v[4 * i + 3])};
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) p[i * 64 + lane] = f2bf(v[i]);
  }
}

// A residual-stream row (XT = float or _Float16, lc_common.h), same lane layouts as above.
// nt: nontemporal loads (a saved activation read once)
template <int V, typename XT>
LC_DEV void load_row_x(const XT* __restrict__ p, int lane, float (&v)[V], bool nt = false) {
  if constexpr (sizeof(XT) == 4) {
    if constexpr (V % 4 == 0) {
      if (nt) {
#pragma unroll
        for (int i = 0; i < V / 4; ++i) {
          const f32x4 t = __builtin_nontemporal_load(
              reinterpret_cast<const f32x4*>((const float*)p + i * 256 + lane * 4));
          v[4 * i] = t[0]; v[4 * i + 1] = t[1]; v[4 * i + 2] = t[2]; v[4 * i + 3] = t[3];
        }
        return;
      }
    }
    load_row_f32<V>((const float*)p, lane, v);
  } else if constexpr (V % 4 == 0) {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int i = 0; i < V / 4; ++i) {
      const u32x2* q = reinterpret_cast<const u32x2*>((const uint16_t*)p + i * 256 + lane * 4);
      const u32x2 t = nt ? __builtin_nontemporal_load(q) : *q;
      v[4 * i] = h2f(t[0] & 0xffff); v[4 * i + 1] = h2f(t[0] >> 16);
      v[4 * i + 2] = h2f(t[1] & 0xffff); v[4 * i + 3] = h2f(t[1] >> 16);
    }
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = h2f(((const uint16_t*)p)[i * 64 + lane]);
  }
}
template <int V, typename XT>
LC_DEV void store_row_x(XT* __restrict__ p, int lane, const float (&v)[V]) {
  if constexpr (sizeof(XT) == 4) {
    store_row_f32<V>((float*)p, lane, v);
  } else if constexpr (V % 4 == 0) {
#pragma unroll
    for (int i = 0; i < V / 4; ++i)
      *reinterpret_cast<uint2*>((uint16_t*)p + i * 256 + lane * 4) =
          uint2{pack2h(v[4 * i], v[4 * i + 1]), pack2h(v[4 * i + 2], v[4 * i + 3])};
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i)
      ((uint16_t*)p)[i * 64 + lane] = __builtin_bit_cast(uint16_t, (_Float16)v[i]);
  }
}

// A row (V % 4 == 0 layout) as e4m3 codes + E8M0 scales in the fp8 GEMM operand format: a
// 32-column block is 8 consecutive lanes' 4 values; the arithmetic is quant_fp8_kernel's
// (quant.hip) on the bf16-rounded values, so the codes equal bf16 output + quant_fp8.
template <int V>
LC_DEV void store_row_fp8(uint8_t* __restrict__ p, uint8_t* __restrict__ scales, long rows_pad,
                          long row, int lane, const float (&v)[V]) {
  static_assert(V % 4 == 0, "fp8 rows need D % 256 == 0");
#pragma unroll
  for (int i = 0; i < V / 4; ++i) {
    float q[4];
    uint32_t amax = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      q[j] = bf2f(f2bf(v[4 * i + j]));
      amax = lc_amax_bits(amax, q[j]);
    }
    amax = max(amax, (uint32_t)__shfl_xor((int)amax, 1));
    amax = max(amax, (uint32_t)__shfl_xor((int)amax, 2));
    amax = max(amax, (uint32_t)__shfl_xor((int)amax, 4));
    const uint32_t byte = e8m0_of_bits(amax);
    const float inv = e8m0_inv(byte);
    const int k = i * 256 + lane * 4;
    *reinterpret_cast<uint32_t*>(p + k) = pack4_fp8(q[0] * inv, q[1] * inv, q[2] * inv, q[3] * inv);
    if ((lane & 7) == 0) scales[fp8_scale_index(row, k >> 5, rows_pad)] = (uint8_t)byte;
  }
}

// y (bf16 / f32, optional when q is set) and / or q: the fp8 operand of the next GEMM
template <int V, typename XT = float>
__global__ void __launch_bounds__(256)
ln_fwd_kernel(int rows, const XT* __restrict__ x, long ldx, const int* __restrict__ row_idx,
              const float* __restrict__ gamma, const float* __restrict__ beta, void* __restrict__ y,
              int y_f32, long ldy, float* __restrict__ mean_out, float* __restrict__ rstd_out,
              uint8_t* __restrict__ qo, long ldq, uint8_t* __restrict__ q_scale, long q_rows) {
  constexpr int D = V * 64;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const long src = row_idx ? (long)row_idx[row] : (long)row;
  // every load of the row issued before the first reduction: one HBM round trip per row
  float v[V], gm[V], bt[V];
  load_row_x<V, XT>(x + src * ldx, lane, v);
  load_row_f32<V>(gamma, lane, gm);
  load_row_f32<V>(beta, lane, bt);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) s += v[i];
  const float mean = wave_sum(s) * (1.0f / D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    v[i] -= mean;
    q += v[i] * v[i];
  }
  const float rstd = rsqrtf(wave_sum(q) * (1.0f / D) + 1e-5f);
#pragma unroll
  for (int i = 0; i < V; ++i) v[i] = v[i] * rstd * gm[i] + bt[i];
  if (y != nullptr) {
    if (y_f32) store_row_f32<V>((float*)y + (long)row * ldy, lane, v);
    else store_row_bf16<V>((bf16_t*)y + (long)row * ldy, lane, v);
  }
  if constexpr (V % 4 == 0)
    if (qo) store_row_fp8<V>(qo + (long)row * ldq, q_scale, q_rows, row, lane, v);
  if (lane == 0 && mean_out) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * gamma; total = dres + dx.
// XT: x's element type; GT: the residual gradient's (dres in, dx out): float, or _Float16 (the
// half residual stream's gradient, scaled by a power of two upstream)
template <int V, typename XT = float, typename GT = float>
__global__ void __launch_bounds__(256)
ln_bwd_kernel(int rows, const void* __restrict__ dy, int dy_f32, long ldy,
              const XT* __restrict__ x, long ldx, const float* __restrict__ mean,
              const float* __restrict__ rstd, const float* __restrict__ gamma,
              const GT* __restrict__ dres, GT* __restrict__ dx, bf16_t* __restrict__ dxb,
              long ldo, const int* __restrict__ row_idx, uint8_t* __restrict__ qo, long ldq,
              uint8_t* __restrict__ q_scale, long q_rows) {
  constexpr int D = V * 64;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const long xr = row_idx ? (long)row_idx[row] : (long)row;
  float g[V], xv[V], gm[V];
  if (dy_f32) load_row_f32<V>((const float*)dy + (long)row * ldy, lane, g);
  else load_row_bf16<V>((const bf16_t*)dy + (long)row * ldy, lane, g);
  // the forward's saved input, read once: nontemporal (step +0.5 %, profiles/r02/epilogue_knockout.txt)
  load_row_x<V, XT>(x + xr * ldx, lane, xv, true);
  load_row_f32<V>(gamma, lane, gm);
  // the residual gradient too, before the reductions (it was a second exposed round trip)
  float r[V];
  if (dres) load_row_x<V, GT>(dres + xr * ldo, lane, r);
  const float mu = mean[row], rs = rstd[row];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    xv[i] = (xv[i] - mu) * rs;
    g[i] *= gm[i];
    s1 += g[i];
    s2 += g[i] * xv[i];
  }
  s1 = wave_sum(s1) * (1.0f / D);
  s2 = wave_sum(s2) * (1.0f / D);
  float out[V];
#pragma unroll
  for (int i = 0; i < V; ++i) out[i] = rs * (g[i] - s1 - xv[i] * s2);
  if (dres) {
#pragma unroll
    for (int i = 0; i < V; ++i) out[i] += r[i];
  }
  if constexpr (sizeof(GT) == 2) {
#pragma unroll
    for (int i = 0; i < V; ++i) out[i] = xround<GT>(out[i]);  // the bf16 copy of the stored value
  }
  store_row_x<V, GT>(dx + xr * ldo, lane, out);
  if (dxb) store_row_bf16<V>(dxb + xr * ldo, lane, out);
  // the bf16 result also as the next fp8 GEMM's operand (the codes of dxb + quant_fp8)
  if constexpr (V % 4 == 0)
    if (qo) store_row_fp8<V>(qo + xr * ldq, q_scale, q_rows, xr, lane, out);
}

// im2col for conv1 (k = s = P): out[(n*g*g + py*g + px)][c*P*P + ky*P + kx] = img[n][c][py*P+ky][px*P+kx]
__global__ void patchify_kernel(int n_img, int res, int P, const float* __restrict__ img,
                                bf16_t* __restrict__ out) {
  const int g = res / P;
  const int cols = 3 * P * P;
  const long total8 = (long)n_img * g * g * cols / 8;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total8;
       e += (long)gridDim.x * blockDim.x) {
    const long flat = e * 8;
    const long row = flat / cols;
    const int col = (int)(flat % cols);
    const int n = (int)(row / (g * g)), pp = (int)(row % (g * g));
    const int py = pp / g, px = pp % g;
    const int c = col / (P * P), rem = col % (P * P), ky = rem / P, kx = rem % P;
    const float* src = img + (((long)n * 3 + c) * res + (py * P + ky)) * res + px * P + kx;
    const float4 a = *reinterpret_cast<const float4*>(src);
    const float4 b = *reinterpret_cast<const float4*>(src + 4);
    *reinterpret_cast<uint4*>(out + flat) =
        uint4{pack2bf(a.x, a.y), pack2bf(a.z, a.w), pack2bf(b.x, b.y), pack2bf(b.z, b.w)};
  }
}

// x[n][0] = cls + pos[0]; x[n][1+p] = patch[n*np + p] + pos[1+p]   (model.py:759-764)
__global__ void vit_assemble_kernel(int n_img, int np, int D, const float* __restrict__ patch,
                                    const float* __restrict__ cls, const float* __restrict__ pos,
                                    float* __restrict__ x) {
  const int L = np + 1;
  const long total4 = (long)n_img * L * D / 4;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total4;
       e += (long)gridDim.x * blockDim.x) {
    const long flat = e * 4;
    const long row = flat / D;
    const int col = (int)(flat % D);
    const int n = (int)(row / L), t = (int)(row % L);
    float4 v = t == 0 ? *reinterpret_cast<const float4*>(cls + col)
                      : *reinterpret_cast<const float4*>(patch + ((long)n * np + t - 1) * D + col);
    const float4 p = *reinterpret_cast<const float4*>(pos + (long)t * D + col);
    *reinterpret_cast<float4*>(x + flat) = make_float4(v.x + p.x, v.y + p.y, v.z + p.z, v.w + p.w);
  }
}

// conv1 output -> CLS / positional embedding -> ln_pre -> the first block's ln_1, one wave per
// sequence row and every value of the row in registers (model.py:759-766, 194-200): x0 (f32,
// the residual stream) and ln_1(x0) (bf16, the QKV GEMM operand) with ln_1's statistics. The
// separate path writes and re-reads the assembled rows and x0 (vit_assemble, ln_pre, ln_1:
// ≈ 465 MB more HBM traffic at batch 256). Both LayerNorms two-pass, as ln_fwd_kernel.
template <int V, typename XT = float>
__global__ void __launch_bounds__(256)
vit_embed_ln_kernel(int rows, int np, const float* __restrict__ patch,
                    const float* __restrict__ cls, const float* __restrict__ pos,
                    const float* __restrict__ g_pre, const float* __restrict__ b_pre,
                    XT* __restrict__ x0, const float* __restrict__ g1,
                    const float* __restrict__ b1, bf16_t* __restrict__ y,
                    float* __restrict__ mean1, float* __restrict__ rstd1) {
  constexpr int D = V * 64;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int L = np + 1, n = row / L, t = row % L;
  float v[V], p[V], ga[V], be[V];
  if (t == 0) load_row_f32<V>(cls, lane, v);  // wave-uniform
  else load_row_f32<V>(patch + ((long)n * np + t - 1) * D, lane, v);
  load_row_f32<V>(pos + (long)t * D, lane, p);
  load_row_f32<V>(g_pre, lane, ga);
  load_row_f32<V>(b_pre, lane, be);
  auto norm = [&](float (&u)[V], float& mean, float& rstd) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < V; ++i) s += u[i];
    mean = wave_sum(s) * (1.0f / D);
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      u[i] -= mean;
      q += u[i] * u[i];
    }
    rstd = rsqrtf(wave_sum(q) * (1.0f / D) + 1e-5f);
  };
  float m0, r0, m1, r1;
#pragma unroll
  for (int i = 0; i < V; ++i) v[i] += p[i];
  norm(v, m0, r0);
#pragma unroll
  for (int i = 0; i < V; ++i) v[i] = xround<XT>(v[i] * r0 * ga[i] + be[i]);  // ln_1 reads x0 as stored
  store_row_x<V, XT>(x0 + (long)row * D, lane, v);
  load_row_f32<V>(g1, lane, ga);
  load_row_f32<V>(b1, lane, be);
  norm(v, m1, r1);
#pragma unroll
  for (int i = 0; i < V; ++i) v[i] = v[i] * r1 * ga[i] + be[i];
  store_row_bf16<V>(y + (long)row * D, lane, v);
  if (lane == 0) {
    mean1[row] = m1;
    rstd1[row] = r1;
  }
}

// x[c][t] = tok_emb[tokens[c][t]] + pos[t]   (model.py:943-946)
__global__ void text_embed_kernel(int C, int L, int D, const int64_t* __restrict__ tokens,
                                  const float* __restrict__ emb, const float* __restrict__ pos,
                                  float* __restrict__ x) {
  const long total4 = (long)C * L * D / 4;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total4;
       e += (long)gridDim.x * blockDim.x) {
    const long flat = e * 4;
    const long row = flat / D;
    const int col = (int)(flat % D);
    const int t = (int)(row % L);
    const long tok = tokens[row];
    const float4 a = *reinterpret_cast<const float4*>(emb + tok * D + col);
    const float4 p = *reinterpret_cast<const float4*>(pos + (long)t * D + col);
    *reinterpret_cast<float4*>(x + flat) = make_float4(a.x + p.x, a.y + p.y, a.z + p.z, a.w + p.w);
  }
}

// row_idx[c] = c*L + argmax_t tokens[c][t]  (first maximum, as torch.argmax)
__global__ void eot_rows_kernel(int C, int L, const int64_t* __restrict__ tokens,
                                int* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  int best = 0;
  int64_t bv = tokens[(long)c * L];
  for (int t = 1; t < L; ++t) {
    int64_t v = tokens[(long)c * L + t];
    if (v > bv) { bv = v; best = t; }
  }
  out[c] = c * L + best;
}

int grid_for(long work, int block) {
  long g = (work + block - 1) / block;
  if (g > 8192) g = 8192;
  return (int)(g < 1 ? 1 : g);
}

// x16: x (the forward's LayerNorm input, the residual stream) is IEEE half
int ln_bwd(hipStream_t st, int rows, int D, const void* dy, int dy_f32, long ldy, const void* x,
           long ldx, const float* mean, const float* rstd, const float* gamma, const void* dres,
           void* dx, void* dx_bf16, long ldo, const int* row_idx, void* q, long ldq,
           void* q_scale, long q_rows, int x16 = 0, int g16 = 0) {
  LC_CHECK_ARG(rows >= 0 && D % 64 == 0 && D >= 64 && D <= 1024);
  if (rows == 0) return LC_OK;
  dim3 grid((rows + 3) / 4), block(256);
  switch (D / 64) {
#define LC_LN_B(V)                                                                              \
  case V:                                                                                      \
    if (g16)                                                                                   \
      hipLaunchKernelGGL((ln_bwd_kernel<V, _Float16, _Float16>), grid, block, 0, st, rows, dy, \
                         dy_f32, ldy, (const _Float16*)x, ldx, mean, rstd, gamma,              \
                         (const _Float16*)dres, (_Float16*)dx, (bf16_t*)dx_bf16, ldo, row_idx,  \
                         (uint8_t*)q, ldq, (uint8_t*)q_scale, q_rows);                          \
    else if (x16)                                                                              \
      hipLaunchKernelGGL((ln_bwd_kernel<V, _Float16>), grid, block, 0, st, rows, dy, dy_f32,   \
                         ldy, (const _Float16*)x, ldx, mean, rstd, gamma, (const float*)dres,  \
                         (float*)dx, (bf16_t*)dx_bf16, ldo, row_idx, (uint8_t*)q, ldq,          \
                         (uint8_t*)q_scale, q_rows);                                            \
    else                                                                                       \
      hipLaunchKernelGGL(ln_bwd_kernel<V>, grid, block, 0, st, rows, dy, dy_f32, ldy,          \
                         (const float*)x, ldx, mean, rstd, gamma, (const float*)dres,          \
                         (float*)dx, (bf16_t*)dx_bf16, ldo, row_idx, (uint8_t*)q, ldq,          \
                         (uint8_t*)q_scale, q_rows);                                            \
    break;
    LC_LN_B(1) LC_LN_B(2) LC_LN_B(4) LC_LN_B(8) LC_LN_B(12) LC_LN_B(16)
    default:
      return LC_EINVAL;
#undef LC_LN_B
  }
  LC_LAUNCH_RET();
}
}  // namespace

extern "C" {

static int ln_fwd(hipStream_t st, int rows, int D, const void* x, long ldx, const int* row_idx,
                  const float* gamma, const float* beta, void* y, int y_f32, long ldy, float* mean,
                  float* rstd, void* q, long ldq, void* q_scale, long q_rows, int x16 = 0) {
  LC_CHECK_ARG(rows >= 0 && D % 64 == 0 && D >= 64 && D <= 1024);
  if (rows == 0) return LC_OK;
  dim3 grid((rows + 3) / 4), block(256);
  switch (D / 64) {
#define LC_LN_F(V)                                                                               \
  case V:                                                                                       \
    if (x16)                                                                                    \
      hipLaunchKernelGGL((ln_fwd_kernel<V, _Float16>), grid, block, 0, st, rows,                \
                         (const _Float16*)x, ldx, row_idx, gamma, beta, y, y_f32, ldy, mean,     \
                         rstd, (uint8_t*)q, ldq, (uint8_t*)q_scale, q_rows);                     \
    else                                                                                        \
      hipLaunchKernelGGL(ln_fwd_kernel<V>, grid, block, 0, st, rows, (const float*)x, ldx,      \
                         row_idx, gamma, beta, y, y_f32, ldy, mean, rstd, (uint8_t*)q, ldq,      \
                         (uint8_t*)q_scale, q_rows);                                             \
    break;
    LC_LN_F(1) LC_LN_F(2) LC_LN_F(4) LC_LN_F(8) LC_LN_F(12) LC_LN_F(16)
    default:
      return LC_EINVAL;
#undef LC_LN_F
  }
  LC_LAUNCH_RET();
}

int lc_layernorm_fwd(hipStream_t st, int rows, int D, const float* x, long ldx, const int* row_idx,
                     const float* gamma, const float* beta, void* y, int y_f32, long ldy,
                     float* mean, float* rstd) {
  LC_CHECK_ARG(y != nullptr);
  return ln_fwd(st, rows, D, x, ldx, row_idx, gamma, beta, y, y_f32, ldy, mean, rstd, nullptr, 0,
                nullptr, 0);
}

int lc_layernorm_fwd_fp8(hipStream_t st, int rows, int D, const float* x, long ldx,
                         const int* row_idx, const float* gamma, const float* beta, void* y,
                         long ldy, float* mean, float* rstd, void* q, long ldq, void* q_scale,
                         long q_rows) {
  LC_CHECK_ARG(D % 256 == 0 && q != nullptr && q_scale != nullptr && ldq >= D && ldq % 16 == 0 &&
               ((uintptr_t)q & 15) == 0 && q_rows >= (rows + 255) / 256 * 256 && q_rows % 256 == 0);
  return ln_fwd(st, rows, D, x, ldx, row_idx, gamma, beta, y, 0, ldy, mean, rstd, q, ldq, q_scale,
                q_rows);
}


int lc_layernorm_bwd(hipStream_t st, int rows, int D, const void* dy, int dy_f32, long ldy,
                     const float* x, long ldx, const float* mean, const float* rstd,
                     const float* gamma, const float* dres, float* dx, void* dx_bf16, long ldo,
                     const int* row_idx) {
  return ln_bwd(st, rows, D, dy, dy_f32, ldy, x, ldx, mean, rstd, gamma, dres, dx, dx_bf16, ldo,
                row_idx, nullptr, 0, nullptr, 0);
}

#ifndef LC_F16  // the image tower's half residual stream (bf16 storage build only)
int lc_layernorm_fwd_x16(hipStream_t st, int rows, int D, const void* x, long ldx,
                         const int* row_idx, const float* gamma, const float* beta, void* y,
                         int y_f32, long ldy, float* mean, float* rstd) {
  LC_CHECK_ARG(y != nullptr && x != nullptr && ldx % 4 == 0 && ((uintptr_t)x & 7) == 0);
  return ln_fwd(st, rows, D, x, ldx, row_idx, gamma, beta, y, y_f32, ldy, mean, rstd, nullptr, 0,
                nullptr, 0, 1);
}

int lc_layernorm_bwd_x16(hipStream_t st, int rows, int D, const void* dy, int dy_f32, long ldy,
                         const void* x, long ldx, const float* mean, const float* rstd,
                         const float* gamma, const float* dres, float* dx, void* dx_bf16,
                         long ldo, const int* row_idx) {
  LC_CHECK_ARG(x != nullptr && ldx % 4 == 0 && ((uintptr_t)x & 7) == 0);
  return ln_bwd(st, rows, D, dy, dy_f32, ldy, x, ldx, mean, rstd, gamma, dres, dx, dx_bf16, ldo,
                row_idx, nullptr, 0, nullptr, 0, 1);
}

int lc_layernorm_bwd_g16(hipStream_t st, int rows, int D, const void* dy, int dy_f32, long ldy,
                         const void* x, long ldx, const float* mean, const float* rstd,
                         const float* gamma, const void* dres, void* dx, void* dx_bf16, long ldo,
                         const int* row_idx) {
  LC_CHECK_ARG(x != nullptr && ldx % 4 == 0 && ((uintptr_t)x & 7) == 0 && ldo % 4 == 0 &&
               ((uintptr_t)dx & 7) == 0 && ((uintptr_t)dres & 7) == 0);
  return ln_bwd(st, rows, D, dy, dy_f32, ldy, x, ldx, mean, rstd, gamma, dres, dx, dx_bf16, ldo,
                row_idx, nullptr, 0, nullptr, 0, 1, 1);
}

// the prompt towers' (MVP, MaPLe) half residual stream under fp8 GEMMs: x IEEE half
int lc_layernorm_fwd_fp8_x16(hipStream_t st, int rows, int D, const void* x, long ldx,
                             const int* row_idx, const float* gamma, const float* beta, void* y,
                             long ldy, float* mean, float* rstd, void* q, long ldq, void* q_scale,
                             long q_rows) {
  LC_CHECK_ARG(D % 256 == 0 && q != nullptr && q_scale != nullptr && ldq >= D && ldq % 16 == 0 &&
               ((uintptr_t)q & 15) == 0 && q_rows >= (rows + 255) / 256 * 256 && q_rows % 256 == 0);
  LC_CHECK_ARG(x != nullptr && ldx % 4 == 0 && ((uintptr_t)x & 7) == 0);
  return ln_fwd(st, rows, D, x, ldx, row_idx, gamma, beta, y, 0, ldy, mean, rstd, q, ldq, q_scale,
                q_rows, 1);
}

int lc_layernorm_bwd_fp8_x16(hipStream_t st, int rows, int D, const void* dy, int dy_f32,
                             long ldy, const void* x, long ldx, const float* mean,
                             const float* rstd, const float* gamma, const float* dres, float* dx,
                             void* dx_bf16, long ldo, const int* row_idx, void* q, long ldq,
                             void* q_scale, long q_rows) {
  LC_CHECK_ARG(D % 256 == 0 && q != nullptr && q_scale != nullptr && ldq >= D && ldq % 16 == 0 &&
               ((uintptr_t)q & 15) == 0 && q_rows % 256 == 0 && row_idx == nullptr &&
               q_rows >= (rows + 255) / 256 * 256);
  LC_CHECK_ARG(x != nullptr && ldx % 4 == 0 && ((uintptr_t)x & 7) == 0);
  return ln_bwd(st, rows, D, dy, dy_f32, ldy, x, ldx, mean, rstd, gamma, dres, dx, dx_bf16, ldo,
                row_idx, q, ldq, q_scale, q_rows, 1);
}
#endif

int lc_layernorm_bwd_fp8(hipStream_t st, int rows, int D, const void* dy, int dy_f32, long ldy,
                         const float* x, long ldx, const float* mean, const float* rstd,
                         const float* gamma, const float* dres, float* dx, void* dx_bf16,
                         long ldo, const int* row_idx, void* q, long ldq, void* q_scale,
                         long q_rows) {
  LC_CHECK_ARG(D % 256 == 0 && q != nullptr && q_scale != nullptr && ldq >= D && ldq % 16 == 0 &&
               ((uintptr_t)q & 15) == 0 && q_rows % 256 == 0 && row_idx == nullptr &&
               q_rows >= (rows + 255) / 256 * 256);
  return ln_bwd(st, rows, D, dy, dy_f32, ldy, x, ldx, mean, rstd, gamma, dres, dx, dx_bf16, ldo,
                row_idx, q, ldq, q_scale, q_rows);
}

int lc_patchify(hipStream_t st, int n_img, int res, int patch, const float* img, void* out) {
  LC_CHECK_ARG(n_img > 0 && patch % 8 == 0 && res % patch == 0);
  const long work = (long)n_img * res * res * 3 / 8;
  hipLaunchKernelGGL(patchify_kernel, dim3(grid_for(work, 256)), dim3(256), 0, st, n_img, res,
                     patch, img, (bf16_t*)out);
  LC_LAUNCH_RET();
}

int lc_vit_assemble(hipStream_t st, int n_img, int n_patch, int D, const float* patch,
                    const float* cls, const float* pos, float* x) {
  LC_CHECK_ARG(n_img > 0 && D % 4 == 0);
  const long work = (long)n_img * (n_patch + 1) * D / 4;
  hipLaunchKernelGGL(vit_assemble_kernel, dim3(grid_for(work, 256)), dim3(256), 0, st, n_img,
                     n_patch, D, patch, cls, pos, x);
  LC_LAUNCH_RET();
}

static int vit_embed_ln(hipStream_t st, int n_img, int n_patch, int D, const float* patch,
                        const float* cls, const float* pos, const float* ln_pre_w,
                        const float* ln_pre_b, void* x0, const float* ln1_w, const float* ln1_b,
                        void* y, float* mean1, float* rstd1, int x16) {
  LC_CHECK_ARG(n_img > 0 && n_patch > 0 && (D == 512 || D == 768 || D == 1024));
  LC_CHECK_ARG(patch && cls && pos && ln_pre_w && ln_pre_b && x0 && ln1_w && ln1_b && y && mean1 &&
               rstd1);
  const long rows = (long)n_img * (n_patch + 1);
  LC_CHECK_ARG(rows < (1L << 31) - 4);
  dim3 grid((unsigned)((rows + 3) / 4)), block(256);
#define LC_VE(V)                                                                                 \
  if (x16)                                                                                       \
    hipLaunchKernelGGL((vit_embed_ln_kernel<V, _Float16>), grid, block, 0, st, (int)rows,        \
                       n_patch, patch, cls, pos, ln_pre_w, ln_pre_b, (_Float16*)x0, ln1_w, ln1_b,  \
                       (bf16_t*)y, mean1, rstd1);                                                \
  else                                                                                           \
    hipLaunchKernelGGL(vit_embed_ln_kernel<V>, grid, block, 0, st, (int)rows, n_patch, patch,     \
                       cls, pos, ln_pre_w, ln_pre_b, (float*)x0, ln1_w, ln1_b, (bf16_t*)y, mean1, \
                       rstd1)
  if (D == 512) LC_VE(8);
  else if (D == 768) LC_VE(12);
  else LC_VE(16);
#undef LC_VE
  LC_LAUNCH_RET();
}

int lc_vit_embed_ln(hipStream_t st, int n_img, int n_patch, int D, const float* patch,
                    const float* cls, const float* pos, const float* ln_pre_w,
                    const float* ln_pre_b, float* x0, const float* ln1_w, const float* ln1_b,
                    void* y, float* mean1, float* rstd1) {
  return vit_embed_ln(st, n_img, n_patch, D, patch, cls, pos, ln_pre_w, ln_pre_b, x0, ln1_w, ln1_b,
                      y, mean1, rstd1, 0);
}

#ifndef LC_F16
int lc_vit_embed_ln_x16(hipStream_t st, int n_img, int n_patch, int D, const float* patch,
                        const float* cls, const float* pos, const float* ln_pre_w,
                        const float* ln_pre_b, void* x0, const float* ln1_w, const float* ln1_b,
                        void* y, float* mean1, float* rstd1) {
  return vit_embed_ln(st, n_img, n_patch, D, patch, cls, pos, ln_pre_w, ln_pre_b, x0, ln1_w, ln1_b,
                      y, mean1, rstd1, 1);
}
#endif

int lc_text_embed(hipStream_t st, int C, int L, int D, const int64_t* tokens, const float* emb,
                  const float* pos, float* x) {
  LC_CHECK_ARG(C > 0 && L > 0 && D % 4 == 0);
  const long work = (long)C * L * D / 4;
  hipLaunchKernelGGL(text_embed_kernel, dim3(grid_for(work, 256)), dim3(256), 0, st, C, L, D,
                     tokens, emb, pos, x);
  LC_LAUNCH_RET();
}

int lc_eot_rows(hipStream_t st, int C, int L, const int64_t* tokens, int* row_idx) {
  LC_CHECK_ARG(C > 0 && L > 0);
  hipLaunchKernelGGL(eot_rows_kernel, dim3((C + 255) / 256), dim3(256), 0, st, C, L, tokens,
                     row_idx);
  LC_LAUNCH_RET();
}

}  // extern "C"
