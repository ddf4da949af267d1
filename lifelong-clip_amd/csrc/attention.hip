// Fused multi-head attention core for CLIP towers (d_head = 64), forward and backward.
// Reference semantics: lora.py:950 (q *= d_h^-0.5), 1043 (S = q k^T), 1047-1051 (additive
// -inf causal mask for the text tower, model.py:926-932), 1063 (softmax), 1068 (O = P v); the
// vanilla/adapter towers use torch's nn.MultiheadAttention, same math (model.py:217,230).
//
// Layout: qkv = [rows = batch*L, 3*D] bf16 (q | k | v, head h at columns h*64), as produced by
// the fused QKV GEMM; O = [rows, D] bf16; lse = [batch*H, L] f32 (log2 domain).
//
// MI355X design: sequence lengths are short (197 image tokens, 77 text tokens), so one
// workgroup owns one (image, head) pair and keeps the WHOLE key range on chip: K and V in LDS,
// the full score row of 32 queries per wave in registers (no online-softmax rescaling). The
// grid is batch*H workgroups (3072 at B=256). Keys are padded to Lp = 32*NQB; padded keys are
// masked to -inf and padded V rows are zero.
//   fwd: S^T = K Q^T (keys on the accumulator rows, queries on lanes), row max / sum across
//        the 4 lane groups, P^T packed to bf16 straight from the accumulators into the
//        B-operand of O^T = V^T P^T; V^T fragments come from ds_read_b64_tr_b16 (hardware
//        transpose) of a row-major V image padded to 160-B rows (conflict-free tr reads).
//   bwd: phase 1 — each wave owns 32 keys, sweeps all queries: S = Q K^T, dP = dO V^T,
//        P = exp2(S*c - lse), dS = P (dP - D); dV^T += dO^T P and dK^T += Q^T dS with P / dS
//        used directly as MFMA B-operands; dS^T is parked in LDS. phase 2 — each wave owns 32
//        queries: dQ^T = K^T dS^T from transposed LDS reads. No atomics, no HBM round trip of
//        S or P.
#include "lc_common.h"

namespace {

constexpr float LOG2E = 1.4426950408889634f;

LC_DEV int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// 16 B fragment from a swizzled [rows][64 bf16] image (128 B rows)
LC_DEV bf16x8 rd_row(const char* base, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(base + row * 128 + swz(row, chunk) * 16);
}
// transposed 4x16 read from the swizzled 128-B-row image; col multiple of 4
LC_DEV bf16x4 tr_swz(const char* base, int row, int col) {
  const int off = row * 128 + swz(row, col >> 3) * 16 + (col & 7) * 2;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) bf16x4*)(base + off));
}
// transposed read from a plain image with a given row stride (bytes)
LC_DEV bf16x4 tr_plain(const char* base, int stride, int row, int col) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) bf16x4*)(base + row * stride + col * 2));
}
LC_DEV bf16x8 cat4(bf16x4 a, bf16x4 b) { return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]}; }
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

LC_DEV uint4 ld16_or_zero(const bf16_t* p, bool ok) {
  return ok ? *reinterpret_cast<const uint4*>(p) : uint4{0, 0, 0, 0};
}

constexpr int V_STRIDE = 160;  // bytes per V row in LDS (conflict-free tr reads)

template <int NQB>
__global__ void __launch_bounds__(64 * NQB)
attn_fwd_kernel(int L, int H, int D, const bf16_t* __restrict__ qkv, long ldq,
                bf16_t* __restrict__ O, long ldo, float* __restrict__ lse, int causal,
                float scale) {
  constexpr int LP = 32 * NQB;
  constexpr int NKT = 2 * NQB;
  constexpr int NTH = 64 * NQB;
  __shared__ __attribute__((aligned(16))) char smem[LP * 128 + LP * V_STRIDE];
  char* Ks = smem;
  char* Vs = smem + LP * 128;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, t = lane & 15;
  const int nh = blockIdx.x, n = nh / H, h = nh % H;
  const long base = (long)n * L;
  const float c = scale * LOG2E;

  for (int idx = tid; idx < LP * 8; idx += NTH) {
    const int r = idx >> 3, ch = idx & 7;
    const bf16_t* src = qkv + (base + r) * ldq + h * 64 + ch * 8;
    const uint4 kv = ld16_or_zero(src + D, r < L);
    const uint4 vv = ld16_or_zero(src + 2 * D, r < L);
    *reinterpret_cast<uint4*>(Ks + r * 128 + swz(r, ch) * 16) = kv;
    *reinterpret_cast<uint4*>(Vs + r * V_STRIDE + ch * 16) = vv;
  }

  // Q fragments (B operand of S^T = K Q^T): Q[q][32s + 8g .. +7]
  const int qb = 32 * w;
  bf16x8 qf[2][2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = qb + qt * 16 + t;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      uint4 u = ld16_or_zero(qkv + (base + q) * ldq + h * 64 + s * 32 + g * 8, q < L);
      qf[qt][s] = *reinterpret_cast<bf16x8*>(&u);
    }
  }
  __syncthreads();

  f32x4 S[NKT][2];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    S[kt][0] = f32x4{0.f, 0.f, 0.f, 0.f};
    S[kt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 kf = rd_row(Ks, kt * 16 + t, s * 4 + g);
      S[kt][0] = mfma16(kf, qf[0][s], S[kt][0]);
      S[kt][1] = mfma16(kf, qf[1][s], S[kt][1]);
    }
  }
  // lane holds S^T[key = kt*16 + 4g + r][q = qb + qt*16 + t]
  float mx[2], sm[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = qb + qt * 16 + t;
    float m = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kt * 16 + 4 * g + r;
        float v = S[kt][qt][r] * c;
        if (key >= L || (causal && key > q)) v = -INFINITY;
        S[kt][qt][r] = v;
        m = fmaxf(m, v);
      }
    m = fmaxf(m, __shfl_xor(m, 16));
    m = fmaxf(m, __shfl_xor(m, 32));
    float l = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = exp2f(S[kt][qt][r] - m);
        S[kt][qt][r] = p;
        l += p;
      }
    l += __shfl_xor(l, 16);
    l += __shfl_xor(l, 32);
    mx[qt] = m;
    sm[qt] = l;
  }

  f32x4 Oa[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) Oa[dt][0] = Oa[dt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NQB; ++s) {
    const bf16x8 pb0 = pack8(S[2 * s][0], S[2 * s + 1][0]);
    const bf16x8 pb1 = pack8(S[2 * s][1], S[2 * s + 1][1]);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int col = dt * 16 + (t & 3) * 4;
      const bf16x4 lo = tr_plain(Vs, V_STRIDE, 32 * s + 4 * g + (t >> 2), col);
      const bf16x4 hi = tr_plain(Vs, V_STRIDE, 32 * s + 16 + 4 * g + (t >> 2), col);
      const bf16x8 vf = cat4(lo, hi);
      Oa[dt][0] = mfma16(vf, pb0, Oa[dt][0]);
      Oa[dt][1] = mfma16(vf, pb1, Oa[dt][1]);
    }
  }
  // lane holds O^T[d = dt*16 + 4g + r][q = qb + qt*16 + t]
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = qb + qt * 16 + t;
    if (q < L) {
      const float inv = 1.0f / sm[qt];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const f32x4 o = Oa[dt][qt];
        *reinterpret_cast<uint2*>(O + (base + q) * ldo + h * 64 + dt * 16 + 4 * g) =
            uint2{pack2bf(o[0] * inv, o[1] * inv), pack2bf(o[2] * inv, o[3] * inv)};
      }
      if (g == 0) lse[(long)nh * L + q] = mx[qt] + log2f(sm[qt]);
    }
  }
}

template <int NQB>
struct BwdLds {
  static constexpr int LP = 32 * NQB;
  static constexpr int DST_STRIDE = LP * 2 + 16;  // bytes per dS^T row
  static constexpr int Q_OFF = 0;
  static constexpr int DO_OFF = LP * 128;
  static constexpr int DST_OFF = 2 * LP * 128;
  static constexpr int LSE_OFF = DST_OFF + LP * DST_STRIDE;
  static constexpr int DQ_OFF = LSE_OFF + LP * 4;
  static constexpr int BYTES = DQ_OFF + LP * 4;
};

template <int NQB>
__global__ void __launch_bounds__(64 * NQB)
attn_bwd_kernel(int L, int H, int D, const bf16_t* __restrict__ qkv, long ldq,
                const bf16_t* __restrict__ O, const bf16_t* __restrict__ dO, long ldo,
                const float* __restrict__ lse, bf16_t* __restrict__ dqkv, long lddq, int causal,
                float scale) {
  using Lay = BwdLds<NQB>;
  constexpr int LP = Lay::LP;
  constexpr int NTH = 64 * NQB;
  __shared__ __attribute__((aligned(16))) char smem[Lay::BYTES];
  char* Qs = smem + Lay::Q_OFF;
  char* dOs = smem + Lay::DO_OFF;
  char* dSTs = smem + Lay::DST_OFF;
  float* lse_s = reinterpret_cast<float*>(smem + Lay::LSE_OFF);
  float* dq_s = reinterpret_cast<float*>(smem + Lay::DQ_OFF);

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, t = lane & 15;
  const int nh = blockIdx.x, n = nh / H, h = nh % H;
  const long base = (long)n * L;
  const float c = scale * LOG2E;

  for (int idx = tid; idx < LP * 8; idx += NTH) {
    const int r = idx >> 3, ch = idx & 7;
    const uint4 qv = ld16_or_zero(qkv + (base + r) * ldq + h * 64 + ch * 8, r < L);
    const uint4 dv = ld16_or_zero(dO + (base + r) * ldo + h * 64 + ch * 8, r < L);
    *reinterpret_cast<uint4*>(Qs + r * 128 + swz(r, ch) * 16) = qv;
    *reinterpret_cast<uint4*>(dOs + r * 128 + swz(r, ch) * 16) = dv;
  }
  for (int q = tid; q < LP; q += NTH) {
    float dsum = 0.f, lv = 1e30f;
    if (q < L) {
      const bf16_t* po = O + (base + q) * ldo + h * 64;
      const bf16_t* pd = dO + (base + q) * ldo + h * 64;
#pragma unroll
      for (int ch = 0; ch < 8; ++ch) {
        const uint4 a = *reinterpret_cast<const uint4*>(po + ch * 8);
        const uint4 b = *reinterpret_cast<const uint4*>(pd + ch * 8);
        const uint32_t aa[4] = {a.x, a.y, a.z, a.w}, bb[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
          dsum += bf2f(aa[k] & 0xffff) * bf2f(bb[k] & 0xffff) + bf2f(aa[k] >> 16) * bf2f(bb[k] >> 16);
      }
      lv = lse[(long)nh * L + q];
    }
    dq_s[q] = dsum;
    lse_s[q] = lv;
  }

  // own key block: K / V rows kb + kt2*16 + t, as B-operand fragments
  const int kb = 32 * w;
  bf16x8 kf[2][2], vf[2][2];
#pragma unroll
  for (int kt2 = 0; kt2 < 2; ++kt2) {
    const int key = kb + kt2 * 16 + t;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16_t* src = qkv + (base + key) * ldq + h * 64 + s * 32 + g * 8;
      uint4 ku = ld16_or_zero(src + D, key < L), vu = ld16_or_zero(src + 2 * D, key < L);
      kf[kt2][s] = *reinterpret_cast<bf16x8*>(&ku);
      vf[kt2][s] = *reinterpret_cast<bf16x8*>(&vu);
    }
  }
  __syncthreads();

  f32x4 dV[4][2], dK[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) dV[dt][k2] = dK[dt][k2] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int qc = 0; qc < NQB; ++qc) {
    f32x4 S[2][2], dP[2][2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) S[qt][k2] = dP[qt][k2] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int row = qc * 32 + qt * 16 + t;
        const bf16x8 qa = rd_row(Qs, row, s * 4 + g);
        const bf16x8 da = rd_row(dOs, row, s * 4 + g);
#pragma unroll
        for (int k2 = 0; k2 < 2; ++k2) {
          S[qt][k2] = mfma16(qa, kf[k2][s], S[qt][k2]);
          dP[qt][k2] = mfma16(da, vf[k2][s], dP[qt][k2]);
        }
      }
    }
    // lane holds X[q = qc*32 + qt*16 + 4g + r][key = kb + k2*16 + t]
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = qc * 32 + qt * 16 + 4 * g + r;
          const int key = kb + k2 * 16 + t;
          float p = exp2f(S[qt][k2][r] * c - lse_s[q]);
          if (key >= L || (causal && key > q)) p = 0.f;
          S[qt][k2][r] = p;
          dP[qt][k2][r] = p * (dP[qt][k2][r] - dq_s[q]);
        }
    // B operands (k = 32 queries of this chunk): slot j<4 -> q = 4g+j, j>=4 -> 16+4g+(j-4)
    bf16x8 pB[2], sB[2];
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      pB[k2] = pack8(S[0][k2], S[1][k2]);
      sB[k2] = pack8(dP[0][k2], dP[1][k2]);
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int col = dt * 16 + (t & 3) * 4;
      const int r0 = qc * 32 + 4 * g + (t >> 2);
      const bf16x8 doT = cat4(tr_swz(dOs, r0, col), tr_swz(dOs, r0 + 16, col));
      const bf16x8 qT = cat4(tr_swz(Qs, r0, col), tr_swz(Qs, r0 + 16, col));
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        dV[dt][k2] = mfma16(doT, pB[k2], dV[dt][k2]);
        dK[dt][k2] = mfma16(qT, sB[k2], dK[dt][k2]);
      }
    }
    // park dS^T[key][q]: 4 consecutive q per lane -> one 8-B LDS store
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        const int key = kb + k2 * 16 + t;
        const int q0 = qc * 32 + qt * 16 + 4 * g;
        const f32x4 v = dP[qt][k2];
        *reinterpret_cast<uint2*>(dSTs + key * Lay::DST_STRIDE + q0 * 2) =
            uint2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
      }
  }
  // dK, dV of the own key block: lane holds X^T[d = dt*16 + 4g + r][key = kb + k2*16 + t]
#pragma unroll
  for (int k2 = 0; k2 < 2; ++k2) {
    const int key = kb + k2 * 16 + t;
    if (key < L) {
      bf16_t* dst = dqkv + (base + key) * lddq + h * 64;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const f32x4 a = dK[dt][k2], b = dV[dt][k2];
        *reinterpret_cast<uint2*>(dst + D + dt * 16 + 4 * g) =
            uint2{pack2bf(a[0] * scale, a[1] * scale), pack2bf(a[2] * scale, a[3] * scale)};
        *reinterpret_cast<uint2*>(dst + 2 * D + dt * 16 + 4 * g) =
            uint2{pack2bf(b[0], b[1]), pack2bf(b[2], b[3])};
      }
    }
  }
  __syncthreads();  // every wave is done with Qs -> reuse it for K
  char* Ks = Qs;
#pragma unroll
  for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int key = kb + kt2 * 16 + t;
      *reinterpret_cast<bf16x8*>(Ks + key * 128 + swz(key, s * 4 + g) * 16) = kf[kt2][s];
    }
  __syncthreads();

  // phase 2: dQ^T[d][q] = sum_key K^T[d][key] dS^T[key][q] for queries qb..qb+31
  const int qb = 32 * w;
  f32x4 dQ[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dQ[dt][0] = dQ[dt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < NQB; ++s) {
    const int r0 = s * 32 + 8 * g + (t >> 2);
    bf16x8 bq[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int col = qb + qt * 16 + (t & 3) * 4;
      bq[qt] = cat4(tr_plain(dSTs, Lay::DST_STRIDE, r0, col), tr_plain(dSTs, Lay::DST_STRIDE, r0 + 4, col));
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int col = dt * 16 + (t & 3) * 4;
      const bf16x8 ka = cat4(tr_swz(Ks, r0, col), tr_swz(Ks, r0 + 4, col));
      dQ[dt][0] = mfma16(ka, bq[0], dQ[dt][0]);
      dQ[dt][1] = mfma16(ka, bq[1], dQ[dt][1]);
    }
  }
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = qb + qt * 16 + t;
    if (q < L) {
      bf16_t* dst = dqkv + (base + q) * lddq + h * 64;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const f32x4 a = dQ[dt][qt];
        *reinterpret_cast<uint2*>(dst + dt * 16 + 4 * g) =
            uint2{pack2bf(a[0] * scale, a[1] * scale), pack2bf(a[2] * scale, a[3] * scale)};
      }
    }
  }
}

}  // namespace

extern "C" {

int lc_attn_fwd(hipStream_t st, int n_seq, int L, int H, const void* qkv, long ldq, void* O,
                long ldo, float* lse, int causal) {
  LC_CHECK_ARG(n_seq > 0 && L > 0 && L <= 256 && H > 0 && ldq >= 3 * H * 64 && ldo >= H * 64);
  LC_CHECK_ARG(ldq % 8 == 0 && ldo % 8 == 0);
  const int D = H * 64;
  const int nqb = (L + 31) / 32;
  dim3 grid(n_seq * H);
  const float scale = 0.125f;  // 64^-0.5
  switch (nqb) {
#define LC_AF(Q)                                                                                \
  case Q:                                                                                      \
    hipLaunchKernelGGL(attn_fwd_kernel<Q>, grid, dim3(64 * Q), 0, st, L, H, D,                 \
                       (const bf16_t*)qkv, ldq, (bf16_t*)O, ldo, lse, causal, scale);          \
    break;
    LC_AF(1) LC_AF(2) LC_AF(3) LC_AF(4) LC_AF(5) LC_AF(6) LC_AF(7) LC_AF(8)
#undef LC_AF
    default:
      return LC_EINVAL;
  }
  LC_LAUNCH_RET();
}

int lc_attn_bwd(hipStream_t st, int n_seq, int L, int H, const void* qkv, long ldq, const void* O,
                const void* dO, long ldo, const float* lse, void* dqkv, long lddq, int causal) {
  LC_CHECK_ARG(n_seq > 0 && L > 0 && L <= 224 && H > 0 && ldq >= 3 * H * 64 && ldo >= H * 64);
  LC_CHECK_ARG(lddq >= 3 * H * 64 && ldq % 8 == 0 && ldo % 8 == 0 && lddq % 8 == 0);
  const int D = H * 64;
  const int nqb = (L + 31) / 32;
  dim3 grid(n_seq * H);
  const float scale = 0.125f;
  switch (nqb) {
#define LC_AB(Q)                                                                                \
  case Q:                                                                                      \
    hipLaunchKernelGGL(attn_bwd_kernel<Q>, grid, dim3(64 * Q), 0, st, L, H, D,                 \
                       (const bf16_t*)qkv, ldq, (const bf16_t*)O, (const bf16_t*)dO, ldo, lse, \
                       (bf16_t*)dqkv, lddq, causal, scale);                                    \
    break;
    LC_AB(1) LC_AB(2) LC_AB(3) LC_AB(4) LC_AB(5) LC_AB(6) LC_AB(7)
#undef LC_AB
    default:
      return LC_EINVAL;
  }
  LC_LAUNCH_RET();
}

}  // extern "C"
