// Fused multi-head attention core for CLIP towers (d_head = 64), forward and backward.
// Reference semantics: lora.py:950 (q *= d_h^-0.5), 1043 (S = q k^T), 1047-1051 (additive
// -inf causal mask for the text tower, model.py:926-932), 1063 (softmax), 1068 (O = P v); the
// vanilla/adapter towers use torch's nn.MultiheadAttention, same math (model.py:217,230).
//
// Layout: qkv = [rows = batch*L, 3*D] bf16 (q | k | v, head h at columns h*64), as produced by
// the fused QKV GEMM; O = [rows, D] bf16; lse = [batch*H, L] f32 (log2 domain).
//
// MI355X design. Sequences are short (197 image tokens, 77 text tokens): one workgroup owns one
// (sequence, head) pair with the WHOLE key range on chip, one wave per 32 rows (queries or keys),
// keys padded to Lp = 32*NQB (padded keys masked, padded rows zero). At d_head = 64 the
// per-score work is dominated by VALU (scale, max, exp, sum, pack), not MFMA, so the kernels are
// laid out to minimise VALU issue:
//   * LDS images use a row swizzle that is invariant under 16-row steps, so every lane's LDS
//     offsets are computed once; loop steps only add wave-uniform row-block offsets;
//   * masking (padded keys, causal) runs only on the wave-uniform edge blocks, and causal blocks
//     entirely above the diagonal are skipped;
//   * fwd: EXACT softmax in two passes — pass 1 recomputes S^T = K Q^T only for the row max
//     (MFMA is the idle pipe here), pass 2 forms p = exp2(S*c - m*c) with one FMA, packs P^T to
//     bf16 straight from the accumulators into the B operand of O^T = V^T P^T (V^T via
//     ds_read_b64_tr_b16); no online rescaling;
//   * bwd, key-major kernel (dK, dV): each wave keeps its 32 keys' K / V fragments and dK^T, dV^T
//     accumulators in registers and sweeps the queries: S = Q K^T, dP = dO V^T with -D preloaded
//     as the dP accumulator, dS = P * dP, dV^T += dO^T P, dK^T += Q^T dS;
//   * bwd, query-major kernel (dQ): each wave keeps its 32 queries' Q / dO fragments, recomputes
//     S^T, dP^T from K / V in LDS and accumulates dQ^T = K^T dS^T; it walks the heads in reverse
//     order so its reads hit what the key-major kernel left in L2 / the Infinity Cache.
#include "lc_common.h"

namespace {

constexpr float LOG2E = 1.4426950408889634f;

// raw v_exp_f32: arguments are <= 0 here, exp2(-inf) = 0, denormal results flush to 0
LC_DEV float ex2(float x) { return __builtin_amdgcn_exp2f(x); }
// padded key or (text tower) future key; bitwise ops keep it a select, not a branch
LC_DEV bool masked(int key, int q, int L, int causal) {
  return (key >= L) | ((causal != 0) & (key > q));
}

// 128-B-row images: 16-B chunk c of row r lives at chunk c ^ m(r), m(r) = x ^ ((x << 1) & 7) with
// x = (r >> 1) & 7: conflict-free both for row reads (ds_read_b128: lane t reads row t) and for the
// transposed reads (ds_read_b64_tr_b16: 8 rows x 32 B per 32 lanes; the plain x ^ chunk mask put
// rows r and r + 2 on the same banks there, 2-way) — checked exhaustively for every lane group.
// Period 16 rows, so lane offsets stay valid for any 16-row-aligned block.
LC_DEV int swz_mask(int row) {
  const int x = (row >> 1) & 7;
  return x ^ ((x << 1) & 7);
}
LC_DEV int swz(int row, int chunk) { return chunk ^ swz_mask(row); }

LC_DEV bf16x8 lds16(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }
LC_DEV bf16x4 lds_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) bf16x4*)(p));
}
LC_DEV bf16x8 cat4(bf16x4 a, bf16x4 b) { return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]}; }

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
LC_DEV bf16x8 as_bf8(u32x4 v) { return __builtin_bit_cast(bf16x8, v); }
LC_DEV bf16x8 pack8(const f32x4& a, const f32x4& b) {
  return as_bf8(u32x4{pack2bf(a[0], a[1]), pack2bf(a[2], a[3]), pack2bf(b[0], b[1]), pack2bf(b[2], b[3])});
}

// q / k / v, O and dO rows are read once per (sequence, head): nontemporal (step +0.4 %,
// profiles/r02/epilogue_knockout.txt)
LC_DEV uint4 ld16_or_zero(const bf16_t* p, bool ok) {
  if (!ok) return uint4{0, 0, 0, 0};
  const i32x4 v = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(p));
  return make_uint4(v[0], v[1], v[2], v[3]);
}

// Raw-buffer descriptor over `rows` rows of `row_bytes` from row row0 of p (wave-uniform): loads
// past the range read zero and stores there are dropped by the range check, so no branch
// surrounds a memory op and hipcc counts vmcnt across them (a load under a branch is followed by
// vmcnt(0): the loads issued before it stop being in flight together).
LC_DEV __amdgpu_buffer_rsrc_t seq_rsrc(const void* p, long row0, long row_bytes, int rows) {
  const uint64_t a = (uint64_t)(static_cast<const char*>(p) + row0 * row_bytes);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int nb = __builtin_amdgcn_readfirstlane((int)(rows * row_bytes));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, nb, 0x00020000);
}
LC_DEV uint4 seq_ld16(__amdgpu_buffer_rsrc_t r, int off) {  // nontemporal (read once)
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 2);
  return make_uint4(v[0], v[1], v[2], v[3]);
}

// Lane offsets (bytes) into a swizzled 128-B-row image, valid for any row block that starts at a
// multiple of 16 rows:
//   row_off(t, g, s): A/B-operand read of row t (+block), k-chunk s*4+g  (16 B)
//   tr_off(t, g, dt): transposed read of rows 4g + (t>>2) (+16 for the upper half), columns
//                     dt*16 + (t&3)*4 .. +3 — the V^T / K^T / Q^T / dO^T fragment layout whose
//                     k order matches a bf16x8 packed from two 16-row accumulator tiles.
LC_DEV int row_off(int t, int g, int s) { return t * 128 + swz(t, s * 4 + g) * 16; }
LC_DEV int tr_off(int t, int g, int dt) {
  const int row = 4 * g + (t >> 2);
  const int col = dt * 16 + (t & 3) * 4;
  return row * 128 + swz(row, col >> 3) * 16 + (col & 7) * 2;
}

// One output row's 64 head columns from the 4 lanes t + 16g that share it (lane g: packed bf16 of
// columns dt*16 + 4g .. +3 in x[dt]) as two 16-B stores per lane instead of four 8-B ones: one
// v_permlane16_swap per dword exchanges lane groups 1 <-> 0 and 3 <-> 2 between the column-tile
// pairs (0, 1) and (2, 3), after which group g holds columns 32p + 16(g & 1) + 8(g >> 1) .. +7
// of pair p (the epilogue store tail is issue-bound: half the store instructions, same bytes).
// All four lanes of the row must be active (row guards are uniform over them).
LC_DEV void store_row64(bf16_t* row, int g, const uint2 (&x)[4]) {
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const auto s0 = __builtin_amdgcn_permlane16_swap(x[2 * p].x, x[2 * p + 1].x, false, false);
    const auto s1 = __builtin_amdgcn_permlane16_swap(x[2 * p].y, x[2 * p + 1].y, false, false);
    *reinterpret_cast<uint4*>(row + 32 * p + 16 * (g & 1) + 8 * (g >> 1)) =
        uint4{s0[0], s1[0], s0[1], s1[1]};
  }
}

constexpr int V_STRIDE = 160;  // bytes per V row in the forward's plain V image (conflict-free tr)

// ----------------------------------------------------------------------------------- forward
// ONLINE (default): one pass over the keys with a running row max — the O accumulators and row
// sums rescaled by exp2((m_old - m_new) c) per 32-key block — instead of the exact two-pass form
// (a first pass of S = K Q^T for the max alone): a third fewer MFMAs and K reads, image forward
// 103.4 -> 94.8 us standalone (profiles/r03/s2/u_ab_attn_online.txt). LCCLIP_ATTN_FWD_ONLINE=0
// selects the two-pass form (A/Bs).
template <int NQB, bool ONLINE = true>
__global__ void __launch_bounds__(64 * NQB, 4)
attn_fwd_kernel(int L, int H, int D, const bf16_t* __restrict__ qkv, long ldq,
                bf16_t* __restrict__ O, long ldo, float* __restrict__ lse, int causal,
                float scale) {
  constexpr int LP = 32 * NQB;
  constexpr int NTH = 64 * NQB;
  __shared__ __attribute__((aligned(16))) char smem[LP * 128 + LP * V_STRIDE];
  char* Ks = smem;
  char* Vs = smem + LP * 128;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, t = lane & 15;
  const int nh = blockIdx.x, n = nh / H, h = nh % H;
  const long base = (long)n * L;
  const float c = scale * LOG2E;

  // staging: every lane issues all its 16-B loads (through the sequence's descriptor: rows >= L
  // read zero) before its first LDS write
  constexpr int IT = LP * 8 / NTH;  // = 4
  const int ch = tid & 7;
  const auto rq = seq_rsrc(qkv, base, ldq * 2, L);
  uint4 kv[IT], vv[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int r = (tid + i * NTH) >> 3;
    const int off = r * (int)ldq * 2 + (h * 64 + ch * 8) * 2;
    kv[i] = seq_ld16(rq, off + D * 2);
    vv[i] = seq_ld16(rq, off + D * 4);
  }
  const int qb = 32 * w;
  bf16x8 qf[2][2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = qb + qt * 16 + t;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      uint4 u = seq_ld16(rq, q * (int)ldq * 2 + (h * 64 + s * 32 + g * 8) * 2);
      qf[qt][s] = *reinterpret_cast<bf16x8*>(&u);
    }
  }
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int r = (tid + i * NTH) >> 3;
    *reinterpret_cast<uint4*>(Ks + r * 128 + swz(r, ch) * 16) = kv[i];
    *reinterpret_cast<uint4*>(Vs + r * V_STRIDE + ch * 16) = vv[i];
  }
  __syncthreads();

  const char* k0 = Ks + row_off(t, g, 0);
  const char* k1 = Ks + row_off(t, g, 1);
  const char* vt = Vs + (4 * g + (t >> 2)) * V_STRIDE + (t & 3) * 8;
  // key steps holding a key <= the wave's last query (causal) / < L
  const int s_end = causal ? min(NQB, (qb + 31) / 32 + 1) : NQB;

  // S^T tile pair of key step s: lane holds S^T[key = 32s + 16kk + 4g + r][q = qb + 16qt + t]
  auto scores = [&](int s, f32x4 (&S)[2][2]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ro = (32 * s + 16 * kk) * 128;
      const bf16x8 ka = lds16(k0 + ro), kb = lds16(k1 + ro);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        S[kk][qt] = mfma16(ka, qf[qt][0], f32x4{0.f, 0.f, 0.f, 0.f});
        S[kk][qt] = mfma16(kb, qf[qt][1], S[kk][qt]);
      }
    }
    if (32 * s + 32 > L || (causal && 32 * s + 31 > qb)) {  // wave-uniform edge block
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            S[kk][qt][r] = masked(32 * s + 16 * kk + 4 * g + r, qb + 16 * qt + t, L, causal)
                               ? -INFINITY : S[kk][qt][r];
    }
  };

  // pass 1: exact row max of the raw scores
  float mx[2] = {-INFINITY, -INFINITY};
#pragma unroll 1
  for (int s = 0; s < (ONLINE ? 0 : s_end); ++s) {
    f32x4 S[2][2];
    scores(s, S);
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      float m = mx[qt];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        m = fmaxf(fmaxf(m, fmaxf(S[kk][qt][0], S[kk][qt][1])), fmaxf(S[kk][qt][2], S[kk][qt][3]));
      mx[qt] = m;
    }
  }
  float nm[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    float m = mx[qt];
    m = fmaxf(m, __shfl_xor(m, 16));
    m = fmaxf(m, __shfl_xor(m, 32));
    mx[qt] = m * c;
    nm[qt] = -m * c;
  }

  // pass 2: P = exp2(S*c - m*c), row sums, O^T += V^T P^T
  float sm[2] = {0.f, 0.f};
  f32x4 Oa[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) Oa[dt][0] = Oa[dt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mr[2] = {-INFINITY, -INFINITY};  // ONLINE: running raw-score max per query
#pragma unroll 1
  for (int s = 0; s < s_end; ++s) {
    f32x4 S[2][2];
    scores(s, S);
    if constexpr (ONLINE) {
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        float m = fmaxf(fmaxf(fmaxf(S[0][qt][0], S[0][qt][1]), fmaxf(S[0][qt][2], S[0][qt][3])),
                        fmaxf(fmaxf(S[1][qt][0], S[1][qt][1]), fmaxf(S[1][qt][2], S[1][qt][3])));
        m = fmaxf(m, __shfl_xor(m, 16));
        m = fmaxf(m, __shfl_xor(m, 32));
        const float mn = fmaxf(mr[qt], m);  // finite from block 0 on (key 0 is never masked)
        const float corr = ex2((mr[qt] - mn) * c);
        mr[qt] = mn;
        nm[qt] = -mn * c;
        sm[qt] *= corr;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) Oa[dt][qt] *= corr;
      }
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = ex2(__builtin_fmaf(S[kk][qt][r], c, nm[qt]));
          S[kk][qt][r] = p;
          sm[qt] += p;
        }
    const bf16x8 pb0 = pack8(S[0][0], S[1][0]);
    const bf16x8 pb1 = pack8(S[0][1], S[1][1]);
    const char* vs = vt + 32 * s * V_STRIDE;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x8 vf = cat4(lds_tr(vs + dt * 32), lds_tr(vs + 16 * V_STRIDE + dt * 32));
      Oa[dt][0] = mfma16(vf, pb0, Oa[dt][0]);
      Oa[dt][1] = mfma16(vf, pb1, Oa[dt][1]);
    }
  }
  if constexpr (ONLINE) mx[0] = mr[0] * c, mx[1] = mr[1] * c;
  // lane holds O^T[d = dt*16 + 4g + r][q = qb + qt*16 + t]
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    float l = sm[qt];
    l += __shfl_xor(l, 16);
    l += __shfl_xor(l, 32);
    const int q = qb + qt * 16 + t;
    if (q < L) {
      const float inv = 1.0f / l;
      uint2 x[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const f32x4 o = Oa[dt][qt];
        x[dt] = uint2{pack2bf(o[0] * inv, o[1] * inv), pack2bf(o[2] * inv, o[3] * inv)};
      }
      store_row64(O + (base + q) * ldo + h * 64, g, x);
      if (g == 0) lse[(long)nh * L + q] = mx[qt] + __log2f(l);
    }
  }
}

// ------------------------------------------------------------------ backward, key-major (dK, dV)
template <int NQB>
__global__ void __launch_bounds__(64 * NQB)
attn_bwd_kv_kernel(int L, int H, int D, const bf16_t* __restrict__ qkv, long ldq,
                   const bf16_t* __restrict__ O, const bf16_t* __restrict__ dO, long ldo,
                   const float* __restrict__ lse, bf16_t* __restrict__ dqkv, long lddq, int causal,
                   float scale) {
  constexpr int LP = 32 * NQB;
  constexpr int NTH = 64 * NQB;
  __shared__ __attribute__((aligned(16))) char smem[2 * LP * 128 + 2 * LP * 4];
  char* Qs = smem;
  char* dOs = smem + LP * 128;
  float* nlse_s = reinterpret_cast<float*>(smem + 2 * LP * 128);  // -lse
  float* nd_s = nlse_s + LP;                                       // -D

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, t = lane & 15;
  const int nh = blockIdx.x, n = nh / H, h = nh % H;
  const long base = (long)n * L;
  const float c = scale * LOG2E;

  // staging: all 16-B loads of Q, dO and O issued before the first LDS write; D = rowsum(dO*O)
  // from the same chunks (8 lanes per row, reduced with xor-shuffles)
  constexpr int IT = LP * 8 / NTH;  // = 4
  const int ch = tid & 7;
  uint4 qv[IT], dv[IT], ov[IT];
  float lv[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int r = (tid + i * NTH) >> 3;
    const long off = h * 64 + ch * 8;
    qv[i] = ld16_or_zero(qkv + (base + r) * ldq + off, r < L);
    dv[i] = ld16_or_zero(dO + (base + r) * ldo + off, r < L);
    ov[i] = ld16_or_zero(O + (base + r) * ldo + off, r < L);
    lv[i] = (r < L) ? lse[(long)nh * L + r] : 1e30f;
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
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int r = (tid + i * NTH) >> 3;
    *reinterpret_cast<uint4*>(Qs + r * 128 + swz(r, ch) * 16) = qv[i];
    *reinterpret_cast<uint4*>(dOs + r * 128 + swz(r, ch) * 16) = dv[i];
    const uint32_t aa[4] = {ov[i].x, ov[i].y, ov[i].z, ov[i].w};
    const uint32_t bb[4] = {dv[i].x, dv[i].y, dv[i].z, dv[i].w};
    float dsum = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      dsum += bf2f(aa[k] & 0xffff) * bf2f(bb[k] & 0xffff) + bf2f(aa[k] >> 16) * bf2f(bb[k] >> 16);
    dsum += __shfl_xor(dsum, 1);
    dsum += __shfl_xor(dsum, 2);
    dsum += __shfl_xor(dsum, 4);
    if (ch == 0) {
      nd_s[r] = -dsum;
      nlse_s[r] = r < L ? -lv[i] : -1e30f;
    }
  }
  __syncthreads();

  const int ro0 = row_off(t, g, 0), ro1 = row_off(t, g, 1);
  const int tr0 = tr_off(t, g, 0), tr1 = tr_off(t, g, 1), tr2 = tr_off(t, g, 2), tr3 = tr_off(t, g, 3);
  const int tro[4] = {tr0, tr1, tr2, tr3};

  f32x4 dV[4][2], dK[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) dV[dt][k2] = dK[dt][k2] = f32x4{0.f, 0.f, 0.f, 0.f};

  // causal: queries before the block's first key see none of its keys
  const int qc0 = causal ? w : 0;
#pragma unroll 1
  for (int qc = qc0; qc < NQB; ++qc) {
    const bool edge = (kb + 32 > L) || (causal && kb + 31 > qc * 32);
    // B operands (k = 32 queries of this chunk): slot j<4 -> q = 4g+j, j>=4 -> 16+4g+(j-4);
    // one 16-query tile of S / dP is live at a time and packed to bf16 straight away.
    u32x4 pw[2], sw[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int q0 = qc * 32 + qt * 16 + 4 * g;
      const f32x4 nl = *reinterpret_cast<const f32x4*>(nlse_s + q0);
      const f32x4 nd = *reinterpret_cast<const f32x4*>(nd_s + q0);
      const char* qrow = Qs + (qc * 32 + qt * 16) * 128;
      const char* drow = dOs + (qc * 32 + qt * 16) * 128;
      const bf16x8 qa0 = lds16(qrow + ro0), qa1 = lds16(qrow + ro1);
      const bf16x8 da0 = lds16(drow + ro0), da1 = lds16(drow + ro1);
      f32x4 S[2], dP[2];
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        S[k2] = mfma16(qa0, kf[k2][0], f32x4{0.f, 0.f, 0.f, 0.f});
        S[k2] = mfma16(qa1, kf[k2][1], S[k2]);
        dP[k2] = mfma16(da0, vf[k2][0], nd);  // dP - D
        dP[k2] = mfma16(da1, vf[k2][1], dP[k2]);
      }
      // lane holds X[q = q0 + r][key = kb + k2*16 + t]
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        f32x4 p;
#pragma unroll
        for (int r = 0; r < 4; ++r) p[r] = ex2(__builtin_fmaf(S[k2][r], c, nl[r]));
        if (edge) {
#pragma unroll
          for (int r = 0; r < 4; ++r) p[r] = masked(kb + k2 * 16 + t, q0 + r, L, causal) ? 0.f : p[r];
        }
        const f32x4 ds = p * dP[k2];
        pw[k2][2 * qt] = pack2bf(p[0], p[1]);
        pw[k2][2 * qt + 1] = pack2bf(p[2], p[3]);
        sw[k2][2 * qt] = pack2bf(ds[0], ds[1]);
        sw[k2][2 * qt + 1] = pack2bf(ds[2], ds[3]);
      }
    }
    const bf16x8 pB[2] = {as_bf8(pw[0]), as_bf8(pw[1])};
    const bf16x8 sB[2] = {as_bf8(sw[0]), as_bf8(sw[1])};
    const char* qblk = Qs + qc * 32 * 128;
    const char* dblk = dOs + qc * 32 * 128;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x8 doT = cat4(lds_tr(dblk + tro[dt]), lds_tr(dblk + 16 * 128 + tro[dt]));
      const bf16x8 qT = cat4(lds_tr(qblk + tro[dt]), lds_tr(qblk + 16 * 128 + tro[dt]));
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        dV[dt][k2] = mfma16(doT, pB[k2], dV[dt][k2]);
        dK[dt][k2] = mfma16(qT, sB[k2], dK[dt][k2]);
      }
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
}

// ------------------------------------------------------------- backward, fused (dK, dV, then dQ)
template <int NQB>
struct BwdLds {
  static constexpr int LP = 32 * NQB;
  static constexpr int DST_STRIDE = LP * 2 + 16;  // bytes per dS^T row (conflict-free tr reads)
  static constexpr int Q_OFF = 0;
  static constexpr int DO_OFF = LP * 128;
  static constexpr int DST_OFF = 2 * LP * 128;
  static constexpr int NLSE_OFF = DST_OFF + LP * DST_STRIDE;
  static constexpr int ND_OFF = NLSE_OFF + LP * 4;
  static constexpr int BYTES = ND_OFF + LP * 4;
};

// Persistent: a workgroup walks (sequence, head) items blockIdx.x, + gridDim.x, ...; the next
// item's Q / dO / O / lse rows and K / V fragments are loaded into registers while the current
// one computes (rows after the current item's LDS image is written, K / V after its phase 1), so
// the item's HBM traffic (~230 KB at L = 197) overlaps the MFMA / exp work of the previous one.
//
// Q8: dQ / dK / dV written as the A operand of the fp8 QKV input-gradient GEMM (MaPLe's fp8
// mode): e4m3 codes (lddq in bytes) + E8M0 scales (q_scale, q_rows), the arithmetic of
// quant_fp8_kernel on the bf16-rounded values, so the codes equal bf16 output + quant_fp8.
template <int NQB, bool PERSIST = (NQB >= 5), bool Q8 = false>
__global__ void __launch_bounds__(64 * NQB)
attn_bwd_kernel(int n_items, int L, int H, int D, const bf16_t* __restrict__ qkv, long ldq,
                   const bf16_t* __restrict__ O, const bf16_t* __restrict__ dO, long ldo,
                   const float* __restrict__ lse, bf16_t* __restrict__ dqkv, long lddq, int causal,
                   float scale, uint8_t* __restrict__ q_scale = nullptr, long q_rows = 0) {
  constexpr int LP = 32 * NQB;
  constexpr int NTH = 64 * NQB;
  using Lay = BwdLds<NQB>;
  __shared__ __attribute__((aligned(16))) char smem[Lay::BYTES];
  char* Qs = smem + Lay::Q_OFF;
  char* dOs = smem + Lay::DO_OFF;
  char* dSTs = smem + Lay::DST_OFF;
  float* nlse_s = reinterpret_cast<float*>(smem + Lay::NLSE_OFF);  // -lse
  float* nd_s = reinterpret_cast<float*>(smem + Lay::ND_OFF);      // -D

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, t = lane & 15;
  const float c = scale * LOG2E;
  int item = blockIdx.x;
  if (item >= n_items) return;

  // staging: 16-B chunks of Q, dO and O rows (8 lanes per row); D = rowsum(dO*O) from the same
  // chunks (xor-shuffles) when they are written to LDS
  constexpr int IT = LP * 8 / NTH;  // = 4
  uint4 qv[IT], dv[IT], ov[IT];
  float lv[IT];
  // Every global access of an item goes through a raw-buffer descriptor over that sequence's L
  // rows (wave-uniform): rows >= L fall outside it, so their loads return zero and their stores
  // are dropped by the range check. No branch surrounds a memory op, so hipcc can count vmcnt
  // across them — with a store under a branch it waits vmcnt(0) at the next use of any earlier
  // load, i.e. for every store still in flight (the whole store latency once per item).
  // (ok = false: an empty descriptor — the past-the-end prefetch and the first item's deferred
  // dQ are issued unconditionally and read zeros / store nothing, so their count never depends
  // on a branch either)
  auto rows_rsrc = [&](const void* p, long row0, long row_bytes, bool ok = true) {
    const uint64_t a = (uint64_t)(static_cast<const char*>(p) + (ok ? row0 * row_bytes : 0));
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const int n = __builtin_amdgcn_readfirstlane(ok ? (int)(L * row_bytes) : 0);
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, n, 0x00020000);
  };
  auto bld16 = [](__amdgpu_buffer_rsrc_t r, int off) {  // nontemporal (read once)
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 2);
    return make_uint4(v[0], v[1], v[2], v[3]);
  };
  // Q rows and lse (prefetched during phase 1), dO and O rows (during phase 2: registers). The
  // per-lane row offsets are recomputed from an opaque copy of tid at every call: hoisted out of
  // the item loop they would stay live through both phases (and spill).
  auto lane_tid = [&]() {
    int v = tid;
    asm volatile("" : "+v"(v));
    return v;
  };
  auto load_rows = [&](int it_) {
    const int tv = lane_tid();
    const bool ok = it_ < n_items;
    const auto rq = rows_rsrc(qkv, (long)(it_ / H) * L, ldq * 2, ok);
    const auto rl = rows_rsrc(lse, (long)it_ * L, 4, ok);  // this item's L lse values
    const int cb = ((it_ % H) * 64 + (tv & 7) * 8) * 2;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int r = (tv + i * NTH) >> 3;
      qv[i] = bld16(rq, r * (int)ldq * 2 + cb);
      // rows >= L read 0 here; the padded-row value (1e30) is substituted where lv is used
      lv[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rl, r * 4, 0, 0));
    }
  };
  auto load_o = [&](int it_) {
    const int tv = lane_tid();
    const bool ok = it_ < n_items;
    const auto rd = rows_rsrc(dO, (long)(it_ / H) * L, ldo * 2, ok);
    const auto ro = rows_rsrc(O, (long)(it_ / H) * L, ldo * 2, ok);
    const int cb = ((it_ % H) * 64 + (tv & 7) * 8) * 2;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int r = (tv + i * NTH) >> 3;
      dv[i] = bld16(rd, r * (int)ldo * 2 + cb);
      ov[i] = bld16(ro, r * (int)ldo * 2 + cb);
    }
  };
  // own key block: K / V rows kb + kt2*16 + t, as B-operand fragments
  const int kb = 32 * w;
  bf16x8 kf[2][2], vf[2][2];
  auto load_kv = [&](int it_) {
    const int tv = lane_tid() & 63;
    const auto rq = rows_rsrc(qkv, (long)(it_ / H) * L, ldq * 2, it_ < n_items);
    const int cb = ((it_ % H) * 64 + D + (tv >> 4) * 8) * 2;
#pragma unroll
    for (int kt2 = 0; kt2 < 2; ++kt2) {
      const int key = kb + kt2 * 16 + (tv & 15);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int off = key * (int)ldq * 2 + cb + s * 64;
        uint4 ku = bld16(rq, off), vu = bld16(rq, off + D * 2);
        kf[kt2][s] = *reinterpret_cast<bf16x8*>(&ku);
        vf[kt2][s] = *reinterpret_cast<bf16x8*>(&vu);
      }
    }
  };
  load_rows(item);
  load_o(item);
  load_kv(item);

  // one row's 64 head columns (lane g holds columns dt*16 + 4g + {0..3} in x[dt], the 4 lanes
  // t, t+16, t+32, t+48 share the row) times mul, to dqkv columns col0..col0+63
  // bf16 rows through the sequence's descriptor (row r of the sequence starting at row0; rows
  // >= L dropped by the range check): store_row64's two 16-B pieces per lane
  auto put_row_b = [&](long row0, int r, int col0, f32x4 x0, f32x4 x1, f32x4 x2, f32x4 x3,
                       float mul) {
    const f32x4 x[4] = {x0, x1, x2, x3};
    const auto rs = rows_rsrc(dqkv, row0, lddq * 2, row0 >= 0);
    uint2 xp[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
      xp[dt] = uint2{pack2bf(x[dt][0] * mul, x[dt][1] * mul), pack2bf(x[dt][2] * mul, x[dt][3] * mul)};
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const auto s0 = __builtin_amdgcn_permlane16_swap(xp[2 * p].x, xp[2 * p + 1].x, false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(xp[2 * p].y, xp[2 * p + 1].y, false, false);
      typedef unsigned int v4u __attribute__((ext_vector_type(4)));
      const v4u v = v4u{s0[0], s1[0], s0[1], s1[1]};
#ifdef ATT_KO_STORES  // diagnostic builds only: the stores replaced by a keep-alive (results wrong)
      asm volatile("" ::"v"(v));
      (void)rs;
#else
      __builtin_amdgcn_raw_buffer_store_b128(
          v, rs, r * (int)lddq * 2 + (col0 + 32 * p + 16 * (g & 1) + 8 * (g >> 1)) * 2, 0, 0);
#endif
    }
  };
  auto put_row = [&](long row, int col0, f32x4 x0, f32x4 x1, f32x4 x2, f32x4 x3, float mul) {
    const f32x4 x[4] = {x0, x1, x2, x3};
    if constexpr (!Q8) {
      uint2 xp[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        xp[dt] = uint2{pack2bf(x[dt][0] * mul, x[dt][1] * mul), pack2bf(x[dt][2] * mul, x[dt][3] * mul)};
      store_row64(dqkv + row * lddq + col0, g, xp);
    } else {
      uint8_t* dst = reinterpret_cast<uint8_t*>(dqkv) + row * lddq + col0;
#pragma unroll
      for (int b = 0; b < 2; ++b) {  // 32-column scale blocks: dt = 2b, 2b + 1
        float v[8];
        uint32_t amax = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          v[i] = bf2f(f2bf(x[2 * b + (i >> 2)][i & 3] * mul));
          amax = lc_amax_bits(amax, v[i]);
        }
        amax = max(amax, (uint32_t)__shfl_xor((int)amax, 16));
        amax = max(amax, (uint32_t)__shfl_xor((int)amax, 32));
        const uint32_t byte = e8m0_of_bits(amax);
        const float inv = e8m0_inv(byte);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          *reinterpret_cast<uint32_t*>(dst + (2 * b + j) * 16 + 4 * g) =
              pack4_fp8(v[4 * j] * inv, v[4 * j + 1] * inv, v[4 * j + 2] * inv, v[4 * j + 3] * inv);
        if (g == 0) q_scale[fp8_scale_index(row, (col0 >> 5) + b, q_rows)] = (uint8_t)byte;
      }
    }
  };
  // Persistent: item i's dQ rows are stored after item i+1's first barrier, not at the end of
  // item i. CDNA's vmcnt retires loads and stores in issue order, so the wait for the prefetched
  // rows at the top of item i+1 (hipcc emits vmcnt(0) there) would otherwise also wait for the
  // dQ stores issued just before it — their whole latency exposed once per item.
  f32x4 dQp[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dQp[dt][0] = dQp[dt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  long pbase = -1;
  int ph = 0;
  auto put_dq = [&](long pb, int hh, const f32x4 (&x)[4][2]) {
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int q = 32 * w + qt * 16 + t;
      if constexpr (!Q8)
        put_row_b(pb, q, hh * 64, x[0][qt], x[1][qt], x[2][qt], x[3][qt], scale);
      else if (pb >= 0 && q < L)
        put_row(pb + q, hh * 64, x[0][qt], x[1][qt], x[2][qt], x[3][qt], scale);
    }
  };
#pragma unroll 1
  for (; item < n_items; item += gridDim.x) {
  const int next = item + gridDim.x;
  const int h = item % H;
  const long base = (long)(item / H) * L;
  const int tvh = lane_tid();  // LDS addresses recomputed per item (hoisted, they spilled)
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int r = (tvh + i * NTH) >> 3;
    const int ch = tvh & 7;
    *reinterpret_cast<uint4*>(Qs + r * 128 + swz(r, ch) * 16) = qv[i];
    *reinterpret_cast<uint4*>(dOs + r * 128 + swz(r, ch) * 16) = dv[i];
    const uint32_t aa[4] = {ov[i].x, ov[i].y, ov[i].z, ov[i].w};
    const uint32_t bb[4] = {dv[i].x, dv[i].y, dv[i].z, dv[i].w};
    float dsum = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      dsum += bf2f(aa[k] & 0xffff) * bf2f(bb[k] & 0xffff) + bf2f(aa[k] >> 16) * bf2f(bb[k] >> 16);
    dsum += __shfl_xor(dsum, 1);
    dsum += __shfl_xor(dsum, 2);
    dsum += __shfl_xor(dsum, 4);
    if (ch == 0) {
      nd_s[r] = -dsum;
      nlse_s[r] = r < L ? -lv[i] : -1e30f;
    }
  }
  __syncthreads();
  if constexpr (PERSIST) {
    put_dq(pbase, ph, dQp);  // the previous item's dQ (see above; none before the first item)
    load_rows(next);         // in flight through phases 1 and 2 (zeros past the last item)
  }

  const int ro0 = row_off(t, g, 0), ro1 = row_off(t, g, 1);
  const int tr0 = tr_off(t, g, 0), tr1 = tr_off(t, g, 1), tr2 = tr_off(t, g, 2), tr3 = tr_off(t, g, 3);
  const int tro[4] = {tr0, tr1, tr2, tr3};

  f32x4 dV[4][2], dK[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) dV[dt][k2] = dK[dt][k2] = f32x4{0.f, 0.f, 0.f, 0.f};

  // causal: queries before the block's first key see none of its keys
  const int qc0 = causal ? w : 0;
#pragma unroll 1
  for (int qc = qc0; qc < NQB; ++qc) {
    const bool edge = (kb + 32 > L) || (causal && kb + 31 > qc * 32);
    // B operands (k = 32 queries of this chunk): slot j<4 -> q = 4g+j, j>=4 -> 16+4g+(j-4);
    // one 16-query tile of S / dP is live at a time and packed to bf16 straight away.
    u32x4 pw[2], sw[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int q0 = qc * 32 + qt * 16 + 4 * g;
      const f32x4 nl = *reinterpret_cast<const f32x4*>(nlse_s + q0);
      const f32x4 nd = *reinterpret_cast<const f32x4*>(nd_s + q0);
      const char* qrow = Qs + (qc * 32 + qt * 16) * 128;
      const char* drow = dOs + (qc * 32 + qt * 16) * 128;
      const bf16x8 qa0 = lds16(qrow + ro0), qa1 = lds16(qrow + ro1);
      const bf16x8 da0 = lds16(drow + ro0), da1 = lds16(drow + ro1);
      f32x4 S[2], dP[2];
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        S[k2] = mfma16(qa0, kf[k2][0], f32x4{0.f, 0.f, 0.f, 0.f});
        S[k2] = mfma16(qa1, kf[k2][1], S[k2]);
        dP[k2] = mfma16(da0, vf[k2][0], nd);  // dP - D
        dP[k2] = mfma16(da1, vf[k2][1], dP[k2]);
      }
      // lane holds X[q = q0 + r][key = kb + k2*16 + t]
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        f32x4 p;
#pragma unroll
        for (int r = 0; r < 4; ++r) p[r] = ex2(__builtin_fmaf(S[k2][r], c, nl[r]));
        if (edge) {
#pragma unroll
          for (int r = 0; r < 4; ++r) p[r] = masked(kb + k2 * 16 + t, q0 + r, L, causal) ? 0.f : p[r];
        }
        const f32x4 ds = p * dP[k2];
        pw[k2][2 * qt] = pack2bf(p[0], p[1]);
        pw[k2][2 * qt + 1] = pack2bf(p[2], p[3]);
        sw[k2][2 * qt] = pack2bf(ds[0], ds[1]);
        sw[k2][2 * qt + 1] = pack2bf(ds[2], ds[3]);
        // park dS^T[key][q0..q0+3] for the dQ phase
        *reinterpret_cast<uint2*>(dSTs + (kb + k2 * 16 + t) * Lay::DST_STRIDE + q0 * 2) =
            uint2{sw[k2][2 * qt], sw[k2][2 * qt + 1]};
      }
    }
    const bf16x8 pB[2] = {as_bf8(pw[0]), as_bf8(pw[1])};
    const bf16x8 sB[2] = {as_bf8(sw[0]), as_bf8(sw[1])};
    const char* qblk = Qs + qc * 32 * 128;
    const char* dblk = dOs + qc * 32 * 128;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x8 doT = cat4(lds_tr(dblk + tro[dt]), lds_tr(dblk + 16 * 128 + tro[dt]));
      const bf16x8 qT = cat4(lds_tr(qblk + tro[dt]), lds_tr(qblk + 16 * 128 + tro[dt]));
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        dV[dt][k2] = mfma16(doT, pB[k2], dV[dt][k2]);
        dK[dt][k2] = mfma16(qT, sB[k2], dK[dt][k2]);
      }
    }
  }
  // dK, dV of the own key block: lane holds X^T[d = dt*16 + 4g + r][key = kb + k2*16 + t]
#pragma unroll
  for (int k2 = 0; k2 < 2; ++k2) {
    const int key = kb + k2 * 16 + t;
    if constexpr (!Q8) {
      put_row_b(base, key, D + h * 64, dK[0][k2], dK[1][k2], dK[2][k2], dK[3][k2], scale);
      put_row_b(base, key, 2 * D + h * 64, dV[0][k2], dV[1][k2], dV[2][k2], dV[3][k2], 1.0f);
    } else if (key < L) {  // every lane of the row (same t) takes this branch together
      put_row(base + key, D + h * 64, dK[0][k2], dK[1][k2], dK[2][k2], dK[3][k2], scale);
      put_row(base + key, 2 * D + h * 64, dV[0][k2], dV[1][k2], dV[2][k2], dV[3][k2], 1.0f);
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
  if constexpr (PERSIST) {  // kf / vf, phase-1 accumulators dead until the next item
    load_o(next);
    load_kv(next);
  }
  __syncthreads();

  // phase 2: dQ^T[d][q] = sum_key K^T[d][key] dS^T[key][q] for queries qb..qb+31 (k order:
  // key = 32s + 8g + j, from rows 8g+(t>>2) and 8g+4+(t>>2) of both images)
  const int qb = 32 * w;
  const int s_end = causal ? min(NQB, w + 1) : NQB;
  int klo[4], khi[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const int col = dt * 16 + (t & 3) * 4;
    const int r0 = 8 * g + (t >> 2);
    klo[dt] = r0 * 128 + swz(r0, col >> 3) * 16 + (col & 7) * 2;
    khi[dt] = (r0 + 4) * 128 + swz(r0 + 4, col >> 3) * 16 + (col & 7) * 2;
  }
  const char* dst0 = dSTs + (8 * g + (t >> 2)) * Lay::DST_STRIDE + (qb + (t & 3) * 4) * 2;
  f32x4 dQ[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dQ[dt][0] = dQ[dt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int s = 0; s < s_end; ++s) {
    const char* ds = dst0 + 32 * s * Lay::DST_STRIDE;
    const bf16x8 bq0 = cat4(lds_tr(ds), lds_tr(ds + 4 * Lay::DST_STRIDE));
    const bf16x8 bq1 = cat4(lds_tr(ds + 32), lds_tr(ds + 4 * Lay::DST_STRIDE + 32));
    const char* kblk = Ks + 32 * s * 128;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x8 ka = cat4(lds_tr(kblk + klo[dt]), lds_tr(kblk + khi[dt]));
      dQ[dt][0] = mfma16(ka, bq0, dQ[dt][0]);
      dQ[dt][1] = mfma16(ka, bq1, dQ[dt][1]);
    }
  }
  if constexpr (!PERSIST) {  // one item per workgroup (short sequences: many workgroups)
    put_dq(base, h, dQ);
    break;
  }
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dQp[dt][0] = dQ[dt][0], dQp[dt][1] = dQ[dt][1];
  pbase = base;
  ph = h;
  __syncthreads();  // phase 2 done with Ks / dS^T before the next item's LDS image
  }
  if (PERSIST && pbase >= 0) put_dq(pbase, ph, dQp);
}

// ------------------------------------------------------------------ backward, query-major (dQ)
template <int NQB>
__global__ void __launch_bounds__(64 * NQB, 4)
attn_bwd_q_kernel(int L, int H, int D, const bf16_t* __restrict__ qkv, long ldq,
                  const bf16_t* __restrict__ O, const bf16_t* __restrict__ dO, long ldo,
                  const float* __restrict__ lse, bf16_t* __restrict__ dqkv, long lddq, int causal,
                  float scale) {
  constexpr int LP = 32 * NQB;
  constexpr int NTH = 64 * NQB;
  __shared__ __attribute__((aligned(16))) char smem[2 * LP * 128];
  char* Ks = smem;
  char* Vs = smem + LP * 128;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, t = lane & 15;
  // reverse order: the key-major kernel touched the last heads most recently (L2 / Infinity Cache)
  const int nh = gridDim.x - 1 - blockIdx.x, n = nh / H, h = nh % H;
  const long base = (long)n * L;
  const float c = scale * LOG2E;

  constexpr int IT = LP * 8 / NTH;  // = 4
  const int ch = tid & 7;
  uint4 kv[IT], vv[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int r = (tid + i * NTH) >> 3;
    const bf16_t* src = qkv + (base + r) * ldq + h * 64 + ch * 8;
    kv[i] = ld16_or_zero(src + D, r < L);
    vv[i] = ld16_or_zero(src + 2 * D, r < L);
  }
  const int qb = 32 * w;
  bf16x8 qf[2][2], df[2][2];
  float nl[2], nd[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = qb + qt * 16 + t;
    float dsum = 0.f;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const long off = h * 64 + s * 32 + g * 8;
      uint4 u = ld16_or_zero(qkv + (base + q) * ldq + off, q < L);
      uint4 d = ld16_or_zero(dO + (base + q) * ldo + off, q < L);
      uint4 o = ld16_or_zero(O + (base + q) * ldo + off, q < L);
      qf[qt][s] = *reinterpret_cast<bf16x8*>(&u);
      df[qt][s] = *reinterpret_cast<bf16x8*>(&d);
      const uint32_t oo[4] = {o.x, o.y, o.z, o.w}, dd[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        dsum += bf2f(oo[k] & 0xffff) * bf2f(dd[k] & 0xffff) + bf2f(oo[k] >> 16) * bf2f(dd[k] >> 16);
    }
    dsum += __shfl_xor(dsum, 16);
    dsum += __shfl_xor(dsum, 32);
    nd[qt] = -dsum;
    nl[qt] = q < L ? -lse[(long)nh * L + q] : -1e30f;
  }
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int r = (tid + i * NTH) >> 3;
    *reinterpret_cast<uint4*>(Ks + r * 128 + swz(r, ch) * 16) = kv[i];
    *reinterpret_cast<uint4*>(Vs + r * 128 + swz(r, ch) * 16) = vv[i];
  }
  __syncthreads();

  const int ro0 = row_off(t, g, 0), ro1 = row_off(t, g, 1);
  const int tro[4] = {tr_off(t, g, 0), tr_off(t, g, 1), tr_off(t, g, 2), tr_off(t, g, 3)};
  const int s_end = causal ? min(NQB, (qb + 31) / 32 + 1) : NQB;

  f32x4 dQ[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dQ[dt][0] = dQ[dt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int s = 0; s < s_end; ++s) {
    const bool edge = (32 * s + 32 > L) || (causal && 32 * s + 31 > qb);
    // one 16-key tile of S^T / dP^T live at a time, packed to bf16 straight away
    u32x4 sw[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ro = (32 * s + 16 * kk) * 128;
      const bf16x8 ka0 = lds16(Ks + ro + ro0), ka1 = lds16(Ks + ro + ro1);
      const bf16x8 va0 = lds16(Vs + ro + ro0), va1 = lds16(Vs + ro + ro1);
      f32x4 S[2], dP[2];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        S[qt] = mfma16(ka0, qf[qt][0], f32x4{0.f, 0.f, 0.f, 0.f});
        S[qt] = mfma16(ka1, qf[qt][1], S[qt]);
        dP[qt] = mfma16(va0, df[qt][0], f32x4{nd[qt], nd[qt], nd[qt], nd[qt]});
        dP[qt] = mfma16(va1, df[qt][1], dP[qt]);
      }
      // lane holds X^T[key = 32s + 16kk + 4g + r][q = qb + qt*16 + t]
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        f32x4 p;
#pragma unroll
        for (int r = 0; r < 4; ++r) p[r] = ex2(__builtin_fmaf(S[qt][r], c, nl[qt]));
        if (edge) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            p[r] = masked(32 * s + 16 * kk + 4 * g + r, qb + qt * 16 + t, L, causal) ? 0.f : p[r];
        }
        const f32x4 ds = p * dP[qt];
        sw[qt][2 * kk] = pack2bf(ds[0], ds[1]);
        sw[qt][2 * kk + 1] = pack2bf(ds[2], ds[3]);
      }
    }
    const bf16x8 sb0 = as_bf8(sw[0]);
    const bf16x8 sb1 = as_bf8(sw[1]);
    const char* kblk = Ks + 32 * s * 128;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x8 kT = cat4(lds_tr(kblk + tro[dt]), lds_tr(kblk + 16 * 128 + tro[dt]));
      dQ[dt][0] = mfma16(kT, sb0, dQ[dt][0]);
      dQ[dt][1] = mfma16(kT, sb1, dQ[dt][1]);
    }
  }
  // lane holds dQ^T[d = dt*16 + 4g + r][q = qb + qt*16 + t]
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

// ------------------------------------------------ backward, two-phase (dQ, then dK / dV), 2 per CU
// One workgroup per (sequence, head), NQB waves; wave w owns the 16-row blocks w and w + NQB
// (its queries in phase 1, its keys in phase 2). LDS holds one pair of row images at a time
// (K | V, then Q | dO) plus the -lse / -D rows: 59 KB at L <= 224, so two workgroups share a CU
// and one's loads and stores run under the other's MFMA / exp chain. The fused kernel parks
// the whole dS^T (163 KB: one workgroup per CU, 1.75 waves per SIMD, its memory instructions
// exposed: profiles/r03/j_attn_bwd_knockouts.txt). The price is S and dP formed twice.
//   phase 1 (query-major, attn_bwd_q_kernel's math): S^T = K Q^T, dP^T = V dO^T - D from the
//     K / V images and the wave's Q / dO fragments; dQ^T += K^T dS^T.
//   hand-over: each wave reads its key blocks' K / V fragments from the images, then writes its
//     query blocks' Q / dO fragments as the Q / dO images (every row is one wave's block).
//   phase 2 (key-major, attn_bwd_kv_kernel's math on 16-key blocks): S = Q K^T,
//     dP = dO V^T - D; dV^T += dO^T P, dK^T += Q^T dS.
template <int NQB, bool CAUSAL>
__global__ void __launch_bounds__(64 * NQB) __attribute__((amdgpu_waves_per_eu(4)))
attn_bwd2_kernel(int L, int H, int D, const bf16_t* __restrict__ qkv, long ldq,
                 const bf16_t* __restrict__ O, const bf16_t* __restrict__ dO, long ldo,
                 const float* __restrict__ lse, bf16_t* __restrict__ dqkv, long lddq, float scale,
                 int ko) {
  constexpr int causal = CAUSAL;
  // non-causal: both query / key chunk loops fully unrolled (LDS offsets in the instructions,
  // the edge chunk known at compile time); causal: runtime bounds, rolled
  constexpr int UNR = CAUSAL ? 1 : NQB;
  // ko: timing knockouts of DIAG builds (LC_ATT2_KO; results wrong), 0 otherwise: 1 no phase-1
  // loop, 2 no phase-2 loop, 4 stores replaced by keep-alives, 8 every item loads item 0's rows
  constexpr int LP = 32 * NQB;
  constexpr int NTH = 64 * NQB;
  __shared__ __attribute__((aligned(16))) char smem[2 * LP * 128 + 2 * LP * 4];
  char* I0 = smem;             // K rows, then Q rows
  char* I1 = smem + LP * 128;  // V rows, then dO rows
  float* nlse_s = reinterpret_cast<float*>(smem + 2 * LP * 128);  // -lse
  float* nd_s = nlse_s + LP;                                       // -D

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar block bounds
  const int g = lane >> 4, t = lane & 15;
  const int nh = blockIdx.x, n = nh / H, h = nh % H;
  const long base = (long)n * L;
  const float c = scale * LOG2E;

  // every global load first, through raw-buffer descriptors over this sequence's L rows (rows
  // >= L read zeros from the range check: no branch around a load, so no vmcnt(0) between them):
  // K / V rows for the images, then the wave's two query blocks' Q / dO fragments (B operands
  // of S^T / dP^T: lane holds row q = qb + t, columns s*32 + 8g ..), O rows and lse
  auto rows_rsrc = [&](const void* p, long row0, long row_bytes) {
    const uint64_t a = (uint64_t)(static_cast<const char*>(p) + row0 * row_bytes);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const int nb = __builtin_amdgcn_readfirstlane((int)(L * row_bytes));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, nb, 0x00020000);
  };
  auto bld16 = [](__amdgpu_buffer_rsrc_t r, int off) {  // nontemporal (read once)
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 2);
    return make_uint4(v[0], v[1], v[2], v[3]);
  };
  const long lb = (ko & 8) ? 0 : base;
  const int hl = (ko & 8) ? 0 : h;
  const auto rq = rows_rsrc(qkv, lb, ldq * 2);
  const auto rd = rows_rsrc(dO, lb, ldo * 2);
  const auto rO = rows_rsrc(O, lb, ldo * 2);
  const auto rl = rows_rsrc(lse, (ko & 8) ? 0 : (long)nh * L, 4);
  constexpr int IT = LP * 8 / NTH;  // = 4
  const int ch = tid & 7;
  uint4 kv[IT], vv[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int r = (tid + i * NTH) >> 3;
    const int off = r * (int)ldq * 2 + (hl * 64 + ch * 8) * 2;
    kv[i] = bld16(rq, off + D * 2);
    vv[i] = bld16(rq, off + D * 4);
  }
  bf16x8 qf[2][2], df[2][2];
  uint4 of[2][2];
  float lv[2];
#pragma unroll
  for (int bk = 0; bk < 2; ++bk) {
    const int q = 16 * (w + NQB * bk) + t;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int cb = (hl * 64 + s * 32 + g * 8) * 2;
      uint4 u = bld16(rq, q * (int)ldq * 2 + cb);
      uint4 d = bld16(rd, q * (int)ldo * 2 + cb);
      of[bk][s] = bld16(rO, q * (int)ldo * 2 + cb);
      qf[bk][s] = *reinterpret_cast<bf16x8*>(&u);
      df[bk][s] = *reinterpret_cast<bf16x8*>(&d);
    }
    lv[bk] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rl, q * 4, 0, 0));
    asm volatile("" : "+v"(lv[bk]));  // issued here, not sunk into the q < L select below
  }
  float nl[2], nd[2];
#pragma unroll
  for (int bk = 0; bk < 2; ++bk) {
    const int q = 16 * (w + NQB * bk) + t;
    float dsum = 0.f;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 d8 = df[bk][s];
      const u32x4 dd = __builtin_bit_cast(u32x4, d8);
      const uint32_t oo[4] = {of[bk][s].x, of[bk][s].y, of[bk][s].z, of[bk][s].w};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        dsum += bf2f(oo[k] & 0xffff) * bf2f(dd[k] & 0xffff) + bf2f(oo[k] >> 16) * bf2f(dd[k] >> 16);
    }
    dsum += __shfl_xor(dsum, 16);
    dsum += __shfl_xor(dsum, 32);
    nd[bk] = -dsum;
    nl[bk] = q < L ? -lv[bk] : -1e30f;
    if (g == 0) {  // phase 2 reads every query's -lse / -D from LDS
      nd_s[q] = nd[bk];
      nlse_s[q] = nl[bk];
    }
  }
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int r = (tid + i * NTH) >> 3;
    *reinterpret_cast<uint4*>(I0 + r * 128 + swz(r, ch) * 16) = kv[i];
    *reinterpret_cast<uint4*>(I1 + r * 128 + swz(r, ch) * 16) = vv[i];
  }
  __syncthreads();

  const int ro0 = row_off(t, g, 0), ro1 = row_off(t, g, 1);
  const int tro[4] = {tr_off(t, g, 0), tr_off(t, g, 1), tr_off(t, g, 2), tr_off(t, g, 3)};

  // ---- phase 1: dQ of the wave's query blocks
#pragma unroll
  for (int bk = 0; bk < 2; ++bk) {
    const int qb = 16 * (w + NQB * bk);
    if (qb >= L) continue;  // wave-uniform
    const int s_end = (ko & 1) ? 0 : causal ? (qb + 15) / 32 + 1 : NQB;
    f32x4 dQ[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dQ[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll UNR
    for (int s = 0; s < NQB; ++s) {
      if (s >= s_end) break;
      const bool edge = (32 * s + 32 > L) || (causal && 32 * s + 31 > qb);
      // one 16-key tile of S^T / dP^T live at a time, packed to bf16 straight away; k slots of
      // the dS^T operand: j < 4 -> key 32s + 4g + j, j >= 4 -> 32s + 16 + 4g + (j - 4)
      u32x4 sw;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int ro = (32 * s + 16 * kk) * 128;
        const bf16x8 ka0 = lds16(I0 + ro + ro0), ka1 = lds16(I0 + ro + ro1);
        const bf16x8 va0 = lds16(I1 + ro + ro0), va1 = lds16(I1 + ro + ro1);
        f32x4 S = mfma16(ka0, qf[bk][0], f32x4{0.f, 0.f, 0.f, 0.f});
        S = mfma16(ka1, qf[bk][1], S);
        f32x4 dP = mfma16(va0, df[bk][0], f32x4{nd[bk], nd[bk], nd[bk], nd[bk]});
        dP = mfma16(va1, df[bk][1], dP);
        // lane holds X^T[key = 32s + 16kk + 4g + r][q = qb + t]
        f32x4 p;
#pragma unroll
        for (int r = 0; r < 4; ++r) p[r] = ex2(__builtin_fmaf(S[r], c, nl[bk]));
        if (edge) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            p[r] = masked(32 * s + 16 * kk + 4 * g + r, qb + t, L, causal) ? 0.f : p[r];
        }
        const f32x4 ds = p * dP;
        sw[2 * kk] = pack2bf(ds[0], ds[1]);
        sw[2 * kk + 1] = pack2bf(ds[2], ds[3]);
      }
      const bf16x8 sb = as_bf8(sw);
      const char* kblk = I0 + 32 * s * 128;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 kT = cat4(lds_tr(kblk + tro[dt]), lds_tr(kblk + 16 * 128 + tro[dt]));
        dQ[dt] = mfma16(kT, sb, dQ[dt]);
      }
    }
    // lane holds dQ^T[d = dt*16 + 4g + r][q = qb + t]
    const int q = qb + t;
    if (q < L) {  // the 4 lanes of the row agree
      uint2 x[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        x[dt] = uint2{pack2bf(dQ[dt][0] * scale, dQ[dt][1] * scale),
                      pack2bf(dQ[dt][2] * scale, dQ[dt][3] * scale)};
      if (ko & 4)
        asm volatile("" ::"v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]));
      else
        store_row64(dqkv + (base + q) * lddq + h * 64, g, x);
    }
  }

  // ---- hand-over: K / V fragments of the wave's key blocks (B operands of S = Q K^T,
  // dP = dO V^T: lane holds row key = kb + t, columns s*32 + 8g ..), then the Q / dO images
  bf16x8 kf[2][2], vf[2][2];
#pragma unroll
  for (int bk = 0; bk < 2; ++bk) {
    const int kb = 16 * (w + NQB * bk);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      kf[bk][s] = lds16(I0 + kb * 128 + (s ? ro1 : ro0));
      vf[bk][s] = lds16(I1 + kb * 128 + (s ? ro1 : ro0));
    }
  }
  __syncthreads();  // every wave holds its K / V fragments
#pragma unroll
  for (int bk = 0; bk < 2; ++bk) {
    const int qb = 16 * (w + NQB * bk);  // rows >= L: zeros (loaded so)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      *reinterpret_cast<bf16x8*>(I0 + qb * 128 + (s ? ro1 : ro0)) = qf[bk][s];
      *reinterpret_cast<bf16x8*>(I1 + qb * 128 + (s ? ro1 : ro0)) = df[bk][s];
    }
  }
  __syncthreads();

  // ---- phase 2: dK, dV of the wave's key blocks
#pragma unroll
  for (int bk = 0; bk < 2; ++bk) {
    const int kb = 16 * (w + NQB * bk);
    if (kb >= L) continue;  // wave-uniform
    f32x4 dV[4], dK[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dV[dt] = dK[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int qc0 = (ko & 2) ? NQB : causal ? kb / 32 : 0;  // (causal: earlier queries see none of it)
#pragma unroll UNR
    for (int qc = 0; qc < NQB; ++qc) {
      if (qc < qc0) continue;
      const bool edge = (kb + 16 > L) || (causal && kb + 15 > qc * 32);
      // k slots of the P / dS operands: j < 4 -> q = 32qc + 4g + j, j >= 4 -> 32qc + 16 + 4g + j-4
      u32x4 pw, sw;
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const int q0 = qc * 32 + qt * 16 + 4 * g;
        const f32x4 nlv = *reinterpret_cast<const f32x4*>(nlse_s + q0);
        const f32x4 ndv = *reinterpret_cast<const f32x4*>(nd_s + q0);
        const int ro = (qc * 32 + qt * 16) * 128;
        const bf16x8 qa0 = lds16(I0 + ro + ro0), qa1 = lds16(I0 + ro + ro1);
        const bf16x8 da0 = lds16(I1 + ro + ro0), da1 = lds16(I1 + ro + ro1);
        f32x4 S = mfma16(qa0, kf[bk][0], f32x4{0.f, 0.f, 0.f, 0.f});
        S = mfma16(qa1, kf[bk][1], S);
        f32x4 dP = mfma16(da0, vf[bk][0], ndv);
        dP = mfma16(da1, vf[bk][1], dP);
        // lane holds X[q = q0 + r][key = kb + t]
        f32x4 p;
#pragma unroll
        for (int r = 0; r < 4; ++r) p[r] = ex2(__builtin_fmaf(S[r], c, nlv[r]));
        if (edge) {
#pragma unroll
          for (int r = 0; r < 4; ++r) p[r] = masked(kb + t, q0 + r, L, causal) ? 0.f : p[r];
        }
        const f32x4 ds = p * dP;
        pw[2 * qt] = pack2bf(p[0], p[1]);
        pw[2 * qt + 1] = pack2bf(p[2], p[3]);
        sw[2 * qt] = pack2bf(ds[0], ds[1]);
        sw[2 * qt + 1] = pack2bf(ds[2], ds[3]);
      }
      const bf16x8 pB = as_bf8(pw), sB = as_bf8(sw);
      const char* qblk = I0 + qc * 32 * 128;
      const char* dblk = I1 + qc * 32 * 128;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 doT = cat4(lds_tr(dblk + tro[dt]), lds_tr(dblk + 16 * 128 + tro[dt]));
        const bf16x8 qT = cat4(lds_tr(qblk + tro[dt]), lds_tr(qblk + 16 * 128 + tro[dt]));
        dV[dt] = mfma16(doT, pB, dV[dt]);
        dK[dt] = mfma16(qT, sB, dK[dt]);
      }
    }
    // lane holds X^T[d = dt*16 + 4g + r][key = kb + t]
    const int key = kb + t;
    if (key < L) {
      uint2 xk[4], xv[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        xk[dt] = uint2{pack2bf(dK[dt][0] * scale, dK[dt][1] * scale),
                       pack2bf(dK[dt][2] * scale, dK[dt][3] * scale)};
        xv[dt] = uint2{pack2bf(dV[dt][0], dV[dt][1]), pack2bf(dV[dt][2], dV[dt][3])};
      }
      bf16_t* dst = dqkv + (base + key) * lddq + h * 64;
      if (ko & 4) {
        asm volatile("" ::"v"(xk[0]), "v"(xk[1]), "v"(xk[2]), "v"(xk[3]));
        asm volatile("" ::"v"(xv[0]), "v"(xv[1]), "v"(xv[2]), "v"(xv[3]));
      } else {
        store_row64(dst + D, g, xk);
        store_row64(dst + 2 * D, g, xv);
      }
    }
  }
}

// workgroups of a persistent launch: as many as fit on the chip at once (LDS-limited) when there
// are many items per workgroup (L = 197: 3072 items, 12 per workgroup), else one per item
int persistent_grid(int items, int lds_bytes) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  int per_cu = (160 * 1024) / lds_bytes;
  per_cu = per_cu < 1 ? 1 : (per_cu > 4 ? 4 : per_cu);
  const int g = cus * per_cu;
  // a few items per workgroup would leave a ragged last round: one item each (no pipelining)
  return items < 4 * g ? items : g;
}

// lc_attn_bwd_set_form: 0 automatic, else one of these
enum { ATTN_BWD_FUSED = 1, ATTN_BWD_SPLIT = 2, ATTN_BWD_TWO_PHASE = 3 };
const int g_att2_ko = [] {  // DIAG builds: attn_bwd2_kernel timing knockouts
  const char* e = lc_diag_env("LC_ATT2_KO");
  return e ? atoi(e) : 0;
}();
int g_attn_bwd_form = [] {  // DIAG builds: LC_ATTN_BWD_FORM=<form>, LC_ATTN_BWD_SPLIT=1 (A/Bs)
  const char* f = lc_diag_env("LC_ATTN_BWD_FORM");
  if (f) return atoi(f);
  const char* e = lc_diag_env("LC_ATTN_BWD_SPLIT");
  return e && atoi(e) ? (int)ATTN_BWD_SPLIT : 0;
}();

}  // namespace

extern "C" {

int lc_attn_fwd(hipStream_t st, int n_seq, int L, int H, const void* qkv, long ldq, void* O,
                long ldo, float* lse, int causal) {
  LC_CHECK_ARG(n_seq > 0 && L > 0 && L <= 256 && H > 0 && ldq >= 3 * H * 64 && ldo >= H * 64);
  LC_CHECK_ARG(ldq % 8 == 0 && ldo % 8 == 0 && ((uintptr_t)O & 15) == 0);  // 16-B row stores
  const int D = H * 64;
  const int nqb = (L + 31) / 32;
  dim3 grid(n_seq * H);
  const float scale = 0.125f;  // 64^-0.5
  static const bool online = [] {
    const char* e = lc_diag_env("LCCLIP_ATTN_FWD_ONLINE");
    return !(e && e[0] == '0');
  }();
  switch (nqb) {
#define LC_AF(Q)                                                                                \
  case Q:                                                                                      \
    if (online)                                                                                \
      hipLaunchKernelGGL((attn_fwd_kernel<Q, true>), grid, dim3(64 * Q), 0, st, L, H, D,       \
                         (const bf16_t*)qkv, ldq, (bf16_t*)O, ldo, lse, causal, scale);        \
    else                                                                                       \
      hipLaunchKernelGGL((attn_fwd_kernel<Q, false>), grid, dim3(64 * Q), 0, st, L, H, D,      \
                         (const bf16_t*)qkv, ldq, (bf16_t*)O, ldo, lse, causal, scale);        \
    break;
    LC_AF(1) LC_AF(2) LC_AF(3) LC_AF(4) LC_AF(5) LC_AF(6) LC_AF(7) LC_AF(8)
#undef LC_AF
    default:
      return LC_EINVAL;
  }
  LC_LAUNCH_RET();
}

int lc_attn_bwd_fp8(hipStream_t st, int n_seq, int L, int H, const void* qkv, long ldq,
                    const void* O, const void* dO, long ldo, const float* lse, void* dqkv, long lddq,
                    void* q_scale, long q_rows, int causal) {
  LC_CHECK_ARG(n_seq > 0 && L > 0 && L <= 224 && H > 0 && ldq >= 3 * H * 64 && ldo >= H * 64);
  LC_CHECK_ARG(lddq >= 3 * H * 64 && lddq % 16 == 0 && ((uintptr_t)dqkv & 15) == 0 &&
               ldq % 8 == 0 && ldo % 8 == 0 && q_scale != nullptr && q_rows % 256 == 0 &&
               q_rows >= ((long)n_seq * L + 255) / 256 * 256);
  const int D = H * 64;
  const float scale = 0.125f;
  switch ((L + 31) / 32) {
#define LC_ABQ(Q)                                                                               \
  case Q:                                                                                      \
    hipLaunchKernelGGL((attn_bwd_kernel<Q, (Q >= 5), true>),                                   \
                       dim3(Q >= 5 ? persistent_grid(n_seq * H, BwdLds<Q>::BYTES) : n_seq * H),  \
                       dim3(64 * Q), 0, st, n_seq * H, L, H, D, (const bf16_t*)qkv, ldq,        \
                       (const bf16_t*)O, (const bf16_t*)dO, ldo, lse, (bf16_t*)dqkv, lddq,      \
                       causal, scale, (uint8_t*)q_scale, q_rows);                               \
    break;
    LC_ABQ(1) LC_ABQ(2) LC_ABQ(3) LC_ABQ(4) LC_ABQ(5) LC_ABQ(6) LC_ABQ(7)
#undef LC_ABQ
    default:
      return LC_EINVAL;
  }
  LC_LAUNCH_RET();
}

int lc_attn_bwd_set_form(int form) {
  if (form < 0 || form > ATTN_BWD_TWO_PHASE) return LC_EINVAL;
  g_attn_bwd_form = form;
  return LC_OK;
}

int lc_attn_bwd(hipStream_t st, int n_seq, int L, int H, const void* qkv, long ldq, const void* O,
                const void* dO, long ldo, const float* lse, void* dqkv, long lddq, int causal) {
  LC_CHECK_ARG(n_seq > 0 && L > 0 && L <= 256 && H > 0 && ldq >= 3 * H * 64 && ldo >= H * 64);
  LC_CHECK_ARG(lddq >= 3 * H * 64 && ldq % 8 == 0 && ldo % 8 == 0 && lddq % 8 == 0 &&
               ((uintptr_t)dqkv & 15) == 0);  // 16-B row stores
  const int D = H * 64;
  const int nqb = (L + 31) / 32;
  dim3 grid(n_seq * H);
  const float scale = 0.125f;
  // fused single-pass kernel (dS^T parked in LDS, 1 workgroup per CU) up to 224 keys; the split
  // key-major + query-major pair beyond that (LDS); lc_attn_bwd_set_form selects another form
  const int form = g_attn_bwd_form ? g_attn_bwd_form : ATTN_BWD_FUSED;
  const bool split = form == ATTN_BWD_SPLIT;
  if (form == ATTN_BWD_TWO_PHASE && nqb <= 7) {
    switch (nqb) {
#define LC_AB2(Q)                                                                               \
  case Q:                                                                                      \
    if (causal)                                                                                \
      hipLaunchKernelGGL((attn_bwd2_kernel<Q, true>), grid, dim3(64 * Q), 0, st, L, H, D,      \
                         (const bf16_t*)qkv, ldq, (const bf16_t*)O, (const bf16_t*)dO, ldo,    \
                         lse, (bf16_t*)dqkv, lddq, scale, g_att2_ko);                          \
    else                                                                                       \
      hipLaunchKernelGGL((attn_bwd2_kernel<Q, false>), grid, dim3(64 * Q), 0, st, L, H, D,     \
                         (const bf16_t*)qkv, ldq, (const bf16_t*)O, (const bf16_t*)dO, ldo,    \
                         lse, (bf16_t*)dqkv, lddq, scale, g_att2_ko);                          \
    break;
      LC_AB2(1) LC_AB2(2) LC_AB2(3) LC_AB2(4) LC_AB2(5) LC_AB2(6) LC_AB2(7)
#undef LC_AB2
      default:
        return LC_EINVAL;
    }
    LC_LAUNCH_RET();
  }
  if (nqb == 8) {
    hipLaunchKernelGGL(attn_bwd_kv_kernel<8>, grid, dim3(512), 0, st, L, H, D, (const bf16_t*)qkv,
                       ldq, (const bf16_t*)O, (const bf16_t*)dO, ldo, lse, (bf16_t*)dqkv, lddq,
                       causal, scale);
    hipLaunchKernelGGL(attn_bwd_q_kernel<8>, grid, dim3(512), 0, st, L, H, D, (const bf16_t*)qkv,
                       ldq, (const bf16_t*)O, (const bf16_t*)dO, ldo, lse, (bf16_t*)dqkv, lddq,
                       causal, scale);
    LC_LAUNCH_RET();
  }
  switch (nqb) {
#define LC_AB(Q)                                                                                \
  case Q:                                                                                      \
    if (split)                                                                                 \
      hipLaunchKernelGGL(attn_bwd_kv_kernel<Q>, grid, dim3(64 * Q), 0, st, L, H, D,            \
                         (const bf16_t*)qkv, ldq, (const bf16_t*)O, (const bf16_t*)dO, ldo,    \
                         lse, (bf16_t*)dqkv, lddq, causal, scale);                             \
    if (split)                                                                                 \
      hipLaunchKernelGGL(attn_bwd_q_kernel<Q>, grid, dim3(64 * Q), 0, st, L, H, D,             \
                         (const bf16_t*)qkv, ldq, (const bf16_t*)O, (const bf16_t*)dO, ldo,    \
                         lse, (bf16_t*)dqkv, lddq, causal, scale);                             \
    else                                                                                       \
      hipLaunchKernelGGL(attn_bwd_kernel<Q>,                                                   \
                         dim3(Q >= 5 ? persistent_grid(n_seq * H, BwdLds<Q>::BYTES) : n_seq * H),\
                         dim3(64 * Q), 0, st, n_seq * H, L, H, D, (const bf16_t*)qkv, ldq,      \
                         (const bf16_t*)O, (const bf16_t*)dO, ldo, lse, (bf16_t*)dqkv, lddq,    \
                         causal, scale);                                                       \
    break;
    LC_AB(1) LC_AB(2) LC_AB(3) LC_AB(4) LC_AB(5) LC_AB(6) LC_AB(7)
#undef LC_AB
    default:
      return LC_EINVAL;
  }
  LC_LAUNCH_RET();
}

}  // extern "C"
