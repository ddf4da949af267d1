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
#include <stdlib.h>

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

// out = bf16(W[N,K] + s * B[N,r] @ A[r,K]) in [N,K] layout and optionally outT in [K,N].
// 64x64 tile per 256-thread workgroup: the r rows of A and r columns of B for the tile staged in
// LDS once, each thread 4 rows x 4 columns (float4 loads of W, 8-byte bf16 stores), and the
// transposed copy written from an LDS tile as 4 consecutive columns per store.
constexpr int MERGE_RMAX = 8;
LC_DEV void merge_tile(int N, int K, int r, const float* __restrict__ W, const float* __restrict__ A,
                       const float* __restrict__ B, float s, bf16_t* __restrict__ out,
                       bf16_t* __restrict__ outT, int n0, int k0) {
  __shared__ float tile[64][65];
  __shared__ float As[MERGE_RMAX][64];
  __shared__ float Bs[64][MERGE_RMAX];
  const int tid = threadIdx.x;
  for (int i = tid; i < r * 64; i += 256) {
    const int j = i / 64, kk = i % 64;
    As[j][kk] = (k0 + kk < K) ? A[(long)j * K + k0 + kk] : 0.f;
  }
  for (int i = tid; i < 64 * r; i += 256) {
    const int nn = i / r, j = i % r;
    Bs[nn][j] = (n0 + nn < N) ? B[(long)(n0 + nn) * r + j] : 0.f;
  }
  if (r > 0) __syncthreads();
  const int nn0 = (tid >> 4) * 4, kk0 = (tid & 15) * 4;
  const int kb = k0 + kk0;
  const bool vec = (K % 4 == 0) && (kb + 3 < K);
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int nn = nn0 + rr, n = n0 + nn;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (n < N) {
      if (vec) {
        const float4 w = *reinterpret_cast<const float4*>(W + (long)n * K + kb);
        v[0] = w.x; v[1] = w.y; v[2] = w.z; v[3] = w.w;
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = (kb + c < K) ? W[(long)n * K + kb + c] : 0.f;
      }
      for (int j = 0; j < r; ++j) {
        const float bj = s * Bs[nn][j];
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] += bj * As[j][kk0 + c];
      }
      if (vec) {
        *reinterpret_cast<uint2*>(out + (long)n * K + kb) = uint2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (kb + c < K) out[(long)n * K + kb + c] = f2bf(v[c]);
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) tile[nn][kk0 + c] = v[c];
  }
  if (!outT) return;
  __syncthreads();
  // transposed: thread -> 4 k rows x 4 consecutive n
  const int kt0 = (tid >> 4) * 4, nt0 = (tid & 15) * 4;
  const int nb = n0 + nt0;
  const bool vecT = (N % 4 == 0) && (nb + 3 < N);
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int k = k0 + kt0 + rr;
    if (k >= K) continue;
    const float* tcol = &tile[0][kt0 + rr];
    if (vecT) {
      *reinterpret_cast<uint2*>(outT + (long)k * N + nb) =
          uint2{pack2bf(tcol[(nt0 + 0) * 65], tcol[(nt0 + 1) * 65]),
                pack2bf(tcol[(nt0 + 2) * 65], tcol[(nt0 + 3) * 65])};
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (nb + c < N) outT[(long)k * N + nb + c] = f2bf(tcol[(nt0 + c) * 65]);
    }
  }
}

__global__ void __launch_bounds__(256)
merge_kernel(int N, int K, int r, const float* __restrict__ W, const float* __restrict__ A,
             const float* __restrict__ B, float s, bf16_t* __restrict__ out,
             bf16_t* __restrict__ outT) {
  merge_tile(N, K, r, W, A, B, s, out, outT, blockIdx.y * 64, blockIdx.x * 64);
}

// Many plain casts in one launch (the adapter weights of every block after each optimizer step:
// 2 x 2 small matrices per block, 48 launches of ~5 us each on the step's critical path before).
// blockIdx.y = item, blockIdx.x = 64x64 tile of that item.
// The same batch form carries LoRA merges (A, B, r, s per item; the LoRA towers' 6 merges per
// block after each optimizer step).
struct CastBatch {
  const float* W[LC_CAST_MAX];
  const float* A[LC_CAST_MAX];
  const float* B[LC_CAST_MAX];
  bf16_t* out[LC_CAST_MAX];
  bf16_t* outT[LC_CAST_MAX];
  int N[LC_CAST_MAX], K[LC_CAST_MAX], r[LC_CAST_MAX];
  float s[LC_CAST_MAX];
};
static_assert(sizeof(CastBatch) <= 4096, "kernel argument block");
__global__ void __launch_bounds__(256) cast_batch_kernel(CastBatch b) {
  const int it = blockIdx.y;
  const int N = b.N[it], K = b.K[it];
  const int tk = (K + 63) / 64;
  if ((int)blockIdx.x >= tk * ((N + 63) / 64)) return;
  merge_tile(N, K, b.r[it], b.W[it], b.A[it], b.B[it], b.s[it], b.out[it], b.outT[it],
             (blockIdx.x / tk) * 64, (blockIdx.x % tk) * 64);
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
constexpr int AD_H = 64;  // adapter.py:38 hard-codes the down width (Q7)

// ------------------------------------------------------------ adapter backward, one pass
// dpre = (h > 0) ? scale * (g Wu) / keep : 0   [M, 64]   (adapter.py:59-72 autograd: the ReLU
// dz   = g + dpre Wd                           [M, D]    mask, dropout and up-projection scale)
// Row-block walker: a persistent workgroup (8 waves, two per SIMD) per CU streams 32-row blocks
// of g through a 3-deep LDS ring (two blocks in flight behind the one computing); both weights
// stay in registers for the whole launch (MFMA fragments staged once through LDS), and g is read
// from HBM once for both products (the two-GEMM form reads it twice and round-trips dpre).
// Arithmetic is the GEMM epilogues' (EPI_AD_MASK, EPI_AD_ADD) with the same MFMA operand order
// and k order, so the results are bit-identical to that path.
// GH: g is the half residual gradient (IEEE half, the image tower's backward), read as written
// (no bf16 copy from the LayerNorm backward: 77 MB less written per layer): phase 1 runs on the
// f16 MFMA with Wu^T's fragments cast to half once per launch (the reference's fp16 autocast
// product, methods/adapter_clip.py:87; rounding g to bf16 per fragment instead cost the walker
// 42 -> 51 us), and phase 2 adds the exact half g.
//   phase 1: dpre^T[j][m]: wave w owns the 16x16 tile j = 16 (w & 3) .., m = 16 (w >> 2) ..
//   phase 2: dz^T[n][m] (K = 64): wave w owns n-tiles w ND/2 .. +ND/2-1 for both row tiles;
//            dz is written over g in the LDS image and stored as whole rows
// The g image is row-major with 16-B units XOR-swizzled by (row & 15), so the 16 rows an MFMA
// fragment read touches land in distinct banks.
constexpr int AD_MT = 2;          // 16-row tiles per block
constexpr int AD_R = 16 * AD_MT;  // rows per block
constexpr int AD_NS = 3;          // ring depth
constexpr int AD_NW = 8;          // waves
template <int ND>
struct AdBwdLds {
  static constexpr int D = 64 * ND;
  static constexpr int XB = AD_R * D * 2;               // one g block (bf16)
  static constexpr int HB = AD_R * AD_H * 2;            // one h block
  static constexpr int X0 = 0, H0 = AD_NS * XB, S0 = H0 + AD_NS * HB;
  static constexpr int BYTES = S0 + AD_R * AD_H * 2;    // + the dpre block (phase-2 operand)
  static_assert(AD_NS * XB >= AD_H * D * 2, "the weight staging reuses the g ring");
};

LC_DEV int ad_swz(int row, int unit) { return unit ^ (row & 15); }
LC_DEV int ad_swz_s(int row, int unit) { return unit ^ ((row >> 1) & 7); }
template <int N>
LC_DEV void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// s_waitcnt vmcnt(n) for a count known only at run time (the ring's ramp-up / drain)
LC_DEV void wait_vm_dyn(int n) {
  switch (n) {
#define LC_WV(k) case k: wait_vm<k>(); break;
    LC_WV(0) LC_WV(1) LC_WV(2) LC_WV(3) LC_WV(4) LC_WV(5) LC_WV(6) LC_WV(7) LC_WV(8) LC_WV(9)
    LC_WV(10) LC_WV(11) LC_WV(12) LC_WV(13) LC_WV(14) LC_WV(15) LC_WV(16) LC_WV(17) LC_WV(18)
    LC_WV(19) LC_WV(20) LC_WV(21) LC_WV(22) LC_WV(23) LC_WV(24) LC_WV(25) LC_WV(26) LC_WV(27)
    LC_WV(28) LC_WV(29) LC_WV(30) LC_WV(31)
#undef LC_WV
    default: wait_vm<0>(); break;
  }
}

template <int ND, bool DZ, bool GH = false>
__global__ void __launch_bounds__(64 * AD_NW, 1)
adapter_bwd_fused_kernel(int M, const bf16_t* __restrict__ G, long ldg,
                         const bf16_t* __restrict__ Hs, const bf16_t* __restrict__ WuT,
                         const bf16_t* __restrict__ WdT, float scale, float keep,
                         bf16_t* __restrict__ dpre, bf16_t* __restrict__ dz, long ldz) {
  using Lay = AdBwdLds<ND>;
  constexpr int D = Lay::D, RU = D / 8;  // 16-B units per g row
  constexpr int NT2 = ND / 2;            // phase-2 n-tiles per wave
  __shared__ __attribute__((aligned(16))) char smem[Lay::BYTES];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int t = lane & 15, g = lane >> 4;
  const int nt1 = w & 3, mt1 = w >> 2;
  const int nb = (M + AD_R - 1) / AD_R;
  int blk = blockIdx.x;
  if (blk >= nb) return;

  // g block: wave w fills 1-KiB pieces w*XP .. +XP-1; LDS unit u = piece*64 + lane holds row
  // u / RU, source unit (u % RU) ^ (row & 15). h block: 2 x 256 B per wave (4-B lanes), linear.
  constexpr int XP = Lay::XB / 1024 / AD_NW, HP = Lay::HB / 256 / AD_NW;
  static_assert(XP * 1024 * AD_NW == Lay::XB && HP * 256 * AD_NW == Lay::HB, "even split");
  auto dma_block = [&](int b, int slot) {
    char* xs = smem + Lay::X0 + slot * Lay::XB;
#pragma unroll
    for (int i = 0; i < XP; ++i) {
      const int piece = w * XP + i, u = piece * 64 + lane;
      const int row = u / RU, cu = ad_swz(row, u % RU);
      const int r = min(b * AD_R + row, M - 1);  // tail rows: computed, never stored
      glds16(G + (long)r * ldg + cu * 8, xs + piece * 1024);
    }
#pragma unroll
    for (int i = 0; i < HP; ++i) {
      const int piece = w * HP + i, e = piece * 64 + lane;  // 4-B element pairs
      const int row = e >> 5;
      const int r = min(b * AD_R + row, M - 1);
      glds4(Hs + (long)r * AD_H + (e & 31) * 2, smem + Lay::H0 + slot * Lay::HB + piece * 256);
    }
  };

  // prologue: both weights' fragments into registers, staged through the (still free) ring
  bf16x8 wu[2 * ND];  // Wu^T rows 16 nt1 + t, k-slice ks
  bf16x8 wd[NT2][2];  // Wd^T rows (w NT2 + j) 16 + t, k-slice ks
  {
    constexpr int UP = AD_H * D * 2 / 1024 / AD_NW;  // Wu^T [64][D], linear
#pragma unroll
    for (int i = 0; i < UP; ++i) {
      const int piece = w * UP + i;
      glds16(WuT + (long)(piece * 64 + lane) * 8, smem + piece * 1024);
    }
    wait_vm<0>();
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 2 * ND; ++ks)
      wu[ks] = *reinterpret_cast<const bf16x8*>(smem + (16 * nt1 + t) * (D * 2) + (ks * 4 + g) * 16);
    if constexpr (GH) {
#pragma unroll
      for (int ks = 0; ks < 2 * ND; ++ks) wu[ks] = b2h8(wu[ks]);
    }
    __syncthreads();
  }
  if constexpr (DZ) {
    constexpr int WP = D * AD_H * 2 / 1024 / AD_NW;  // Wd^T [D][64], linear
#pragma unroll
    for (int i = 0; i < WP; ++i) {
      const int piece = w * WP + i;
      glds16(WdT + (long)(piece * 64 + lane) * 8, smem + piece * 1024);
    }
    wait_vm<0>();
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NT2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int n = (w * NT2 + j) * 16 + t;
        wd[j][ks] = *reinterpret_cast<const bf16x8*>(smem + n * 128 + (ks * 4 + g) * 16);
      }
    __syncthreads();  // every wave holds its fragments before the ring is overwritten
  }
  // ring: this walker's blocks i = 0 .. n-1 (block blockIdx.x + i * gridDim.x) in slot i % NS;
  // the prologue issues blocks 0 .. NS-2, iteration i issues block i + NS - 1 after its barrier
  // and then stores block i. Issue order per wave: D0 .. D(P-1), then per iteration D(i+P), S(i)
  // (P = NS - 1), so when iteration i waits for Di the memory ops issued after it are
  // min(P-1, n-1-i) later blocks' DMAs (LP each) and min(i, P) blocks' stores (SP each).
  constexpr int P = AD_NS - 1, LP = XP + HP, SP = 1 + (DZ ? XP : 0);
  static_assert((P - 1) * LP + P * SP < 32, "wait_vm_dyn range");
  const int n = (nb - 1 - (int)blockIdx.x) / (int)gridDim.x + 1;
#pragma unroll
  for (int i = 0; i < P; ++i)
    if (i < n) dma_block(blk + i * gridDim.x, i);
  const float inv = 1.0f / keep;
  // Every LDS access in the loop is inline asm and every barrier a raw one (lds_barrier): hipcc
  // puts vmcnt(0) in front of __syncthreads() and of any plain access that may alias the ring
  // (the whole smem array), which drained the two blocks in flight at each of them.
  const uint32_t lds0 = lds_addr(smem);
  constexpr int GK = 4, NG = 2 * ND / GK;  // phase-1 fragment reads in groups, one group ahead
  static_assert(NG * GK == 2 * ND, "phase-1 groups");
#pragma unroll 1
  for (int i = 0; i < n; ++i, blk += gridDim.x) {
    const int slot = i % AD_NS;
    // block i's DMA landed; the barrier also retires every wave's use of the slot the next DMA
    // overwrites (block i-1's) and of the dpre image
    wait_vm_dyn(min(P - 1, n - 1 - i) * LP + min(i, P) * SP);
    lds_barrier();
    if (i + P < n) dma_block(blk + P * gridDim.x, (i + P) % AD_NS);
    const uint32_t xs = lds0 + Lay::X0 + slot * Lay::XB;
    const uint32_t hs = lds0 + Lay::H0 + slot * Lay::HB;
    const uint32_t s0 = lds0 + Lay::S0;
    // an opaque copy of t per block: the LDS addresses are recomputed (a few VALU) instead of
    // being hoisted out of the loop as ~30 loop-invariant registers (the ND = 12 walker spilled)
    int tq = t;
    asm volatile("" : "+v"(tq));
    {
      // phase 1: lane holds dpre^T[j = 16 nt1 + 4g + r][m = 16 mt1 + t]
      const int row = 16 * mt1 + tq, m = blk * AD_R + row;
      const uint32_t xrow = xs + row * (D * 2);
      // unit ks*4 + g swizzled by t (< 16): ((ks & 3) * 4 + g) ^ t, + 16 units per 4 k-slices,
      // so four base addresses and the instruction's offset field cover all 2 ND reads
      uint32_t xa[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) xa[q] = xrow + ((q * 4 + g) ^ tq) * 16;
      bf16x8 fb[2][GK];
      auto rd = [&](int grp, bf16x8* dst) {
#pragma unroll
        for (int e = 0; e < GK; ++e) {
          const int ks = grp * GK + e;
          asm volatile("ds_read_b128 %0, %1 offset:%2"
                       : "=v"(dst[e]) : "v"(xa[ks & 3]), "i"((ks >> 2) * 256));
        }
      };
      rd(0, fb[0]);
      f32x4 a1 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int grp = 0; grp < NG; ++grp) {
        if (grp + 1 < NG) {
          rd(grp + 1, fb[(grp + 1) & 1]);
          asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(GK) : "memory");
        } else {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int e = 0; e < GK; ++e)
          a1 = GH ? mfma16_h(wu[grp * GK + e], fb[grp & 1][e], a1)
                  : mfma16(wu[grp * GK + e], fb[grp & 1][e], a1);
      }
      // EPI_AD_MASK: v = acc * scale (+ no bias); (h > 0) ? v / keep : 0
      const int col = 16 * nt1 + 4 * g;
      uint2 hb;
      asm volatile("ds_read_b64 %0, %1" : "=v"(hb) : "v"(hs + row * 128 + col * 2));
      lds_wait0();
      const uint32_t hh[2] = {hb.x, hb.y};
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float hv = bf2f((r & 1) ? (hh[r >> 1] >> 16) : (hh[r >> 1] & 0xffff));
        const float v = a1[r] * scale + 0.0f;
        o[r] = hv > 0.f ? v * inv : 0.f;
      }
      const uint2 ob = uint2{pack2bf(o[0], o[1]), pack2bf(o[2], o[3])};
      if (m < M) *reinterpret_cast<uint2*>(dpre + (long)m * AD_H + col) = ob;
      if constexpr (DZ)
        asm volatile("ds_write_b64 %0, %1"
                     :: "v"(s0 + row * 128 + ad_swz_s(row, col >> 3) * 16 + (col & 7) * 2), "v"(ob)
                     : "memory");
    }
    if constexpr (DZ) {
      lds_barrier();  // the whole dpre block is in LDS; phase 1's g reads are done
#pragma unroll
      for (int mt = 0; mt < AD_MT; ++mt) {
        const int row = 16 * mt + tq;
        bf16x8 fs[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          asm volatile("ds_read_b128 %0, %1"
                       : "=v"(fs[ks]) : "v"(s0 + row * 128 + ad_swz_s(row, ks * 4 + g) * 16));
        const uint32_t xrow = xs + row * (D * 2);
        constexpr int JH = NT2 % 2 == 0 ? NT2 / 2 : NT2;  // tiles in flight (register budget)
#pragma unroll
        for (int j0 = 0; j0 < NT2; j0 += JH) {
          // g values of this lane's JH tiles, read while the MFMAs run
          uint2 gb[JH];
#pragma unroll
          for (int j = 0; j < JH; ++j) {
            const int nn = (w * NT2 + j0 + j) * 16 + 4 * g;
            asm volatile("ds_read_b64 %0, %1"
                         : "=v"(gb[j]) : "v"(xrow + ad_swz(tq, nn >> 3) * 16 + (nn & 7) * 2));
          }
          lds_wait0();
          f32x4 a2[JH];
#pragma unroll
          for (int j = 0; j < JH; ++j) {
            a2[j] = mfma16(wd[j0 + j][0], fs[0], f32x4{0.f, 0.f, 0.f, 0.f});
            a2[j] = mfma16(wd[j0 + j][1], fs[1], a2[j]);
          }
#pragma unroll
          for (int j = 0; j < JH; ++j) {
            // EPI_AD_ADD: g + acc; lane holds dz[m][n = 16 (w NT2 + j) + 4g + r], written over its
            // own g values in the image (each element is read and rewritten by the same lane)
            const int nn = (w * NT2 + j0 + j) * 16 + 4 * g;
            const uint32_t gg[2] = {gb[j].x, gb[j].y};
            float o[4];
#pragma unroll
            for (int r = 0; r < 4; ++r)
              o[r] = (GH ? h2f((uint16_t)((r & 1) ? (gg[r >> 1] >> 16) : (gg[r >> 1] & 0xffff)))
                         : bf2f((r & 1) ? (gg[r >> 1] >> 16) : (gg[r >> 1] & 0xffff))) +
                     (a2[j][r] * 1.0f + 0.0f);
            const uint2 ob = uint2{pack2bf(o[0], o[1]), pack2bf(o[2], o[3])};
            asm volatile("ds_write_b64 %0, %1"
                         :: "v"(xrow + ad_swz(tq, nn >> 3) * 16 + (nn & 7) * 2), "v"(ob) : "memory");
          }
        }
      }
      lds_barrier();  // the dz block is complete in the image
      // whole-row stores: wave w writes the image's 1-KiB pieces w*XP .. (16 B per lane)
      uint4 v[XP];
#pragma unroll
      for (int i2 = 0; i2 < XP; ++i2)
        asm volatile("ds_read_b128 %0, %1" : "=v"(v[i2]) : "v"(xs + (w * XP + i2) * 1024 + lane * 16));
      lds_wait0();
#pragma unroll
      for (int i2 = 0; i2 < XP; ++i2) {
        const int piece = w * XP + i2, u = piece * 64 + lane;
        const int row = u / RU, cu = ad_swz(row, u % RU);
        const int m = blk * AD_R + row;
        if (m < M) *reinterpret_cast<uint4*>(dz + (long)m * ldz + cu * 8) = v[i2];
      }
    }
  }
}

int ad_cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    n = v;
  }
  return n;
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
                             const int* __restrict__ skip, const long long* __restrict__ step_dev) {
  if (skip && *skip) return;
  if (step_dev) {  // bias corrections from the device-side step counter (graph replay)
    const float st = (float)*step_dev;
    bc1 = 1.0f - powf(b1, st);
    bc2 = 1.0f - powf(b2, st);
  }
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

__global__ void counter_add_kernel(int n, long long* ctr, long long delta) {
  if ((int)threadIdx.x < n) ctr[threadIdx.x] += delta;
}

// AdamW's state['step'] advances only when the update is applied: GradScaler.step skips
// optimizer.step() on non-finite gradients (methods/adapter_clip.py:94), so torch's counter
// does not move either.
__global__ void step_advance_kernel(long long* ctr, const int* skip) {
  if (threadIdx.x == 0 && !(skip && *skip)) *ctr += 1;
}

int grid_for(long work, int block) {
  long gsz = (work + block - 1) / block;
  if (gsz > 4096) gsz = 4096;
  return (int)(gsz < 1 ? 1 : gsz);
}

// ---------------------------------------------------------------- LoRA gradients, one pass
// Rank-r (r <= 4) LoRA gradients of one projection site (lora.py:838-839 / 1073-1074 autograd):
//   XA = X A^T [M, r],  dYB = dY B [M, r],  dB[N, r] += s dY^T XA,  dA[r, K] += s dYB^T X
// reading X [M, K] and dY [M, N] ONCE (the four-GEMM form streams each of them twice). Rows are
// independent, so a 32-row block b needs only its own rows: X_b (32 x K, whole, in LDS) gives
// XA_b; dY_b streams through a 3-slot ring in 128-column chunks, each chunk feeding both dYB_b
// (row reads) and dB (transposed reads, with XA_b as the other operand); once dY_b has passed,
// dA += dYB_b^T X_b (transposed reads of X_b). MFMA 16x16x32 with r padded to 16 (A / B^T staged
// as bf16 [>= 16, K] / [>= 16, N] with zero rows >= r).
// One persistent workgroup (8 waves) per CU walks row blocks cidx, cidx + walkers, ...; X of
// the next block and the ring's next chunks are in flight while the current block computes.
// dB (waves own one 16-column tile of every chunk) and dA (waves own KT/8... column tiles) stay
// in registers; each walker writes its partial to a workspace slot and lora_reduce_kernel sums
// the slots in walker order (deterministic, no atomics).
// Reductions across waves (XA_b: each wave a third of K; dYB_b: each wave one k-step of every
// chunk) go through LDS. Rows >= M are loaded clamped and their XA / dYB rows set to zero.
template <int KT, int NC>
struct LoraGeom {
  static constexpr int K = KT * 32;
  static constexpr int XROW = K * 2;              // X image row bytes
  static constexpr int XIMG = 32 * XROW;          // one X block
  static constexpr int CHUNK = 32 * 256;          // 32 rows x 128 cols of dY
  static constexpr int XPIECES = XIMG / 1024 / 8; // X DMA pieces per wave
  static constexpr int RED = 8 * 32 * 16 * 4;     // per-wave [32][16] f32 partials
  static constexpr int X_OFF = 0;
  static constexpr int RING_OFF = 2 * XIMG;
  static constexpr int RED_OFF = RING_OFF + 3 * CHUNK;
  static constexpr int XAT_OFF = RED_OFF + RED;   // bf16 [16][32]
  static constexpr int DYBT_OFF = XAT_OFF + 1024;
  static constexpr int BT_OFF = DYBT_OFF + 1024;  // B^T rows 0..3 (r <= 4), bf16 [4][N]
  static constexpr int BYTES = BT_OFF + 4 * NC * 128 * 2;
  static constexpr int XKS = KT / 8;              // XA k-steps per wave
  static constexpr int DAT = KT * 2 / 8;          // dA 16-column tiles per wave
  // walker slot: dB [N][r] then dA [r][K] (only the real rank is stored)
};

LC_DEV void vm_wait_n(int n) {
  switch (n) {
#define LC_VM(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    LC_VM(0) LC_VM(1) LC_VM(2) LC_VM(3) LC_VM(4) LC_VM(5) LC_VM(6) LC_VM(7) LC_VM(8)
    LC_VM(9) LC_VM(10) LC_VM(11) LC_VM(12) LC_VM(13) LC_VM(14)
    default: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
#undef LC_VM
  }
}

template <int KT, int NC>
__global__ void __launch_bounds__(512, 1)
lora_grad1p_kernel(int M, const bf16_t* __restrict__ X, long ldx, const bf16_t* __restrict__ dY,
                   long ldy, const bf16_t* __restrict__ apad, long lda,
                   const bf16_t* __restrict__ btpad, long ldbt, float* __restrict__ part,
                   int walkers, int r) {
  using G = LoraGeom<KT, NC>;
  constexpr int K = G::K, XROW = G::XROW;
  __shared__ __attribute__((aligned(16))) char smem[G::BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, t = lane & 15;
  const int nblk = (M + 31) / 32;
  const int cidx = blockIdx.x;
  const int nb = cidx < nblk ? (nblk - 1 - cidx) / walkers + 1 : 0;  // blocks of this walker
  auto blk_row = [&](int i) { return (cidx + i * walkers) * 32; };

  // DMA: X block i into buffer i & 1 (XPIECES 1-KiB pieces per wave), dY chunk (i, c) into ring
  // slot q (one piece per wave). Lane -> (row, 16-B position) inverts the 32-B unit swizzle.
  auto dma_x = [&](int i) {
    char* dst = smem + G::X_OFF + (i & 1) * G::XIMG;
    const int r0 = blk_row(i);
#pragma unroll
    for (int pp = 0; pp < G::XPIECES; ++pp) {
      const int piece = wave * G::XPIECES + pp;
      const int idx = piece * 64 + lane;          // 16-B position in the image
      const int row = idx / (XROW / 16), pc = idx % (XROW / 16);
      const int c = (((pc >> 1) ^ swz_w(row)) << 1) | (pc & 1);
      const int m = min(r0 + row, M - 1);
      glds16(X + (long)m * ldx + c * 8, dst + piece * 1024);
    }
  };
  auto dma_c = [&](int i, int c, int q) {
    char* dst = smem + G::RING_OFF + q * G::CHUNK;
    const int idx = wave * 64 + lane;
    const int row = idx >> 4, pc = idx & 15;
    const int cc = (((pc >> 1) ^ swz_w(row)) << 1) | (pc & 1);
    const int m = min(blk_row(i) + row, M - 1);
    glds16(dY + (long)m * ldy + c * 128 + cc * 8, dst + wave * 1024);
  };
  // LDS reads of the DMA'd images as inline asm (a plain read of an LDS-DMA target makes hipcc
  // wait vmcnt(0) first — it cannot tell the slot apart from the ones in flight — which drained
  // the ring once per chunk); each use follows an explicit lgkmcnt wait + sched_barrier.
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  // row read (A operand): row `row` (lane t's), 16-B chunk `ch` of an image with ROWB-byte rows
  auto row_frag = [&](uint32_t img, int rowb, int row, int ch) {
    const int u = (ch >> 1) ^ swz_w(row);
    bf16x8 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(img + row * rowb + u * 32 + (ch & 1) * 16));
    return v;
  };
  // transposed read: tr_frag's operand (rows row, row + 4 at column col) by two ds_read_b64_tr_b16
  auto tr_frag_asm = [&](uint32_t img, int rowb, int row, int col) {
    auto addr = [&](int r) {
      const int byte = col * 2;
      const int u = (byte >> 5) ^ swz_w(r);
      return img + r * rowb + u * 32 + (byte & 31);
    };
    bf16x4 lo, hi;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(addr(row)));
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(addr(row + 4)));
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  auto lgkm0 = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  // per-walker constant fragments: A rows (XA's B operand) for this wave's k-steps; B^T rows
  // (dYB's B operand) are read per chunk from an LDS copy of its r <= 4 nonzero rows
  bf16x8 af[G::XKS];
  // (inline-asm loads: hipcc would otherwise wait vmcnt(0) — draining the LDS-DMA ring — at
  // every use inside the loop; the explicit wait below retires them before the first DMA)
#pragma unroll
  for (int k = 0; k < G::XKS; ++k)
    asm volatile("global_load_dwordx4 %0, %1, off"
                 : "=v"(af[k])
                 : "v"(apad + (long)t * lda + (wave * G::XKS + k) * 32 + g * 8));
  {
    uint4* bt_l = reinterpret_cast<uint4*>(smem + G::BT_OFF);
    for (int e = tid; e < 4 * NC * 128 / 8; e += 512) {
      const int row = e / (NC * 16), c8 = e % (NC * 16);
      bt_l[e] = *reinterpret_cast<const uint4*>(btpad + (long)row * ldbt + c8 * 8);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // the B^T copy (no LDS-DMA in flight yet)
  // LDS hand-offs between waves with LDS-DMA in flight: a raw barrier behind lgkmcnt(0)
  // (__syncthreads() would wait vmcnt(0) and drain the ring)
  auto lds_barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  f32x4 accB[NC], accA[G::DAT];
#pragma unroll
  for (int c = 0; c < NC; ++c) accB[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < G::DAT; ++j) accA[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float* red = reinterpret_cast<float*>(smem + G::RED_OFF);
  bf16_t* xat = reinterpret_cast<bf16_t*>(smem + G::XAT_OFF);
  bf16_t* dybt = reinterpret_cast<bf16_t*>(smem + G::DYBT_OFF);

  // issue order per block i: [X_{i+1}], then one chunk piece per chunk step (the ring runs two
  // chunks ahead, across block seams); prologue: X_0, chunks (0,0), (0,1)
  if (nb > 0) {
    dma_x(0);
    dma_c(0, 0, 0);
    if (NC > 1) dma_c(0, 1, 1);
  }
  int slot = 0;  // ring slot of the current chunk
  for (int i = 0; i < nb; ++i) {
    const bool more = i + 1 < nb;
    // X_i landed: younger ops are the two ring pieces issued after it
    vm_wait_n(NC > 1 ? 2 : 1);
    __builtin_amdgcn_s_barrier();
    const uint32_t ximg = lds0 + G::X_OFF + (i & 1) * G::XIMG;
    // ---- XA_i partial: wave's k-steps, both 16-row subtiles
    {
      f32x4 xa[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int k = 0; k < G::XKS; ++k) {
        bf16x8 xf[2];
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
          xf[sub] = row_frag(ximg, XROW, sub * 16 + t, (wave * G::XKS + k) * 4 + g);
        lgkm0();
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) xa[sub] = mfma16(xf[sub], af[k], xa[sub]);
      }
      // lane holds XA[m = sub*16 + 4g + rr][r = t]
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) red[(wave * 32 + sub * 16 + 4 * g + rr) * 16 + t] = xa[sub][rr];
    }
    if (more) dma_x(i + 1);  // buffer (i+1)&1 was last read by block i-1's dA (before its end barrier)
    lds_barrier();
    {
      const int m = tid >> 4, r = tid & 15;  // 512 threads = 32 rows x 16
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) v += red[(w * 32 + m) * 16 + r];
      xat[r * 32 + m] = f2bf(blk_row(i) + m < M ? v : 0.f);
    }
    lds_barrier();
    const bf16x8 xaf = *reinterpret_cast<const bf16x8*>(xat + t * 32 + g * 8);  // XA[8g..8g+7][t]
    f32x4 dyb = f32x4{0.f, 0.f, 0.f, 0.f};
    const int sub = wave & 1, ks = wave >> 1;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      // chunk c landed (younger: the next chunk's piece, and X_{i+1} for c < 2)
      // ops younger than chunk c: the piece issued at step c - 1 (c == 0: chunk 1, issued one
      // block earlier or in the prologue) and X_{i+1} (issued after chunks 0 and 1)
      const int younger = (c == 0 ? (NC > 1 ? 1 : 0) : ((c + 1 < NC || more) ? 1 : 0)) +
                          (c < 2 && more ? G::XPIECES : 0);
      vm_wait_n(younger);
      __builtin_amdgcn_s_barrier();  // also: every wave done with the slot the next DMA reuses
      // the ring stays two chunks ahead, across the block seam
      {
        const int nc = c + 2, nq = slot >= 1 ? slot - 1 : 2;  // slot of chunk c + 2 (== c - 1)
        if (nc < NC) dma_c(i, nc, nq);
        else if (more && nc - NC < NC) dma_c(i + 1, nc - NC, nq);
      }
      const uint32_t cimg = lds0 + G::RING_OFF + slot * G::CHUNK;
      bf16x8 bfc;  // B^T[r = t][chunk c, k-step ks, 8g ..]: rows >= 4 are zero (r <= 4)
      asm volatile("ds_read_b128 %0, %1"
                   : "=v"(bfc)
                   : "v"(lds0 + G::BT_OFF + ((t & 3) * NC * 128 + c * 128 + ks * 32 + 8 * g) * 2));
      const bf16x8 dya = row_frag(cimg, 256, sub * 16 + t, ks * 4 + g);
      const bf16x8 dyt = tr_frag_asm(cimg, 256, 8 * g + (t >> 2), wave * 16 + (t & 3) * 4);
      lgkm0();
      if (t >= 4) bfc = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      // dYB partial: rows sub*16 + t, k-step ks of this chunk
      dyb = mfma16(dya, bfc, dyb);
      // dB tile `wave` of this chunk: A = dY^T (transposed reads), B = XA
      accB[c] = mfma16(dyt, xaf, accB[c]);
      slot = slot == 2 ? 0 : slot + 1;
    }
    // ---- dYB_i: sum the 4 waves of each subtile (each did a quarter of the k-steps)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) red[(wave * 32 + sub * 16 + 4 * g + rr) * 16 + t] = dyb[rr];
    lds_barrier();
    {
      const int m = tid >> 4, r = tid & 15, sb = m >> 4;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) v += red[((2 * w + sb) * 32 + m) * 16 + r];
      dybt[r * 32 + m] = f2bf(blk_row(i) + m < M ? v : 0.f);
    }
    lds_barrier();
    // ---- dA += dYB_i^T X_i: A = dYB^T rows, B = X_i columns (transposed reads)
    const bf16x8 dyf = *reinterpret_cast<const bf16x8*>(dybt + t * 32 + g * 8);
#pragma unroll
    for (int j = 0; j < G::DAT; j += 2) {
      const bf16x8 x0 = tr_frag_asm(ximg, XROW, 8 * g + (t >> 2), (wave * G::DAT + j) * 16 + (t & 3) * 4);
      const bf16x8 x1 = tr_frag_asm(ximg, XROW, 8 * g + (t >> 2), (wave * G::DAT + j + 1) * 16 + (t & 3) * 4);
      lgkm0();
      accA[j] = mfma16(dyf, x0, accA[j]);
      accA[j + 1] = mfma16(dyf, x1, accA[j + 1]);
    }
  }
  // walker partial: dB [N][r] (lane: rows n = c*128 + wave*16 + 4g + rr, column t < r), dA [r][K]
  // (lane: rows 4g + rr < r, column k = (wave*DAT + j)*16 + t)
  constexpr int N = NC * 128;
  float* slot_p = part + (long)cidx * ((long)N * r + (long)r * K);
  if (t < r) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        slot_p[(c * 128 + wave * 16 + 4 * g + rr) * r + t] = accB[c][rr];
  }
#pragma unroll
  for (int j = 0; j < G::DAT; ++j)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr)
      if (4 * g + rr < r)
        slot_p[(long)N * r + (4 * g + rr) * K + (wave * G::DAT + j) * 16 + t] = accA[j][rr];
}

// dB[n][j] += s * sum_w part_w dB[n][j],  dA[j][k] += s * sum_w part_w dA[j][k]  (j < r): the
// walker slots are [N r | r K] floats (the output's own layout), so output e sums element e of
// every slot. 8 threads per output each sum every 8th walker, then one of them adds the 8 in
// order (deterministic); 32 outputs per 256-thread workgroup.
__global__ void __launch_bounds__(256)
lora_reduce_kernel(const float* __restrict__ part, int walkers, long slot_floats, long nb,
                   float s, float* __restrict__ dA, float* __restrict__ dB,
                   const float* __restrict__ div) {
  __shared__ float red[8][33];
  const int lo = threadIdx.x & 31, wg = threadIdx.x >> 5;
  const long e = (long)blockIdx.x * 32 + lo;
  float v = 0.f;
  if (e < slot_floats) {
    int w = wg;
    for (; w + 56 < walkers; w += 64) {
      float q[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) q[u] = part[(long)(w + 8 * u) * slot_floats + e];
      v += ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
    }
    for (; w < walkers; w += 8) v += part[(long)w * slot_floats + e];
  }
  red[wg][lo] = v;
  __syncthreads();
  if (wg == 0 && e < slot_floats) {
    float tot = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) tot += red[k][lo];
    if (div) tot /= *div;  // the scaled half gradient's power of two: exact
    if (e < nb) dB[e] += s * tot;
    else dA[e - nb] += s * tot;
  }
}


// ------------------------------------------------- adapter forward + residual + LayerNorm, fused
// One launch for the adapter sub-block of a block (adapter.py:53-72, model.py:440-441) and the
// LayerNorm that reads its output next (ln_2 of the same block, or ln_1 of the next one,
// model.py:194-200):
//   h     = drop(relu(z Wd^T + bd))                (saved, bf16 [M, 64])
//   x_out = resid + z + scale * (h Wu^T + bu)      (f32, the residual stream)
//   y     = LN(x_out) * gamma + beta               (bf16, the next GEMM's A operand; mean, rstd saved)
// Separately these are two skinny GEMM launches and a LayerNorm launch that re-reads x_out
// (and z twice); here z, resid and x_out each cross HBM once. 16-row blocks; one persistent
// 8-wave workgroup per CU. Both weights live in registers as MFMA fragments: the down
// projection splits K = D over the waves (partials summed through LDS), the up projection gives
// each wave D/8 output columns of all 16 rows. The row statistics of the LayerNorm (two-pass:
// mean, then the mean of squared deviations, as ln_fwd_kernel) are summed over the waves in LDS.
// The dropout mask is drop_mul(seed, row, j) — the EPI_AD_DOWN epilogue's — so the forward is
// the separate path's, and the backward regenerates the same mask.
// Streaming: z and resid arrive by LDS-DMA. resid (the larger stream) is double-buffered and
// issued a whole block ahead, at the top of the block before; z is single-buffered and issued as
// soon as the current block's z has been read (after the down projection, whose operands and the
// epilogue's z values are read first), so both have most of a block of lead time. The only VMEM
// instructions inside a block are those DMAs and the stores, and the wait at the top of a block
// is COUNTED: the stores issued after the last DMA stay in flight while the next block computes.
// Down projection: wave w computes the 16 bottleneck columns 16 (w & 3) over the K half (w >> 2),
// so the cross-wave sum is one partial per output (4 KiB of LDS instead of eight).
template <int D, int XB = 4>  // XB: bytes per residual element (4 f32, 2 IEEE half)
struct AdLnLay {
  static constexpr int ZROW = D * 2;                 // z image row bytes
  static constexpr int ZIMG = 16 * ZROW;             // one 16-row z block
  static constexpr int ZP = ZIMG / 1024 / 8;         // z DMA pieces per wave
  static constexpr int XIMG = 16 * D * XB;           // one 16-row resid block (plain rows)
  static constexpr int XP = XIMG / 1024 / 8;         // resid DMA pieces per wave
  static constexpr int Z_OFF = 0;                    // one z buffer
  static constexpr int X_OFF = ZIMG;                 // two resid buffers
  static constexpr int PRM_OFF = X_OFF + 2 * XIMG;   // bu, gamma, beta [3][D], bd [64] f32
  static constexpr int ST_OFF = PRM_OFF + (3 * D + 64) * 4;  // [2][8][16] f32 row sums
  static constexpr int RED_OFF = ST_OFF + 2 * 8 * 16 * 4;    // [16][64] f32 down partials (K half 1)
  static constexpr int H_OFF = RED_OFF + 16 * 64 * 4;        // h block bf16 [16][64]
  // y staging over RED / H (both dead by then): [16][YSTR] bf16, rows padded by 16 B so that
  // the 16 rows of a ds_write_b64 group fall on distinct banks
  static constexpr int YSTR = D * 2 + 16;
  static constexpr int Y_OFF = RED_OFF;
  static constexpr int BYTES = RED_OFF + (16 * YSTR > 16 * 64 * 6 ? 16 * YSTR : 16 * 64 * 6);
  static constexpr int KS = D / 32 / 2;              // down-projection k-steps per wave (K half)
  static constexpr int NU = D / 8 / 16;              // up-projection 16-column tiles per wave
  static_assert(BYTES <= 160 * 1024, "LDS");
};

template <int N>
LC_DEV void vmcnt_le() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// XT: the residual stream's element type (float, or _Float16 — the reference's autocast
// residual, lc_common.h): resid in, x_out out; the LayerNorm reads x_out as stored.
template <int D, typename XT = float>
__global__ void __launch_bounds__(512, 1)
adapter_ln_fwd_kernel(int M, const bf16_t* __restrict__ z, long ldz, const bf16_t* __restrict__ Wd,
                      const float* __restrict__ bd, const bf16_t* __restrict__ Wu,
                      const float* __restrict__ bu, float scale, float keep, uint64_t seed,
                      const unsigned long long* __restrict__ seed_dev,
                      const XT* __restrict__ resid, XT* __restrict__ xout, long ldx,
                      bf16_t* __restrict__ hout, const float* __restrict__ gamma,
                      const float* __restrict__ beta, bf16_t* __restrict__ y, long ldy,
                      float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  constexpr int XB = (int)sizeof(XT);
  using L = AdLnLay<D, XB>;
  constexpr int KS = L::KS, NU = L::NU;
  __shared__ __attribute__((aligned(16))) char smem[L::BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, t = lane & 15;
  const int nd = wave & 3, kh = wave >> 2;  // down projection: column tile, K half
  const int nblk = (M + 15) / 16;
  if ((int)blockIdx.x >= nblk) return;
  if (seed_dev) seed += *seed_dev * 0xD1B54A32D192ED03ull;
  float* red = reinterpret_cast<float*>(smem + L::RED_OFF);
  bf16_t* hs = reinterpret_cast<bf16_t*>(smem + L::H_OFF);
  float* st = reinterpret_cast<float*>(smem + L::ST_OFF);
  float* prm = reinterpret_cast<float*>(smem + L::PRM_OFF);
  for (int e = tid; e < D; e += 512) {
    prm[e] = bu[e];
    prm[D + e] = gamma[e];
    prm[2 * D + e] = beta[e];
  }
  if (tid < 64) prm[3 * D + tid] = bd[tid];
  // weights as fragments (inline-asm loads: invisible to hipcc's vmcnt bookkeeping, retired
  // by the explicit wait below before any LDS-DMA is in flight)
  //   down: B[k][j] = Wd[j][k], lane (t, g): Wd row (16 nd + t), k = (kh KS + ks) 32 + 8g ..
  //   up:   B[k][j] = Wu[j][k], lane (t, g): Wu row (wave D/8 + 16 u + t), k = 32 ks + 8g ..
  bf16x8 wdf[KS], wuf[NU][2];
#pragma unroll
  for (int k = 0; k < KS; ++k)
    asm volatile("global_load_dwordx4 %0, %1, off"
                 : "=v"(wdf[k])
                 : "v"(Wd + (long)(16 * nd + t) * D + (kh * KS + k) * 32 + 8 * g));
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int k = 0; k < 2; ++k)
      asm volatile("global_load_dwordx4 %0, %1, off"
                   : "=v"(wuf[u][k])
                   : "v"(Wu + (long)(wave * (D / 8) + 16 * u + t) * 64 + 32 * k + 8 * g));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // z block b -> the z buffer: 1-KiB pieces, lane -> (row, 16-B position) inverting the 32-B
  // unit swizzle (swz_w: conflict-free row reads and 8-B epilogue reads)
  auto dma_z = [&](int b) {
    char* dst = smem + L::Z_OFF;
    const int r0 = b * 16;
#pragma unroll
    for (int pp = 0; pp < L::ZP; ++pp) {
      const int piece = wave * L::ZP + pp;
      const int idx = piece * 64 + lane;
      const int row = idx / (L::ZROW / 16), pc = idx % (L::ZROW / 16);
      const int c = (((pc >> 1) ^ swz_w(row)) << 1) | (pc & 1);
      const int m = min(r0 + row, M - 1);
      glds16(z + (long)m * ldz + c * 8, dst + piece * 1024);
    }
  };
  // resid block b -> resid buffer buf, plain row-major [16][D] (the epilogue's reads of 16 rows
  // at one column are spread by the row stride: 2-way at worst); 16-B chunks of EPC elements
  constexpr int EPC = 16 / XB;
  auto dma_x = [&](int b, int buf) {
    char* dst = smem + L::X_OFF + buf * L::XIMG;
#pragma unroll
    for (int pp = 0; pp < L::XP; ++pp) {
      const int piece = wave * L::XP + pp;
      const int idx = piece * 64 + lane;
      const int row = idx / (D / EPC), c = idx % (D / EPC);
      const int m = min(b * 16 + row, M - 1);
      glds16(resid + (long)m * ldx + c * EPC, dst + piece * 1024);
    }
  };
  const uint32_t lds0 = lds_addr(smem);
  auto zaddr = [&](int row, int byte) {  // LDS address of z image byte `byte` of row `row`
    const int u = (byte >> 5) ^ swz_w(row);
    return lds0 + L::Z_OFF + row * L::ZROW + u * 32 + (byte & 31);
  };
  // stores issued after the last DMA of a full block, per wave: h (waves 0-1), mean and rstd
  // (wave 0), then NST full-row pieces (x_out 2 rows x D x 4 B and y 2 rows x D x 2 B, 1 KiB each)
  constexpr int XPR = D * XB / 512;  // x_out pieces per wave (2 rows x D x XB bytes, 1-KiB each)
#ifdef ADLN_KO  // (the knocked-out stores are not in flight: the counted waits below stay exact)
  constexpr int NST = ((ADLN_KO & 1) ? 0 : XPR) + ((ADLN_KO & 2) ? 0 : D / 256);
#else
  constexpr int NST = XPR + D / 256;
#endif
  const int tail = NST + (wave < 2 ? 1 : 0) + (wave == 0 ? 2 : 0);

  int b = blockIdx.x;
  dma_x(b, 0);
  dma_z(b);
  __syncthreads();  // prm (no LDS-DMA waited on here: the first block's wait comes next)
  bool prev_full = false;
#pragma unroll 1
  for (int k = 0; b < nblk; ++k, b += gridDim.x) {
    const int buf = k & 1;
    const int r0 = b * 16;
    // this block's z and resid landed; the previous block's tail stores may stay in flight
    if (prev_full) {
      if (tail == NST + 3) vmcnt_le<NST + 3>();
      else if (tail == NST + 1) vmcnt_le<NST + 1>();
      else vmcnt_le<NST>();
    } else {
      vmcnt_le<0>();
    }
    lds_barrier();
    const int bn = b + gridDim.x;
    if (bn < nblk) dma_x(bn, buf ^ 1);  // the other buffer: read by the previous block only
    // ---- down projection: this wave's column tile over its K half (A = z rows t)
    f32x4 pd = f32x4{0.f, 0.f, 0.f, 0.f};
    uint2 zz[NU];
    {
      constexpr int GK = KS / 2;  // two groups of reads, the second in flight under the first's MFMAs
      bf16x8 za[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        asm volatile("ds_read_b128 %0, %1"
                     : "=v"(za[ks]) : "v"(zaddr(t, ((kh * KS + ks) * 32 + 8 * g) * 2)));
      // the epilogue's z values (row t, this wave's up-projection columns), read now so that the
      // z buffer is free for the next block's DMA after the barrier below
#pragma unroll
      for (int u = 0; u < NU; ++u)
        asm volatile("ds_read_b64 %0, %1"
                     : "=v"(zz[u]) : "v"(zaddr(t, (wave * (D / 8) + 16 * u + 4 * g) * 2)));
      asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(NU + KS - GK) : "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < GK; ++ks) pd = mfma16(za[ks], wdf[ks], pd);
      asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(NU) : "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = GK; ks < KS; ++ks) pd = mfma16(za[ks], wdf[ks], pd);
    }
    // lane holds P[m = 4g + rr][j = 16 nd + t] over K half kh
    if (kh == 1)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) red[(4 * g + rr) * 64 + 16 * nd + t] = pd[rr];
    lds_barrier();  // also: every wave's z reads are done (lgkmcnt(0) above the barrier)
    if (bn < nblk) dma_z(bn);
    if (kh == 0) {
      const int j = 16 * nd + t;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int m = 4 * g + rr;
        float v = pd[rr] + red[m * 64 + j];
        v = fmaxf(v + prm[3 * D + j], 0.f) * drop_mul(seed, (long)(r0 + m), j, keep);
        hs[m * 64 + j] = f2bf(v);
      }
    }
    lds_barrier();
    // (every LDS read from here on is inline asm: hipcc treats a plain read as possibly aliasing
    // the LDS-DMA in flight and waits vmcnt(0) first)
    const uint32_t hl = lds0 + L::H_OFF;
    if (wave < 2) {  // the h block (2 KiB, contiguous in hout) as 16-B row pieces
      const int e = tid;  // 128 pieces: row e >> 3, 8 columns (e & 7) * 8
      uint4 v;
      asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(hl + e * 16));
      lds_wait0();
      if (r0 + (e >> 3) < M) *reinterpret_cast<uint4*>(hout + (long)r0 * 64 + e * 8) = v;
    }
    // ---- up projection: rows t of the block (A = h), this wave's D/8 columns (B = Wu)
    bf16x8 ha0, ha1;
    asm volatile("ds_read_b128 %0, %1" : "=v"(ha0) : "v"(hl + (t * 64 + 8 * g) * 2));
    asm volatile("ds_read_b128 %0, %1" : "=v"(ha1) : "v"(hl + (t * 64 + 32 + 8 * g) * 2));
    f32x4 xo[NU];
    float s1 = 0.f;
    // resid of this lane's outputs from the DMA'd image
    f32x4 xr4[NU];
    uint2 xh4[NU];  // (XB == 2: the 4 halves)
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int col = wave * (D / 8) + 16 * u + 4 * g;
      if constexpr (XB == 4)
        asm volatile("ds_read_b128 %0, %1"
                     : "=v"(xr4[u]) : "v"(lds0 + L::X_OFF + buf * L::XIMG + (t * D + col) * 4));
      else
        asm volatile("ds_read_b64 %0, %1"
                     : "=v"(xh4[u]) : "v"(lds0 + L::X_OFF + buf * L::XIMG + (t * D + col) * 2));
    }
    lds_wait0();
    if constexpr (XB == 2) {
#pragma unroll
      for (int u = 0; u < NU; ++u)
        xr4[u] = f32x4{h2f(xh4[u].x & 0xffff), h2f(xh4[u].x >> 16), h2f(xh4[u].y & 0xffff),
                       h2f(xh4[u].y >> 16)};
    }
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      f32x4 acc = mfma16(wuf[u][0], ha0, f32x4{0.f, 0.f, 0.f, 0.f});
      acc = mfma16(wuf[u][1], ha1, acc);
      // lane holds U[m = t][n = col + rr], col = wave D/8 + 16u + 4g (the swapped layout)
      const int col = wave * (D / 8) + 16 * u + 4 * g;
      const float zf[4] = {bf2f(zz[u].x & 0xffff), bf2f(zz[u].x >> 16), bf2f(zz[u].y & 0xffff),
                           bf2f(zz[u].y >> 16)};
      const f32x4 xr = xr4[u];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const float v = acc[rr] + prm[col + rr];
        xo[u][rr] = xround<XT>(xr[rr] + zf[rr] + scale * v);  // the LayerNorm reads x_out as stored
        s1 += xo[u][rr];
      }
    }
    // ---- LayerNorm of the 16 rows: sums over the 4 lanes of a row, then over the waves
    s1 += __shfl_xor(s1, 16);
    s1 += __shfl_xor(s1, 32);
    if (g == 0) st[wave * 16 + t] = s1;
    lds_barrier();
    const bool live = r0 + t < M;
    // x_out and y leave as whole rows: both are staged in LDS (x_out in this block's resid
    // buffer, read for the last time above; y over the dead RED / H region) and stored after one
    // more barrier as 1-KiB contiguous pieces through descriptors over the block's rows < M.
    // Stored straight from the MFMA layout, every store instruction covered 16 rows x 64 B
    // (x_out) / 32 B (y): those stores were 45 of the kernel's 105 us (knockout builds).
    // x_out image: plain [16][D] f32 rows, 16-B chunk c of row r at chunk (c & ~7) | ((c ^ r) & 7)
    // (the 8 rows of a write group on distinct banks); y image: [16][YSTR] bf16 rows (padded).
    const uint32_t xs = lds0 + L::X_OFF + buf * L::XIMG;
    const uint32_t ys = lds0 + L::Y_OFF;
    if constexpr (XB == 4) {
      // this lane's 16-B chunk of row t for tile u: c = wave D/32 + 4u + g (wave D/32 is a
      // multiple of 8), so its swizzled position is a per-lane base for even / odd u plus u x 64 B
      static_assert((D / 32) % 8 == 0, "wave column block must be whole 128-B groups");
      const uint32_t xb = xs + t * D * 4 + wave * (D / 32) * 16;
      const uint32_t x0 = xb + ((g ^ t) & 7) * 16, x1 = xb + (((4 + g) ^ t) & 7) * 16 - 64;
#pragma unroll
      for (int u = 0; u < NU; ++u)
        asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"((u & 1) ? x1 : x0), "v"(xo[u]),
                     "n"(u * 64) : "memory");
    } else {
      // half image [16][2 D B]: 16-B chunk c of row r at (c & ~7) | ((c ^ r) & 7); this lane's
      // 8 B of tile u are half g & 1 of chunk c = wave D/64 + 2u + (g >> 1)
      const uint32_t xb = xs + t * D * 2 + (g & 1) * 8;
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int c = wave * (D / 64) + 2 * u + (g >> 1);
        const uint32_t a = xb + ((c & ~7) | ((c ^ t) & 7)) * 16;
        asm volatile("ds_write_b64 %0, %1" ::"v"(a),
                     "v"(uint2{pack2h(xo[u][0], xo[u][1]), pack2h(xo[u][2], xo[u][3])}) : "memory");
      }
    }
    float mean = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) mean += st[w * 16 + t];
    mean *= 1.0f / D;
    float s2 = 0.f;
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        xo[u][rr] -= mean;
        s2 += xo[u][rr] * xo[u][rr];
      }
    s2 += __shfl_xor(s2, 16);
    s2 += __shfl_xor(s2, 32);
    if (g == 0) st[128 + wave * 16 + t] = s2;
    lds_barrier();
    float var = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) var += st[128 + w * 16 + t];
    const float rstd = rsqrtf(var * (1.0f / D) + 1e-5f);
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int col = wave * (D / 8) + 16 * u + 4 * g;
      float o[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) o[rr] = xo[u][rr] * rstd * prm[D + col + rr] + prm[2 * D + col + rr];
      const uint2 ov = uint2{pack2bf(o[0], o[1]), pack2bf(o[2], o[3])};
      asm volatile("ds_write_b64 %0, %1 offset:%2"
                   ::"v"(ys + t * L::YSTR + (wave * (D / 8) + 4 * g) * 2), "v"(ov), "n"(u * 32)
                   : "memory");
    }
    if (live && wave == 0 && g == 0) {
      mean_out[r0 + t] = mean;
      rstd_out[r0 + t] = rstd;
    }
    lds_barrier();  // both images complete (and every st read done)
    {
      const int rows_here = min(16, M - r0);
      const __amdgpu_buffer_rsrc_t rx = lc_rsrc(xout + (long)r0 * ldx, (long)rows_here * ldx * XB);
      const __amdgpu_buffer_rsrc_t ry = lc_rsrc(y + (long)r0 * ldy, (long)rows_here * ldy * 2);
      // wave w: rows 2w, 2w + 1; f32 x_out: D / 256 pieces of 64 chunks per row (h = 0, 1); half
      // x_out: its 2 x 2 D bytes as D / 256 pieces of 1 KiB (h = 1 only); then y's 2 x 2 D bytes
      // as D / 256 pieces (h = 2) — one row (or y) at a time: few registers in flight
      constexpr int YPR = D / 256;
#pragma unroll
      for (int h = (XB == 4 ? 0 : 1); h < 3; ++h) {
        uint4 v[YPR];
#pragma unroll
        for (int j = 0; j < YPR; ++j) {
          if (h < 2 && XB == 4) {
            const int r = 2 * wave + h, c = j * 64 + lane;
            asm volatile("ds_read_b128 %0, %1"
                         : "=v"(v[j]) : "v"(xs + r * D * 4 + ((c & ~7) | ((c ^ r) & 7)) * 16));
          } else if (h < 2) {
            const int bb = j * 1024 + lane * 16, r = 2 * wave + bb / (2 * D), o = bb % (2 * D);
            const int c = o >> 4;
            asm volatile("ds_read_b128 %0, %1"
                         : "=v"(v[j]) : "v"(xs + r * D * 2 + ((c & ~7) | ((c ^ r) & 7)) * 16));
          } else {
            const int bb = j * 1024 + lane * 16, r = 2 * wave + bb / (2 * D), o = bb % (2 * D);
            asm volatile("ds_read_b128 %0, %1" : "=v"(v[j]) : "v"(ys + r * L::YSTR + o));
          }
        }
        lds_wait0();
#pragma unroll
        for (int j = 0; j < YPR; ++j) {
          const lc_u32x4 d = lc_u32x4{v[j].x, v[j].y, v[j].z, v[j].w};
          if (h < 2) {
#if !(defined(ADLN_KO) && (ADLN_KO & 1))  // (diagnostic builds: x_out stores off)
            if constexpr (XB == 4) {
              const int r = 2 * wave + h, c = j * 64 + lane;
              __builtin_amdgcn_raw_buffer_store_b128(d, rx, (int)(r * ldx * 4 + c * 16), 0, 0);
            } else {
              const int bb = j * 1024 + lane * 16, r = 2 * wave + bb / (2 * D), o = bb % (2 * D);
              __builtin_amdgcn_raw_buffer_store_b128(d, rx, (int)(r * ldx * 2 + o), 0, 0);
            }
#else
            asm volatile("" ::"v"(d));
#endif
          } else {
#if !(defined(ADLN_KO) && (ADLN_KO & 2))  // (diagnostic builds: y stores off)
            const int bb = j * 1024 + lane * 16, r = 2 * wave + bb / (2 * D), o = bb % (2 * D);
            __builtin_amdgcn_raw_buffer_store_b128(d, ry, (int)(r * ldy * 2 + o), 0, 0);
#else
            asm volatile("" ::"v"(d));
#endif
          }
        }
      }
    }
    // st is rewritten by the next block only after its first two barriers
    prev_full = r0 + 16 <= M;
  }
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
  LC_CHECK_ARG(N > 0 && K > 0 && r >= 0 && r <= MERGE_RMAX && (r == 0 || (A && B)));
  dim3 grid((K + 63) / 64, (N + 63) / 64);
  hipLaunchKernelGGL(merge_kernel, grid, dim3(256), 0, st, N, K, r, W, A, B, scaling,
                     (bf16_t*)out, (bf16_t*)outT);
  LC_LAUNCH_RET();
}

int lc_cast_weights_bf16(hipStream_t st, int n, const float* const* W, const int* N,
                         const int* K, void* const* out, void* const* outT) {
  LC_CHECK_ARG(n >= 0 && n <= LC_CAST_MAX && (n == 0 || (W && N && K && out && outT)));
  if (n == 0) return LC_OK;
  return lc_merge_weights_bf16(st, n, W, nullptr, nullptr, nullptr, nullptr, N, K, out, outT);
}

int lc_merge_weights_bf16(hipStream_t st, int n, const float* const* W, const float* const* A,
                          const float* const* B, const int* r, const float* scaling, const int* N,
                          const int* K, void* const* out, void* const* outT) {
  LC_CHECK_ARG(n >= 0 && n <= LC_CAST_MAX && (n == 0 || (W && N && K && out && outT)));
  LC_CHECK_ARG((r == nullptr) == (scaling == nullptr));
  if (n == 0) return LC_OK;
  CastBatch b{};
  int tiles = 0;
  for (int i = 0; i < n; ++i) {
    LC_CHECK_ARG(W[i] != nullptr && out[i] != nullptr && N[i] > 0 && K[i] > 0);
    const int ri = r ? r[i] : 0;
    LC_CHECK_ARG(ri >= 0 && ri <= MERGE_RMAX && (ri == 0 || (A && B && A[i] && B[i])));
    b.W[i] = W[i];
    b.A[i] = ri ? A[i] : nullptr;
    b.B[i] = ri ? B[i] : nullptr;
    b.r[i] = ri;
    b.s[i] = ri ? scaling[i] : 0.f;
    b.out[i] = static_cast<bf16_t*>(out[i]);
    b.outT[i] = static_cast<bf16_t*>(outT[i]);
    b.N[i] = N[i];
    b.K[i] = K[i];
    const int t = ((N[i] + 63) / 64) * ((K[i] + 63) / 64);
    tiles = t > tiles ? t : tiles;
  }
  hipLaunchKernelGGL(cast_batch_kernel, dim3(tiles, n), dim3(256), 0, st, b);
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

static int lora_grad_ws(hipStream_t st, int M, int N, int K, int r, const void* dY, long ldy,
                        const void* X, long ldx, const void* apad, long lda, const void* btpad,
                        long ldbt, float scaling, float* dA, float* dB, void* ws, long ws_bytes,
                        const float* div) {
  LC_CHECK_ARG(M > 0 && r >= 1 && r <= 4 && dY && X && apad && btpad && dA && dB && ws);
  LC_CHECK_ARG(ldy % 8 == 0 && ldx % 8 == 0 && lda % 8 == 0 && ldbt % 8 == 0);
  LC_CHECK_ARG(ldy >= N && ldx >= K && lda >= K && ldbt >= N);
  const int nblk = (M + 31) / 32;
  int walkers = 0;
  {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    walkers = nblk < cus ? nblk : cus;
  }
  const long slot = (long)N * r + (long)r * K;
  LC_CHECK_ARG(ws_bytes >= LC_SPLITK_TICKET_BYTES + (long)walkers * slot * 4);
  float* part = reinterpret_cast<float*>(static_cast<char*>(ws) + LC_SPLITK_TICKET_BYTES);
#define LC_LG(KT, NC)                                                                           \
  if (K == KT * 32 && N == NC * 128) {                                                         \
    hipLaunchKernelGGL((lora_grad1p_kernel<KT, NC>), dim3(walkers), dim3(512), 0, st, M,        \
                       (const bf16_t*)X, ldx, (const bf16_t*)dY, ldy, (const bf16_t*)apad, lda, \
                       (const bf16_t*)btpad, ldbt, part, walkers, r);                          \
  } else
  LC_LG(24, 18) LC_LG(24, 6) LC_LG(16, 12) LC_LG(16, 4)
  { return LC_EINVAL; }
#undef LC_LG
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return LC_ELAUNCH;
  hipLaunchKernelGGL(lora_reduce_kernel, dim3((unsigned)((slot + 31) / 32)), dim3(256), 0, st,
                     part, walkers, slot, (long)N * r, scaling, dA, dB, div);
  LC_LAUNCH_RET();
}

int lc_lora_grad_ws(hipStream_t st, int M, int N, int K, int r, const void* dY, long ldy,
                    const void* X, long ldx, const void* apad, long lda, const void* btpad,
                    long ldbt, float scaling, float* dA, float* dB, void* ws, long ws_bytes) {
  return lora_grad_ws(st, M, N, K, r, dY, ldy, X, ldx, apad, lda, btpad, ldbt, scaling, dA, dB, ws,
                      ws_bytes, nullptr);
}

#ifndef LC_F16  // the image tower's half residual gradient (bf16 storage build only)
int lc_lora_grad_ws_unscaled(hipStream_t st, int M, int N, int K, int r, const void* dY, long ldy,
                             const void* X, long ldx, const void* apad, long lda,
                             const void* btpad, long ldbt, float scaling, float* dA, float* dB,
                             void* ws, long ws_bytes, const float* gscale) {
  LC_CHECK_ARG(gscale != nullptr);
  return lora_grad_ws(st, M, N, K, r, dY, ldy, X, ldx, apad, lda, btpad, ldbt, scaling, dA, dB, ws,
                      ws_bytes, gscale);
}
#endif

// The adapter as two skinny GEMMs through lc_gemm_nt's LDS-staged MFMA template (the weights
// are staged once per workgroup by global_load_lds instead of being re-read by every wave):
//   h    = drop(relu(z Wd^T + bd))                 [M,64]  N = 64,  K = D
//   xout = resid + z + scale * (h Wu^T + bu)       [M,D]   N = D,   K = 64
int lc_adapter_fwd(hipStream_t st, int M, int D, const void* z, long ldz, const void* Wd,
                   const float* bd, const void* Wu, const float* bu, float scale, float keep,
                   unsigned long long seed, const unsigned long long* seed_dev,
                   const float* resid, float* xout, long ldx, void* hout) {
  LC_CHECK_ARG(M > 0 && D % 64 == 0 && ldz % 8 == 0 && ldx % 4 == 0);
  LC_CHECK_ARG(keep > 0.f && keep <= 1.f);
  EpiParams ep{z, ldz, scale, keep, (uint64_t)seed, nullptr, seed_dev};
  int rc = lc_gemm_nt_ex(st, 8 /*EPI_AD_DOWN*/, M, AD_H, D, z, ldz, Wd, D, bd, 1.0f, hout, AD_H,
                         nullptr, 0, nullptr, 0, ep);
  if (rc) return rc;
  return lc_gemm_nt_ex(st, 9 /*EPI_AD_UP*/, M, D, AD_H, hout, AD_H, Wu, AD_H, bu, 1.0f, xout, ldx,
                       nullptr, 0, resid, ldx, ep);
}

static int adapter_ln_fwd(hipStream_t st, int M, int D, const void* z, long ldz, const void* Wd,
                          const float* bd, const void* Wu, const float* bu, float scale,
                          float keep, unsigned long long seed,
                          const unsigned long long* seed_dev, const void* resid, void* xout,
                          long ldx, void* hout, const float* gamma, const float* beta, void* y,
                          long ldy, float* mean, float* rstd, int x16) {
  const int xb = x16 ? 2 : 4;
  LC_CHECK_ARG(M > 0 && (D == 768 || D == 512) && ldz % 8 == 0 && ldx % (16 / xb) == 0 &&
               ldy % 8 == 0);
  // x_out / y leave as 16-B pieces through descriptors over a 16-row block (32-bit offsets)
  LC_CHECK_ARG(ldx < (1L << 24) && ldy < (1L << 24));
  LC_CHECK_ARG(((uintptr_t)xout & 15) == 0 && ((uintptr_t)y & 15) == 0 &&
               ((uintptr_t)resid & 15) == 0);
  LC_CHECK_ARG(ldz >= D && ldx >= D && ldy >= D && keep > 0.f && keep <= 1.f);
  LC_CHECK_ARG(z && Wd && bd && Wu && bu && resid && xout && hout && gamma && beta && y && mean && rstd);
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  const int nblk = (M + 15) / 16;
  const int grid = nblk < cus ? nblk : cus;
#define LC_ALN(DD, XT)                                                                           \
  hipLaunchKernelGGL((adapter_ln_fwd_kernel<DD, XT>), dim3(grid), dim3(512), 0, st, M,           \
                     (const bf16_t*)z, ldz, (const bf16_t*)Wd, bd, (const bf16_t*)Wu, bu, scale,  \
                     keep, (uint64_t)seed, seed_dev, (const XT*)resid, (XT*)xout, ldx,           \
                     (bf16_t*)hout, gamma, beta, (bf16_t*)y, ldy, mean, rstd)
  if (x16) {
    if (D == 768) LC_ALN(768, _Float16);
    else LC_ALN(512, _Float16);
  } else {
    if (D == 768) LC_ALN(768, float);
    else LC_ALN(512, float);
  }
#undef LC_ALN
  LC_LAUNCH_RET();
}

int lc_adapter_ln_fwd(hipStream_t st, int M, int D, const void* z, long ldz, const void* Wd,
                      const float* bd, const void* Wu, const float* bu, float scale, float keep,
                      unsigned long long seed, const unsigned long long* seed_dev,
                      const float* resid, float* xout, long ldx, void* hout,
                      const float* gamma, const float* beta, void* y, long ldy, float* mean,
                      float* rstd) {
  return adapter_ln_fwd(st, M, D, z, ldz, Wd, bd, Wu, bu, scale, keep, seed, seed_dev, resid, xout,
                        ldx, hout, gamma, beta, y, ldy, mean, rstd, 0);
}

#ifndef LC_F16  // the image tower's half residual stream (bf16 storage build only)
int lc_adapter_ln_fwd_x16(hipStream_t st, int M, int D, const void* z, long ldz, const void* Wd,
                          const float* bd, const void* Wu, const float* bu, float scale,
                          float keep, unsigned long long seed,
                          const unsigned long long* seed_dev, const void* resid, void* xout,
                          long ldx, void* hout, const float* gamma, const float* beta, void* y,
                          long ldy, float* mean, float* rstd) {
  return adapter_ln_fwd(st, M, D, z, ldz, Wd, bd, Wu, bu, scale, keep, seed, seed_dev, resid, xout,
                        ldx, hout, gamma, beta, y, ldy, mean, rstd, 1);
}
#endif

static int g_adapter_bwd_fused = 1;

int lc_adapter_bwd_set_form(int fused) {
  g_adapter_bwd_fused = fused != 0;
  return LC_OK;
}

//   dpre = (h > 0) ? scale * (gout Wu) / keep : 0    [M,64]  N = 64, K = D   (B = Wu^T)
//   dz   = gout + dpre Wd                            [M,D]   N = D,  K = 64  (B = Wd^T)
#ifndef LC_F16
// gout IEEE half (the image tower's half residual gradient), everything else bf16: the
// row-block kernel reading gout directly (any M; dz may be NULL: dpre only)
int lc_adapter_bwd_g16(hipStream_t st, int M, int D, const void* gout, long ldg, const void* h,
                       const void* WuT, const void* WdT, float scale, float keep, void* dpre,
                       void* dz, long ldz) {
  LC_CHECK_ARG(M > 0 && (D == 768 || D == 512) && ldg % 8 == 0 && ldz % 8 == 0);
  LC_CHECK_ARG(keep > 0.f && keep <= 1.f);
  LC_CHECK_ARG(((uintptr_t)gout & 15) == 0 && ((uintptr_t)h & 15) == 0 &&
               ((uintptr_t)WuT & 15) == 0 && ((uintptr_t)WdT & 15) == 0 &&
               (dz == nullptr || ((uintptr_t)dz & 15) == 0));
  const int nb = (M + AD_R - 1) / AD_R;
  const dim3 grid(nb < ad_cu_count() ? nb : ad_cu_count()), block(64 * AD_NW);
  auto G = static_cast<const bf16_t*>(gout);
  auto H = static_cast<const bf16_t*>(h);
  auto U = static_cast<const bf16_t*>(WuT);
  auto Wd = static_cast<const bf16_t*>(WdT);
  auto P = static_cast<bf16_t*>(dpre);
  auto Z = static_cast<bf16_t*>(dz);
#define LC_ADB(ND, DZ)                                                                            \
  hipLaunchKernelGGL((adapter_bwd_fused_kernel<ND, DZ, true>), grid, block, 0, st, M, G, ldg, H,  \
                     U, Wd, scale, keep, P, Z, ldz)
  if (D == 768) {
    if (dz) LC_ADB(12, true);
    else LC_ADB(12, false);
  } else {
    if (dz) LC_ADB(8, true);
    else LC_ADB(8, false);
  }
#undef LC_ADB
  LC_LAUNCH_RET();
}
#endif

int lc_adapter_bwd(hipStream_t st, int M, int D, const void* gout, long ldg, const void* h,
                   const void* WuT, const void* WdT, float scale, float keep, void* dpre,
                   void* dz, long ldz) {
  LC_CHECK_ARG(M > 0 && D % 64 == 0 && ldg % 8 == 0 && ldz % 8 == 0);
  LC_CHECK_ARG(keep > 0.f && keep <= 1.f);
  // one-pass row-block kernel at the towers' widths (lc_adapter_bwd_set_form(0): the two-GEMM
  // form, which the tests compare it with)
  const bool fused = g_adapter_bwd_fused != 0;
  // (dpre alone stays on the GEMM: 17.6 vs 22.8 us standalone; with dz 40.4 vs 44.9 us)
  if (fused && dz != nullptr && (D == 768 || D == 512) && M >= 1024 && ((uintptr_t)gout & 15) == 0 &&
      ((uintptr_t)h & 15) == 0 && ((uintptr_t)WuT & 15) == 0 && ((uintptr_t)WdT & 15) == 0) {
    const int nb = (M + AD_R - 1) / AD_R;
    const dim3 grid(nb < ad_cu_count() ? nb : ad_cu_count()), block(64 * AD_NW);
    auto G = static_cast<const bf16_t*>(gout);
    auto H = static_cast<const bf16_t*>(h);
    auto U = static_cast<const bf16_t*>(WuT);
    auto Wd = static_cast<const bf16_t*>(WdT);
    auto P = static_cast<bf16_t*>(dpre);
    auto Z = static_cast<bf16_t*>(dz);
#define LC_ADB(ND, DZ)                                                                            \
  hipLaunchKernelGGL((adapter_bwd_fused_kernel<ND, DZ>), grid, block, 0, st, M, G, ldg, H, U, Wd, \
                     scale, keep, P, Z, ldz)
    if (D == 768) LC_ADB(12, true);
    else LC_ADB(8, true);
#undef LC_ADB
    LC_LAUNCH_RET();
  }
  EpiParams ep{nullptr, 0, scale, keep, 0, nullptr};
  int rc = lc_gemm_nt_ex(st, 10 /*EPI_AD_MASK*/, M, AD_H, D, gout, ldg, WuT, D, nullptr, scale, dpre,
                         AD_H, nullptr, 0, h, AD_H, ep);
  if (rc) return rc;
  if (dz == nullptr) return LC_OK;  // dpre only (the input gradient is not needed)
  return lc_gemm_nt_ex(st, 11 /*EPI_AD_ADD*/, M, D, AD_H, dpre, AD_H, WdT, AD_H, nullptr, 1.0f, dz,
                       ldz, nullptr, 0, gout, ldg, ep);
}

int lc_check_finite(hipStream_t st, long n, const float* g, int* flag) {
  LC_CHECK_ARG(n >= 0);
  if (n == 0) return LC_OK;
  hipLaunchKernelGGL(finite_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, n, g, flag);
  LC_LAUNCH_RET();
}

int lc_adamw(hipStream_t st, long n, float* p, const float* g, float* m, float* v, float lr,
             float b1, float b2, float eps, float wd, int step, const int* skip,
             const long long* step_dev) {
  LC_CHECK_ARG(n >= 0 && (step >= 1 || step_dev != nullptr));
  if (n == 0) return LC_OK;
  const float fs = (float)(step >= 1 ? step : 1);
  const float bc1 = 1.0f - powf(b1, fs), bc2 = 1.0f - powf(b2, fs);
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, n, p, g, m, v, lr, b1,
                     b2, eps, wd, bc1, bc2, skip, step_dev);
  LC_LAUNCH_RET();
}

int lc_counter_add(hipStream_t st, int n, long long* ctr, long long delta) {
  LC_CHECK_ARG(n > 0 && n <= 64 && ctr != nullptr);
  hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(64), 0, st, n, ctr, delta);
  LC_LAUNCH_RET();
}

int lc_adam_step_advance(hipStream_t st, long long* ctr, const int* skip) {
  LC_CHECK_ARG(ctr != nullptr);
  hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(64), 0, st, ctr, skip);
  LC_LAUNCH_RET();
}

}  // extern "C"
