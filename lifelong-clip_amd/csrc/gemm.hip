// bf16 MFMA GEMMs for the CLIP PEFT step on gfx950.
//
//  lc_gemm_nt : C[M,N] = A[M,K] . B[N,K]^T (+bias) with a fused epilogue. Both operands are
//               K-contiguous: activations [rows, features] and nn.Linear weights [out, in]
//               (models/clip/model.py:219-222, lora.py:837/1072). The backward dX GEMMs use a
//               transposed copy of each frozen weight kept resident in HBM, so every GEMM of
//               the step (fwd and dX) runs through this one NT kernel.
//  lc_gemm_tn : C[N1,N2] += alpha * A[M,N1]^T . B[M,N2], reduction over the M = batch*tokens
//               rows, split over M across workgroups (PEFT weight gradients: adapter
//               down/up, adapter.py:38-40).
//
// Tiling (NT): BM x BN x 64 block tile, 256 threads = 4 waves in a WM x WN grid, 16x16x32
// bf16 MFMA. The MFMA is issued "swapped" (A-operand = weight rows, B-operand = activation
// rows) so each lane's accumulator holds 4 consecutive output columns of one row: epilogue
// stores are 8 B (bf16) / 16 B (f32) per lane. Tiles are staged global->LDS with
// global_load_lds_dwordx4 into a lane-linear image; bank conflicts of the ds_read_b128 fragment
// reads are removed by an XOR swizzle applied to the per-lane SOURCE chunk (chunk ^ ((row>>1)&7))
// and to the read address. Two LDS buffers: the next K-tile's DMA overlaps this tile's MFMAs.
// Grid: one workgroup per output tile, XCD-aware bijective remap so that the tiles an XCD
// runs are contiguous in (m, n) order and share A row-panels in its L2.
#include "lc_common.h"
#include <stdlib.h>
#include <type_traits>

enum {
  EPI_BF16 = 0,        // out0 bf16 = acc*alpha + bias
  EPI_F32 = 1,         // out0 f32  = acc*alpha + bias
  EPI_RESID = 2,       // out0 f32  = aux_f32 + acc*alpha + bias          (residual add)
  EPI_GELU = 3,        // out0 bf16 = pre = acc+bias ; out1 bf16 = quick_gelu(pre)
  EPI_GELU_BWD = 4,    // out0 bf16 = (acc*alpha) * quick_gelu'(aux_bf16)
  EPI_BF16_F32 = 5,    // out0 bf16 and out1 f32 of acc*alpha + bias
  EPI_GELU_D = 6,      // out0 bf16 = quick_gelu'(pre) ; out1 bf16 = quick_gelu(pre), pre = acc+bias
  EPI_MUL = 7,         // out0 bf16 = (acc*alpha) * aux_bf16
  // fused adapter epilogues (internal; adapter.py:59-72 as two skinny GEMMs)
  EPI_AD_DOWN = 8,     // out0 bf16 = relu(acc + bias) * dropmask(seed, m, n) / keep
  EPI_AD_UP = 9,       // out0 f32 = aux_f32 + aux2_bf16 + scale * (acc + bias)
  EPI_AD_MASK = 10,    // out0 bf16 = aux_bf16 > 0 ? alpha * acc / keep : 0
  EPI_AD_ADD = 11,     // out0 bf16 = aux_bf16 + acc
  // fp8-output epilogues of the fp8 GEMM (MaPLe's fp8 mode): out1 = e4m3 codes (ldo1 in bytes)
  // + E8M0 scales (ep.q_scale, ep.q_rows) of the bf16-rounded value, bit-identical to the bf16
  // epilogue followed by quant_fp8 (quant.hip) — the next fp8 GEMM's A operand straight from here
  EPI_GELU_D_Q8 = 12,  // out0 bf16 = quick_gelu'(pre) ; out1 fp8 = quick_gelu(pre), pre = acc+bias
  EPI_MUL_Q8 = 13,     // out1 fp8 = (acc*alpha) * aux_bf16 (out0 unused)
  // the half residual stream (lc_common.h xres): out0 half = aux_half + acc*alpha + bias
  EPI_RESID16 = 14,
};

namespace {

constexpr int BK = 64;


LC_DEV int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// Tile raster of the 256x256 GEMMs: linear tile index -> (row panel tm, column tile tn), in groups
// of gm row panels walked column-major inside the group, so that the workgroups one XCD runs at
// once (a contiguous index range, see the XCD remap) share a few B column slices across gm
// A panels instead of all of B across ~tiles/XCD / tiles_n panels (B = the weight, 4.7 MB at
// N = 3072, K = 768, more than one XCD's 4 MB L2). gm <= 1: row-major.
LC_DEV void tile_coords(int tile, int tiles_m, int tiles_n, int gm, int& tm, int& tn) {
  if (gm <= 1) {
    tm = tile / tiles_n;
    tn = tile % tiles_n;
    return;
  }
  const int per = gm * tiles_n;
  const int grp = tile / per, idx = tile % per;
  const int rows = min(gm, tiles_m - grp * gm);
  tm = grp * gm + idx % rows;
  tn = idx / rows;
}

template <int ROWS, int NW>
LC_DEV void stage_tile(const bf16_t* __restrict__ g, long ld, int row0, int rows_valid, int k0,
                       char* lds, int tid) {
  // ROWS x 64 bf16 tile = ROWS*128 bytes; one wave-instruction moves 8 rows (1 KiB).
  constexpr int INSTR = ROWS / 8 / NW;  // per wave
  static_assert(INSTR * 8 * NW == ROWS, "tile rows must split evenly over the waves");
  const int wave = tid >> 6, lane = tid & 63;
#pragma unroll
  for (int i = 0; i < INSTR; ++i) {
    int r = (wave * INSTR + i) * 8 + (lane >> 3);
    int p = lane & 7;
    int c = swz(r, p);  // global chunk that lands at LDS position p of row r
    int gr = row0 + r;
    gr = gr < rows_valid ? gr : rows_valid - 1;  // clamp: tail rows are computed, never stored
    const bf16_t* src = g + (long)gr * ld + k0 + c * 8;
    glds16(src, lds + (wave * INSTR + i) * 1024);
  }
}

LC_DEV bf16x8 read_frag(const char* lds, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(lds + row * 128 + swz(row, chunk) * 16);
}

template <int N>
LC_DEV void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Epilogue shared by the GEMM kernels: acc holds the swapped MFMA layout (lane: 4 consecutive
// columns n of one row m per 16x16 subtile).
template <int BM, int BN, int WM, int WN, int EPI, int PASS_MAX = 32, int TM, int TN>
LC_DEV void store_tile(f32x4 (&acc)[TM][TN], char* smem, int smem_bytes, int m0, int n0, int M,
                       const float* __restrict__ bias, float alpha, void* __restrict__ out0,
                       long ldo0, void* __restrict__ out1, long ldo1, const void* __restrict__ aux,
                       long ldaux, const EpiParams& ep, int tid = -1) {
  // tid: the caller's (opaque) thread id, so that a caller looping over tiles recomputes the
  // lane-dependent addresses per tile instead of keeping them live (default: threadIdx.x)
  if (tid < 0) tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  constexpr int NW = WM * WN;
#if defined(G8_NOSTORE) && G8_NOSTORE == 1  // diagnostic builds only: epilogue off (results wrong)
  if (ep.dbg == nullptr) return;
#endif
  // Through LDS. The swapped MFMA leaves 4 consecutive columns of one row per lane, so
  // a direct store would touch 16 rows x 64 B per instruction. Each wave instead parks 32 rows
  // of its accumulator tile in the (now idle) stage ring and reads them back row-contiguous:
  // every global load/store of the epilogue covers whole 256-B row segments.
  constexpr int WT_M = BM / WM, WT_N = BN / WN;
  constexpr int PASS = (WT_M % PASS_MAX == 0) ? PASS_MAX : 16;
  constexpr int LSTR = WT_N + 4;          // floats per staged row (pad: bank spread)
  // columns per lane on the read-back: 8 when every output is bf16 (one 16-B store per lane and
  // output: half the store instructions of 4 columns — the epilogue tail is store-issue bound),
  // 4 when an output is f32 (already 16 B per lane)
  constexpr bool F32OUT = (EPI == EPI_F32 || EPI == EPI_RESID || EPI == EPI_BF16_F32 ||
                           EPI == EPI_AD_UP);
  constexpr int CPL = F32OUT ? 4 : 8;
  constexpr int NQ = CPL / 4;             // float4 groups per lane
  constexpr int LPR = WT_N / CPL;         // lanes per row
  constexpr int RPI = 64 / LPR;           // rows per read-back instruction
  (void)smem_bytes;
  float* stg = reinterpret_cast<float*>(smem) + wave * PASS * LSTR;
  const int lc = (lane % LPR) * CPL;
  const int n = n0 + wn * WT_N + lc;
  float bb[CPL];
#pragma unroll
  for (int q = 0; q < CPL; ++q) bb[q] = 0.f;
  if (EPI != EPI_GELU_BWD && EPI != EPI_MUL && EPI != EPI_AD_MASK && EPI != EPI_AD_ADD &&
      EPI != EPI_MUL_Q8 && bias != nullptr) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const float4 b4 = *reinterpret_cast<const float4*>(bias + n + 4 * q);
      bb[4 * q] = b4.x, bb[4 * q + 1] = b4.y, bb[4 * q + 2] = b4.z, bb[4 * q + 3] = b4.w;
    }
  }
  // side inputs (residual / pre-activation / adapter z / h) of a pass are fetched one pass
  // ahead, before the stores of the current pass: CDNA's vmcnt also counts stores, so a load
  // issued after them would wait for their acknowledgement.
  constexpr bool AUXF = (EPI == EPI_RESID || EPI == EPI_AD_UP);
  constexpr bool AUXB = (EPI == EPI_GELU_BWD || EPI == EPI_MUL || EPI == EPI_AD_MASK ||
                         EPI == EPI_AD_ADD || EPI == EPI_MUL_Q8 || EPI == EPI_RESID16);
  constexpr bool AUX2 = (EPI == EPI_AD_UP);
  constexpr int NIT = PASS / RPI;
  float pf_f[2][NIT][CPL];
  uint32_t pf_b[2][NIT][CPL / 2];
  auto prefetch = [&](int pass, int slot) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      long m = m0 + wm * WT_M + pass * PASS + it * RPI + lane / LPR;
      m = m < M ? m : M - 1;
      if constexpr (AUXF) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          // side inputs are read once: nontemporal (step +0.5 %, profiles/r02/epilogue_knockout.txt)
          const f32x4 fv = __builtin_nontemporal_load(
              reinterpret_cast<const f32x4*>((const float*)aux + m * ldaux + n + 4 * q));
          const float4 f = make_float4(fv[0], fv[1], fv[2], fv[3]);
          pf_f[slot][it][4 * q] = f.x, pf_f[slot][it][4 * q + 1] = f.y;
          pf_f[slot][it][4 * q + 2] = f.z, pf_f[slot][it][4 * q + 3] = f.w;
        }
      }
      if constexpr (AUXB || AUX2) {
        const bf16_t* bsrc = AUXB ? (const bf16_t*)aux + m * ldaux + n
                                  : (const bf16_t*)ep.aux2 + m * ep.ldaux2 + n;
        if constexpr (CPL == 8) {
          const i32x4 uv = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(bsrc));
          const uint4 u = make_uint4(uv[0], uv[1], uv[2], uv[3]);
          pf_b[slot][it][0] = u.x, pf_b[slot][it][1] = u.y, pf_b[slot][it][2] = u.z, pf_b[slot][it][3] = u.w;
        } else {
          const uint2 u = *reinterpret_cast<const uint2*>(bsrc);
          pf_b[slot][it][0] = u.x, pf_b[slot][it][1] = u.y;
        }
      }
    }
  };
  // one lane's CPL outputs of row m: a single 8-B / 16-B bf16 store, or NQ 16-B f32 stores,
  // through a descriptor over this tile's rows < M (rows past M dropped by the range check: no
  // row-guard branch, so hipcc keeps the stores in flight instead of draining them with
  // vmcnt(0) at every row group — 16 store-latency waits per 256x256 tile before)
  const int rows_here = (M - m0) < BM ? (M - m0) : BM;
  auto tile_rsrc = [&](void* base, long ld, int esize) {
    return lc_rsrc(static_cast<char*>(base) + (long)m0 * ld * esize, (long)rows_here * ld * esize);
  };
  auto store_bf = [&](const __amdgpu_buffer_rsrc_t& rs, long ld, long m, const float (&w)[CPL]) {
    const int off = (int)(((m - m0) * ld + n) * 2);
    if constexpr (CPL == 8)  // nontemporal (aux 2): the consumer is the next kernel
      __builtin_amdgcn_raw_buffer_store_b128(
          lc_u32x4{pack2bf(w[0], w[1]), pack2bf(w[2], w[3]), pack2bf(w[4], w[5]), pack2bf(w[6], w[7])},
          rs, off, 0, 2);
    else
      __builtin_amdgcn_raw_buffer_store_b64(lc_u32x2{pack2bf(w[0], w[1]), pack2bf(w[2], w[3])}, rs,
                                            off, 0, 0);
  };
  auto store_f = [&](const __amdgpu_buffer_rsrc_t& rs, long ld, long m, const float (&w)[CPL]) {
    const int off = (int)(((m - m0) * ld + n) * 4);
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(lc_u32x4, f32x4{w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]}),
          rs, off + 16 * q, 0, 0);
  };
  constexpr bool OUT0_F = (EPI == EPI_F32 || EPI == EPI_RESID || EPI == EPI_AD_UP);
  constexpr bool HAS_OUT1 = (EPI == EPI_GELU || EPI == EPI_BF16_F32 || EPI == EPI_GELU_D);
  constexpr bool Q8OUT = (EPI == EPI_GELU_D_Q8 || EPI == EPI_MUL_Q8);
  // (descriptors of absent outputs are built from their null pointer and never used; the fp8
  // outputs' ldo1 is in bytes)
  const __amdgpu_buffer_rsrc_t rs0 = tile_rsrc(EPI != EPI_MUL_Q8 ? out0 : nullptr, ldo0, OUT0_F ? 4 : 2);
  const __amdgpu_buffer_rsrc_t rs1 = tile_rsrc(HAS_OUT1 || Q8OUT ? out1 : nullptr,
                                               HAS_OUT1 || Q8OUT ? ldo1 : 0,
                                               EPI == EPI_BF16_F32 ? 4 : (Q8OUT ? 1 : 2));
  // one lane's 8 outputs of row m as e4m3 in the fp8 operand format: the 4 lanes of a 32-column
  // block (consecutive, 4-aligned: LPR is a multiple of 4) share one E8M0 scale; the arithmetic
  // is quant_fp8_kernel's on the bf16-rounded values. All 4 lanes of a block hold the same row
  // (every lane is active: rows >= M are dropped by the descriptor, not skipped).
  auto store_q8 = [&](void*, long ld, long m, const float (&w)[CPL]) {
    if constexpr (CPL == 8) {  // every fp8-output epilogue (no f32 output)
      float q[8];
      uint32_t amax = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        q[i] = bf2f(f2bf(w[i]));
        amax = lc_amax_bits(amax, q[i]);
      }
      amax = max(amax, (uint32_t)__shfl_xor((int)amax, 1));
      amax = max(amax, (uint32_t)__shfl_xor((int)amax, 2));
      const uint32_t byte = e8m0_of_bits(amax);
      const float inv = e8m0_inv(byte);
      // codes through the tile descriptor (rows >= M dropped); the scale byte from all 4 lanes
      // of the block (the same value to the same address; rows up to the tile end stay inside
      // the 256-row-padded scale array) — no branch, like the bf16 stores
      __builtin_amdgcn_raw_buffer_store_b64(
          lc_u32x2{pack4_fp8(q[0] * inv, q[1] * inv, q[2] * inv, q[3] * inv),
                   pack4_fp8(q[4] * inv, q[5] * inv, q[6] * inv, q[7] * inv)},
          rs1, (int)((m - m0) * ld + n), 0, 0);
      ep.q_scale[fp8_scale_index(m, n >> 5, ep.q_rows)] = (uint8_t)byte;
    }
  };
  // bf16 element i of a lane's packed side input (hfv: IEEE half, the half residual stream)
  auto bfv = [](const uint32_t* x, int i) { return bf2f((i & 1) ? (x[i >> 1] >> 16) : (x[i >> 1] & 0xffff)); };
  auto hfv = [](const uint32_t* x, int i) { return h2f((i & 1) ? (x[i >> 1] >> 16) : (x[i >> 1] & 0xffff)); };
  if constexpr (AUXF || AUXB) prefetch(0, 0);
  uint64_t seed = ep.seed;
  if constexpr (EPI == EPI_AD_DOWN)
    if (ep.seed_dev) seed += *ep.seed_dev * 0xD1B54A32D192ED03ull;
#pragma unroll
  for (int pass = 0; pass < WT_M / PASS; ++pass) {
#pragma unroll
    for (int ii = 0; ii < PASS / 16; ++ii)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        *reinterpret_cast<f32x4*>(stg + (ii * 16 + (lane & 15)) * LSTR + j * 16 + (lane >> 4) * 4) =
            acc[pass * (PASS / 16) + ii][j];
    if constexpr (AUXF || AUXB)
      if (pass + 1 < WT_M / PASS) prefetch(pass + 1, (pass + 1) & 1);
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int lr = it * RPI + lane / LPR;
      const long m = m0 + wm * WT_M + pass * PASS + lr;
      float v[CPL];
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const f32x4 a4 = *reinterpret_cast<const f32x4*>(stg + lr * LSTR + lc + 4 * q);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[4 * q + r] = a4[r] * alpha + bb[4 * q + r];
      }
      const float* xf = pf_f[pass & 1][it];
      const uint32_t* xb = pf_b[pass & 1][it];
#if defined(G8_NOSTORE) && G8_NOSTORE == 2  // diagnostic builds only: global stores off
      if (ep.dbg == nullptr) continue;
#endif
      float w[CPL];
      if constexpr (EPI == EPI_BF16 || EPI == EPI_BF16_F32) {
        store_bf(rs0, ldo0, m, v);
        if constexpr (EPI == EPI_BF16_F32) store_f(rs1, ldo1, m, v);
      } else if constexpr (EPI == EPI_F32) {
        store_f(rs0, ldo0, m, v);
      } else if constexpr (EPI == EPI_RESID) {
#pragma unroll
        for (int i = 0; i < CPL; ++i) w[i] = xf[i] + v[i];
        store_f(rs0, ldo0, m, w);
      } else if constexpr (EPI == EPI_RESID16) {
        static_assert(CPL == 8, "8 halves (16 B) per lane");
#pragma unroll
        for (int i = 0; i < CPL; ++i) w[i] = hfv(xb, i) + v[i];
        // temporal: the next LayerNorm reads it at once, the backward later
        __builtin_amdgcn_raw_buffer_store_b128(
            lc_u32x4{pack2h(w[0], w[1]), pack2h(w[2], w[3]), pack2h(w[4], w[5]), pack2h(w[6], w[7])},
            rs0, (int)(((m - m0) * ldo0 + n) * 2), 0, 0);
      } else if constexpr (EPI == EPI_GELU) {
        store_bf(rs0, ldo0, m, v);
#pragma unroll
        for (int i = 0; i < CPL; ++i) w[i] = quick_gelu(v[i]);
        store_bf(rs1, ldo1, m, w);
      } else if constexpr (EPI == EPI_GELU_BWD) {
#pragma unroll
        for (int i = 0; i < CPL; ++i) w[i] = v[i] * quick_gelu_grad(bfv(xb, i));
        store_bf(rs0, ldo0, m, w);
      } else if constexpr (EPI == EPI_GELU_D || EPI == EPI_GELU_D_Q8) {
#pragma unroll
        for (int i = 0; i < CPL; ++i) {
          const float sg = lc_sigmoid1702(v[i]);
          w[i] = v[i] * sg;                                            // QuickGELU
          v[i] = sg * __builtin_fmaf(1.702f * v[i], 1.0f - sg, 1.0f);  // QuickGELU'
        }
        store_bf(rs0, ldo0, m, v);
        if constexpr (EPI == EPI_GELU_D_Q8)
          store_q8(out1, ldo1, m, w);
        else
          store_bf(rs1, ldo1, m, w);
      } else if constexpr (EPI == EPI_MUL || EPI == EPI_MUL_Q8) {
#pragma unroll
        for (int i = 0; i < CPL; ++i) w[i] = v[i] * bfv(xb, i);
        if constexpr (EPI == EPI_MUL_Q8)
          store_q8(out1, ldo1, m, w);
        else
          store_bf(rs0, ldo0, m, w);
      } else if constexpr (EPI == EPI_AD_DOWN) {
#pragma unroll
        for (int i = 0; i < CPL; ++i) w[i] = fmaxf(v[i], 0.f) * drop_mul(seed, m, n + i, ep.keep);
        store_bf(rs0, ldo0, m, w);
      } else if constexpr (EPI == EPI_AD_UP) {
#pragma unroll
        for (int i = 0; i < CPL; ++i) w[i] = xf[i] + bfv(xb, i) + ep.scale * v[i];
        store_f(rs0, ldo0, m, w);
      } else if constexpr (EPI == EPI_AD_MASK) {
        const float inv = 1.0f / ep.keep;
#pragma unroll
        for (int i = 0; i < CPL; ++i) w[i] = bfv(xb, i) > 0.f ? v[i] * inv : 0.f;
        store_bf(rs0, ldo0, m, w);
      } else if constexpr (EPI == EPI_AD_ADD) {
#pragma unroll
        for (int i = 0; i < CPL; ++i) w[i] = bfv(xb, i) + v[i];
        store_bf(rs0, ldo0, m, w);
      }
    }
  }
}

// BM x BN block tile, WM x WN waves, STAGES-deep LDS ring filled by global_load_lds.
// Loop body per K-tile t: issue the DMA of tile t+STAGES-1, read fragments of tile t from LDS,
// MFMA cluster under s_setprio(1), then a COUNTED vmcnt (tile t+1 has landed, later tiles stay
// in flight) and a raw s_barrier (no implicit vmcnt(0) drain).
template <int BM, int BN, int WM, int WN, int STAGES, int EPI>
__global__ void __launch_bounds__(64 * WM * WN, (WM * WN == 4 ? 2 : 1))
gemm_nt_kernel(int M, int N, int K, const bf16_t* __restrict__ A, long lda,
               const bf16_t* __restrict__ B, long ldb, const float* __restrict__ bias,
               float alpha, void* __restrict__ out0, long ldo0, void* __restrict__ out1,
               long ldo1, const void* __restrict__ aux, long ldaux, EpiParams ep) {
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM / 16;  // 16-row subtiles per wave (activation rows)
  constexpr int TN = BN / WN / 16;  // 16-col subtiles per wave (output features)
  constexpr int STAGE_BYTES = (BM + BN) * 128;
  constexpr int LOADS = (BM + BN) / 8 / NW;  // glds instructions per wave per stage
  // the epilogue stages PASS rows of each wave's accumulator tile through the same LDS
  // (16-row passes for the one-stage variant: half the staging LDS and prefetch registers)
  constexpr int PASS_MAX = STAGES == 1 ? 16 : 32;
  constexpr int EPI_BYTES = NW * ((BM / WM) % PASS_MAX == 0 ? PASS_MAX : 16) * (BN / WN + 4) * 4;
  constexpr int SMEM = STAGES * STAGE_BYTES > EPI_BYTES ? STAGES * STAGE_BYTES : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  // XCD-aware bijective block remap.
  const int tiles_n = N / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  int bid = blockIdx.x;
  {
    int q = nwg / 8, r = nwg % 8, x = bid % 8, loc = bid / 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + loc;
  }
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  // LDS-DMA through per-tile buffer descriptors (as gemm8_kernel): lane offsets fixed for the
  // loop, the k-tile in the SGPR offset; tile rows past M read as zero (computed, never stored)
  constexpr int IA = BM / 8 / NW, IB = BN / 8 / NW;  // 1-KiB pieces per wave and stage
  static_assert(IA * 8 * NW == BM && IB * 8 * NW == BN, "tile rows must split evenly over the waves");
  const __amdgpu_buffer_rsrc_t rsA = lc_rsrc(A + (long)m0 * lda, (long)min(M - m0, BM) * lda * 2);
  const __amdgpu_buffer_rsrc_t rsB = lc_rsrc(B + (long)n0 * ldb, (long)BN * ldb * 2);
  // (the lane offsets are loop-invariant: hoisted out of the k loop by the compiler. Held in
  // arrays captured by the lambda instead, hipcc's host pass dropped the kernel's launch stub.)
  auto stage = [&](int buf, int kt) {
    char* s = smem + buf * STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const int r = (wave * IA + i) * 8 + (lane >> 3);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, LDS_PTR(s + (wave * IA + i) * 1024), 16,
                                               (uint32_t)(r * lda * 2 + swz(r, lane & 7) * 16),
                                               kt * BK * 2, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const int r = (wave * IB + i) * 8 + (lane >> 3);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, LDS_PTR(s + BM * 128 + (wave * IB + i) * 1024),
                                               16, (uint32_t)(r * ldb * 2 + swz(r, lane & 7) * 16),
                                               kt * BK * 2, 0, 0);
    }
  };

  auto compute = [&](const char* sa) {
    const char* sb = sa + BM * 128;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int chunk = ks * 4 + (lane >> 4);
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = read_frag(sa, wm * (BM / WM) + i * 16 + (lane & 15), chunk);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = read_frag(sb, wn * (BN / WN) + j * 16 + (lane & 15), chunk);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(fb[j], fa[i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
  };

  if constexpr (STAGES == 1) {
    // one LDS stage (the one-k-tile streams, K = 64: more workgroups per CU); the closing
    // barrier of a tile also guards the next tile's DMA and the epilogue's reuse of the LDS
    for (int kt = 0; kt < nk; ++kt) {
      stage(0, kt);
      wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      compute(smem);
      __builtin_amdgcn_s_barrier();
    }
  } else {
    // prologue: STAGES-1 tiles in flight, wait for the first
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
      if (s < nk) stage(s, s);
    if (nk >= STAGES - 1) wait_vmcnt<LOADS * (STAGES - 2)>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();

    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      const int pre = kt + STAGES - 1;
      int pbuf = cur + STAGES - 1;
      if (pbuf >= STAGES) pbuf -= STAGES;
      if (pre < nk) stage(pbuf, pre);
      compute(smem + cur * STAGE_BYTES);
      // tile kt+1 must have landed; tiles up to kt+STAGES-1 may stay in flight
      if (pre < nk) wait_vmcnt<LOADS * (STAGES - 2)>();
      else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      cur = cur + 1 == STAGES ? 0 : cur + 1;
    }
  }

  store_tile<BM, BN, WM, WN, EPI, PASS_MAX>(acc, smem, SMEM, m0, n0, M, bias, alpha, out0, ldo0,
                                            out1, ldo1, aux, ldaux, ep);
}

// ---------------------------------------------------------------------------------------------
// Ping-pong GEMM (BM x BN = 256 x 256 or 128 x 256..., 8 waves as 2 x 4).
// Waves 0-3 (group 0) and 4-7 (group 1) place one wave of each group on every SIMD. The groups
// are staggered by one s_barrier, so each SIMD alternates: one wave runs an MFMA segment while
// its partner runs a LOAD segment (ds_read of its fragments + global_load_lds prefetch).
// K is consumed in 32-deep halves through a 4-slot LDS ring (slot = A [BM][32] + B [BN][32]
// bf16, 64-B rows); the DMA of half h+3 is issued in the LOAD segment of half h, so a half has
// three segments to land. Row swizzle for conflict-free ds_read_b128 on 64-B rows:
// chunk' = chunk ^ (((row >> 3) & 1) << 1).
// Hazards (every wave): RAW — a wave's own DMA of half h+1 is retired by the counted vmcnt at
// the end of its LOAD(h); both groups' LOAD(h) precede the barrier that precedes LOAD(h+1) of
// either group. WAR — slot (h+3)%4 == (h-1)%4 was last read in LOAD(h-1) of both groups, whose
// lgkmcnt(0) precedes the barriers in front of LOAD(h) of either group.
LC_DEV int swz64(int row, int chunk) { return chunk ^ (((row >> 3) & 1) << 1); }

// Split-K tail of the ping-pong GEMM. A launch of T output tiles on C CUs runs ceil(T/C) rounds;
// when the last round is only partly filled (N = 768 at M = 50 432: 591 tiles = 2.31 rounds),
// its R = T mod C tiles are instead cut along K into S slices (R*S <= C workgroups, one extra
// short round). Each slice workgroup writes its f32 accumulators to a slab (register-image
// layout, 256 KiB per tile slice), publishes with an agent-scope release + ticket atomic; the
// workgroup that draws the last ticket acquires, adds the other slabs and runs the normal fused
// epilogue, then resets the ticket (counters start zeroed: the caller's workspace).
struct SplitK {
  int dp_tiles;   // tiles [0, dp_tiles) run whole; tiles [dp_tiles, T) are split
  int splits;     // S (1 = no split-K)
  float* slabs;   // [(T - dp_tiles) * S][256 * 256] f32
  int* tickets;   // [T - dp_tiles], zero between launches
};

// Slice workgroup s_id (0 .. (T - dp) * S - 1, after the dp tiles) -> (tail tile, slice): groups
// of 8 tail tiles x S slices, slice k of tile x at s_id = 8 S g + x + 8 k, so a tile's slices
// have equal workgroup ids mod 8 — one XCD under round-robin placement (speed only: the
// publication below is correct for any placement) — and the last arriver reads the other slabs
// from its own L2. A last, partial group of Tg < 8 tiles is dealt the same way modulo Tg.
LC_DEV void splitk_slice(int s_id, int tail_tiles, int S, int& tail, int& split) {
#ifdef LC_SPLITK_SPREAD
  // diagnostic build (make SPREAD=1): slice k of tile x at s_id = S x + k, i.e. a tile's slices
  // on consecutive workgroups and so on different XCDs, to pin the publication protocol's
  // cross-XCD case (tests/test_kernels_gpu.py split-K cases under LCCLIP_LIB)
  tail = s_id / S;
  split = s_id % S;
  return;
#endif
  const int grp = s_id / (8 * S), rem = s_id % (8 * S);
  const int tg = min(8, tail_tiles - grp * 8);
  tail = grp * 8 + rem % tg;
  split = rem / tg;
}

// The last-arriving slice's sum of every slice's partial tile, in slice order (bit-identical to
// adding the S slabs one after another: its own partial, exact in the slab, is taken from the
// registers instead of re-read). The slabs are read with sc1 loads (the publication protocol of
// gemm8_kernel's split path: sc1 stores, no fences). All S <= 4 slabs are addressed through buffer descriptors that
// are empty for the own slice and for k >= S, so the loads are unconditional (no branch around
// a load: hipcc would wait vmcnt(0) at every join) and read zero there; CH tiles of every slab in
// flight per round.
template <int TM, int TN, int CH>
LC_DEV void splitk_sum(f32x4 (&acc)[TM][TN], const SplitK& sk, int tail, int split, int lane_off) {
  constexpr int SLAB = 256 * 256;
  __amdgpu_buffer_rsrc_t rs[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool use = k < sk.splits && k != split;
    rs[k] = lc_rsrc(sk.slabs + ((long)tail * sk.splits + (use ? k : 0)) * SLAB,
                    use ? (long)SLAB * 4 : 0);
  }
  static_assert((TM * TN) % CH == 0, "chunking");
#pragma unroll
  for (int c = 0; c < TM * TN; c += CH) {
    f32x4 v[4][CH];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int e = 0; e < CH; ++e)
        v[k][e] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs[k], (lane_off + (c + e) * 256) * 4, 0, 16));
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      f32x4& a = acc[(c + e) / TN][(c + e) % TN];
      f32x4 sum = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 4; ++k) sum += (k == split) ? a : v[k][e];  // zero for k >= S
      a = sum;
    }
  }
}

template <int EPI>
__global__ void __launch_bounds__(512, 1)
gemm_pp_kernel(int M, int N, int K, const bf16_t* __restrict__ A, long lda,
               const bf16_t* __restrict__ B, long ldb, const float* __restrict__ bias,
               float alpha, void* __restrict__ out0, long ldo0, void* __restrict__ out1,
               long ldo1, const void* __restrict__ aux, long ldaux, EpiParams ep, SplitK sk) {
  constexpr int BM = 256, BN = 256, WM = 2, WN = 4;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;  // 8 x 4 subtiles per wave
  constexpr int SLOT = (BM + BN) * 64;                 // one k-half: 32 KiB
  constexpr int NSLOT = 4;
  constexpr int PIECES = (BM + BN) / 16 / 8;           // 1-KiB DMA pieces per wave per half (4)
  constexpr int P_LOAD = 2;                            // issued in the LOAD segment
  constexpr int P_COMP = PIECES - P_LOAD;              // interleaved into the MFMA segment
  __shared__ __attribute__((aligned(16))) char smem[NSLOT * SLOT];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;  // wm = group
  const int tiles_n = N / BN;
  int bid = blockIdx.x;
  int split = -1;  // >= 0: this workgroup computes K-slice `split` of a tail tile
  int hb = 0, he = K / 32;  // k-halves [hb, he) of this workgroup
  if (bid < sk.dp_tiles) {
    const int nwg = sk.dp_tiles;  // XCD-aware bijective remap over the whole-tile part
    int q = nwg / 8, r = nwg % 8, x = bid % 8, loc = bid / 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + loc;
  } else {
    const int s_id = bid - sk.dp_tiles;
    split = s_id % sk.splits;
    bid = sk.dp_tiles + s_id / sk.splits;
    const int nh_all = K / 32;
    hb = split * nh_all / sk.splits;
    he = (split + 1) * nh_all / sk.splits;
  }
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nh = he - hb;  // halves of this workgroup; h below counts from 0 (slot = h % 4)
  const bf16_t* __restrict__ Ak = A + hb * 32;
  const bf16_t* __restrict__ Bk = B + hb * 32;
  // piece p of this wave = 16-row block p*8 + wave of half h (A blocks 0..15, B blocks 16..31)
  auto dma_piece = [&](int h, int p) {
    const int blk = p * 8 + wave;
    char* sl = smem + (h % NSLOT) * SLOT;
    const bool isA = blk < BM / 16;
    const int b = isA ? blk : blk - BM / 16;
    const int r = b * 16 + (lane >> 2);
    const int c = swz64(r, lane & 3);
    const int rows_valid = isA ? M : N;
    int gr = (isA ? m0 : n0) + r;
    gr = gr < rows_valid ? gr : rows_valid - 1;
    const bf16_t* src = isA ? Ak + (long)gr * lda : Bk + (long)gr * ldb;
    glds16(src + h * 32 + c * 8, sl + (isA ? 0 : BM * 64) + b * 1024);
  };
  auto dma_half = [&](int h) {
#pragma unroll
    for (int p = 0; p < PIECES; ++p) dma_piece(h, p);
  };
  // segment timestamps for tools/gemm_trace.py / gemm_phases.py: compiled in only with
  // -DLC_GEMM_TRACE (make TRACE=1) — even disabled, each stamp site costs an exec-masked branch
  // inside the MFMA stream
#ifdef LC_GEMM_TRACE
  const bool diag = ep.dbg != nullptr && blockIdx.x == 0 && (wave == 0 || wave == 4) && lane == 0;
  auto stamp = [&](int idx) {
    if (diag && idx < 256) {
      unsigned long long t;
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
      ep.dbg[(wave / 4) * 256 + idx] = t;
    }
  };
#else
  auto stamp = [](int) {};
#endif

  // prologue: halves 0..2 in flight; wait for this wave's part of half 0
  dma_half(0);
  if (nh > 1) dma_half(1);
  if (nh > 2) dma_half(2);
  if (nh > 2) wait_vmcnt<2 * PIECES>();
  else if (nh > 1) wait_vmcnt<PIECES>();
  else wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();
  if (wm == 1) __builtin_amdgcn_s_barrier();  // stagger group 1 by one segment

  const int g = lane >> 4, t = lane & 15;
  for (int h = 0; h < nh; ++h) {
    stamp(4 * h);
    // ---------------- LOAD segment: fragments of half h + the first DMA pieces of half h+3
    // (slot (h+3)%4 == (h-1)%4 was last read in LOAD(h-1) of both groups)
    const char* sa = smem + (h % NSLOT) * SLOT;
    const char* sb = sa + BM * 64;
    bf16x8 fa[TM], fb[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int r = wm * (BM / WM) + i * 16 + t;
      fa[i] = *reinterpret_cast<const bf16x8*>(sa + r * 64 + swz64(r, g) * 16);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int r = wn * (BN / WN) + j * 16 + t;
      fb[j] = *reinterpret_cast<const bf16x8*>(sb + r * 64 + swz64(r, g) * 16);
    }
    const bool pre = h + 3 < nh;
    if (pre) {
#pragma unroll
      for (int p = 0; p < P_LOAD; ++p) dma_piece(h + 3, p);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    stamp(4 * h + 1);
    // this wave's DMA of half h+1 must have landed before the barrier in front of LOAD(h+1);
    // in flight behind it: half h+2 (all pieces) and the pieces of h+3 issued just now
    if (pre) wait_vmcnt<PIECES + P_LOAD>();
    else if (h + 2 < nh) wait_vmcnt<PIECES>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    stamp(4 * h + 2);
    // ---------------- COMPUTE segment (remaining DMA pieces in the MFMA issue gaps)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(fb[j], fa[i], acc[i][j]);
      if (P_COMP > 0 && pre && (i * P_COMP) / TM != ((i + 1) * P_COMP) / TM)
        dma_piece(h + 3, P_LOAD + (i * P_COMP) / TM);
    }
    __builtin_amdgcn_s_setprio(0);
    stamp(4 * h + 3);
    __builtin_amdgcn_s_barrier();
  }
  if (wm == 0) __builtin_amdgcn_s_barrier();  // match group 1's stagger barrier
  if (split >= 0) {
    // publish this K-slice (G16 recipe: stores drained, barrier, agent release, ticket)
    const int tail = bid - sk.dp_tiles;
    constexpr int SLAB = BM * BN;  // floats
    float* mine = sk.slabs + ((long)tail * sk.splits + split) * SLAB;
    const int lane_off = (wave * TM * TN * 64 + lane) * 4;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        *reinterpret_cast<f32x4*>(mine + lane_off + (i * TN + j) * 256) = acc[i][j];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem);
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int ticket = __hip_atomic_fetch_add(sk.tickets + tail, 1, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
      const int last = ticket == sk.splits - 1;
      if (last) {
        __hip_atomic_store(sk.tickets + tail, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      flag[0] = last;
    }
    __syncthreads();
    const int last = flag[0];
    __syncthreads();  // flag read by every wave before the epilogue reuses the LDS
    if (!last) return;
    // sum every slice's slab (own included) in slice order: the result does not depend on
    // which slice arrived last
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < sk.splits; ++s) {
      const float* other = sk.slabs + ((long)tail * sk.splits + s) * SLAB;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] += *reinterpret_cast<const f32x4*>(other + lane_off + (i * TN + j) * 256);
    }
  }
  store_tile<BM, BN, WM, WN, EPI>(acc, smem, NSLOT * SLOT, m0, n0, M, bias, alpha, out0, ldo0,
                                  out1, ldo1, aux, ldaux, ep);
}

// ---------------------------------------------------------------------------------------------
// Phase-interleaved GEMM, bf16 or block-scaled fp8 (256 x 256 tile, 512 threads).
// 8 waves = 2 groups (wr = wave / 4: A rows 128 wr .. +127) x 4 (wc: B rows 64 wc .. +63); each
// wave owns a 128 x 64 output = 8 x 4 subtiles of 16 x 16 (128 accumulator VGPRs). K goes in
// k-tiles of 128 B per row (64 bf16 or 128 e4m3), double-buffered in LDS: A [256][128 B] + B
// [256][128 B] (+ 2 KiB of E8M0 scales for fp8) per buffer = 129 / 131 KiB in total.
// A k-tile is 4 phases, one per quadrant (qm, qn) of the wave's output, in the order (0,0),
// (0,1), (1,0), (1,1): LOAD part (this quadrant's fragments not yet in registers — A(qm0) + B(qn0)
// = 12 ds_read_b128, B(qn1) = 4, A(qm1) = 8, then none — plus one quarter of the DMA of a later
// k-tile), barrier, MFMA part (16 bf16 16x16x32 or 8 scaled 16x16x128 MFMAs = 256 cycles),
// barrier. Group 1 runs one barrier behind group 0, so on every SIMD one wave's MFMA part
// overlaps the other's LOAD part.
// DMA quarters (16 KiB, 2 global_load_lds per thread), issued well ahead of their use: phase 0
// of k-tile t: A rows 0..127 of t+1 (+ the scale piece of t+1); phase 1: A rows 128..255 of
// t+1; phase 3: B rows 0..255 of t+2 (two quarters). Hazards (barriers numbered by interval;
// G0's LOAD(P) is interval 2P, G1's 2P+1): WAR — B(t) is last read by G1's phase-1 LOAD,
// retired in its phase-1 MFMA, 2 intervals before the first B(t+2) DMA; A(t-1) / scales(t-1)
// are last read in phase 2 of t-1, >= 3 intervals before A(t+1) is issued. RAW — before G0
// reads k-tile t+1 (phase 0: A rows 0..127, B, scales) every wave has retired them: G0 at the
// end of its phase-3 MFMA, G1 at the end of its phase-3 LOAD (both leave A rows 128..255 of t+1
// and B of t+2 in flight: vmcnt(6)); before G1 reads A rows 128..255 of t+1, G0 retires them at
// the end of its next phase-0 LOAD (B(t+2), A rows 0..127 (t+2) in flight) and G1 at the end of
// its phase-3 MFMA (B(t+2) in flight). So a quarter has 5-8 intervals to land.
// A lane (g = lane >> 4) reads 16-B chunks g and g + 4 of a 128-B row in both forms: the bf16
// operand's k-steps 0 and 1, and for fp8 exactly the bytes v_mfma_scale_f32_16x16x128_f8f6f4
// takes from lane group g (k 16g..16g+15 in bytes 0-15, 64+16g.. in bytes 16-31; measured with
// tools/dbg_fp8.py: hardware scale block b = k / 32 takes lane group b's scale byte, so each
// lane passes the scale of block g). Conflict-free under the row XOR swizzle chunk ^ ((row >> 1) & 7).
constexpr int TRACE_STAMPS_LOOP_END = 638;

// SKM (stream-K): gridDim.x workgroups, workgroup range r = an XCD-major renumbering of
// blockIdx.x, owns the k-units [U r / G, U (r + 1) / G) of the T x KT units (tile-major), i.e.
// whole tiles plus at most one partial tile at each end (the host guarantees U / G >= KT, so a
// tile is cut at most once). The two parts of a cut tile meet through one slab per range
// boundary b (between ranges b and b + 1) and a ticket: the first arriver writes its partial
// (sc1 stores), drains, then adds 2 to the ticket; the second waits for the ticket to reach 4
// (1 + 1 + 2), adds the slab (sc1 loads) to its registers, resets the ticket and runs the
// epilogue. The wait is only ever on a workgroup that has already taken its ticket, i.e. is
// resident and past its main loop. a + b = b + a in IEEE, so the result does not depend on
// which part arrives first.
template <int EPI, bool FP8, bool SKM = false>
__global__ void __launch_bounds__(512, 1)
gemm8_kernel(int M, int N, int K, const void* __restrict__ Av, long lda,
             const void* __restrict__ Bv, long ldb, const float* __restrict__ bias, float alpha,
             void* __restrict__ out0, long ldo0, void* __restrict__ out1, long ldo1,
             const void* __restrict__ aux, long ldaux, EpiParams ep, SplitK sk, Fp8Scales sc) {
  constexpr int BM = 256, BN = 256, WM = 2, WN = 4;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;  // 8 x 4 subtiles per wave
  constexpr int TILE_A = BM * 128, TILE_B = BN * 128;
  constexpr int SCALES = FP8 ? 2048 : 0;
  constexpr int BUF = TILE_A + TILE_B + SCALES;
  constexpr int SWM = 7;
  constexpr int KT = FP8 ? 128 : 64;  // k per k-tile
#ifdef LC_GEMM_TRACE
  // s_memtime stamps of waves 0 and 4 kept in LDS (global stores would break the counted
  // vmcnt waits), copied out at the end: [group][640]
  constexpr int TRACE_N = 640;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF + 2 * TRACE_N * 8];
#else
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
#endif

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WN, wc = wave % WN;
  const int tiles_n = N / BN;
  // One tile (or k-slice of a tile): k-tiles [tb, te) of tile bid; split >= 0: slice `split` of
  // a split-K tail tile; skb >= 0 (SKM): a cut tile meeting its other part at range boundary skb.
  // Lane-dependent values are derived from an opaque copy of the thread id inside, so that hipcc
  // cannot hoist them out of the SKM segment loop (they would stay live through the epilogue).
  auto body = [&](int bid, int split, int tb, int te, int skb) {
  int tid_o = tid;
  if constexpr (SKM) asm volatile("" : "+v"(tid_o));
  const int lane = tid_o & 63;
  int tm, tn;
  tile_coords(bid, (M + BM - 1) / BM, tiles_n, ep.group_m, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int nt = te - tb;
  const char* __restrict__ A = static_cast<const char*>(Av) + (long)tb * 128;
  const char* __restrict__ B = static_cast<const char*>(Bv) + (long)tb * 128;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // DMA quarter `kind` of k-tile t: 0 = B rows 0..127, 1 = B rows 128..255, 2 = A rows 0..127
  // (+ scales), 3 = A rows 128..255
  // Buffer-descriptor DMA: one 32-bit lane offset per piece, fixed for the whole loop, and the
  // k-tile in the SGPR offset — no per-k-tile 64-bit address VALU and half the address VGPRs of
  // global_load_lds (same-box: every step shape 2-5 % faster, step +1.4 %). Tile rows past M
  // read as zero through the range check (computed, never stored).
  const __amdgpu_buffer_rsrc_t rsA = lc_rsrc(A + (long)m0 * lda, (long)min(M - m0, BM) * lda);
  const __amdgpu_buffer_rsrc_t rsB = lc_rsrc(B + (long)n0 * ldb, (long)BN * ldb);
  uint32_t voA[2][2], voB[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = h * 128 + (wave * 2 + i) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & SWM);
      voA[h][i] = (uint32_t)(row * lda + c * 16);
      voB[h][i] = (uint32_t)(row * ldb + c * 16);
    }
  auto dma = [&](int t, int kind) {
#ifdef G8_NODMA  // diagnostic builds only: main-loop DMA off (results wrong)
    if (t > 0) return;
#endif
    char* buf = smem + (t & 1) * BUF;
    const bool isA = kind >= 2;
    const int half = kind & 1;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row0 = half * 128 + (wave * 2 + i) * 8;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? rsA : rsB,
                                               LDS_PTR(buf + (isA ? 0 : TILE_A) + row0 * 128), 16,
                                               isA ? voA[half][i] : voB[half][i], t * 128, 0, 0);
    }
    if constexpr (FP8) {
      if (kind == 2) {
        // 2 KiB of scales: waves 0-3 -> A rows 64 w .. +63, waves 4-7 -> B rows
        const bool sA = wave < 4;
        const long rows_pad = sA ? sc.sa_rows : sc.sb_rows;
        const uint8_t* s = sA ? sc.sa : sc.sb;
        const int row = (wave & 3) * 64 + lane;
        glds4(s + ((long)(tb + t) * rows_pad + (sA ? m0 : n0) + row) * 4,
              buf + TILE_A + TILE_B + (sA ? 0 : 1024) + (wave & 3) * 256);
      }
    }
  };

  const int g = lane >> 4, t16 = lane & 15;
  using Frag = typename std::conditional<FP8, i32x8, bf16x8[2]>::type;
  Frag fa[4], fb[2][2];
  uint32_t sfa[4], sfb[2][2];
  (void)sfa;
  (void)sfb;
  // Lane-constant parts of the fragment addresses: the swizzle term (row >> 1) & SWM only
  // depends on t16 (subtile rows start at multiples of 16), so every read is a per-lane base plus
  // an immediate. Chunks g and g + 4: c1 = c0 ^ 64.
  const int sw = (t16 >> 1) & SWM;
  const int c0 = (g ^ sw) << 4;
  const int c1 = c0 ^ 64;
  const int a_row = (wr * 128 + t16) * 128, b_row = TILE_A + (wc * 64 + t16) * 128;
  auto read_frag = [&](const char* p0, const char* p1, auto& f) {
    if constexpr (FP8) {
      const i32x4 lo = *reinterpret_cast<const i32x4*>(p0);
      const i32x4 hi = *reinterpret_cast<const i32x4*>(p1);
      f = i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    } else {
      f[0] = *reinterpret_cast<const bf16x8*>(p0);
      f[1] = *reinterpret_cast<const bf16x8*>(p1);
    }
  };
  // scale byte of (row, this lane's k-block g): byte g of the row's k-tile dword
  auto read_scale = [&](const char* p) -> uint32_t {
    return *reinterpret_cast<const uint8_t*>(p + g);
  };
  auto load_a = [&](const char* buf, int qm) {
#ifdef G8_NOREAD  // diagnostic builds only: fragment reads off after the first k-tile
    if (buf != smem) return;
#endif
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ro = (qm * 64 + i * 16) * 128;
      read_frag(buf + a_row + ro + c0, buf + a_row + ro + c1, fa[i]);
      if constexpr (FP8)
        sfa[i] = read_scale(buf + TILE_A + TILE_B + (wr * 128 + t16 + qm * 64 + i * 16) * 4);
    }
  };
  auto load_b = [&](const char* buf, int qn) {
#ifdef G8_NOREAD
    if (buf != smem) return;
#endif
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ro = (qn * 32 + j * 16) * 128;
      read_frag(buf + b_row + ro + c0, buf + b_row + ro + c1, fb[qn][j]);
      if constexpr (FP8)
        sfb[qn][j] = read_scale(buf + TILE_A + TILE_B + 1024 + (wc * 64 + t16 + qn * 32 + j * 16) * 4);
    }
  };
  // The MFMA cluster is pinned between its barriers: the empty asm statements redefine the
  // quadrant's accumulators before the cluster and consume them after it, and volatile asm stays
  // in order with s_barrier. (hipcc otherwise sinks the register-only scaled MFMAs into the
  // loop latch: all fragments of a k-tile stay live and spill.)
  auto pin = [&](int qm, int qn) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(acc[qm * 4 + i][qn * 2 + j]));
  };
  auto mma = [&](int qm, int qn) {
    pin(qm, qn);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f32x4& c = acc[qm * 4 + i][qn * 2 + j];
        if constexpr (FP8) {
          c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fb[qn][j], fa[i], c, 0, 0, 0,
                                                               sfb[qn][j], 0, sfa[i]);
        } else {
          c = mfma16(fb[qn][j][0], fa[i][0], c);
          c = mfma16(fb[qn][j][1], fa[i][1], c);
        }
      }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    pin(qm, qn);
  };
  const bool g0 = wr == 0;
#ifdef LC_GEMM_TRACE
  const int trace_wg = ep.dbg ? (int)(ep.dbg[0] >> 32) : -1;  // workgroup to trace (host-set)
  const bool diag = ep.dbg != nullptr && (int)blockIdx.x == trace_wg && (wave & 3) == 0;
  unsigned long long* tr = reinterpret_cast<unsigned long long*>(smem + 2 * BUF) + wr * TRACE_N;
  auto stamp = [&](int idx) {
    if (diag && idx < TRACE_N) {
      const unsigned long long tt = __builtin_amdgcn_s_memtime();
      if (lane == 0) tr[idx] = tt;
    }
  };
#else
  auto stamp = [](int) {};
#endif
#ifdef LC_GEMM_CLOCK
  // in-kernel clock (tools/g8_clock.py, make CLOCK=1): shader-clock and 100 MHz stamps around
  // the workgroup's tile, kept in SGPRs and written once at the end
  const unsigned long long ck_t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long ck_r0 = __builtin_amdgcn_s_memrealtime();
  auto clock_out = [&]() {
    if (ep.dbg == nullptr) return;
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) {
      unsigned long long* d = ep.dbg + 4L * blockIdx.x;
      d[0] = t1 - ck_t0;
      d[1] = r1 - ck_r0;
      d[2] = ck_r0;
      d[3] = r1;
    }
  };
#endif
  stamp(0);

  // prologue: k-tile 0 whole, then B rows 0..255 of k-tile 1 (in flight across the barrier)
  dma(0, 0);
  dma(0, 1);
  dma(0, 2);
  dma(0, 3);
  if (nt > 1) {
    dma(1, 0);
    dma(1, 1);
    wait_vmcnt<4>();
  } else {
    wait_vmcnt<0>();
  }
  __builtin_amdgcn_s_barrier();
  if (!g0) __builtin_amdgcn_s_barrier();  // group 1 one barrier behind
  stamp(1);

  constexpr int S = FP8 ? 1 : 0;  // scale glds riding with the A rows 0..127 quarter
  for (int t = 0; t < nt; ++t) {
    const char* buf = smem + (t & 1) * BUF;
    const bool n1 = t + 1 < nt, n2 = t + 2 < nt;
    const int sb = 2 + t * 12;  // stamps of this k-tile: per phase [MFMA start, MFMA end, next start]
    // ---- phase 0: quadrant (0,0); DMA A rows 0..127 (+ scales) of t+1
    load_a(buf, 0);
    load_b(buf, 0);
    if (n1) dma(t + 1, 2);
    if (g0) {  // A rows 128..255 of k-tile t retired (group 1 reads them next interval); B
               // (t+1) and A rows 0..127 (t+1) may stay in flight
      if (n1) wait_vmcnt<6 + S>();
      else wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    stamp(sb + 0);
    mma(0, 0);
    stamp(sb + 1);
    __builtin_amdgcn_s_barrier();
    stamp(sb + 2);
    // ---- phase 1: quadrant (0,1); DMA A rows 128..255 of t+1
    load_b(buf, 1);
    if (n1) dma(t + 1, 3);
    __builtin_amdgcn_s_barrier();
    stamp(sb + 3);
    mma(0, 1);
    stamp(sb + 4);
    __builtin_amdgcn_s_barrier();
    stamp(sb + 5);
    // ---- phase 2: quadrant (1,0), no DMA
    load_a(buf, 1);
    __builtin_amdgcn_s_barrier();
    stamp(sb + 6);
    mma(1, 0);
    stamp(sb + 7);
    __builtin_amdgcn_s_barrier();
    stamp(sb + 8);
    // ---- phase 3: quadrant (1,1), no reads; DMA B of t+2 (B(t) was last read in phase 1)
    if (n2) {
      dma(t + 2, 0);
      dma(t + 2, 1);
    }
    if (!g0) {  // B and A rows 0..127 (+ scales) of k-tile t+1 retired
      if (n2) wait_vmcnt<6>();
      else if (n1) wait_vmcnt<2>();
    }
    __builtin_amdgcn_s_barrier();
    stamp(sb + 9);
    mma(1, 1);
    stamp(sb + 10);
    if (g0) {
      if (n2) wait_vmcnt<6>();
      else if (n1) wait_vmcnt<2>();
    } else {  // A rows 128..255 of k-tile t+1 retired
      if (n2) wait_vmcnt<4>();
      else wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    stamp(sb + 11);
  }
  if (g0) __builtin_amdgcn_s_barrier();  // match group 1's stagger barrier
  stamp(TRACE_STAMPS_LOOP_END);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if (split >= 0) {
    const int tail = bid - sk.dp_tiles;
    constexpr int SLAB = BM * BN;
    const int lane_off = (wave * TM * TN * 64 + lane) * 4;
    // publication without fences (MI355X_MICROARCH.md, valid forms: sc1 write-through 16-B slab
    // stores drained by every wave, a barrier, then one lane's relaxed agent-scope ticket add;
    // the workgroup whose add returns S-1 reads every other slab with sc1 16-B loads after a
    // barrier, splitk_sum): no L2 write-back of the XCD's dirty lines (release) and no L1
    // invalidate (acquire) on the tail's critical path
    const __amdgpu_buffer_rsrc_t rs_mine =
        lc_rsrc(sk.slabs + ((long)tail * sk.splits + split) * SLAB, (long)SLAB * 4);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(lc_u32x4, acc[i][j]), rs_mine,
                                               (lane_off + (i * TN + j) * 256) * 4, 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(630);
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem);
    if (tid == 0) {
      const int ticket = __hip_atomic_fetch_add(sk.tickets + tail, 1, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
      const int last = ticket == sk.splits - 1;
      if (last) __hip_atomic_store(sk.tickets + tail, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = last;
    }
    __syncthreads();
    const int last = flag[0];
    __syncthreads();
    stamp(631);
    if (!last) {
#ifdef LC_GEMM_CLOCK
      clock_out();  // a slice that only wrote its slab
#endif
      return;
    }
    splitk_sum<TM, TN, 4>(acc, sk, tail, split, lane_off);
    stamp(632);
  } else if (SKM && skb >= 0) {
    // a cut tile (see the kernel comment): first arriver publishes, second adds and stores
    constexpr int SLAB = BM * BN;
    const int lane_off = (wave * TM * TN * 64 + lane) * 4;
    int* tk = sk.tickets + skb;
    int* flag = reinterpret_cast<int*>(smem);
    __builtin_amdgcn_s_barrier();  // every wave done with the ring (lgkmcnt(0) above)
    if (tid == 0) flag[0] = __hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int order = flag[0];
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rs = lc_rsrc(sk.slabs + (long)skb * SLAB, (long)SLAB * 4);
    if (order == 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(lc_u32x4, acc[i][j]), rs,
                                                 (lane_off + (i * TN + j) * 256) * 4, 0, 16);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(tk, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef LC_GEMM_CLOCK
      clock_out();
#endif
      return;
    }
    if (tid == 0) {
      while (__hip_atomic_load(tk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < 4)
        __builtin_amdgcn_s_sleep(2);
      __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < TM * TN; c += 4) {
      f32x4 v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        v[e] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (lane_off + (c + e) * 256) * 4, 0, 16));
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[(c + e) / TN][(c + e) % TN] += v[e];
      __builtin_amdgcn_sched_barrier(0);  // 4 slab loads in flight at a time (registers)
    }
    // its own epilogue call: merged with the whole-tile path, the summed accumulators came out
    // of register allocation as copies with spills
    store_tile<BM, BN, WM, WN, EPI>(acc, smem, 2 * BUF, m0, n0, M, bias, alpha, out0, ldo0, out1,
                                    ldo1, aux, ldaux, ep, tid_o);
    return;
  } else {
    __builtin_amdgcn_s_barrier();  // every wave done with the ring: the epilogue reuses it
  }
  store_tile<BM, BN, WM, WN, EPI>(acc, smem, 2 * BUF, m0, n0, M, bias, alpha, out0, ldo0, out1,
                                  ldo1, aux, ldaux, ep, SKM ? tid_o : -1);
#ifdef LC_GEMM_TRACE
  stamp(TRACE_N - 1);
  __syncthreads();
  if (diag)
    for (int k = lane; k < TRACE_N; k += 64) ep.dbg[1 + wr * TRACE_N + k] = tr[k];
#endif
#ifdef LC_GEMM_CLOCK
  clock_out();
#endif
  };  // body

  const int nt_all = K / KT;
  if constexpr (!SKM) {
    int bid = blockIdx.x;
    int split = -1;
    int tb = 0, te = nt_all;  // k-tiles [tb, te) of this workgroup
    if (bid < sk.dp_tiles) {
      const int nwg = sk.dp_tiles;
      int q = nwg / 8, r = nwg % 8, x = bid % 8, loc = bid / 8;
      bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + loc;
    } else {
      int tail;
      splitk_slice(bid - sk.dp_tiles, ((M + BM - 1) / BM) * tiles_n - sk.dp_tiles, sk.splits,
                   tail, split);
      bid = sk.dp_tiles + tail;
      tb = split * nt_all / sk.splits;
      te = (split + 1) * nt_all / sk.splits;
    }
    body(bid, split, tb, te, -1);
  } else {
    // XCD-major range numbering: ranges r and r + 1 (which may share a cut tile) run on the same
    // XCD under round-robin placement, except where one XCD's block of ranges ends
    const int G = gridDim.x, w = blockIdx.x;
    const int r = (G % 8 == 0) ? (w % 8) * (G / 8) + w / 8 : w;
    const long U = (long)((M + BM - 1) / BM) * tiles_n * nt_all;
    long u = U * r / G;
    const long ue = U * (r + 1) / G;
    bool first = true;
#pragma unroll 1
    while (u < ue) {
      const int tile = (int)(u / nt_all), k0 = (int)(u % nt_all);
      const int k1 = (int)min((long)nt_all, k0 + (ue - u));
      const int skb = (k0 == 0 && k1 == nt_all) ? -1 : (k0 == 0 ? r : r - 1);
      if (!first) {  // the previous segment's epilogue staged through the ring
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
      body(tile, -1, k0, k1, skb);
      first = false;
      u += k1 - k0;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// 4-wave 256x256 GEMM (one wave per SIMD, each wave a 128x128 sub-tile: 64 accumulator tiles in
// AGPRs). K is consumed in 32-deep steps through a 4-slot LDS ring (slot = A [256][32] + B
// [256][32] bf16 in 64-B rows, the ping-pong kernel's layout and swizzle); the DMA of step s+3 is
// issued at step s, so every step has three steps of MFMA time to land. Per step: one barrier,
// then the 16 fragment reads of step s+1 are issued ahead of step s's 64 MFMAs (fragments double-
// buffered in VGPRs), so LDS latency hides behind the MFMA stream of the same wave.
// Hazards: slot (s+3)%4 == (s-1)%4 was last read by fragment reads issued in step s-2 and waited
// (lgkmcnt(0)) before the barrier of step s-1; step s+1's slot has landed for this wave (counted
// vmcnt) and for every wave after the barrier of step s+1... the reads of step s+1 are issued
// after the barrier of step s, which every wave passes only after its own DMA of step s+1 landed.
template <int EPI>
__global__ void __launch_bounds__(256, 1)
gemm_w4_kernel(int M, int N, int K, const bf16_t* __restrict__ A, long lda,
               const bf16_t* __restrict__ B, long ldb, const float* __restrict__ bias,
               float alpha, void* __restrict__ out0, long ldo0, void* __restrict__ out1,
               long ldo1, const void* __restrict__ aux, long ldaux, EpiParams ep) {
  constexpr int BM = 256, BN = 256, WM = 2, WN = 2;
  constexpr int TM = 8, TN = 8;
  constexpr int SLOT = (BM + BN) * 64;   // 32 KiB
  constexpr int NSLOT = 4;
  constexpr int PIECES = (BM + BN) / 16 / 4;  // 1-KiB DMA pieces per wave per step (8)
  static_assert(PIECES == TM, "one DMA piece per MFMA row group");
  __shared__ __attribute__((aligned(16))) char smem[NSLOT * SLOT];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_n = N / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  int bid = blockIdx.x;
  {
    int q = nwg / 8, r = nwg % 8, x = bid % 8, loc = bid / 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + loc;
  }
  int tm, tn;
  tile_coords(bid, tiles_m, tiles_n, ep.group_m, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int ns = K / 32;

  // piece p of this wave = 16-row block p*4 + wave (A blocks 0..15, B blocks 16..31); source
  // row pointers and LDS destinations computed once, a step only adds its k offset
  const bf16_t* psrc[PIECES];
  int pdst[PIECES];
#pragma unroll
  for (int p = 0; p < PIECES; ++p) {
    const int blk = p * 4 + wave;
    const bool isA = blk < BM / 16;
    const int b = isA ? blk : blk - BM / 16;
    const int r = b * 16 + (lane >> 2);
    const int c = swz64(r, lane & 3);
    const int rows_valid = isA ? M : N;
    int gr = (isA ? m0 : n0) + r;
    gr = gr < rows_valid ? gr : rows_valid - 1;
    psrc[p] = (isA ? A + (long)gr * lda : B + (long)gr * ldb) + c * 8;
    pdst[p] = (isA ? 0 : BM * 64) + b * 1024;
  }
  auto dma_piece = [&](int s, int p) {
    glds16(psrc[p] + s * 32, smem + (s % NSLOT) * SLOT + pdst[p]);
  };
  auto dma_step = [&](int s) {
#pragma unroll
    for (int p = 0; p < PIECES; ++p) dma_piece(s, p);
  };
  const int g = lane >> 4, t = lane & 15;
  // fragment reads of the NEXT step as inline asm: the compiler does not track them, so it puts
  // no lgkmcnt wait in front of this step's MFMAs; the explicit lgkmcnt(0) before the next
  // step's barrier is what orders them (the registers are consumed one step later)
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  uint32_t fa_off[TM], fb_off[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = wm * (BM / WM) + i * 16 + t;
    fa_off[i] = r * 64 + swz64(r, g) * 16;
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int r = wn * (BN / WN) + j * 16 + t;
    fb_off[j] = BM * 64 + r * 64 + swz64(r, g) * 16;
  }
  auto read_frags = [&](int s, bf16x8 (&fa)[TM], bf16x8 (&fb)[TN]) {
    const uint32_t base = lds0 + (s % NSLOT) * SLOT;
#pragma unroll
    for (int i = 0; i < TM; ++i)
      asm volatile("ds_read_b128 %0, %1" : "=v"(fa[i]) : "v"(base + fa_off[i]));
#pragma unroll
    for (int j = 0; j < TN; ++j)
      asm volatile("ds_read_b128 %0, %1" : "=v"(fb[j]) : "v"(base + fb_off[j]));
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: steps 0..2 in flight; step 0 landed everywhere; its fragments read
  dma_step(0);
  if (ns > 1) dma_step(1);
  if (ns > 2) dma_step(2);
  if (ns > 2) wait_vmcnt<2 * PIECES>();
  else if (ns > 1) wait_vmcnt<PIECES>();
  else wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();
  bf16x8 fa0[TM], fb0[TN], fa1[TM], fb1[TN];
  read_frags(0, fa0, fb0);

  // accumulators pinned to AGPRs: the MFMA as inline asm with an "a" operand, so the compiler
  // neither splits their live ranges nor shuffles them through VGPRs between steps
  // one step: wait for step s+1 (own DMA), barrier, then step s's MFMAs with DMA s+3 and the
  // fragment reads of s+1 (into the other buffer) interleaved
#ifdef LC_GEMM_TRACE
  const bool diag = ep.dbg != nullptr && blockIdx.x == 0 && lane == 0 && wave == 0;
  auto stamp = [&](int idx) {
    if (diag && idx < 512) {
      unsigned long long tt;
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tt)::"memory");
      ep.dbg[idx] = tt;
    }
  };
#else
  auto stamp = [](int) {};
#endif
  // FULL (std::true_type): steady state, s + 3 < ns, no per-group branches
  auto step = [&](int s, auto full, const bf16x8 (&fa)[TM], const bf16x8 (&fb)[TN],
                  bf16x8 (&na)[TM], bf16x8 (&nb)[TN]) {
    constexpr bool FULL = decltype(full)::value;
    stamp(3 * s);
    if (FULL || s + 2 < ns) wait_vmcnt<PIECES>();  // s+1 landed; s+2 may fly
    else if (s + 1 < ns) wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this step's fragments are in VGPRs
    __builtin_amdgcn_s_barrier();
    stamp(3 * s + 1);
    // memory work spread through the MFMA stream: row group i of the 8x8 sub-tile grid carries
    // DMA piece i of step s+3 and the A/B fragments i of step s+1 between its MFMAs, so the
    // wave never queues 24 memory instructions in front of its matrix work
#if defined(W4_NODMA)  // trace-only experiments: memory streams switched off (wrong results)
    const bool dma = false, rd = FULL || s + 1 < ns;
#elif defined(W4_NOREAD)
    const bool dma = FULL || s + 3 < ns, rd = false;
#else
    const bool dma = FULL || s + 3 < ns, rd = FULL || s + 1 < ns;
#endif
    const uint32_t nbase = lds0 + ((s + 1) % NSLOT) * SLOT;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int j = 0; j < TN / 2; ++j)
        asm volatile(LC_MFMA16_ASM " %0, %1, %2, %0"
                     : "+a"(acc[i][j])
                     : "v"(fb[j]), "v"(fa[i]));
      if (dma) dma_piece(s + 3, i);
      if (rd) {
        asm volatile("ds_read_b128 %0, %1" : "=v"(na[i]) : "v"(nbase + fa_off[i]));
        asm volatile("ds_read_b128 %0, %1" : "=v"(nb[i]) : "v"(nbase + fb_off[i]));
      }
#pragma unroll
      for (int j = TN / 2; j < TN; ++j)
        asm volatile(LC_MFMA16_ASM " %0, %1, %2, %0"
                     : "+a"(acc[i][j])
                     : "v"(fb[j]), "v"(fa[i]));
    }
    stamp(3 * s + 2);
  };
  using Full = std::true_type;
  using Tail = std::false_type;
  int s = 0;
  for (; s + 4 < ns; s += 2) {
    step(s, Full{}, fa0, fb0, fa1, fb1);
    step(s + 1, Full{}, fa1, fb1, fa0, fb0);
  }
  // at most four steps remain (s even)
  if (s < ns) step(s, Tail{}, fa0, fb0, fa1, fb1);
  if (s + 1 < ns) step(s + 1, Tail{}, fa1, fb1, fa0, fb0);
  if (s + 2 < ns) step(s + 2, Tail{}, fa0, fb0, fa1, fb1);
  if (s + 3 < ns) step(s + 3, Tail{}, fa1, fb1, fa0, fb0);
  // the last MFMA results reach the AGPRs before the epilogue reads them (asm MFMAs are opaque
  // to the hazard recognizer)
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // every wave done with the ring: the epilogue reuses it
  store_tile<BM, BN, WM, WN, EPI>(acc, smem, NSLOT * SLOT, m0, n0, M, bias, alpha, out0, ldo0,
                                  out1, ldo1, aux, ldaux, ep);
}

// ---------------------------------------------------------------------------------------------
// TN split-K GEMM: C[N1,N2] += alpha * sum_m A[m][n1] * B[m][n2].
// 64x64 output tile per workgroup, 4 waves (2x2, 32x32 each), K-step = 64 rows of M staged
// row-major in LDS and read TRANSPOSED with ds_read_b64_tr_b16 (4 rows x 16 cols per 16-lane
// group -> lane i gets column i), which is exactly the k-major fragment the MFMA needs.
// Each workgroup reduces one chunk of M and adds its tile into C with f32 atomics.
constexpr int TN_BM = 64;

LC_DEV bf16x4 tr_read(const char* lds, int row, int col) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) bf16x4*)(lds + row * 128 + col * 2));
}

__global__ void __launch_bounds__(256)
gemm_tn_kernel(int M, int N1, int N2, int chunk_rows, const bf16_t* __restrict__ A, long lda,
               const bf16_t* __restrict__ B, long ldb, float alpha, float* __restrict__ C,
               long ldc, float* __restrict__ colsum, float colsum_scale) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TN_BM * 128 + 4 * 64 * 4];
  float* red = reinterpret_cast<float*>(smem + 2 * 2 * TN_BM * 128);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wa = wave >> 1, wb = wave & 1;
  const int tiles_n2 = (N2 + 63) / 64;
  const int t1 = blockIdx.x / tiles_n2, t2 = blockIdx.x % tiles_n2;
  const int c1 = t1 * 64, c2 = t2 * 64;
  const int mbeg = blockIdx.y * chunk_rows;
  const int mend = min(M, mbeg + chunk_rows);
  if (mbeg >= mend) return;
  // bias gradient fused in: column sums of the A tile (only the t2 == 0 column of workgroups,
  // so every A column is summed exactly once)
  const bool do_cs = colsum != nullptr && t2 == 0;
  float cs = 0.f;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stage = [&](int buf, int mrow) {
    char* s = smem + buf * (2 * TN_BM * 128);
    // 64 rows x 128 B per operand = 8 wave-instructions; 2 per wave per operand.
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int r = (wave * 2 + i) * 8 + (lane >> 3);
      int gr = min(mrow + r, mend - 1);
      glds16(A + (long)gr * lda + c1 + (lane & 7) * 8, s + (wave * 2 + i) * 1024);
      glds16(B + (long)gr * ldb + c2 + (lane & 7) * 8, s + TN_BM * 128 + (wave * 2 + i) * 1024);
    }
  };

  const int nsteps = (mend - mbeg + TN_BM - 1) / TN_BM;
  stage(0, mbeg);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int st = 0; st < nsteps; ++st) {
    const int cur = st & 1;
    const int mrow = mbeg + st * TN_BM;
    if (st + 1 < nsteps) stage(cur ^ 1, mrow + TN_BM);
    char* sa = smem + cur * (2 * TN_BM * 128);
    char* sb = sa + TN_BM * 128;
    const int valid = mend - mrow;
    if (valid < TN_BM) {
      // zero the rows past the end of M (they were loaded clamped)
      for (int idx = tid; idx < (TN_BM - valid) * 16; idx += 256) {
        int r = valid + idx / 16, c = (idx % 16) * 8;
        if (c < 64) *reinterpret_cast<uint4*>(sa + r * 128 + c * 2) = uint4{0, 0, 0, 0};
        else *reinterpret_cast<uint4*>(sb + r * 128 + (c - 64) * 2) = uint4{0, 0, 0, 0};
      }
      __syncthreads();
    }
    if (do_cs) {
      const bf16_t* col = reinterpret_cast<const bf16_t*>(sa) + (tid & 63);
#pragma unroll
      for (int i = 0; i < 16; ++i) cs += bf2f(col[((tid >> 6) + 4 * i) * 64]);
    }
    const int g = lane >> 4, t = lane & 15;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        // rows (k) 32ks + 8g + {0..3}, {4..7}; cols block; lane 4q+p -> row q, cols 4p..4p+3
        const int row = ks * 32 + g * 8 + (t >> 2);
        const int cola = wa * 32 + i * 16 + (t & 3) * 4;
        bf16x4 lo = tr_read(sa, row, cola), hi = tr_read(sa, row + 4, cola);
        fa[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const int colb = wb * 32 + i * 16 + (t & 3) * 4;
        bf16x4 lo2 = tr_read(sb, row, colb), hi2 = tr_read(sb, row + 4, colb);
        fb[i] = bf16x8{lo2[0], lo2[1], lo2[2], lo2[3], hi2[0], hi2[1], hi2[2], hi2[3]};
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(fa[i], fb[j], acc[i][j]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (do_cs) {
    red[tid] = cs;
    __syncthreads();
    if (tid < 64 && c1 + tid < N1)
      atomicAdd(colsum + c1 + tid, colsum_scale * (red[tid] + red[tid + 64] + red[tid + 128] + red[tid + 192]));
  }
  // acc[i][j]: lane holds D[n1 = 4g + r][n2 = t] of subtile (i, j)
  const int g = lane >> 4, t = lane & 15;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n1 = c1 + wa * 32 + i * 16 + g * 4 + r;
        const int n2 = c2 + wb * 32 + j * 16 + t;
        if (n1 < N1 && n2 < N2) atomicAdd(C + (long)n1 * ldc + n2, acc[i][j][r] * alpha);
      }
}

// ---------------------------------------------------------------------------------------------
// Wide x skinny TN reduction (the PEFT weight gradients): P[n][j] = sum_m W[m][n] S[m][j] for a
// wide operand W [M, Nw] (activations / output gradients, Nw = 768 / 2304) and a skinny one
// S [M, 64] (adapter bottleneck, zero-padded LoRA rank), stored as C[n][j] or, transposed, C[j][n].
// These are HBM streams (≈128 FLOP per byte of W at most), so the design is about bytes in flight:
// one 512-thread workgroup per CU owns a 128-column W panel and a long contiguous chunk of rows,
// streamed through a 5-slot global_load_lds ring (64 rows x (256 + 128) B = 24 KiB per slot, four
// slots in flight), and adds its 128 x 64 partial once with f32 atomics at the end (one partial
// per workgroup instead of one per 64x64 tile and short chunk). Column sums (bias gradients) ride
// on the MFMA as products with a ones fragment. Up to two problems per launch (adapter: dWu and
// dWd in one grid).
struct TnProb {
  const bf16_t* W;
  long ldw;
  const bf16_t* S;
  long lds;
  float* C;
  long ldc;
  int Nw, ns, trans;  // P is Nw x ns; trans: C[j][n] instead of C[n][j]
  float alpha;
  float* cs_w;        // += cs_w_scale * sum_m W[m][n]   (n < Nw), or nullptr
  float cs_w_scale;
  float* cs_s;        // += cs_s_scale * sum_m S[m][j]   (j < ns), or nullptr
  float cs_s_scale;
  int M, n_chunks, n_tiles, wgs;  // row-block walkers per panel, W panels, workgroups
  float* part;        // two-stage mode: one partial slot per workgroup (tn_reduce_kernel sums
                      // them into C / the column sums); nullptr: f32 atomics into C
  int pw;             // W panel width of the launch (128 or 256)
  const float* div;   // optional device scalar every result is divided by (a power-of-two
                      // gradient scale: exact), or nullptr
  int w16;            // W holds IEEE halves (the half residual gradient): its fragments are
                      // rounded to bf16 as read (h2s8: the values of ln_bwd's bf16 copy)
};
LC_DEV float tn_unscale(const TnProb& p, float v) { return p.div ? v / *p.div : v; }

// Geometry of the wide x skinny reduction for a W panel of PW columns (128 or 256; 256 halves
// the re-reads of S, one per panel, for the adapter's D = 768: 3 panels instead of 6).
template <int PW>
struct TnGeom {
  static constexpr int ROWB = PW * 2;              // W panel row bytes (256 / 512)
  static constexpr int WB = 64 * ROWB;             // W bytes of one 64-row step
  static constexpr int SLOT = WB + 64 * 128;       // + S 64 x 64 bf16
#ifndef TNW256_STAGES
#define TNW256_STAGES 3
#endif
  static constexpr int STAGES = PW == 256 ? TNW256_STAGES : 5;  // 120 KiB of ring (160 at 4)
  static constexpr int WPW = WB / 1024 / 8;        // W 1-KiB pieces per wave per step (2 / 4)
  static constexpr int LOADS = WPW + 1;            // glds per wave per step (+ one S piece)
  static constexpr int TI = PW / 64;               // 16-column W blocks per wave (2 / 4)
};

// partial slot of one walker (two-stage mode): P [pw panel columns][64], pw W column sums,
// 64 S column sums
__host__ __device__ inline int tn_pslot(int pw) { return pw * 64 + pw + 64; }

// 8 waves: wave w owns W columns (PW/4) (w & 3) .. +PW/4 and S columns 32 (w >> 2) .. +31.
template <int PW>
__global__ void __launch_bounds__(512, 1)
gemm_tn_wide_kernel(TnProb p0, TnProb p1) {
  using Geo = TnGeom<PW>;
  constexpr int STAGES = Geo::STAGES, SLOT = Geo::SLOT, LOADS = Geo::LOADS, TI = Geo::TI;
  constexpr int ROWB = Geo::ROWB, LPRW = ROWB / 16, RPP = 64 / LPRW;  // lanes / rows per W piece
  constexpr int PSLOT = PW * 64 + PW + 64;
  __shared__ __attribute__((aligned(16))) char smem[STAGES * SLOT];
  const bool second = (int)blockIdx.x >= p0.wgs;
  const TnProb& p = second ? p1 : p0;
  const int bid = second ? blockIdx.x - p0.wgs : blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave & 3, wsv = wave >> 2;
  const int g = lane >> 4, t = lane & 15;
  const int tile = bid % p.n_tiles, cidx = bid / p.n_tiles;
  // block-cyclic rows: walker cidx takes 64-row blocks cidx, cidx + n_chunks, ... so that the
  // workgroups of the grid sweep one contiguous band of rows together (DRAM-page locality)
  const int nblk = (p.M + 63) / 64;
  float* slot = p.part ? p.part + (long)(tile * p.n_chunks + cidx) * PSLOT : nullptr;
  if (cidx >= nblk) {  // no rows (plan_tn never makes such walkers): an empty partial
    if (slot)
      for (int e = tid; e < PSLOT; e += 512) slot[e] = 0.f;
    return;
  }
  const int nsteps = (nblk - 1 - cidx) / p.n_chunks + 1;
  auto blk_row = [&](int s) { return (cidx + s * p.n_chunks) * 64; };
  const int nw_pad = (p.Nw + 63) & ~63;
  const bool do_csw = p.cs_w != nullptr && wsv == 0;
  const bool do_css = p.cs_s != nullptr && tile == 0 && wn == 0;

  // DMA of step s into slot s % STAGES. A wave-instruction fills 1 KiB of LDS linearly; the
  // lane -> (row, unit) map inverts the swizzle (source chosen so that lane*16 is its slot).
  //   W: RPP rows per piece, lane -> row lane / LPRW, position 16-B chunk lane % LPRW
  //   S: 8 rows per piece, lane -> row lane >> 3, position chunk lane & 7
  auto dma = [&](int s) {
    char* sl = smem + (s % STAGES) * SLOT;
    const int r0 = blk_row(s);
#pragma unroll
    for (int i = 0; i < Geo::WPW; ++i) {
      const int piece = wave * Geo::WPW + i;
      const int lr = piece * RPP + lane / LPRW;
      const int pc = lane % LPRW;
      const int c = (((pc >> 1) ^ swz_w(lr)) << 1) | (pc & 1);  // source 16-B chunk
      const int r = min(r0 + lr, p.M - 1);
      int col = tile * PW + c * 8;
      col = col < nw_pad ? col : col - 64;  // past a 64-multiple Nw: re-read, masked at the store
      glds16(p.W + (long)r * p.ldw + col, sl + piece * 1024);
    }
    {
      const int piece = wave;  // 8 S pieces
      const int lr = piece * 8 + (lane >> 3);
      const int pc = lane & 7;
      const int c = (((pc >> 1) ^ swz_s(lr)) << 1) | (pc & 1);
      const int r = min(r0 + lr, p.M - 1);
      glds16(p.S + (long)r * p.lds + c * 8, sl + Geo::WB + piece * 1024);
    }
  };

  f32x4 acc[TI][2], csw[TI], css[2];
#pragma unroll
  for (int i = 0; i < TI; ++i) {
    csw[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  css[0] = css[1] = f32x4{0.f, 0.f, 0.f, 0.f};
  const short one = LC_ONE16;

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nsteps) dma(s);
  for (int s = 0; s < nsteps; ++s) {
    // own DMA of step s landed (up to STAGES-2 later steps may stay in flight); after the
    // barrier every wave's has, and every wave is done reading slot (s-1) % STAGES, which the
    // DMA of step s + STAGES - 1 overwrites
    const int ahead = min(nsteps - 1 - s, STAGES - 2);
    if (STAGES > 4 && ahead >= 3) wait_vmcnt<3 * LOADS>();
    else if (STAGES > 3 && ahead == 2) wait_vmcnt<2 * LOADS>();
    else if (ahead >= 1) wait_vmcnt<LOADS>();
    else wait_vmcnt<0>();
    lds_barrier();  // (__syncthreads would wait vmcnt(0): the whole ring)
    if (s + STAGES - 1 < nsteps) dma(s + STAGES - 1);
    const uint32_t sw = lds_addr(smem + (s % STAGES) * SLOT);
    const uint32_t ss = sw + Geo::WB;
    const int valid = p.M - blk_row(s);  // rows of this block inside M (>= 64: all)
    // both k-slices' fragments issued up front (asm reads: no compiler drain), one wait
    bf16x8 fwk[2][TI], fsk[2][2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int row = ks * 32 + g * 8 + (t >> 2);
#pragma unroll
      for (int i = 0; i < TI; ++i)
        fwk[ks][i] = tr_frag_asm<ROWB>(sw, row, wn * (PW / 4) + i * 16 + (t & 3) * 4);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        fsk[ks][j] = tr_frag_asm<128>(ss, row, wsv * 32 + j * 16 + (t & 3) * 4);
    }
    lds_wait0();
    if (p.w16) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < TI; ++i) fwk[ks][i] = h2s8(fwk[ks][i]);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int kb = ks * 32 + g * 8;
      bf16x8* fw = fwk[ks];
      bf16x8* fs = fsk[ks];
      bf16x8 ones;
#pragma unroll
      for (int e = 0; e < 8; ++e) ones[e] = (kb + e < valid) ? one : (short)0;
      if (valid < 64) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int e = 0; e < 8; ++e) fs[j][e] = (kb + e < valid) ? fs[j][e] : (short)0;
      }
#pragma unroll
      for (int i = 0; i < TI; ++i) {
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(fw[i], fs[j], acc[i][j]);
        if (do_csw) csw[i] = mfma16(fw[i], ones, csw[i]);
      }
      if (do_css) {
#pragma unroll
        for (int j = 0; j < 2; ++j) css[j] = mfma16(ones, fs[j], css[j]);
      }
    }
  }
  // lane holds P[n = tile*PW + (PW/4) wn + 16i + 4g + r][j = 32wsv + 16jj + t]
  if (slot) {  // two-stage: plain stores of the whole partial (masking happens in the reduce)
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int nl = wn * (PW / 4) + i * 16 + g * 4 + r;
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) slot[nl * 64 + wsv * 32 + jj * 16 + t] = acc[i][jj][r];
        if (wsv == 0 && t == 0) slot[PW * 64 + nl] = do_csw ? csw[i][r] : 0.f;
      }
    if (wn == 0 && g == 0)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
        slot[PW * 64 + PW + wsv * 32 + jj * 16 + t] = do_css ? css[jj][0] : 0.f;
    return;
  }
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = tile * PW + wn * (PW / 4) + i * 16 + g * 4 + r;
      if (n >= p.Nw) continue;
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int j = wsv * 32 + jj * 16 + t;
        if (j < p.ns) {
          float* dst = p.trans ? p.C + (long)j * p.ldc + n : p.C + (long)n * p.ldc + j;
          atomicAdd(dst, tn_unscale(p, acc[i][jj][r] * p.alpha));
        }
      }
      if (do_csw && t == 0) atomicAdd(p.cs_w + n, tn_unscale(p, csw[i][r] * p.cs_w_scale));
    }
  if (do_css && g == 0) {
    // css[jj]: lane holds sum_k S[k][32wsv + 16jj + t] in every r
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = wsv * 32 + jj * 16 + t;
      if (j < p.ns) atomicAdd(p.cs_s + j, tn_unscale(p, css[jj][0] * p.cs_s_scale));
    }
  }
}

// sum of n partial slots (stride ps floats): loads issued 8 at a time, so a thread waits for
// ceil(n / 8) memory round trips instead of n (~42 walkers per panel: the plain loop was a
// 31 us latency chain in the step)
LC_DEV float sum_slots(const float* __restrict__ src, int n, long ps) {
  float v = 0.f;
  int c = 0;
  for (; c + 8 <= n; c += 8) {
    float t[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = src[(c + i) * ps];
    v += ((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7]));
  }
  for (; c < n; ++c) v += src[c * ps];
  return v;
}

// Second stage of the two-stage PEFT weight-gradient reduction: one thread per output (P
// element, W column sum or S column sum) of both problems sums the walkers' partial slots and
// adds the result into C / the column sums (each output owned by one thread: no atomics).
__global__ void __launch_bounds__(256)
tn_reduce_kernel(TnProb p0, TnProb p1) {
  const int np0 = p0.Nw * 64 + p0.Nw + 64;
  const int np1 = p1.part ? p1.Nw * 64 + p1.Nw + 64 : 0;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < np0 + np1; e += gridDim.x * 256) {
    const bool second = e >= np0;
    const TnProb& p = second ? p1 : p0;
    const int k = second ? e - np0 : e;
    const int pw = p.pw;
    const long ps = tn_pslot(pw);
    if (k < p.Nw * 64) {  // P[n][j]
      const int n = k / 64, j = k % 64;
      if (j >= p.ns) continue;
      const int tile = n / pw, nl = n % pw;
      const float v = sum_slots(p.part + (long)tile * p.n_chunks * ps + nl * 64 + j, p.n_chunks, ps);
      float* dst = p.trans ? p.C + (long)j * p.ldc + n : p.C + (long)n * p.ldc + j;
      *dst += tn_unscale(p, v * p.alpha);
    } else if (k < p.Nw * 64 + p.Nw) {  // column sums of W
      if (!p.cs_w) continue;
      const int n = k - p.Nw * 64, tile = n / pw, nl = n % pw;
      const float v = sum_slots(p.part + (long)tile * p.n_chunks * ps + pw * 64 + nl, p.n_chunks, ps);
      p.cs_w[n] += tn_unscale(p, v * p.cs_w_scale);
    } else {  // column sums of S (tile 0's walkers carry them)
      const int j = k - p.Nw * 64 - p.Nw;
      if (!p.cs_s || j >= p.ns) continue;
      const float v = sum_slots(p.part + pw * 64 + pw + j, p.n_chunks, ps);
      p.cs_s[j] += tn_unscale(p, v * p.cs_s_scale);
    }
  }
}

int cu_count();

// Walkers per panel so that the problems of one launch fill about one workgroup per CU.
void plan_tn(TnProb& p, int total_panels) {
  // measured (adapter dW, M = 50 432): one walker per CU 60 us; 2 per CU 80 us (twice the
  // partials to add atomically); contiguous per-walker chunks instead of block-cyclic 80-88 us
  static int walkers = -1;
  if (walkers < 0) {
    const char* e = lc_diag_env("LC_TN_WALKERS");
    walkers = e ? atoi(e) : 0;
  }
  const int cus = walkers > 0 ? walkers : cu_count();
  const int nblk = (p.M + 63) / 64;
  int chunks = cus / total_panels;
  chunks = chunks < 1 ? 1 : chunks;
  // at least 4 blocks per walker (ring fill)
  chunks = chunks > nblk / 4 ? (nblk / 4 > 0 ? nblk / 4 : 1) : chunks;
  p.n_chunks = chunks;
  p.wgs = p.n_tiles * chunks;
}

template <int BM, int BN, int WM, int WN, int STAGES>
int launch_nt(hipStream_t st, int epi, int M, int N, int K, const bf16_t* A, long lda,
              const bf16_t* B, long ldb, const float* bias, float alpha, void* o0, long l0,
              void* o1, long l1, const void* aux, long la, const EpiParams& ep) {
  // the main-loop DMA descriptors span one tile of A / B rows with 32-bit byte offsets
  LC_CHECK_ARG(lda < (1L << 22) && ldb < (1L << 22));
  const int tiles = ((M + BM - 1) / BM) * (N / BN);
  dim3 grid(tiles), block(64 * WM * WN);
#define LC_NT_CASE(E)                                                                       \
  case E:                                                                                     \
    hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, WM, WN, STAGES, E>), grid, block, 0, st, M, N, \
                       K, A, lda, B, ldb, bias, alpha, o0, l0, o1, l1, aux, la, ep);          \
    break;
  switch (epi) {
    LC_NT_CASE(EPI_BF16)
    LC_NT_CASE(EPI_F32)
    LC_NT_CASE(EPI_RESID)
    LC_NT_CASE(EPI_RESID16)
    LC_NT_CASE(EPI_GELU)
    LC_NT_CASE(EPI_GELU_BWD)
    LC_NT_CASE(EPI_BF16_F32)
    LC_NT_CASE(EPI_GELU_D)
    LC_NT_CASE(EPI_MUL)
    LC_NT_CASE(EPI_AD_DOWN)
    LC_NT_CASE(EPI_AD_UP)
    LC_NT_CASE(EPI_AD_MASK)
    LC_NT_CASE(EPI_AD_ADD)
    default:
      return LC_EINVAL;
  }
#undef LC_NT_CASE
  LC_LAUNCH_RET();
}

int g_split_mode = -1;  // LC_GEMM_SPLITK=0 disables the split-K tail (A/B experiments)

int cu_count() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cus[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

// Split-K plan for the tail round (see SplitK): S slices of >= min_units k-units each (units =
// the kernel's k-steps), R*S <= CUs, only when the last round is at most half full and the
// workspace holds the slabs.
SplitK plan_split(int tiles, int units, int min_units, void* ws, long ws_bytes, int per_cu = 1,
                  long slab_floats = 256 * 256) {
  SplitK sk{tiles, 1, nullptr, nullptr};
  if (g_split_mode < 0) {
    const char* e = lc_diag_env("LC_GEMM_SPLITK");
    g_split_mode = e ? atoi(e) : 1;
  }
  if (!g_split_mode || ws == nullptr) return sk;
  const int cus = cu_count() * per_cu;  // workgroup slots per round
  const int rem = tiles % cus;
  if (tiles < cus || rem == 0 || rem > cus / 2) return sk;
  int S = cus / rem;
  S = S > 4 ? 4 : S;
  if (S > units / min_units) S = units / min_units;  // measured: slices under 16 halves (K = 768) lose
  if (S < 2) return sk;
  const long tick_bytes = LC_SPLITK_TICKET_BYTES;
  if ((long)rem * 4 > tick_bytes || tick_bytes + (long)rem * S * slab_floats * 4 > ws_bytes) return sk;
  sk.dp_tiles = tiles - rem;
  sk.splits = S;
  sk.tickets = static_cast<int*>(ws);
  sk.slabs = reinterpret_cast<float*>(static_cast<char*>(ws) + tick_bytes);
  return sk;
}

// Stream-K plan (gemm8_kernel<.., SKM>): one workgroup per CU, each owning U / G >= one tile of
// k-units, cut tiles meeting through one slab per range boundary (G - 1 slabs and tickets in the
// split-K workspace). Only for launches with a ragged last round of more than one tile per CU.
// g_sk_mode (lc_gemm_set_streamk): 0 off, 1 N = 768 with K >= 2048, 2 every N = 768 launch,
// 3 every ragged bf16 launch, 4 N = 768 as whole row panels (one workgroup per panel).
int g_sk_mode = 0;
bool plan_sk(int tiles, int units, void* ws, long ws_bytes, SplitK& sk, int& G, int panels = 0) {
  G = panels > 0 ? panels : cu_count();
  if (panels > 0 && tiles % panels == 0 && ws != nullptr) {  // whole row panels: no cut tiles
    sk.dp_tiles = 0;
    sk.splits = 1;
    sk.tickets = static_cast<int*>(ws);
    sk.slabs = reinterpret_cast<float*>(static_cast<char*>(ws) + LC_SPLITK_TICKET_BYTES);
    return true;
  }
  if (ws == nullptr || tiles <= G || tiles % G == 0) return false;
  if ((long)tiles * units / G < units) return false;
  if ((long)(G - 1) * 4 > LC_SPLITK_TICKET_BYTES ||
      LC_SPLITK_TICKET_BYTES + (long)(G - 1) * 256 * 256 * 4 > ws_bytes)
    return false;
  sk.dp_tiles = 0;
  sk.splits = 1;
  sk.tickets = static_cast<int*>(ws);
  sk.slabs = reinterpret_cast<float*>(static_cast<char*>(ws) + LC_SPLITK_TICKET_BYTES);
  return true;
}
bool sk_wanted(int epi, int N, int K) {
  if (epi != EPI_BF16 && epi != EPI_F32 && epi != EPI_RESID) return false;
  switch (g_sk_mode) {
    case 1: return N == 768 && K >= 2048;
    case 2: return N == 768;
    case 3: return true;
    case 4: return N == 768;
    default: return false;
  }
}

// row panels per tile-raster group of the 256x256 GEMMs (tile_coords; env LC_GEMM_GM forces one).
// Measured (tools/gpu_gm.sh, M = 50 432): groups of 8 panels help the wide-N shapes (QKV fwd
// N = 2304: 181 -> 174 us, c_fc fwd N = 3072: 311 -> 303-307 us, c_proj dX -1 %) and cost the
// N = 768 ones 1-3 % (3 column tiles: the row-major raster already shares B)
int group_m(int N) {
  static const int forced = [] {
    const char* e = lc_diag_env("LC_GEMM_GM");
    return e ? atoi(e) : 0;
  }();
  if (forced) return forced;
  return N >= 2304 ? 8 : 1;
}

int launch_w4(hipStream_t st, int epi, int M, int N, int K, const bf16_t* A, long lda,
              const bf16_t* B, long ldb, const float* bias, float alpha, void* o0, long l0,
              void* o1, long l1, const void* aux, long la, const EpiParams& ep_in) {
  EpiParams ep = ep_in;
  ep.group_m = group_m(N);
  const int tiles = ((M + 255) / 256) * (N / 256);
  dim3 grid(tiles), block(256);
#define LC_W4_CASE(E)                                                                          \
  case E:                                                                                      \
    hipLaunchKernelGGL((gemm_w4_kernel<E>), grid, block, 0, st, M, N, K, A, lda, B, ldb, bias, \
                       alpha, o0, l0, o1, l1, aux, la, ep);                                    \
    break;
  switch (epi) {
    LC_W4_CASE(EPI_BF16)
    LC_W4_CASE(EPI_F32)
    LC_W4_CASE(EPI_RESID)
    LC_W4_CASE(EPI_GELU_D)
    LC_W4_CASE(EPI_MUL)
    default:
      return LC_EINVAL;
  }
#undef LC_W4_CASE
  LC_LAUNCH_RET();
}

int launch_pp(hipStream_t st, int epi, int M, int N, int K, const bf16_t* A, long lda,
              const bf16_t* B, long ldb, const float* bias, float alpha, void* o0, long l0,
              void* o1, long l1, const void* aux, long la, const EpiParams& ep, void* ws,
              long ws_bytes) {
  const int tiles = ((M + 255) / 256) * (N / 256);
  const SplitK sk = plan_split(tiles, K / 32, 16, ws, ws_bytes);
  dim3 grid(sk.dp_tiles + (tiles - sk.dp_tiles) * sk.splits), block(512);
#define LC_PP_CASE(E)                                                                          \
  case E:                                                                                      \
    hipLaunchKernelGGL((gemm_pp_kernel<E>), grid, block, 0, st, M, N, K, A, lda, B, ldb, bias, \
                       alpha, o0, l0, o1, l1, aux, la, ep, sk);                                \
    break;
  switch (epi) {
    LC_PP_CASE(EPI_BF16)
    LC_PP_CASE(EPI_F32)
    LC_PP_CASE(EPI_RESID)
    LC_PP_CASE(EPI_GELU)
    LC_PP_CASE(EPI_GELU_BWD)
    LC_PP_CASE(EPI_BF16_F32)
    LC_PP_CASE(EPI_GELU_D)
    LC_PP_CASE(EPI_MUL)
    LC_PP_CASE(EPI_AD_DOWN)
    LC_PP_CASE(EPI_AD_UP)
    LC_PP_CASE(EPI_AD_MASK)
    LC_PP_CASE(EPI_AD_ADD)
    default:
      return LC_EINVAL;
  }
#undef LC_PP_CASE
  LC_LAUNCH_RET();
}

// Phase-interleaved 256x256 GEMM (gemm8_kernel). bf16: A, B bf16 with lda/ldb in elements;
// fp8: A, B e4m3 with lda/ldb in bytes and their E8M0 scales in sc.
template <bool FP8>
int launch_g8(hipStream_t st, int epi, int M, int N, int K, const void* A, long lda,
              const void* B, long ldb, const float* bias, float alpha, void* o0, long l0,
              void* o1, long l1, const void* aux, long la, const EpiParams& ep_in, void* ws,
              long ws_bytes, const Fp8Scales& sc) {
  EpiParams ep = ep_in;
  ep.group_m = group_m(N);
  const int tiles = ((M + 255) / 256) * (N / 256);
  const int units = K / (FP8 ? 128 : 64);
  // (LC_GEMM_SPLIT_MIN overrides the minimum k-tiles per split-K slice: in-step A/Bs)
  static const int split_min = [] {
    const char* e = lc_diag_env("LC_GEMM_SPLIT_MIN");
    return e && atoi(e) > 0 ? atoi(e) : 8;
  }();
  const SplitK sk = plan_split(tiles, units, split_min, ws, ws_bytes);
  const long ea = FP8 ? 1 : 2;  // bytes per element
  // the main-loop DMA descriptors span one 256-row tile of A / B with 32-bit byte offsets
  LC_CHECK_ARG(lda * ea < (1L << 23) && ldb * ea < (1L << 23));
  if constexpr (!FP8) {
    SplitK skm{};
    int G = 0;
    // mode 4: one workgroup per 256-row panel walking its N / 256 column tiles (hipBLASLt's
    // N = 768 schedule: 197 workgroups at M = 50 432, no tile cut)
    const int panels = g_sk_mode == 4 ? (M + 255) / 256 : 0;
    if (sk_wanted(epi, N, K) && plan_sk(tiles, units, ws, ws_bytes, skm, G, panels)) {
#define LC_G8SK_CASE(E)                                                                          \
  case E:                                                                                        \
    hipLaunchKernelGGL((gemm8_kernel<E, false, true>), dim3(G), dim3(512), 0, st, M, N, K, A,    \
                       lda * ea, B, ldb * ea, bias, alpha, o0, l0, o1, l1, aux, la, ep, skm, sc); \
    break;
      switch (epi) {
        LC_G8SK_CASE(EPI_BF16)
        LC_G8SK_CASE(EPI_F32)
        LC_G8SK_CASE(EPI_RESID)
        default:
          return LC_EINVAL;
      }
#undef LC_G8SK_CASE
      LC_LAUNCH_RET();
    }
  }
  dim3 grid(sk.dp_tiles + (tiles - sk.dp_tiles) * sk.splits), block(512);
#define LC_G8_CASE(E)                                                                          \
  case E:                                                                                      \
    hipLaunchKernelGGL((gemm8_kernel<E, FP8>), grid, block, 0, st, M, N, K, A, lda * ea, B,    \
                       ldb * ea, bias, alpha, o0, l0, o1, l1, aux, la, ep, sk, sc);            \
    break;
  switch (epi) {
    LC_G8_CASE(EPI_BF16)
    LC_G8_CASE(EPI_F32)
    LC_G8_CASE(EPI_RESID)
    LC_G8_CASE(EPI_RESID16)
    LC_G8_CASE(EPI_GELU)
    LC_G8_CASE(EPI_GELU_D)
    LC_G8_CASE(EPI_MUL)
    LC_G8_CASE(EPI_GELU_D_Q8)
    LC_G8_CASE(EPI_MUL_Q8)
    default:
      return LC_EINVAL;
  }
#undef LC_G8_CASE
  LC_LAUNCH_RET();
}

// tile-shape selector (env LC_GEMM_TILE forces one for experiments: 0 auto, 1 = 128x128x2,
// 2 = 256x128x3, 3 = 256x256x2, 4 = 128x64x2)
int g_force_tile = -1;
unsigned long long* g_dbg = nullptr;

}  // namespace

extern "C" {

}  // extern "C"

int lc_gemm_nt_ex(hipStream_t stream, int epi, int M, int N, int K, const void* A, long lda,
                  const void* B, long ldb, const float* bias, float alpha, void* out0, long ldo0,
                  void* out1, long ldo1, const void* aux, long ldaux, const EpiParams& ep,
                  void* ws, long ws_bytes) {
  LC_CHECK_ARG(M > 0 && N > 0 && K > 0 && K % 64 == 0 && N % 64 == 0);
  LC_CHECK_ARG(lda % 8 == 0 && ldb % 8 == 0 && lda >= K && ldb >= K);
  LC_CHECK_ARG(lda < (1L << 22) && ldb < (1L << 22));  // tile descriptors: 32-bit byte offsets
  // epilogue rows are written / side inputs read 8 elements (16 B of bf16) per lane
  LC_CHECK_ARG(ldo0 % 8 == 0 && ldo0 >= N);
  // the epilogue's buffer descriptors span one 256-row tile with 32-bit byte offsets: 256 rows
  // x ldo x 4 B (f32 outputs) must stay below 2^31 (num_records and the int offsets)
  LC_CHECK_ARG(ldo0 < (1L << 21) && ldo1 < (1L << 21));
  LC_CHECK_ARG((epi >= 0 && epi <= EPI_AD_ADD) || epi == EPI_RESID16);
  if (epi == EPI_GELU || epi == EPI_BF16_F32 || epi == EPI_GELU_D)
    LC_CHECK_ARG(out1 != nullptr && ldo1 >= N && ldo1 % 8 == 0);
  if (epi == EPI_RESID || epi == EPI_GELU_BWD || epi == EPI_MUL || epi >= EPI_AD_UP)
    LC_CHECK_ARG(aux != nullptr && ldaux >= N && ldaux % 8 == 0);
  if (epi == EPI_AD_UP) LC_CHECK_ARG(ep.aux2 != nullptr && ep.ldaux2 >= N && ep.ldaux2 % 8 == 0);
  auto a = static_cast<const bf16_t*>(A);
  auto b = static_cast<const bf16_t*>(B);
  if (g_force_tile < 0) {
    const char* e = lc_diag_env("LC_GEMM_TILE");
    g_force_tile = e ? atoi(e) : 0;
  }
  int tile = g_force_tile;
#ifndef LC_F16
#ifndef LC_BLASLT_MIN_M  // (A/B builds override it)
#define LC_BLASLT_MIN_M 32768
#endif
  // the QKV input-gradient GEMM of a 256-image step (plain: no epilogue, no bias) on hipBLASLt
  // (blaslt.hip: 142 vs 160 us standalone, step +1.2 %); its workspace is the split-K scratch
  // after the tickets. A forced tile (A/B tools) or LC_GEMM_BLASLT=0 (DIAG) keeps gemm8.
  static const bool use_blaslt = [] {
    const char* e = lc_diag_env("LC_GEMM_BLASLT");
    return !(e && e[0] == '0');
  }();
  if (use_blaslt && tile == 0 && epi == EPI_BF16 && bias == nullptr && alpha == 1.0f &&
      M >= LC_BLASLT_MIN_M && N == 768 && K == 2304 && ws != nullptr &&
      ws_bytes >= LC_SPLITK_TICKET_BYTES + (8L << 20) &&
      lc_blaslt_nt_bf16(stream, M, N, K, a, lda, b, ldb, out0, ldo0,
                        static_cast<char*>(ws) + LC_SPLITK_TICKET_BYTES,
                        ws_bytes - LC_SPLITK_TICKET_BYTES))
    return LC_OK;
#endif
  if (tile == 0) {
    // measured on the ViT-B/16 step shapes (tools/bench_gemm.py, M = 50 432): the 256x256
    // phase-interleaved kernel beats the ping-pong one on every shape (776-1113 vs 743-1044 TF)
    // and the 128x128 kernel on N = K = 768 (858 vs ~780 TF); 128x128 at 2 workgroups/CU for
    // launches with fewer 256x256 tiles than CUs (text tower, MaPLe's 64-image batch at N =
    // 768: 150 tiles) — those would leave CUs idle
    // Rounds of 256x256 tiles: a ragged last round costs a whole tile time unless split-K can
    // spread it (K >= 1024: plan_split's 2 x 8 k-tiles) — measured at MaPLe's shapes
    // (tools/gpu_tn.sh, M = 7700 text / 12 800 image): with ~1.1-1.5 rounds the 128x128 kernel
    // wins (QKV fwd 39.7 vs 45.2 us, c_fc fwd 53.5 vs 59.1); with >= 2 full rounds, a tail over
    // half a round or a splittable tail the 256x256 one does (every M = 50 432 shape). Below one
    // round it still wins from half a round on when K is long (N = 768, K >= 2304 at 150 tiles:
    // 65.6 vs 83.4 us for 128x128, 73.8 for 128x64); N = 768 otherwise: 128x64 tiles (K = 768:
    // 24.3 vs 26.7 us; K = 3072 at 93 tiles: 46.5 vs 48.5).
    const int t256 = ((M + 255) / 256) * (N / 256), cus = cu_count();
    const int full = t256 / cus, rem = t256 % cus;
    const bool tail_ok = full >= 2 || rem == 0 || 2 * rem >= cus || (2 * rem <= cus && K >= 1024);
    // N = 768 with one full round and a short ragged tail that split-K cannot spread (K < 1024:
    // LoRA / MVP at 128 images, M = 25 216 .. 27 776, the out-projections): 128x128 at two
    // workgroups per CU (M = 25 216, K = 768: 35.5 / 36.9 us dX / fwd vs 39.4 / 39.9 for 128x64
    // and 42.8 / 43.7 for gemm8, tools/bench_gemm.py, profiles/r05/lo/)
    if (N % 128 != 0) tile = 4;
    else if (M >= 4096 && N % 256 == 0 && t256 >= cus && tail_ok) tile = 8;
    else if (M >= 4096 && N % 256 == 0 && 2 * t256 >= cus && K >= 2048) tile = 8;
    else if (M >= 4096 && N <= 768 && t256 >= cus) tile = 1;
    else if (M >= 4096 && N <= 768) tile = 4;
    // few rows, narrow N, long K (the C = 10 text tower's c_proj fwd / c_fc dX / QKV dX at
    // M = 770): 128x64 tiles give twice the workgroups of 128x128 for the long reduction
    // (15.6 / 15.5 / 12.6 vs 22.4 / 22.3 / 17.8 us, profiles/r05/tw/)
    else if (N <= 768 && K >= 1536) tile = 4;
    else tile = 1;
    // c_proj dX x QuickGELU' (N 3072, K 768): gemm8 since its epilogue stores went branch-free
    // (260 vs 267-271 us for the 4-wave kernel standalone, step +0.4 %, profiles/r03/s2/
    // r_ab_mul_route.txt; before that the 4-wave kernel won, 289 vs 295 us). LC_GEMM_MUL_W4=1
    // routes it to the 4-wave kernel again (A/Bs).
    static const bool mul_w4 = [] {
      const char* e = lc_diag_env("LC_GEMM_MUL_W4");
      return e && e[0] == '1';
    }();
    if (tile == 8 && epi == EPI_MUL && K <= 1024 && N >= 2048 && mul_w4) tile = 7;
    // one-k-tile streams (adapter up-projection / input gradient, K = 64): 128x64 tiles keep
    // more rows in flight per CU (tools/bench_adapter_kernels.py: AD_UP 83 -> 77 us, AD_ADD
    // 37 -> 35 us)
    if (K <= 64) tile = 11;
  }
  if (((tile == 3 || tile == 5 || tile == 6 || tile == 7 || tile == 8) && N % 256) ||
      ((tile == 1 || tile == 2) && N % 128))
    tile = 4;
  switch (tile) {
    case 1:
      return launch_nt<128, 128, 2, 2, 2>(stream, epi, M, N, K, a, lda, b, ldb, bias, alpha, out0,
                                          ldo0, out1, ldo1, aux, ldaux, ep);
    case 2:
      return launch_nt<256, 128, 4, 2, 3>(stream, epi, M, N, K, a, lda, b, ldb, bias, alpha, out0,
                                          ldo0, out1, ldo1, aux, ldaux, ep);
    case 3:
      return launch_nt<256, 256, 2, 4, 2>(stream, epi, M, N, K, a, lda, b, ldb, bias, alpha, out0,
                                          ldo0, out1, ldo1, aux, ldaux, ep);
    case 7:
      return launch_w4(stream, epi, M, N, K, a, lda, b, ldb, bias, alpha, out0, ldo0, out1, ldo1,
                       aux, ldaux, ep);
    case 5:
    case 6:
      return launch_pp(stream, epi, M, N, K, a, lda, b, ldb, bias, alpha, out0, ldo0, out1, ldo1,
                       aux, ldaux, ep, ws, ws_bytes);
    case 8:
      if (epi != EPI_BF16 && epi != EPI_F32 && epi != EPI_RESID && epi != EPI_GELU &&
          epi != EPI_GELU_D && epi != EPI_MUL && epi != EPI_RESID16)
        return launch_pp(stream, epi, M, N, K, a, lda, b, ldb, bias, alpha, out0, ldo0, out1, ldo1,
                         aux, ldaux, ep, ws, ws_bytes);
      return launch_g8<false>(stream, epi, M, N, K, a, lda, b, ldb, bias, alpha, out0, ldo0, out1,
                              ldo1, aux, ldaux, ep, ws, ws_bytes, Fp8Scales{});
    case 11:  // 128x64, one LDS stage
      return launch_nt<128, 64, 4, 1, 1>(stream, epi, M, N, K, a, lda, b, ldb, bias, alpha, out0,
                                         ldo0, out1, ldo1, aux, ldaux, ep);
    default:
      return launch_nt<128, 64, 4, 1, 2>(stream, epi, M, N, K, a, lda, b, ldb, bias, alpha, out0,
                                         ldo0, out1, ldo1, aux, ldaux, ep);
  }
}

extern "C" {

// See include/lc_clip.h for the contract.
int lc_gemm_nt(hipStream_t stream, int epi, int M, int N, int K, const void* A, long lda,
               const void* B, long ldb, const float* bias, float alpha, void* out0, long ldo0,
               void* out1, long ldo1, const void* aux, long ldaux) {
  return lc_gemm_nt_ws(stream, epi, M, N, K, A, lda, B, ldb, bias, alpha, out0, ldo0, out1, ldo1,
                       aux, ldaux, nullptr, 0);
}

int lc_gemm_nt_ws(hipStream_t stream, int epi, int M, int N, int K, const void* A, long lda,
                  const void* B, long ldb, const float* bias, float alpha, void* out0, long ldo0,
                  void* out1, long ldo1, const void* aux, long ldaux, void* ws, long ws_bytes) {
  LC_CHECK_ARG((epi >= 0 && epi <= 7) || epi == EPI_RESID16);
  LC_CHECK_ARG(ws == nullptr || (ws_bytes >= LC_SPLITK_TICKET_BYTES && ((uintptr_t)ws & 255) == 0));
  // the epilogue's buffer descriptors span one 256-row tile with 32-bit byte offsets: 256 rows
  // x ldo x 4 B (f32 outputs) must stay below 2^31 (num_records and the int offsets)
  LC_CHECK_ARG(ldo0 < (1L << 21) && ldo1 < (1L << 21));
  EpiParams ep{nullptr, 0, 1.0f, 1.0f, 0, g_dbg};
  return lc_gemm_nt_ex(stream, epi, M, N, K, A, lda, B, ldb, bias, alpha, out0, ldo0, out1, ldo1,
                       aux, ldaux, ep, ws, ws_bytes);
}

int lc_gemm_set_debug(unsigned long long* p) {
  g_dbg = p;
  return LC_OK;
}

int lc_gemm_nt_fp8(hipStream_t stream, int epi, int M, int N, int K, const void* A, long lda,
                   const void* sa, long sa_rows, const void* B, long ldb, const void* sb,
                   long sb_rows, const float* bias, float alpha, void* out0, long ldo0,
                   void* out1, long ldo1, const void* aux, long ldaux, void* ws, long ws_bytes,
                   void* q_scale, long q_rows) {
  LC_CHECK_ARG(M > 0 && N > 0 && K > 0 && K % 128 == 0 && N % 256 == 0);
  LC_CHECK_ARG(lda % 16 == 0 && ldb % 16 == 0 && lda >= K && ldb >= K);
  LC_CHECK_ARG(sa != nullptr && sb != nullptr && sa_rows >= (M + 255) / 256 * 256 &&
               sb_rows >= N && sa_rows % 256 == 0 && sb_rows % 256 == 0);
  LC_CHECK_ARG(((uintptr_t)sa & 15) == 0 && ((uintptr_t)sb & 15) == 0);
  LC_CHECK_ARG(epi == EPI_BF16 || epi == EPI_F32 || epi == EPI_RESID || epi == EPI_GELU ||
               epi == EPI_GELU_D || epi == EPI_MUL || epi == EPI_GELU_D_Q8 || epi == EPI_MUL_Q8 ||
               epi == EPI_RESID16);
  const bool q8 = epi == EPI_GELU_D_Q8 || epi == EPI_MUL_Q8;
  if (epi != EPI_MUL_Q8) LC_CHECK_ARG(out0 != nullptr && ldo0 % 8 == 0 && ldo0 >= N);
  if (epi == EPI_GELU || epi == EPI_GELU_D) LC_CHECK_ARG(out1 != nullptr && ldo1 >= N && ldo1 % 8 == 0);
  // fp8 output: 8-B code stores per lane, an operand-format scale buffer covering every row
  if (q8)
    LC_CHECK_ARG(out1 != nullptr && ldo1 >= N && ldo1 % 16 == 0 && ((uintptr_t)out1 & 15) == 0 &&
                 q_scale != nullptr && q_rows >= (M + 255) / 256 * 256 && q_rows % 256 == 0);
  if (epi == EPI_RESID || epi == EPI_MUL || epi == EPI_MUL_Q8 || epi == EPI_RESID16)
    LC_CHECK_ARG(aux != nullptr && ldaux >= N && ldaux % 8 == 0);
  LC_CHECK_ARG(ws == nullptr || (ws_bytes >= LC_SPLITK_TICKET_BYTES && ((uintptr_t)ws & 255) == 0));
  // the epilogue's buffer descriptors span one 256-row tile with 32-bit byte offsets: 256 rows
  // x ldo x 4 B (f32 outputs) must stay below 2^31 (num_records and the int offsets)
  LC_CHECK_ARG(ldo0 < (1L << 21) && ldo1 < (1L << 21));
  EpiParams ep{nullptr, 0, 1.0f, 1.0f, 0, g_dbg};
  ep.q_scale = q8 ? static_cast<uint8_t*>(q_scale) : nullptr;
  ep.q_rows = q_rows;
  Fp8Scales sc{static_cast<const uint8_t*>(sa), static_cast<const uint8_t*>(sb), sa_rows, sb_rows};
  return launch_g8<true>(stream, epi, M, N, K, A, lda, B, ldb, bias, alpha, out0, ldo0, out1, ldo1,
                         aux, ldaux, ep, ws, ws_bytes, sc);
}

int lc_gemm_set_tile(int tile) {
  LC_CHECK_ARG(tile >= 0 && tile <= 11);
  g_force_tile = tile;
  return LC_OK;
}

int lc_gemm_set_streamk(int mode) {
  LC_CHECK_ARG(mode >= 0 && mode <= 4);
  g_sk_mode = mode;
  return LC_OK;
}

int lc_gemm_tn(hipStream_t stream, int M, int N1, int N2, const void* A, long lda, const void* B,
               long ldb, float alpha, float* C, long ldc, float* colsum, float colsum_scale) {
  return lc_gemm_tn_ws(stream, M, N1, N2, A, lda, B, ldb, alpha, C, ldc, colsum, colsum_scale,
                       nullptr, 0);
}

int lc_gemm_tn_ws(hipStream_t stream, int M, int N1, int N2, const void* A, long lda,
                  const void* B, long ldb, float alpha, float* C, long ldc, float* colsum,
                  float colsum_scale, void* ws, long ws_bytes) {
  LC_CHECK_ARG(M > 0 && N1 > 0 && N2 > 0);
  // operand rows are read in 64-column blocks: they must be readable up to the next multiple
  // of 64 (zero padding); outputs beyond N1 x N2 are masked
  LC_CHECK_ARG(lda % 8 == 0 && ldb % 8 == 0 && lda >= (N1 + 63) / 64 * 64 &&
               ldb >= (N2 + 63) / 64 * 64 && ldc >= N2);
  if (N1 <= 64 || N2 <= 64) {
    // wide x skinny: the skinny side is the 64-column operand; C transposed when it is A
    const bool a_wide = N2 <= 64;
    TnProb p{};
    p.W = static_cast<const bf16_t*>(a_wide ? A : B);
    p.ldw = a_wide ? lda : ldb;
    p.S = static_cast<const bf16_t*>(a_wide ? B : A);
    p.lds = a_wide ? ldb : lda;
    p.C = C;
    p.ldc = ldc;
    p.Nw = a_wide ? N1 : N2;
    p.ns = a_wide ? N2 : N1;
    p.trans = a_wide ? 0 : 1;
    p.alpha = alpha;
    p.cs_w = a_wide ? colsum : nullptr;
    p.cs_w_scale = colsum_scale;
    p.cs_s = a_wide ? nullptr : colsum;
    p.cs_s_scale = colsum_scale;
    p.M = M;
    // with a workspace: 256-column panels (half the re-reads of the skinny operand) and the
    // two-stage reduction, when the wide side is a multiple of 256
    const bool wide = ws != nullptr && p.Nw % 256 == 0;
    p.pw = wide ? 256 : 128;
    p.n_tiles = (p.Nw + p.pw - 1) / p.pw;
    plan_tn(p, p.n_tiles);
    if (wide && ws_bytes >= LC_SPLITK_TICKET_BYTES + (long)p.wgs * tn_pslot(p.pw) * 4)
      p.part = reinterpret_cast<float*>(static_cast<char*>(ws) + LC_SPLITK_TICKET_BYTES);
    TnProb none{};
    if (p.pw == 256)
      hipLaunchKernelGGL(gemm_tn_wide_kernel<256>, dim3(p.wgs), dim3(512), 0, stream, p, none);
    else
      hipLaunchKernelGGL(gemm_tn_wide_kernel<128>, dim3(p.wgs), dim3(512), 0, stream, p, none);
    if (p.part) {
      const int outs = p.Nw * 64 + p.Nw + 64;
      hipLaunchKernelGGL(tn_reduce_kernel, dim3((outs + 255) / 256), dim3(256), 0, stream, p, none);
    }
    LC_LAUNCH_RET();
  }
  const int tiles = ((N1 + 63) / 64) * ((N2 + 63) / 64);
  // Enough M-chunks to give ~4 workgroups per CU, each chunk a multiple of 64 rows.
  int splits = (1024 + tiles - 1) / tiles;
  int chunk = (M + splits - 1) / splits;
  chunk = ((chunk + 63) / 64) * 64;
  if (chunk < 256) chunk = 256;
  splits = (M + chunk - 1) / chunk;
  dim3 grid(tiles, splits), block(256);
  hipLaunchKernelGGL(gemm_tn_kernel, grid, block, 0, stream, M, N1, N2, chunk,
                     static_cast<const bf16_t*>(A), lda, static_cast<const bf16_t*>(B), ldb, alpha,
                     C, ldc, colsum, colsum_scale);
  LC_LAUNCH_RET();
}

int lc_adapter_wgrad(hipStream_t stream, int M, int D, const void* gout, long ldg, const void* h,
                     const void* z, long ldz, const void* dpre, float scale, float* dWu,
                     float* dbu, float* dWd, float* dbd) {
  return lc_adapter_wgrad_ws(stream, M, D, gout, ldg, h, z, ldz, dpre, scale, dWu, dbu, dWd, dbd,
                             nullptr, 0);
}

static int adapter_wgrad(hipStream_t stream, int M, int D, const void* gout, long ldg,
                         const void* h, const void* z, long ldz, const void* dpre, float scale,
                         float* dWu, float* dbu, float* dWd, float* dbd, void* ws, long ws_bytes,
                         const float* div, int g16 = 0) {
  LC_CHECK_ARG(M > 0 && D > 0 && D % 64 == 0 && ldg % 8 == 0 && ldz % 8 == 0 && ldg >= D &&
               ldz >= D);
  LC_CHECK_ARG(dWu != nullptr && dWd != nullptr);
  TnProb up{}, down{};
  up.div = down.div = div;
  // dWu[D][64] += scale * gout^T h ; dbu += scale * colsum(gout)
  up.W = static_cast<const bf16_t*>(gout);
  up.w16 = g16;
  up.ldw = ldg;
  up.S = static_cast<const bf16_t*>(h);
  up.lds = 64;
  up.C = dWu;
  up.ldc = 64;
  up.Nw = D;
  up.ns = 64;
  up.trans = 0;
  up.alpha = scale;
  up.cs_w = dbu;
  up.cs_w_scale = scale;
  // 256-column W panels when D allows (half the re-reads of h / dpre, one per panel)
  const int pw = D % 256 == 0 ? 256 : 128;
  up.pw = pw;
  up.M = M;
  up.n_tiles = (D + pw - 1) / pw;
  // dWd[64][D] += dpre^T z = (z^T dpre)^T ; dbd += colsum(dpre)
  down.W = static_cast<const bf16_t*>(z);
  down.ldw = ldz;
  down.S = static_cast<const bf16_t*>(dpre);
  down.lds = 64;
  down.C = dWd;
  down.ldc = D;
  down.Nw = D;
  down.ns = 64;
  down.trans = 1;
  down.alpha = 1.0f;
  down.cs_s = dbd;
  down.cs_s_scale = 1.0f;
  down.pw = pw;
  down.M = M;
  down.n_tiles = (D + pw - 1) / pw;
  plan_tn(up, 2 * up.n_tiles);
  plan_tn(down, 2 * down.n_tiles);
#ifdef LC_DIAG_SKIP_WGRAD  // timing-knockout builds only (make EXTRA_FLAGS=-DLC_DIAG_SKIP_WGRAD)
  return LC_OK;
#endif
  // two-stage reduction when the workspace holds every walker's partial (after the split-K
  // ticket region, which must stay zero): plain stores + one small summing launch instead of
  // 8192 f32 atomics per walker
  const long need = (long)(up.wgs + down.wgs) * tn_pslot(pw) * 4;
  if (ws != nullptr && ws_bytes >= LC_SPLITK_TICKET_BYTES + need) {
    up.part = reinterpret_cast<float*>(static_cast<char*>(ws) + LC_SPLITK_TICKET_BYTES);
    down.part = up.part + (long)up.wgs * tn_pslot(pw);
  }
  if (pw == 256)
    hipLaunchKernelGGL(gemm_tn_wide_kernel<256>, dim3(up.wgs + down.wgs), dim3(512), 0, stream, up,
                       down);
  else
    hipLaunchKernelGGL(gemm_tn_wide_kernel<128>, dim3(up.wgs + down.wgs), dim3(512), 0, stream, up,
                       down);
  if (up.part) {
    const int outs = 2 * (D * 64 + D + 64);
    hipLaunchKernelGGL(tn_reduce_kernel, dim3((outs + 255) / 256), dim3(256), 0, stream, up, down);
  }
  LC_LAUNCH_RET();
}

int lc_adapter_wgrad_ws(hipStream_t stream, int M, int D, const void* gout, long ldg,
                        const void* h, const void* z, long ldz, const void* dpre, float scale,
                        float* dWu, float* dbu, float* dWd, float* dbd, void* ws, long ws_bytes) {
  return adapter_wgrad(stream, M, D, gout, ldg, h, z, ldz, dpre, scale, dWu, dbu, dWd, dbd, ws,
                       ws_bytes, nullptr);
}

#ifndef LC_F16
int lc_adapter_wgrad_ws_unscaled(hipStream_t stream, int M, int D, const void* gout, long ldg,
                                 const void* h, const void* z, long ldz, const void* dpre,
                                 float scale, float* dWu, float* dbu, float* dWd, float* dbd,
                                 void* ws, long ws_bytes, const float* gscale) {
  LC_CHECK_ARG(gscale != nullptr);
  return adapter_wgrad(stream, M, D, gout, ldg, h, z, ldz, dpre, scale, dWu, dbu, dWd, dbd, ws,
                       ws_bytes, gscale);
}

// gout IEEE half (the image tower's half residual gradient, carrying the scale gscale)
int lc_adapter_wgrad_ws_unscaled_g16(hipStream_t stream, int M, int D, const void* gout, long ldg,
                                     const void* h, const void* z, long ldz, const void* dpre,
                                     float scale, float* dWu, float* dbu, float* dWd, float* dbd,
                                     void* ws, long ws_bytes, const float* gscale) {
  LC_CHECK_ARG(gscale != nullptr);
  return adapter_wgrad(stream, M, D, gout, ldg, h, z, ldz, dpre, scale, dWu, dbu, dWd, dbd, ws,
                       ws_bytes, gscale, 1);
}
#endif

}  // extern "C"
