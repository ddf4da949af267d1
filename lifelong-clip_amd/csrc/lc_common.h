// Shared device helpers for the MI355X (gfx950 / CDNA4) CLIP PEFT kernels.
// Wave = 64 lanes; MFMA = v_mfma_f32_16x16x32_bf16 (A/B: 8 bf16 per lane, C/D: 4 f32 per lane).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include "lc_clip.h"

// Schedule-changing environment overrides (tile family, split-K, raster groups, kernel forms)
// exist for same-box A/B experiments only: they are read in a diagnostic build (make DIAG=1,
// -DLC_DIAG_ENV). The production library ignores the environment, so a stray variable cannot
// change the shipped kernels' schedule.
inline const char* lc_diag_env(const char* name) {
#ifdef LC_DIAG_ENV
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

typedef uint16_t bf16_t;  // raw bf16 bits in global memory
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));  // 32 fp8 e4m3 (one 16x16x128 operand)

// 16-B nontemporal (streaming) global store: a large producer output that the next kernel reads
// once. Measured on the step's GEMM epilogues: c_fc + QuickGELU/' 297 -> 269 us,
// QKV fwd 171 -> 162 us, step +1.6 % (profiles/r02/epilogue_knockout.txt).
__device__ __forceinline__ void st_nt16(void* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  __builtin_nontemporal_store(i32x4{(int)a, (int)b, (int)c, (int)d}, reinterpret_cast<i32x4*>(p));
}

#define LC_DEV __device__ __forceinline__
#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))
#define GLB_PTR(p) ((const __attribute__((address_space(1))) void*)(p))

// Block-scaled fp8 operand format of the fp8 GEMMs (MX-style, OCP e4m3fn elements): a [rows, K]
// row-major e4m3 matrix plus one E8M0 scale byte per 32 consecutive k of a row (value =
// e4m3 * 2^(byte - 127)). The scale bytes are stored k-tile-major, [K/128][rows_pad][4]: the
// 4 bytes of (k-tile, row) are the 4 blocks of that row's 128 k — one 1-KiB contiguous piece per
// 256-row tile and k-tile. rows_pad = rows rounded up to 256 (tile loads never leave the buffer).
LC_DEV long fp8_scale_index(long row, int kblock, long rows_pad) {
  return ((long)(kblock >> 2) * rows_pad + row) * 4 + (kblock & 3);
}

// The 16-bit storage type. Every kernel reads, writes and multiplies its 16-bit operands only
// through the helpers below, so the same sources compile for two storage types:
//   default: bf16 (the image tower, BASELINE config 2's dtype);
//   -DLC_F16 (the second object of each 16-bit source, entry points suffixed _f16 by
//            lc_f16_names.h): IEEE half, the reference's autocast dtype
//            (methods/adapter_clip.py:87), used by the text tower.
// The names (bf16_t, bf16x8, bf2f, f2bf, pack2bf) stay those of the default build.
typedef float lc_f32x2 __attribute__((ext_vector_type(2)));
#ifdef LC_F16
typedef _Float16 lc_f16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 lc_f16x8 __attribute__((ext_vector_type(8)));
LC_DEV float bf2f(bf16_t h) { return (float)__builtin_bit_cast(_Float16, h); }
LC_DEV float bf2f_s(short h) { return (float)__builtin_bit_cast(_Float16, h); }
// fp32 -> half, round to nearest even (overflow to +-inf)
LC_DEV bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (_Float16)f); }
LC_DEV uint32_t pack2bf(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((lc_f32x2){lo, hi}, lc_f16x2));
}
LC_DEV f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(lc_f16x8, a),
                                                __builtin_bit_cast(lc_f16x8, b), c, 0, 0, 0);
}
#define LC_MFMA16_ASM "v_mfma_f32_16x16x32_f16"
#define LC_ONE16 ((short)0x3C00)  // 1.0
#else
LC_DEV float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
LC_DEV float bf2f_s(short h) { return __uint_as_float(((uint32_t)(uint16_t)h) << 16); }

// fp32 -> bf16, round to nearest even; lowers to v_cvt_pk_bf16_f32 (NaN-preserving).
LC_DEV bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return *reinterpret_cast<bf16_t*>(&b);
}
// Two values in one v_cvt_pk_bf16_f32. (Two scalar f2bf + shift/or made hipcc convert pairs in
// its own order and re-shuffle the halves: 2-3 extra VALU per pair in every bf16 epilogue.)
typedef __bf16 lc_bf16x2 __attribute__((ext_vector_type(2)));
LC_DEV uint32_t pack2bf(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((lc_f32x2){lo, hi}, lc_bf16x2));
}

LC_DEV f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
#define LC_MFMA16_ASM "v_mfma_f32_16x16x32_bf16"
#define LC_ONE16 ((short)0x3F80)  // 1.0
#endif

// The residual stream x of a tower: f32, or IEEE half (the reference's autocast dtype: its
// LayerNorm returns the input dtype, model.py:194-200, so x stays fp16 from conv1 on,
// model.py:756-766 and every `x = x + ...`). Independent of the 16-bit storage build above.
// xres<T>: element type (float or _Float16); load / round / store through these helpers.
typedef _Float16 lc_h16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 lc_h16x4 __attribute__((ext_vector_type(4)));
LC_DEV float h2f(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }
LC_DEV uint32_t pack2h(float lo, float hi) {  // round to nearest even
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((lc_f32x2){lo, hi}, lc_h16x2));
}
// the value a residual element of type XT holds (identity for f32)
template <typename XT>
LC_DEV float xround(float v) {
  if constexpr (sizeof(XT) == 2) return (float)(_Float16)v;
  else return v;
}

// Async 16-byte global -> LDS copy; LDS destination = wave-uniform base + lane * 16.
LC_DEV void glds16(const void* gsrc, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(GLB_PTR(gsrc), LDS_PTR(lds_wave_base), 16, 0, 0);
}
// 4-byte form: LDS destination = wave-uniform base + lane * 4.
LC_DEV void glds4(const void* gsrc, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(GLB_PTR(gsrc), LDS_PTR(lds_wave_base), 4, 0, 0);
}

LC_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
LC_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// QuickGELU (model.py:203-206): x * sigmoid(1.702 x), with the sigmoid as one v_exp_f32 and one
// v_rcp_f32 (1 ulp) — the IEEE division would cost ~10 VALU per element in the GEMM epilogues.
// exp2(-1.702*log2(e)*x) overflows to +inf for very negative x: rcp(inf) = 0, the right limit.
constexpr float LC_GELU_K2 = -1.702f * 1.4426950408889634f;
LC_DEV float lc_sigmoid1702(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(LC_GELU_K2 * x));
}
LC_DEV float quick_gelu(float x) { return x * lc_sigmoid1702(x); }
// d/dx [x s(x)] = s + 1.702 x s (1 - s) = s * (1 + t (1 - s)),  t = 1.702 x
LC_DEV float quick_gelu_grad(float x) {
  const float s = lc_sigmoid1702(x);
  const float t = 1.702f * x;
  return s * __builtin_fmaf(t, 1.0f - s, 1.0f);
}

// Counter-based hash RNG (splitmix-style) for adapter dropout masks: mask(seed, index) is a
// pure function, so backward regenerates the forward's mask without storing it.
LC_DEV uint32_t lc_hash(uint64_t seed, uint64_t idx) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (idx + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}

// Dropout multiplier for adapter bottleneck element (row m, column j): 1/keep or 0.
LC_DEV float drop_mul(uint64_t seed, long m, int j, float keep) {
  if (keep >= 1.0f) return 1.0f;
  const uint32_t hsh = lc_hash(seed, (uint64_t)m * 64 + j);
  const float u = (hsh >> 8) * (1.0f / 16777216.0f);
  return u < keep ? 1.0f / keep : 0.0f;
}

// Extra epilogue operands of the fused GEMM epilogues (internal).
struct EpiParams {
  const void* aux2;  // second side input (bf16), e.g. the adapter input z
  long ldaux2;
  float scale;       // adapter scalar
  float keep;        // 1 - dropout p
  uint64_t seed;     // dropout mask seed
  unsigned long long* dbg;  // diagnostic timestamps (nullptr in production)
  const unsigned long long* seed_dev;  // optional device-side RNG epoch added to seed (graphs)
  uint8_t* q_scale;  // fp8-output epilogues: E8M0 scales of the fp8 output ([N/128][q_rows][4])
  long q_rows;       // padded row count of that scale buffer
  int group_m;       // 256x256 GEMMs: tile raster groups of group_m row panels (0/1: row-major)
};

// fp8 operand scales of a block-scaled GEMM (see fp8_scale_index)
struct Fp8Scales {
  const uint8_t* sa;  // A's scales, rows_pad = sa_rows
  const uint8_t* sb;  // B's scales
  long sa_rows, sb_rows;
};

// E8M0 block scale of a 32-element block with max |x| = amax (OCP MX: 2^(floor(log2 amax) - 8),
// e4m3's largest power being 2^8), clamped to [2^-126, 2^126]; amax = 0 (or below the f32 normal
// range) -> byte 0, every element encodes to 0. A block holding a NaN or an infinity gets the MX
// NaN scale 0xFF and NaN codes (pack4_fp8), so a non-finite input stays non-finite through the
// fp8 GEMM: amax is reduced as the bit pattern of |x| (lc_amax_bits), where NaN and inf order
// above every finite value (fmaxf would drop the NaN).
LC_DEV uint32_t lc_amax_bits(uint32_t acc, float x) {
  const uint32_t b = __float_as_uint(x) & 0x7fffffffu;
  return acc > b ? acc : b;
}
LC_DEV uint32_t e8m0_of_bits(uint32_t amax_bits) {
  const int e = (int)(amax_bits >> 23);  // sign already cleared
  if (e == 0) return 0;
  if (e == 255) return 0xFF;  // NaN / inf in the block
  const int b = e - 8;
  return (uint32_t)(b < 1 ? 1 : (b > 253 ? 253 : b));
}
LC_DEV uint32_t e8m0_of(float amax) { return e8m0_of_bits(__float_as_uint(amax) & 0x7fffffffu); }
// 2^-(byte - 127) as f32 (the multiplier that maps a block into e4m3 range); byte 0 -> 0,
// byte 0xFF (NaN scale) -> NaN
LC_DEV float e8m0_inv(uint32_t byte) {
  if (byte == 0) return 0.f;
  if (byte == 0xFF) return __uint_as_float(0x7fc00000u);
  return __uint_as_float((uint32_t)(254 - byte) << 23);
}
// four f32 -> four e4m3fn bytes (RNE), saturated to +-448 first. The four values come from one
// scale block, so they are NaN together (NaN scale) or finite together: a NaN group encodes as
// the e4m3fn NaN code 0x7F (the clamp alone would turn NaN into -448).
LC_DEV uint32_t pack4_fp8(float a, float b, float c, float d) {
  // integer test: attention.o is built with -fno-honor-nans, where a != a folds to false
  const bool nan = (__float_as_uint(a) & 0x7fffffffu) > 0x7f800000u;
  a = fminf(fmaxf(a, -448.f), 448.f);
  b = fminf(fmaxf(b, -448.f), 448.f);
  c = fminf(fmaxf(c, -448.f), 448.f);
  d = fminf(fmaxf(d, -448.f), 448.f);
  uint32_t r = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  r = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, r, true);
  return nan ? 0x7f7f7f7fu : r;
}

// LDS images are XOR-swizzled in 32-B units so that the 8 rows {0..3, 8..11} (+16) one
// ds_read_b64_tr_b16 pass of 32 lanes touches land in 8 distinct 32-B bank groups.
//   W rows (256 or 512 B): unit u of row r at u ^ ((r & 3) | ((r >> 1) & 4)) (low 3 bits: a
//     row's bank offset only depends on u mod 8 for both widths)
//   S rows (128 B = 4 units; two rows per 256-B bank span): unit u at u ^ (((r >> 1) & 1) | ((r >> 2) & 2))
LC_DEV int swz_w(int r) { return (r & 3) | ((r >> 1) & 4); }
LC_DEV int swz_s(int r) { return ((r >> 1) & 1) | ((r >> 2) & 2); }

// 8 consecutive k-rows (row, row + 4 of the lane's 4-row group) of one 16-column block, as an
// MFMA operand: lane (g, t) gets column col0 + t, k = 8g .. 8g+7 of the 32-row k-slice.
template <int ROWB>
LC_DEV bf16x8 tr_frag(const char* lds, int row, int col) {
  auto addr = [&](int r) {
    const int byte = col * 2;  // within the row
    const int u = (byte >> 5) ^ (ROWB >= 256 ? swz_w(r) : swz_s(r));
    return lds + r * ROWB + u * 32 + (byte & 31);
  };
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) bf16x4*)addr(row));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) bf16x4*)addr(row + 4));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// Reads of LDS-DMA images inside a streaming loop. hipcc cannot tell a ring slot that has landed
// from the ones still in flight, so it puts s_waitcnt vmcnt(0) in front of a builtin LDS read of
// a global_load_lds target and in front of __syncthreads() — draining the ring every step. The
// forms below are inline asm: the caller owns the waits (lds_wait0 before the first use of a
// result, counted vmcnt waits before the barrier that publishes a slot).
// Wave-uniform raw-buffer descriptor over `bytes` bytes at p (stride 0). Accesses at offsets
// outside [0, bytes) are dropped (stores) or read 0 (loads) by the hardware range check, so a
// row guard needs no branch: hipcc's vmcnt bookkeeping stays exact across such accesses (a
// store under a branch makes it wait vmcnt(0) at the next use of an earlier load).
LC_DEV __amdgpu_buffer_rsrc_t lc_rsrc(const void* p, long bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane((int)bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, n, 0x00020000);
}
typedef unsigned int lc_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int lc_u32x2 __attribute__((ext_vector_type(2)));

// A half residual gradient read as a 16-bit MFMA operand (the image tower, bf16 build): 8 IEEE
// halves -> bf16 (round to nearest even), the values ln_bwd's bf16 copy of the same gradient
// held (norm.hip ln_bwd_kernel rounds to half, then to bf16), so consumers reading the half
// gradient directly reproduce the copy's results bit for bit. Identity in the LC_F16 build.
LC_DEV bf16x8 h2s8(bf16x8 v) {
#ifdef LC_F16
  return v;
#else
  // (written out per dword: the same conversion as a loop over u[k] / o[k] compiled to dword 0
  // converted and splatted into all four)
  const lc_u32x4 u = __builtin_bit_cast(lc_u32x4, v);
  const lc_f32x2 f0 = __builtin_convertvector(__builtin_bit_cast(lc_h16x2, (uint32_t)u.x), lc_f32x2);
  const lc_f32x2 f1 = __builtin_convertvector(__builtin_bit_cast(lc_h16x2, (uint32_t)u.y), lc_f32x2);
  const lc_f32x2 f2 = __builtin_convertvector(__builtin_bit_cast(lc_h16x2, (uint32_t)u.z), lc_f32x2);
  const lc_f32x2 f3 = __builtin_convertvector(__builtin_bit_cast(lc_h16x2, (uint32_t)u.w), lc_f32x2);
  return __builtin_bit_cast(bf16x8, (lc_u32x4{pack2bf(f0.x, f0.y), pack2bf(f1.x, f1.y),
                                              pack2bf(f2.x, f2.y), pack2bf(f3.x, f3.y)}));
#endif
}
// 8 bf16 -> IEEE half (round to nearest even; |x| < 2^-24 flushes to zero, as the reference's
// fp16 autocast cast of the same weight, methods/adapter_clip.py:87)
LC_DEV bf16x8 b2h8(bf16x8 v) {
  const lc_u32x4 u = __builtin_bit_cast(lc_u32x4, v);
  auto cv = [](uint32_t w) {
    return pack2h(__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u));
  };
  return __builtin_bit_cast(bf16x8, (lc_u32x4{cv(u.x), cv(u.y), cv(u.z), cv(u.w)}));
}
// v_mfma_f32_16x16x32_f16 on 8-half fragments (either storage build)
LC_DEV f32x4 mfma16_h(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b),
                                                c, 0, 0, 0);
}

LC_DEV uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}
template <int ROWB>
LC_DEV bf16x8 tr_frag_asm(uint32_t img, int row, int col) {
  auto addr = [&](int r) {
    const int byte = col * 2;
    const int u = (byte >> 5) ^ (ROWB >= 256 ? swz_w(r) : swz_s(r));
    return img + r * ROWB + u * 32 + (byte & 31);
  };
  bf16x4 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(addr(row)));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(addr(row + 4)));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
// all issued LDS reads retired; nothing is scheduled across the wait
LC_DEV void lds_wait0() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
// workgroup barrier for LDS hand-offs while LDS-DMA stays in flight (no vmcnt(0))
LC_DEV void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Internal launcher shared by the GEMM-shaped fused kernels (gemm.hip).
int lc_gemm_nt_ex(hipStream_t stream, int epi, int M, int N, int K, const void* A, long lda,
                  const void* B, long ldb, const float* bias, float alpha, void* out0, long ldo0,
                  void* out1, long ldo1, const void* aux, long ldaux, const EpiParams& ep,
                  void* ws = nullptr, long ws_bytes = 0);

// hipBLASLt for plain bf16 GEMMs that the step routes there (blaslt.hip, bf16 build only):
// C[M, N] = A[M, K] . B[N, K]^T, false when hipBLASLt cannot take the launch (nothing written)
bool lc_blaslt_nt_bf16(hipStream_t stream, int M, int N, int K, const void* A, long lda,
                       const void* B, long ldb, void* C, long ldo, void* ws, long ws_bytes);

#define LC_CHECK_ARG(cond) \
  do {                     \
    if (!(cond)) return LC_EINVAL; \
  } while (0)

#define LC_LAUNCH_RET()                                   \
  do {                                                    \
    hipError_t _e = hipGetLastError();                    \
    return _e == hipSuccess ? LC_OK : LC_ELAUNCH;         \
  } while (0)
