// GPU train transform of the online step: the torchvision Compose of
// methods/_trainer.py:236-242 applied to the uint8-quantised batch on the GPU
// (methods/adapter_clip.py:81):
//   [autoaug branch, _trainer.py:216/229: x -> (x*255).type(uint8) -> .float()/255]
//   Resize((R, R))              bilinear, align_corners = False (upsampling: antialias inert)
//   RandomCrop(R, padding=pad)  zero pad on every side, crop at (crop_i, crop_j)
//   RandomHorizontalFlip()      whole batch when flip != 0 (torchvision draws once per call)
//   Normalize(mean, std)        (v - mean[c]) / std[c]  (LDS kernel: v * (1/std) - mean/std)
// One pass, no intermediate image: every output pixel gathers its 4 bilinear taps straight from
// the small input (a 32x32 CIFAR image is 12 KB, L2-resident), so the kernel is bound by its
// output stream. layout 0 writes the f32 NCHW batch the reference feeds the model; layout 1
// writes the bf16 patch rows of conv1's GEMM ([n*g*g, C*P*P], the lc_patchify layout) directly,
// skipping the f32 image round trip.
#include "lc_common.h"

namespace {

struct TfParams {
  float mean[4], std_[4];
  float inv_std[4], nbias[4];  // 1/std and -mean/std (the LDS kernel's fused normalise)
};

// One bilinear blend a (1 - l) + b l as an explicit FMA on the rounded first product, so every
// kernel (f32 NCHW, patch rows, separable) rounds the same way: the f32 image and the patch rows
// stay bit-identical whichever kernel wrote them.
LC_DEV float lerp1(float a, float b, float l) { return __builtin_fmaf(b, l, a * (1.f - l)); }

// torch upsample_bilinear2d (align_corners = False) source index and weight along one axis
LC_DEV void lin_src(int dst, float scale, int in, int& i0, int& i1, float& l1) {
  float src = scale * (dst + 0.5f) - 0.5f;
  src = src < 0.f ? 0.f : src;
  int i = (int)src;  // floor (src >= 0)
  i = i < in - 1 ? i : in - 1;
  float l = src - (float)i;
  l = l < 0.f ? 0.f : (l > 1.f ? 1.f : l);
  i0 = i;
  i1 = i + (i < in - 1 ? 1 : 0);
  l1 = l;
}

LC_DEV float quant(float v, int q) {
  if (!q) return v;
  const float t = v * 255.0f;                       // (x * 255).type(torch.uint8): truncation
  int u = (int)t;
  u = u < 0 ? 0 : (u > 255 ? 255 : u);
  return (float)u / 255.0f;                        // .type(torch.float32) / 255
}

__global__ void __launch_bounds__(256)
train_transform_kernel(int n, int C, int Hin, int Win, const float* __restrict__ x, int R, int pad,
                       int crop_i, int crop_j, int flip, TfParams tp, int quantize, int layout,
                       int P, void* __restrict__ out) {
  const int q4 = R / 4;
  const long total = (long)n * C * R * q4;
  const float sh = (float)Hin / (float)R, sw = (float)Win / (float)R;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const int xq = (int)(e % q4);
    const long r1 = e / q4;
    const int y = (int)(r1 % R);
    const long r2 = r1 / R;
    const int c = (int)(r2 % C);
    const int img = (int)(r2 / C);
    const float* src = x + ((long)img * C + c) * Hin * Win;
    float v[4];
    const int py = y + crop_i - pad;  // row in the resized image (RandomCrop after zero pad)
    int y0 = 0, y1 = 0;
    float ly = 0.f;
    const bool row_in = py >= 0 && py < R;
    if (row_in) lin_src(py, sh, Hin, y0, y1, ly);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int xo = xq * 4 + k;
      const int xs = flip ? (R - 1 - xo) : xo;  // hflip after the crop
      const int px = xs + crop_j - pad;
      float val = 0.f;                           // RandomCrop's zero fill
      if (row_in && px >= 0 && px < R) {
        int x0, x1;
        float lx;
        lin_src(px, sw, Win, x0, x1, lx);
        const float a = quant(src[y0 * Win + x0], quantize), b = quant(src[y0 * Win + x1], quantize);
        const float cc = quant(src[y1 * Win + x0], quantize), d = quant(src[y1 * Win + x1], quantize);
        val = lerp1(lerp1(a, b, lx), lerp1(cc, d, lx), ly);
      }
      v[k] = (val - tp.mean[c]) / tp.std_[c];
    }
    if (layout == 0) {
      float* o = static_cast<float*>(out) + (((long)img * C + c) * R + y) * R + xq * 4;
      *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      const int g = R / P;
      const int pyi = y / P, ky = y % P, pxi = (xq * 4) / P, kx = (xq * 4) % P;
      const long row = ((long)img * g + pyi) * g + pxi;
      bf16_t* o = static_cast<bf16_t*>(out) + row * (C * P * P) + (c * P + ky) * P + kx;
      *reinterpret_cast<uint2*>(o) = uint2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
    }
  }
}

// Per output row / column of the workgroup's image: the two source taps and the weight of the
// second after crop, pad and flip (ok = 0: RandomCrop's zero fill). Built once per workgroup in
// LDS. Each thread owns FIXED output columns (their taps live in registers) and walks rows, so a
// pixel costs four LDS tap reads and seven FMAs; the row tap is one LDS read per row.
struct Tap {
  int i0, i1;
  float l1;
  int ok;
};

// NV pixels of one output row from the LDS-resident (quantised) image; normalise as
// x * (1/std) - mean/std, within one f32 rounding of torchvision's (x - mean) / std.
template <int NV>
LC_DEV void tf_row(const float* __restrict__ simg, const Tap& ry, const Tap (&cx)[NV], int c,
                   int Hin, int Win, float inv, float bias, float (&v)[NV]) {
  const float* r0 = simg + (c * Hin + ry.i0) * Win;
  const float* r1 = simg + (c * Hin + ry.i1) * Win;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    float val = 0.f;
    if (ry.ok & cx[k].ok) {
      const float top = lerp1(r0[cx[k].i0], r0[cx[k].i1], cx[k].l1);
      const float bot = lerp1(r1[cx[k].i0], r1[cx[k].i1], cx[k].l1);
      val = lerp1(top, bot, ry.l1);
    }
    v[k] = __builtin_fmaf(val, inv, bias);
  }
}

// Small inputs (CIFAR: 3 x 32 x 32 f32 = 12 KiB): a workgroup stages the quantised image in LDS
// once and streams its share of the output in the final order, 16 B per lane per store —
// coalesced whole rows (layout 0: NCHW f32) or whole patch rows (layout 1: conv1's bf16 im2col,
// patch 16). Work split: layout 0 — thread = 4 fixed columns, rows strided over the workgroups
// of the image (gridDim.y); layout 1 — thread = one 8-column chunk of a patch row and a fixed
// patch column, walking the patch rows.
template <int LAYOUT>
__global__ void __launch_bounds__(256)
train_transform_lds_kernel(int C, int Hin, int Win, const float* __restrict__ x, int R, int pad,
                           int crop_i, int crop_j, int flip, TfParams tp, int quantize,
                           void* __restrict__ out) {
  extern __shared__ float simg[];  // [C*Hin*Win] image, then the row and column tap tables
  const int img = blockIdx.x;
  const int tot = C * Hin * Win;
  Tap* rows = reinterpret_cast<Tap*>(simg + ((tot + 3) & ~3));
  Tap* cols = rows + R;
  const float* src = x + (long)img * tot;
  for (int k = threadIdx.x; k < tot; k += blockDim.x) simg[k] = quant(src[k], quantize);
  const float sh = (float)Hin / (float)R, sw = (float)Win / (float)R;
  for (int k = threadIdx.x; k < 2 * R; k += blockDim.x) {
    const bool is_row = k < R;
    const int o = is_row ? k : k - R;
    // row: RandomCrop offset only; column: hflip of the cropped window, then the offset
    const int p = is_row ? o + crop_i - pad : (flip ? R - 1 - o : o) + crop_j - pad;
    Tap tp_{0, 0, 0.f, 0};
    if (p >= 0 && p < R) {
      lin_src(p, is_row ? sh : sw, is_row ? Hin : Win, tp_.i0, tp_.i1, tp_.l1);
      tp_.ok = 1;
    }
    (is_row ? rows : cols)[o] = tp_;
  }
  __syncthreads();
  if constexpr (LAYOUT == 0) {
    const int q4 = R / 4, nrg = blockDim.x / q4;
    const int xq = threadIdx.x % q4, rg = threadIdx.x / q4;
    if (rg >= nrg) return;
    Tap cx[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) cx[k] = cols[xq * 4 + k];
    float* o = static_cast<float*>(out) + (long)img * C * R * R + xq * 4;
    for (int r = blockIdx.y * nrg + rg; r < C * R; r += gridDim.y * nrg) {
      const int c = r / R, y = r - c * R;
      float v[4];
      tf_row<4>(simg, rows[y], cx, c, Hin, Win, tp.inv_std[c], tp.nbias[c], v);
      *reinterpret_cast<float4*>(o + (long)r * R) = make_float4(v[0], v[1], v[2], v[3]);
    }
  } else {
    constexpr int P = 16;
    const int g = R / P, row_len = C * P * P, per_row = row_len / 8, npg = blockDim.x / per_row;
    const int chunk = threadIdx.x % per_row, pg = threadIdx.x / per_row;
    const int pxi = blockIdx.y * npg + pg;
    if (pg >= npg || pxi >= g) return;
    const int col = chunk * 8, c = col / (P * P), rem = col % (P * P);
    const int ky = rem / P, x0 = pxi * P + rem % P;
    Tap cx[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) cx[k] = cols[x0 + k];
    const float inv = tp.inv_std[c], bias = tp.nbias[c];
    bf16_t* o = static_cast<bf16_t*>(out) + ((long)img * g * g + pxi) * row_len + col;
    for (int pyi = 0; pyi < g; ++pyi) {
      float v[8];
      tf_row<8>(simg, rows[pyi * P + ky], cx, c, Hin, Win, inv, bias, v);
      *reinterpret_cast<uint4*>(o + (long)pyi * g * row_len) =
          uint4{pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7])};
    }
  }
}

// Separable form of the layout-1 (conv1 patch rows) transform, one workgroup per (image,
// channel): the horizontal pass runs once per SOURCE row — Hs[i][x] = r_i[c0(x)] (1 - lx) +
// r_i[c1(x)] lx for the Hin source rows and the R output columns (crop, flip and zero fill
// folded into the column taps) — and every output pixel is then Hs[y0][x] (1 - ly) + Hs[y1][x] ly,
// read as two 16-B LDS vectors per 8 pixels. Same f32 operations in the same order as tf_row
// (lerp1 top / bottom per source row, then the vertical lerp1 and the normalising FMA: the f32
// image through lc_patchify and these patch rows are bit-identical); the LDS-read
// count per pixel drops from 4 scalar reads to 0.5 vector reads, which bounded tf_row's kernel
// (1.7 TB/s of output). Output: 8 bf16 (16 B) per lane, lanes in patch-row order (512 B runs).
__global__ void __launch_bounds__(256)
train_transform_sep_kernel(int C, int Hin, int Win, const float* __restrict__ x, int R, int pad,
                           int crop_i, int crop_j, int flip, TfParams tp, int quantize,
                           bf16_t* __restrict__ out) {
  extern __shared__ float sep_lds[];
  const int img = blockIdx.x, c = blockIdx.y, tid = threadIdx.x;
  const int npx = Hin * Win;
  float* simg = sep_lds;                               // [Hin][Win]
  float* hs = sep_lds + ((npx + 3) & ~3);              // [Hin][R]
  Tap* rows = reinterpret_cast<Tap*>(hs + Hin * R);    // [R]
  Tap* cols = rows + R;                                // [R]
  const float* src = x + ((long)img * C + c) * npx;
  for (int k = tid; k < npx; k += blockDim.x) simg[k] = quant(src[k], quantize);
  const float sh = (float)Hin / (float)R, sw = (float)Win / (float)R;
  for (int k = tid; k < 2 * R; k += blockDim.x) {
    const bool is_row = k < R;
    const int o = is_row ? k : k - R;
    const int p = is_row ? o + crop_i - pad : (flip ? R - 1 - o : o) + crop_j - pad;
    Tap t{0, 0, 0.f, 0};
    if (p >= 0 && p < R) {
      lin_src(p, is_row ? sh : sw, is_row ? Hin : Win, t.i0, t.i1, t.l1);
      t.ok = 1;
    }
    (is_row ? rows : cols)[o] = t;
  }
  __syncthreads();
  for (int k = tid; k < Hin * R; k += blockDim.x) {
    const int i = k / R, xo = k - i * R;
    const Tap t = cols[xo];
    const float* r = simg + i * Win;
    hs[k] = t.ok ? lerp1(r[t.i0], r[t.i1], t.l1) : 0.f;
  }
  __syncthreads();
  constexpr int P = 16;
  const int g = R / P;
  const float inv = tp.inv_std[c], bias = tp.nbias[c];
  const long row_len = (long)C * P * P;
  bf16_t* o = out + (long)img * g * g * row_len + c * P * P;
  // chunk = ((pyi * g + pxi) * P + ky) * 2 + half: 8 output columns of one patch row
  for (int ch = tid; ch < g * g * P * 2; ch += blockDim.x) {
    const int half = ch & 1, ky = (ch >> 1) & (P - 1), pq = ch >> 5;
    const int pyi = pq / g, pxi = pq - pyi * g;
    const int y = pyi * P + ky, x0 = pxi * P + half * 8;
    const Tap ry = rows[y];
    const float4* a = reinterpret_cast<const float4*>(hs + ry.i0 * R + x0);
    const float4* b = reinterpret_cast<const float4*>(hs + ry.i1 * R + x0);
    const float4 t0 = a[0], t1 = a[1], u0 = b[0], u1 = b[1];
    const float top[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
    const float bot[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float val = ry.ok ? lerp1(top[k], bot[k], ry.l1) : 0.f;
      v[k] = __builtin_fmaf(val, inv, bias);
    }
    *reinterpret_cast<uint4*>(o + (long)pq * row_len + ky * P + half * 8) =
        uint4{pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7])};
  }
}

}  // namespace

extern "C" {

int lc_train_transform(hipStream_t st, int n, int C, int Hin, int Win, const float* x, int R,
                       int pad, int crop_i, int crop_j, int flip, const float* mean_host,
                       const float* std_host, int quantize, int layout, int patch, void* out) {
  LC_CHECK_ARG(n > 0 && C >= 1 && C <= 4 && Hin > 0 && Win > 0 && R > 0 && R % 4 == 0);
  LC_CHECK_ARG(pad >= 0 && crop_i >= 0 && crop_j >= 0 && crop_i <= 2 * pad && crop_j <= 2 * pad);
  LC_CHECK_ARG(mean_host != nullptr && std_host != nullptr && x != nullptr && out != nullptr);
  LC_CHECK_ARG(layout == 0 || (layout == 1 && patch > 0 && patch % 4 == 0 && R % patch == 0));
  TfParams tp{};
  for (int c = 0; c < C; ++c) {
    LC_CHECK_ARG(std_host[c] != 0.f);
    tp.mean[c] = mean_host[c];
    tp.std_[c] = std_host[c];
    tp.inv_std[c] = 1.0f / std_host[c];
    tp.nbias[c] = -mean_host[c] / std_host[c];
  }
  const size_t img_bytes = (size_t)((C * Hin * Win + 3) & ~3) * sizeof(float) + 2 * R * 16;
  if (img_bytes <= 64 * 1024 && layout == 0 && R / 4 <= 256) {
    const int q4 = R / 4, nrg = 256 / q4;
    hipLaunchKernelGGL(train_transform_lds_kernel<0>, dim3(n, 8),  // 8 workgroups per image
                       dim3(nrg * q4), img_bytes, st, C,
                       Hin, Win, x, R, pad, crop_i, crop_j, flip, tp, quantize, out);
    LC_LAUNCH_RET();
  }
  // conv1 patch rows (the product path): the separable kernel when a channel's source rows
  // resized to R columns fit in LDS beside the channel (CIFAR: 4 + 28 + 7 KB)
  const size_t sep_bytes =
      (size_t)(((Hin * Win + 3) & ~3) + Hin * R) * sizeof(float) + 2 * (size_t)R * sizeof(Tap);
  if (layout == 1 && patch == 16 && R % 16 == 0 && sep_bytes <= 64 * 1024) {
    hipLaunchKernelGGL(train_transform_sep_kernel, dim3(n, C), dim3(256), sep_bytes, st, C, Hin,
                       Win, x, R, pad, crop_i, crop_j, flip, tp, quantize, static_cast<bf16_t*>(out));
    LC_LAUNCH_RET();
  }
  if (img_bytes <= 64 * 1024 && layout == 1 && patch == 16 && C * 32 <= 256) {
    const int per_row = C * 32, npg = 256 / per_row, g = R / 16;
    hipLaunchKernelGGL(train_transform_lds_kernel<1>, dim3(n, (g + npg - 1) / npg),
                       dim3(npg * per_row), img_bytes, st, C, Hin, Win, x, R, pad, crop_i, crop_j,
                       flip, tp, quantize, out);
    LC_LAUNCH_RET();
  }
  // large inputs: per-pixel gathers straight from global memory
  const long total = (long)n * C * R * (R / 4);
  long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(train_transform_kernel, dim3((unsigned)blocks), dim3(256), 0, st, n, C, Hin,
                     Win, x, R, pad, crop_i, crop_j, flip, tp, quantize, layout, patch, out);
  LC_LAUNCH_RET();
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// AutoAugment ops on the uint8 batch (the 'autoaug' branch of methods/_trainer.py:215-229:
// (x*255).type(uint8) -> transforms.AutoAugment(policy) -> .float()/255). torchvision draws one
// sub-policy per call for the whole batch tensor; the host (lcclip/transforms.py) draws it and
// passes the active ops, each restated here from torchvision 0.16's tensor functional ops:
//   INVERT      255 - v
//   BLEND       (c1 * v + c2 * other).clamp(0, 255) truncated to uint8 (_blend), with other =
//               0 (adjust_brightness), the uint8-truncated grayscale (adjust_saturation), its
//               per-image mean (adjust_contrast), or the 3x3 [1 1 1; 1 5 1; 1 1 1]/13 blur,
//               rounded, borders kept (adjust_sharpness)
//   POSTERIZE   v & mask;  SOLARIZE  v >= thr ? 255 - v : v
//   AUTOCONTRAST per image+channel ((v - min) * (255 / (max - min))).clamp truncated (min = 0,
//               scale = 1 where max == min; the scale is torch's reciprocal(max - min) * 255)
//   EQUALIZE    per image+channel histogram LUT: step = (sum of the non-zero bins but the last)
//               // 255; lut[k] = (cumsum[k-1] + step // 2) // step (lut[0] = 0), identity when
//               step == 0
//   AFFINE      nearest grid_sample (align_corners = False, zero fill) on torchvision's affine
//               grid: base (x, y) = (j - W/2 + 0.5, i - H/2 + 0.5), g = (x r0 + y r1) + r2 /
//               (x r3 + y r4) + r5 with the host's rescaled inverse matrix, source index =
//               rint(((g + 1) * size - 1) / 2) (ShearX/Y, TranslateX/Y, Rotate)
// One workgroup per image, the image resident in LDS (C*H*W <= 12288: CIFAR 32x32, Tiny-
// ImageNet 64x64). f32 arithmetic is written op by op (no contraction) in torch's order so the
// result is bit-identical to the oracle's restatement (oracle/clip_oracle.py autoaugment).
namespace {

enum { AA_INVERT = 0, AA_BLEND_ZERO = 1, AA_BLEND_GRAY = 2, AA_BLEND_MEAN = 3, AA_BLEND_BLUR = 4,
       AA_POSTERIZE = 5, AA_SOLARIZE = 6, AA_AUTOCONTRAST = 7, AA_EQUALIZE = 8, AA_AFFINE = 9 };

struct AugOps {
  int n;
  int code[2];
  float p[2][6];
};

LC_DEV int trunc_u8(float v) {  // .clamp(0, 255).to(torch.uint8)
  v = fminf(fmaxf(v, 0.f), 255.f);
  return (int)v;
}

LC_DEV int gray_u8(int r, int g, int b) {  // rgb_to_grayscale(uint8): (0.2989r + 0.587g + 0.114b).to(uint8)
  const float s = __fadd_rn(__fadd_rn(__fmul_rn(0.2989f, (float)r), __fmul_rn(0.587f, (float)g)),
                            __fmul_rn(0.114f, (float)b));
  return (int)s;
}

// GLB = false: both working images in LDS (C*H*W <= 12288). GLB = true (larger images, e.g.
// ImageNet-R at 3 x 224 x 224): the current image lives in this image's slice of `out` (as ints,
// converted to f32 in place at the end) and the scratch image in the caller's workspace `ws`;
// the histogram / reductions stay in LDS. Same arithmetic in the same order either way: the two
// forms are bit-identical (tests/test_autoaug_gpu.py).
template <bool GLB>
__global__ void __launch_bounds__(256)
autoaug_kernel(int C, int H, int W, const float* __restrict__ x, float* out, AugOps ops, int* ws) {
  extern __shared__ int sm[];
  const int HW = H * W, tot = C * HW;
  int* a;     // current image
  int* b;     // scratch image
  int* hist;  // [C][256] histogram / LUT
  if constexpr (GLB) {
    a = reinterpret_cast<int*>(out) + (long)blockIdx.x * tot;
    b = ws + (long)blockIdx.x * tot;
    hist = sm;
  } else {
    a = sm;
    b = sm + tot;
    hist = b + tot;
  }
  int* red = hist + 4 * 256;   // reductions: [0..3] min, [4..7] max, [8] gray sum
  const int tid = threadIdx.x;
  const float* src = x + (long)blockIdx.x * tot;
  for (int k = tid; k < tot; k += blockDim.x) {
    const float t = src[k] * 255.0f;  // (x * 255).type(torch.uint8)
    int u = (int)t;
    a[k] = u < 0 ? 0 : (u > 255 ? 255 : u);
  }
  __syncthreads();
  for (int o = 0; o < ops.n; ++o) {
    const int code = ops.code[o];
    const float* p = ops.p[o];
    if (code == AA_INVERT || code == AA_POSTERIZE || code == AA_SOLARIZE) {
      const int mask = (int)p[0];
      for (int k = tid; k < tot; k += blockDim.x) {
        const int v = a[k];
        a[k] = code == AA_INVERT ? 255 - v
               : code == AA_POSTERIZE ? (v & mask)
                                      : ((float)v >= p[0] ? 255 - v : v);
      }
    } else if (code >= AA_BLEND_ZERO && code <= AA_BLEND_BLUR) {
      const float c1 = p[0], c2 = p[1];
      float mean = 0.f;
      if (code == AA_BLEND_MEAN) {
        if (tid == 0) red[8] = 0;
        __syncthreads();
        int s = 0;
        for (int k = tid; k < HW; k += blockDim.x) s += gray_u8(a[k], a[HW + k], a[2 * HW + k]);
        atomicAdd(&red[8], s);
        __syncthreads();
        mean = (float)red[8] / (float)HW;  // exact integer sum, one rounding
      }
      if (code == AA_BLEND_BLUR && (H <= 2 || W <= 2)) continue;  // adjust_sharpness: identity
      for (int k = tid; k < tot; k += blockDim.x) {
        const int c = k / HW, pix = k - c * HW, i = pix / W, j = pix - i * W;
        float other = 0.f;
        if (code == AA_BLEND_GRAY) {
          other = (float)gray_u8(a[pix], a[HW + pix], a[2 * HW + pix]);
        } else if (code == AA_BLEND_MEAN) {
          other = mean;
        } else if (code == AA_BLEND_BLUR) {
          if (i == 0 || j == 0 || i == H - 1 || j == W - 1) {
            other = (float)a[k];
          } else {
            const float w1 = p[2], w5 = p[3];  // f32 1/13 and 5/13
            float s = 0.f;
            for (int di = -1; di <= 1; ++di)
              for (int dj = -1; dj <= 1; ++dj)
                s = __fadd_rn(s, __fmul_rn((float)a[k + di * W + dj], (di | dj) ? w1 : w5));
            other = rintf(s);  // _cast_squeeze_out: round, then uint8
          }
        }
        b[k] = trunc_u8(__fadd_rn(__fmul_rn(c1, (float)a[k]), __fmul_rn(c2, other)));
      }
      __syncthreads();
      int* t = a; a = b; b = t;
    } else if (code == AA_AUTOCONTRAST) {
      if (tid < 4) { red[tid] = 255; red[4 + tid] = 0; }
      __syncthreads();
      for (int k = tid; k < tot; k += blockDim.x) {
        const int c = k / HW;
        atomicMin(&red[c], a[k]);
        atomicMax(&red[4 + c], a[k]);
      }
      __syncthreads();
      for (int k = tid; k < tot; k += blockDim.x) {
        const int c = k / HW;
        float mn = (float)red[c];
        // `bound / (max - min)` with a Python-int numerator is Tensor.__rtruediv__:
        // reciprocal(max - min) * 255, two roundings
        float sc = __fmul_rn(__frcp_rn((float)red[4 + c] - mn), 255.0f);
        if (!isfinite(sc)) { mn = 0.f; sc = 1.0f; }
        a[k] = trunc_u8(__fmul_rn((float)a[k] - mn, sc));
      }
    } else if (code == AA_EQUALIZE) {
      for (int k = tid; k < C * 256; k += blockDim.x) hist[k] = 0;
      __syncthreads();
      for (int k = tid; k < tot; k += blockDim.x) atomicAdd(&hist[(k / HW) * 256 + a[k]], 1);
      __syncthreads();
      // one wave per channel, 4 bins per lane: the last non-zero bin (max), the sum below it and
      // the cumulative sum (wave scans) instead of three 256-step serial loops with a division each
      const int wv = tid >> 6, ln = tid & 63;
      if (wv < C) {
        int* h = hist + wv * 256;
        int hv[4], lastl = -1;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          hv[j] = h[4 * ln + j];
          if (hv[j] != 0) lastl = 4 * ln + j;
        }
        int last = lastl;  // the last non-zero bin (0 when none)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) last = max(last, __shfl_xor(last, o));
        last = last < 0 ? 0 : last;
        int part = 0, cl[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          part += (4 * ln + j < last) ? hv[j] : 0;
          cl[j] = (j ? cl[j - 1] : 0) + hv[j];  // lane-local inclusive cumsum
        }
        int sum = part;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
        const int step = sum / 255;
        if (step == 0) {
#pragma unroll
          for (int j = 0; j < 4; ++j) h[4 * ln + j] = 4 * ln + j;  // unchanged channel
        } else {
          int off = cl[3];  // inclusive scan of the lane totals, then exclusive
#pragma unroll
          for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(off, o);
            if (ln >= o) off += y;
          }
          off -= cl[3];
          int lut[4];  // lut before the shift: (cumsum + step // 2) // step, clamped
#pragma unroll
          for (int j = 0; j < 4; ++j) lut[j] = min((off + cl[j] + step / 2) / step, 255);
          int prev = __shfl_up(lut[3], 1);  // pad [1, 0], drop the last
          if (ln == 0) prev = 0;
          h[4 * ln] = prev;
          h[4 * ln + 1] = lut[0];
          h[4 * ln + 2] = lut[1];
          h[4 * ln + 3] = lut[2];
        }
      }
      __syncthreads();
      for (int k = tid; k < tot; k += blockDim.x) a[k] = hist[(k / HW) * 256 + a[k]];
    } else if (code == AA_AFFINE) {
      for (int k = tid; k < tot; k += blockDim.x) {
        const int c = k / HW, pix = k - c * HW, i = pix / W, j = pix - i * W;
        const float xb = (float)j - 0.5f * (float)W + 0.5f, yb = (float)i - 0.5f * (float)H + 0.5f;
        const float gx = __fadd_rn(__fadd_rn(__fmul_rn(xb, p[0]), __fmul_rn(yb, p[1])), p[2]);
        const float gy = __fadd_rn(__fadd_rn(__fmul_rn(xb, p[3]), __fmul_rn(yb, p[4])), p[5]);
        const float ix = __fdiv_rn(__fsub_rn(__fmul_rn(__fadd_rn(gx, 1.f), (float)W), 1.f), 2.f);
        const float iy = __fdiv_rn(__fsub_rn(__fmul_rn(__fadd_rn(gy, 1.f), (float)H), 1.f), 2.f);
        const int sx = (int)rintf(ix), sy = (int)rintf(iy);
        b[k] = (sx >= 0 && sx < W && sy >= 0 && sy < H) ? a[c * HW + sy * W + sx] : 0;
      }
      __syncthreads();
      int* t = a; a = b; b = t;
    }
    __syncthreads();
  }
  float* dst = out + (long)blockIdx.x * tot;
  // .float() / 255 (GLB: a may be dst itself; each lane converts the elements it reads)
  for (int k = tid; k < tot; k += blockDim.x) dst[k] = (float)a[k] / 255.0f;
}

}  // namespace

extern "C" {

// Images larger than the LDS form (C*H*W > 12288) need ws: n * C*H*W ints (lc_autoaugment_ws)
static int autoaug_launch(hipStream_t st, int n, int C, int H, int W, const float* x, float* out,
                          int n_ops, const int* codes, const float* params, void* ws,
                          long ws_bytes) {
  LC_CHECK_ARG(n > 0 && C >= 1 && C <= 4 && H > 0 && W > 0);
  LC_CHECK_ARG(n_ops >= 0 && n_ops <= 2 && x != nullptr && out != nullptr);
  LC_CHECK_ARG(n_ops == 0 || (codes != nullptr && params != nullptr));
  const long tot = (long)C * H * W;
  const bool glb = tot > 12288;
  LC_CHECK_ARG(tot <= (1L << 30) / n);
  LC_CHECK_ARG(!glb || (ws != nullptr && ws_bytes >= (long)n * tot * (long)sizeof(int) &&
                        (reinterpret_cast<uintptr_t>(out) & 3) == 0));
  AugOps ops{};
  ops.n = n_ops;
  for (int o = 0; o < n_ops; ++o) {
    LC_CHECK_ARG(codes[o] >= AA_INVERT && codes[o] <= AA_AFFINE);
    LC_CHECK_ARG(!(codes[o] == AA_BLEND_GRAY || codes[o] == AA_BLEND_MEAN) || C == 3);
    ops.code[o] = codes[o];
    for (int k = 0; k < 6; ++k) ops.p[o][k] = params[o * 6 + k];
  }
  if (glb) {
    const size_t shm = (size_t)(4 * 256 + 16) * sizeof(int);
    hipLaunchKernelGGL(autoaug_kernel<true>, dim3(n), dim3(256), shm, st, C, H, W, x, out, ops,
                       static_cast<int*>(ws));
  } else {
    const size_t shm = (size_t)(2 * tot + 4 * 256 + 16) * sizeof(int);
    hipLaunchKernelGGL(autoaug_kernel<false>, dim3(n), dim3(256), shm, st, C, H, W, x, out, ops,
                       nullptr);
  }
  LC_LAUNCH_RET();
}

int lc_autoaugment(hipStream_t st, int n, int C, int H, int W, const float* x, float* out,
                   int n_ops, const int* codes, const float* params) {
  LC_CHECK_ARG((long)C * H * W <= 12288);  // larger images: lc_autoaugment_ws
  return autoaug_launch(st, n, C, H, W, x, out, n_ops, codes, params, nullptr, 0);
}

int lc_autoaugment_ws(hipStream_t st, int n, int C, int H, int W, const float* x, float* out,
                      int n_ops, const int* codes, const float* params, void* ws, long ws_bytes) {
  return autoaug_launch(st, n, C, H, W, x, out, n_ops, codes, params, ws, ws_bytes);
}

}  // extern "C"
