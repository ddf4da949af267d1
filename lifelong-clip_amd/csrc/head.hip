// Image-text logit head, forward + backward in one pass over the (small) B x C logit block:
//   models/clip/model.py:966-974  normalise, logits = exp(logit_scale) * I^ T^T
//   models/adapter_clip.py:99      probs = softmax(logits)
//   methods/adapter_clip.py:88-89  loss = CrossEntropyLoss(mean)(probs, y)   (CE on the
//                                  probabilities — the reference's double softmax, Q5)
// logit_scale is read from device memory (no host sync; it is frozen, Q12).
#include "lc_common.h"

namespace {

__global__ void __launch_bounds__(64)
l2norm_kernel(int R, int E, const float* __restrict__ f, long ldf, float* __restrict__ out,
              float* __restrict__ norms) {
  const int r = blockIdx.x, lane = threadIdx.x;
  const float* row = f + (long)r * ldf;
  float s = 0.f;
  for (int k = lane; k < E; k += 64) s += row[k] * row[k];
  const float nrm = sqrtf(wave_sum(s));
  const float inv = 1.0f / nrm;
  for (int k = lane; k < E; k += 64) out[(long)r * E + k] = row[k] * inv;
  if (lane == 0) norms[r] = nrm;
}

// one workgroup (256 threads) per image row b
__global__ void __launch_bounds__(256)
head_rows_kernel(int B, int C, int E, const float* __restrict__ img_n,
                 const float* __restrict__ txt_n, const float* __restrict__ logit_scale,
                 const int64_t* __restrict__ labels, float* __restrict__ probs,
                 float* __restrict__ dlogits, float* __restrict__ loss) {
  extern __shared__ float sh[];  // [E] image row + [C] logits
  float* irow = sh;
  float* lg = sh + E;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float s = __expf(*logit_scale);
  for (int k = tid; k < E; k += 256) irow[k] = img_n[(long)b * E + k];
  __syncthreads();
  for (int c = w; c < C; c += 4) {
    float d = 0.f;
    for (int k = lane; k < E; k += 64) d += irow[k] * txt_n[(long)c * E + k];
    d = wave_sum(d);
    if (lane == 0) lg[c] = s * d;
  }
  __syncthreads();
  if (w != 0) return;
  // softmax over logits -> p ; CE over p: loss_b = logsumexp(p) - p[y]
  float m = -INFINITY;
  for (int c = lane; c < C; c += 64) m = fmaxf(m, lg[c]);
  m = wave_max(m);
  float z = 0.f;
  for (int c = lane; c < C; c += 64) z += __expf(lg[c] - m);
  z = wave_sum(z);
  // p in (0, 1]: logsumexp(p) needs no max shift
  float z2 = 0.f;
  for (int c = lane; c < C; c += 64) {
    const float p = __expf(lg[c] - m) / z;
    lg[c] = p;
    probs[(long)b * C + c] = p;
    z2 += __expf(p);
  }
  z2 = wave_sum(z2);
  const int64_t y64 = labels[b];
  const float invB = 1.0f / B;
  if (y64 < 0 || y64 >= C) {
    // a label outside the class list (e.g. remapped against a rank-local list): poison the loss
    // and this row's gradient, so the non-finite check skips the update instead of training on
    // garbage (torch's CrossEntropyLoss raises here)
    for (int c = lane; c < C; c += 64) dlogits[(long)b * C + c] = __builtin_nanf("");
    if (lane == 0) atomicAdd(loss, __builtin_nanf(""));
    return;
  }
  const int y = (int)y64;
  // dL/dp_c = (softmax(p)_c - [c == y]) / B ; dL/dlogit = p * (dp - sum p*dp)
  float dot = 0.f;
  for (int c = lane; c < C; c += 64) {
    const float p = lg[c];
    const float dp = (__expf(p) / z2 - (c == y ? 1.f : 0.f)) * invB;
    dot += p * dp;
  }
  dot = wave_sum(dot);
  for (int c = lane; c < C; c += 64) {
    const float p = lg[c];
    const float dp = (__expf(p) / z2 - (c == y ? 1.f : 0.f)) * invB;
    dlogits[(long)b * C + c] = p * (dp - dot);
  }
  if (lane == 0) atomicAdd(loss, (logf(z2) - lg[y]) * invB);
}

// dF[r] = (dn - n (n.dn)) / norm[r],  dn[k] = s * sum_c dlog(r, c) * other[c][k] (+ dn_ext)
// dlog(r, c) = dlogits[r*sr + c*sc]. One workgroup per row r; the sum over c is spread over 8
// groups of 32 lanes (c = cg, cg + 8, ...; lane kk owns k = kk + 32 j), so a row with many terms
// (the text side: Co = batch) keeps 8 independent load streams in flight, and the 8 partial sums
// meet in LDS in a fixed order (deterministic).
constexpr int HFG_CG = 8;
__global__ void __launch_bounds__(256)
head_feat_grad_kernel(int R, int Co, int E, const float* __restrict__ dlogits, long sr, long sc,
                      const float* __restrict__ other_n, const float* __restrict__ self_n,
                      const float* __restrict__ norms, const float* __restrict__ logit_scale,
                      const float* __restrict__ dn_ext, float* __restrict__ dF) {
  __shared__ float part_s[HFG_CG][1024];
  __shared__ float red[4];
  const int r = blockIdx.x, tid = threadIdx.x;
  const int cg = tid >> 5, kk = tid & 31;
  const float s = __expf(*logit_scale);
  float acc[32];  // E <= 1024
#pragma unroll
  for (int j = 0; j < 32; ++j) acc[j] = 0.f;
  // unrolled so that several rows' loads are in flight per lane (the FMA order per acc is
  // unchanged: the result is bit-identical to the rolled loop)
#pragma unroll 4
  for (int c = cg; c < Co; c += HFG_CG) {
    const float d = dlogits[(long)r * sr + (long)c * sc];
    const float* o = other_n + (long)c * E + kk;
#pragma unroll
    for (int j = 0; j < 32; ++j)
      if (kk + 32 * j < E) acc[j] += d * o[32 * j];
  }
#pragma unroll
  for (int j = 0; j < 32; ++j)
    if (kk + 32 * j < E) part_s[cg][kk + 32 * j] = acc[j];
  __syncthreads();
  float dn[4] = {0.f, 0.f, 0.f, 0.f};
  float part = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = tid + i * 256;
    if (k < E) {
      float v = 0.f;
#pragma unroll
      for (int g2 = 0; g2 < HFG_CG; ++g2) v += part_s[g2][k];
      dn[i] = v * s;
      if (dn_ext) dn[i] += dn_ext[(long)r * E + k];
      part += dn[i] * self_n[(long)r * E + k];
    }
  }
  part = wave_sum(part);
  if ((tid & 63) == 0) red[tid >> 6] = part;
  __syncthreads();
  const float nd = red[0] + red[1] + red[2] + red[3];
  const float inv = 1.0f / norms[r];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = tid + i * 256;
    if (k < E) dF[(long)r * E + k] = (dn[i] - self_n[(long)r * E + k] * nd) * inv;
  }
}

// The same for E % 4 == 0 with 16-B loads: wave w sums the terms c = w, w + 4, ... (lane l owns
// k = 4 (l + 64 j) .. +3), 4 rows in flight per wave; the 4 waves' partials meet in LDS in a fixed
// order (deterministic). The text side's dL/dT (R = C prompts, Co = the batch: 256 terms) ran
// 155 us on 10 workgroups with 4-B loads one row at a time.
__global__ void __launch_bounds__(256)
head_feat_grad4_kernel(int R, int Co, int E, const float* __restrict__ dlogits, long sr, long sc,
                       const float* __restrict__ other_n, const float* __restrict__ self_n,
                       const float* __restrict__ norms, const float* __restrict__ logit_scale,
                       const float* __restrict__ dn_ext, float* __restrict__ dF) {
  __shared__ float4 part_s[4][256];
  __shared__ float red[4];
  const int r = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int E4 = E >> 2;
  const float s = __expf(*logit_scale);
  float4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
  for (int c = w; c < Co; c += 4) {
    const float d = dlogits[(long)r * sr + (long)c * sc];
    const float4* o = reinterpret_cast<const float4*>(other_n + (long)c * E);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (lane + 64 * j < E4) {
        const float4 v = o[lane + 64 * j];
        acc[j].x += d * v.x, acc[j].y += d * v.y, acc[j].z += d * v.z, acc[j].w += d * v.w;
      }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (lane + 64 * j < E4) part_s[w][lane + 64 * j] = acc[j];
  __syncthreads();
  // thread tid owns float4 group tid (E <= 1024: 256 groups)
  float4 dn = make_float4(0.f, 0.f, 0.f, 0.f);
  float part = 0.f;
  const bool own = tid < E4;
  if (own) {
    const float4 a = part_s[0][tid], b = part_s[1][tid], c2 = part_s[2][tid], d2 = part_s[3][tid];
    dn.x = (((a.x + b.x) + c2.x) + d2.x) * s;
    dn.y = (((a.y + b.y) + c2.y) + d2.y) * s;
    dn.z = (((a.z + b.z) + c2.z) + d2.z) * s;
    dn.w = (((a.w + b.w) + c2.w) + d2.w) * s;
    if (dn_ext) {
      const float4 e = reinterpret_cast<const float4*>(dn_ext + (long)r * E)[tid];
      dn.x += e.x, dn.y += e.y, dn.z += e.z, dn.w += e.w;
    }
    const float4 n4 = reinterpret_cast<const float4*>(self_n + (long)r * E)[tid];
    part = dn.x * n4.x + dn.y * n4.y + dn.z * n4.z + dn.w * n4.w;
  }
  part = wave_sum(part);
  if (lane == 0) red[w] = part;
  __syncthreads();
  const float nd = red[0] + red[1] + red[2] + red[3];
  const float inv = 1.0f / norms[r];
  if (own) {
    const float4 n4 = reinterpret_cast<const float4*>(self_n + (long)r * E)[tid];
    reinterpret_cast<float4*>(dF + (long)r * E)[tid] =
        make_float4((dn.x - n4.x * nd) * inv, (dn.y - n4.y * nd) * inv, (dn.z - n4.z * nd) * inv,
                    (dn.w - n4.w * nd) * inv);
  }
}

// logits[b][c] = exp(logit_scale) * img_n[b] . txt_n[c]; probs = softmax(logits) (optional)
__global__ void __launch_bounds__(256)
head_logits_kernel(int B, int C, int E, const float* __restrict__ img_n,
                   const float* __restrict__ txt_n, const float* __restrict__ logit_scale,
                   float* __restrict__ logits, float* __restrict__ probs) {
  extern __shared__ float sh[];
  float* irow = sh;
  float* lg = sh + E;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float s = __expf(*logit_scale);
  for (int k = tid; k < E; k += 256) irow[k] = img_n[(long)b * E + k];
  __syncthreads();
  for (int c = w; c < C; c += 4) {
    float d = 0.f;
    for (int k = lane; k < E; k += 64) d += irow[k] * txt_n[(long)c * E + k];
    d = wave_sum(d);
    if (lane == 0) {
      lg[c] = s * d;
      logits[(long)b * C + c] = s * d;
    }
  }
  __syncthreads();
  if (w != 0 || probs == nullptr) return;
  float m = -INFINITY;
  for (int c = lane; c < C; c += 64) m = fmaxf(m, lg[c]);
  m = wave_max(m);
  float z = 0.f;
  for (int c = lane; c < C; c += 64) z += __expf(lg[c] - m);
  z = wave_sum(z);
  for (int c = lane; c < C; c += 64) probs[(long)b * C + c] = __expf(lg[c] - m) / z;
}

// dlogits = p * (dp - sum_c p*dp), one wave per row
__global__ void __launch_bounds__(64)
softmax_bwd_kernel(int B, int C, const float* __restrict__ p, const float* __restrict__ dp,
                   float* __restrict__ dl) {
  const int b = blockIdx.x, lane = threadIdx.x;
  float dot = 0.f;
  for (int c = lane; c < C; c += 64) dot += p[(long)b * C + c] * dp[(long)b * C + c];
  dot = wave_sum(dot);
  for (int c = lane; c < C; c += 64)
    dl[(long)b * C + c] = p[(long)b * C + c] * (dp[(long)b * C + c] - dot);
}

// ---------------------------------------------------------------- half-precision gradient scale
// The text tower's backward in IEEE half (lc_*_f16) sees gradients of 1e-9..3e-4 at its 16-bit
// stores (ViT-B/16, C = 10..100: most below half's normal range, 6.1e-5), so its incoming
// gradient is scaled first, as the reference's torch.cuda.amp.GradScaler scales the loss
// (methods/adapter_clip.py:93, _trainer.py:163) — here per call and by a power of two computed
// on the device from the gradient itself: s = 2^(target - floor(log2 max|x|)), which puts
// max|x| in [2^target, 2^(target+1)) (the tower's own stores stay within ~1.4x of its input's
// max, measured: target 10 leaves a 30x margin below half's 65504). A zero or non-finite
// max gives s = 1. Powers of two make scaling and unscaling exact.
__global__ void __launch_bounds__(1024)
grad_pow2_normalize_kernel(long n, float* __restrict__ x, float* __restrict__ s_out, int target) {
  __shared__ float red[16];
  __shared__ float s_sh;
  const int tid = threadIdx.x;
  float m = 0.f;
  // 16-B loads, 8 in flight per lane (one workgroup streams the whole vector twice: a strided
  // scalar loop waited out one load latency per element, 19 us for 256 x 512 floats)
  const bool v4 = ((uintptr_t)x & 15) == 0;
  const long n4 = v4 ? n / 4 : 0;
  const float4* x4 = reinterpret_cast<const float4*>(x);
#pragma unroll 8
  for (long i = tid; i < n4; i += 1024) {
    const float4 a = x4[i];
    m = fmaxf(m, fmaxf(fmaxf(fabsf(a.x), fabsf(a.y)), fmaxf(fabsf(a.z), fabsf(a.w))));
  }
  for (long i = 4 * n4 + tid; i < n; i += 1024) m = fmaxf(m, fabsf(x[i]));
  m = wave_max(m);
  if ((tid & 63) == 0) red[tid >> 6] = m;
  __syncthreads();
  if (tid == 0) {
    float a = 0.f;
    for (int w = 0; w < 16; ++w) a = fmaxf(a, red[w]);
    float s = 1.0f;
    if (a > 0.f && a <= 3.4e38f) {  // finite, nonzero
      const int e = (int)((__float_as_uint(a) >> 23) & 0xff) - 127;  // floor(log2 a), normals
      const int k = min(max(target - e, -126), 127);
      s = __uint_as_float((uint32_t)(k + 127) << 23);
    }
    s_sh = s;
    s_out[0] = s;
  }
  __syncthreads();
  const float s = s_sh;
  float4* y4 = reinterpret_cast<float4*>(x);
#pragma unroll 8
  for (long i = tid; i < n4; i += 1024) {
    float4 a = y4[i];
    a.x *= s, a.y *= s, a.z *= s, a.w *= s;
    y4[i] = a;
  }
  for (long i = 4 * n4 + tid; i < n; i += 1024) x[i] *= s;
}

// y[i] += x[i] / s[0] (s a power of two: exact)
__global__ void __launch_bounds__(256)
add_unscaled_kernel(long n, float* __restrict__ y, const float* __restrict__ x,
                    const float* __restrict__ s) {
  const float inv = 1.0f / s[0];
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    y[i] += x[i] * inv;
}

}  // namespace

extern "C" {

int lc_l2norm_rows(hipStream_t st, int R, int E, const float* f, long ldf, float* out, float* norms) {
  LC_CHECK_ARG(R > 0 && E > 0 && ldf >= E);
  hipLaunchKernelGGL(l2norm_kernel, dim3(R), dim3(64), 0, st, R, E, f, ldf, out, norms);
  LC_LAUNCH_RET();
}

int lc_clip_head(hipStream_t st, int B, int C, int E, const float* img_n, const float* txt_n,
                 const float* logit_scale, const int64_t* labels, float* probs, float* dlogits,
                 float* loss) {
  LC_CHECK_ARG(B > 0 && C > 0 && C <= 8192 && E > 0 && E <= 1024);
  const size_t shm = (size_t)(E + C) * sizeof(float);
  hipLaunchKernelGGL(head_rows_kernel, dim3(B), dim3(256), shm, st, B, C, E, img_n, txt_n,
                     logit_scale, labels, probs, dlogits, loss);
  LC_LAUNCH_RET();
}

int lc_head_feat_grad(hipStream_t st, int R, int Co, int E, const float* dlogits, long sr, long sc,
                      const float* other_n, const float* self_n, const float* norms,
                      const float* logit_scale, const float* dn_ext, float* dF) {
  LC_CHECK_ARG(R > 0 && Co > 0 && E > 0 && E <= 1024);
  const bool v4 = E % 4 == 0 && (((uintptr_t)other_n | (uintptr_t)self_n | (uintptr_t)dF |
                                  (uintptr_t)dn_ext) & 15) == 0;
  if (v4)
    hipLaunchKernelGGL(head_feat_grad4_kernel, dim3(R), dim3(256), 0, st, R, Co, E, dlogits, sr,
                       sc, other_n, self_n, norms, logit_scale, dn_ext, dF);
  else
    hipLaunchKernelGGL(head_feat_grad_kernel, dim3(R), dim3(256), 0, st, R, Co, E, dlogits, sr, sc,
                       other_n, self_n, norms, logit_scale, dn_ext, dF);
  LC_LAUNCH_RET();
}

int lc_head_logits(hipStream_t st, int B, int C, int E, const float* img_n, const float* txt_n,
                   const float* logit_scale, float* logits, float* probs) {
  LC_CHECK_ARG(B > 0 && C > 0 && C <= 8192 && E > 0 && E <= 1024);
  const size_t shm = (size_t)(E + C) * sizeof(float);
  hipLaunchKernelGGL(head_logits_kernel, dim3(B), dim3(256), shm, st, B, C, E, img_n, txt_n,
                     logit_scale, logits, probs);
  LC_LAUNCH_RET();
}

int lc_softmax_bwd_rows(hipStream_t st, int B, int C, const float* probs, const float* dprobs,
                        float* dlogits) {
  LC_CHECK_ARG(B > 0 && C > 0);
  hipLaunchKernelGGL(softmax_bwd_kernel, dim3(B), dim3(64), 0, st, B, C, probs, dprobs, dlogits);
  LC_LAUNCH_RET();
}

int lc_grad_pow2_normalize(hipStream_t st, long n, float* x, float* scale, int target_exp) {
  LC_CHECK_ARG(n > 0 && x != nullptr && scale != nullptr && target_exp >= -100 &&
               target_exp <= 100);
  hipLaunchKernelGGL(grad_pow2_normalize_kernel, dim3(1), dim3(1024), 0, st, n, x, scale,
                     target_exp);
  LC_LAUNCH_RET();
}

int lc_add_unscaled(hipStream_t st, long n, float* y, const float* x, const float* scale) {
  LC_CHECK_ARG(n > 0 && y != nullptr && x != nullptr && scale != nullptr);
  const long blocks = (n + 255) / 256;
  hipLaunchKernelGGL(add_unscaled_kernel, dim3((unsigned)(blocks < 1024 ? blocks : 1024)),
                     dim3(256), 0, st, n, y, x, scale);
  LC_LAUNCH_RET();
}

int lc_device_cu_count(int device, int* n_cu) {
  LC_CHECK_ARG(n_cu != nullptr);
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    return LC_ELAUNCH;
  *n_cu = v;
  return LC_OK;
}

int lc_stream_create_cumask(int device, int first, int count, int stride, void** stream) {
  int n_cu = 0;
  LC_CHECK_ARG(stream != nullptr && first >= 0 && count > 0 && stride > 0);
  if (lc_device_cu_count(device, &n_cu) != LC_OK) return LC_ELAUNCH;
  LC_CHECK_ARG((long)first + (long)(count - 1) * stride < n_cu);
  uint32_t mask[32] = {0};
  LC_CHECK_ARG(n_cu <= 32 * 32);
  for (int i = 0; i < count; ++i) {
    const int cu = first + i * stride;
    mask[cu >> 5] |= 1u << (cu & 31);
  }
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) return LC_ELAUNCH;
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)((n_cu + 31) / 32), mask);
  (void)hipSetDevice(prev);
  if (e != hipSuccess) return LC_ELAUNCH;
  *stream = (void*)s;
  return LC_OK;
}

int lc_stream_destroy(void* stream) {
  LC_CHECK_ARG(stream != nullptr);
  return hipStreamDestroy((hipStream_t)stream) == hipSuccess ? LC_OK : LC_ELAUNCH;
}

}  // extern "C"
