// hipBLASLt for one plain GEMM shape of the step (host code only).
//
// The image tower's QKV input-gradient GEMM (dh = dqkv . Wqkv, M = 50 432, N = 768, K = 2 304,
// bf16 in / out, f32 accumulation, no epilogue: lora.py:1072's in-projection backward, as
// autograd forms it) is a plain library GEMM: no fused epilogue, no side input. hipBLASLt's
// stream-K schedule runs it in 142 us standalone against 160-162 us for gemm8's split-K tail
// (profiles/r05/q, r), and routed there the step gains 1.2 % (profiles/r06/blaslt/). Every other
// step GEMM keeps its hand-written kernel: those carry fused epilogues (bias + QuickGELU /
// QuickGELU', residual adds, the adapter epilogues, the x QuickGELU' side input) or measured
// equal / slower on hipBLASLt (the out-projections, the K = 3 072 shapes).
//
// Row-major C[M, N] = A[M, K] . B[N, K]^T is column-major C^T = B^T' . A with hipBLASLt's
// operands (op_A = T on B stored K x N with ld = ldb, op_B = N on A stored K x M with ld = lda,
// D stored N x M with ld = ldo). One handle per device; the descriptors and the heuristic's
// first algorithm are cached per (device, M, N, K, lda, ldb, ldo, workspace size).
#include "lc_common.h"
#include <hipblaslt/hipblaslt.h>
#include <mutex>
#include <vector>

namespace {

struct Plan {
  int dev, M, N, K;
  long lda, ldb, ldo, ws;
  hipblasLtMatmulDesc_t op;
  hipblasLtMatrixLayout_t la, lb, lc;
  hipblasLtMatmulAlgo_t algo;
  size_t algo_ws;
};

std::mutex g_mu;
std::vector<Plan> g_plans;
hipblasLtHandle_t g_handles[64] = {};
bool g_broken = false;  // a hipBLASLt call failed once: the callers keep their own kernels

bool make_plan(Plan& p) {
  if (!g_handles[p.dev] && hipblasLtCreate(&g_handles[p.dev]) != HIPBLAS_STATUS_SUCCESS) return false;
  if (hipblasLtMatmulDescCreate(&p.op, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS)
    return false;
  const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  if (hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)) ||
      hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)))
    return false;
  if (hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, p.K, p.N, p.ldb) ||
      hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, p.K, p.M, p.lda) ||
      hipblasLtMatrixLayoutCreate(&p.lc, HIP_R_16BF, p.N, p.M, p.ldo))
    return false;
  hipblasLtMatmulPreference_t pref;
  if (hipblasLtMatmulPreferenceCreate(&pref)) return false;
  const uint64_t wsb = (uint64_t)p.ws;
  hipblasLtMatmulHeuristicResult_t res;
  int n = 0;
  const bool ok =
      hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb,
                                            sizeof(wsb)) == HIPBLAS_STATUS_SUCCESS &&
      hipblasLtMatmulAlgoGetHeuristic(g_handles[p.dev], p.op, p.la, p.lb, p.lc, p.lc, pref, 1,
                                      &res, &n) == HIPBLAS_STATUS_SUCCESS &&
      n > 0;
  hipblasLtMatmulPreferenceDestroy(pref);
  if (!ok) return false;
  p.algo = res.algo;
  p.algo_ws = res.workspaceSize;
  return true;
}

}  // namespace

// C[M, N] (bf16, row stride ldo) = A[M, K] . B[N, K]^T (bf16, row strides lda / ldb) on hipBLASLt,
// workspace ws / ws_bytes (the caller's split-K scratch). Returns false when hipBLASLt cannot take
// the launch (the caller then runs its own kernel); no output is written in that case.
bool lc_blaslt_nt_bf16(hipStream_t stream, int M, int N, int K, const void* A, long lda,
                       const void* B, long ldb, void* C, long ldo, void* ws, long ws_bytes) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
  std::lock_guard<std::mutex> lock(g_mu);
  if (g_broken) return false;
  Plan* p = nullptr;
  for (auto& q : g_plans)
    if (q.dev == dev && q.M == M && q.N == N && q.K == K && q.lda == lda && q.ldb == ldb &&
        q.ldo == ldo && q.ws == ws_bytes) {
      p = &q;
      break;
    }
  if (!p) {
    Plan q{dev, M, N, K, lda, ldb, ldo, ws_bytes};
    if (!make_plan(q)) {
      g_broken = true;
      return false;
    }
    g_plans.push_back(q);
    p = &g_plans.back();
  }
  const float one = 1.0f, zero = 0.0f;
  if (hipblasLtMatmul(g_handles[dev], p->op, &one, B, p->la, A, p->lb, &zero, C, p->lc, C, p->lc,
                      &p->algo, ws, p->algo_ws, stream) != HIPBLAS_STATUS_SUCCESS) {
    g_broken = true;
    return false;
  }
  return true;
}
