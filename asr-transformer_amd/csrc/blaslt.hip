// bf16 GEMMs on hipBLASLt: the library path for plain GEMMs — the epilogue-free data gradients, and the bias +
// fp32-residual forward (C fp32 = A.B^T + bias + resid: the library's own bias epilogue and beta = 1 over the residual
// as its C matrix; no dropout, no gating) — where the vendor kernel beats the hand-written ones (asrx_gemm planner,
// gemm.hip: kernel code 7 forces it).  Host code
// only: one handle, one workspace and a per-shape cache of (descriptors, heuristic algorithm), all created outside
// stream capture — during a HIP-graph capture an unseen shape is declined (the caller falls back to its own
// kernel) instead of allocating or querying the library inside the capture.
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

#include "common.h"

namespace {

struct LtPlan {
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr, d = nullptr;
  hipblasLtMatmulAlgo_t algo;
  size_t ws = 0;
  bool ok = false;
};

constexpr size_t LT_WS_BYTES = 64ull << 20;
std::mutex g_lt_mu;
hipblasLtHandle_t g_lt = nullptr;
void* g_lt_ws = nullptr;
bool g_lt_failed = false;
// (m, n, k, lda, ldb, ldc, b_trans, c fp32, bias, ld_resid or -1)
using LtKey = std::tuple<int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int, int, int, int64_t>;
std::map<LtKey, LtPlan> g_lt_plans;

bool capturing(hipStream_t st) {
  hipStreamCaptureStatus s = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(st, &s) == hipSuccess && s != hipStreamCaptureStatusNone;
}

// Row-major C[m x n] = A[m x k] . op(B) (asrx convention: b_trans = 0 -> B is [n x k], C = A B^T; b_trans = 1 ->
// B is [k x n], C = A B) is column-major C^T[n x m] = op'(B) A^T: hipBLASLt (m', n', k') = (n, m, k) with
// A' = B (layout [n x k] ld ldb, N if b_trans else [k x n] T) and B' = A (layout [k x m] ld lda, N).
// bias: the epilogue adds bias[n] (fp32) — a per-row vector of the column-major C^T.  resid: C^T = the fp32 residual
// (ld_resid) with beta = 1, D^T = the output (ldc).
LtPlan make_plan(const asrx_gemm_desc* d) {
  LtPlan p;
  const hipblasOperation_t ta = d->b_trans ? HIPBLAS_OP_N : HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  const hipDataType ct = d->c_dtype == ASRX_F32 ? HIP_R_32F : HIP_R_16BF;
  if (hipblasLtMatmulDescCreate(&p.op, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return p;
  hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
  hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
  if (d->bias) {
    const hipblasLtEpilogue_t ep = HIPBLASLT_EPILOGUE_BIAS;
    const hipDataType bt = HIP_R_32F;
    if (hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep)) != HIPBLAS_STATUS_SUCCESS ||
        hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)) !=
            HIPBLAS_STATUS_SUCCESS ||
        hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &d->bias, sizeof(d->bias)) !=
            HIPBLAS_STATUS_SUCCESS)
      return p;
  }
  const uint64_t ar = d->b_trans ? d->n : d->k, ac = d->b_trans ? d->k : d->n;
  if (hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16BF, ar, ac, d->ldb) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16BF, d->k, d->m, d->lda) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.d, ct, d->n, d->m, d->ldc) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.c, ct, d->n, d->m, d->resid ? d->ld_resid : d->ldc) != HIPBLAS_STATUS_SUCCESS)
    return p;
  hipblasLtMatmulPreference_t pref = nullptr;
  if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return p;
  const uint64_t wsb = LT_WS_BYTES;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb));
  hipblasLtMatmulHeuristicResult_t res[1];
  int nres = 0;
  const hipblasStatus_t hs =
      hipblasLtMatmulAlgoGetHeuristic(g_lt, p.op, p.a, p.b, p.c, p.d, pref, 1, res, &nres);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (hs != HIPBLAS_STATUS_SUCCESS || nres < 1 || res[0].state != HIPBLAS_STATUS_SUCCESS ||
      res[0].workspaceSize > LT_WS_BYTES)
    return p;
  p.algo = res[0].algo;
  p.ws = res[0].workspaceSize;
  p.ok = true;
  return p;
}

}  // namespace

// Returns ASRX_OK after enqueueing the GEMM, 1 when the library path is not available for this call (the caller
// runs its own kernel), or an ASRX error.
int blaslt_gemm_bf16(const asrx_gemm_desc* d, hipStream_t st) {
  std::lock_guard<std::mutex> lock(g_lt_mu);
  if (g_lt_failed) return 1;
  const bool cap = capturing(st);
  if (!g_lt) {
    if (cap) return 1;
    if (hipblasLtCreate(&g_lt) != HIPBLAS_STATUS_SUCCESS || hipMalloc(&g_lt_ws, LT_WS_BYTES) != hipSuccess) {
      g_lt_failed = true;
      return 1;
    }
  }
  const auto key = LtKey((int64_t)d->m, (int64_t)d->n, (int64_t)d->k, (int64_t)d->lda, (int64_t)d->ldb, (int64_t)d->ldc,
                         (int)d->b_trans, (int)(d->c_dtype == ASRX_F32), (int)(d->bias != nullptr),
                         d->resid ? (int64_t)d->ld_resid : (int64_t)-1);
  auto it = g_lt_plans.find(key);
  if (it == g_lt_plans.end()) {
    if (cap) return 1;
    it = g_lt_plans.emplace(key, make_plan(d)).first;
  }
  const LtPlan& p = it->second;
  if (!p.ok) return 1;
  // the bias pointer is an attribute of the (per-shape) descriptor: set for this call (read at enqueue)
  if (d->bias && hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &d->bias,
                                                 sizeof(d->bias)) != HIPBLAS_STATUS_SUCCESS)
    return ASRX_ERR_LAUNCH;
  const float alpha = d->alpha, beta = d->resid ? 1.f : 0.f;
  const void* cin = d->resid ? d->resid : d->c;
  const hipblasStatus_t s = hipblasLtMatmul(g_lt, p.op, &alpha, d->b, p.a, d->a, p.b, &beta, cin, p.c, d->c, p.d,
                                            &p.algo, g_lt_ws, p.ws, st);
  return s == HIPBLAS_STATUS_SUCCESS ? ASRX_OK : ASRX_ERR_LAUNCH;
}
