// Plain library GEMM through hipBLASLt: the vertex projection of inf_project_table
// (out = E [W_0; W_y]^T over the whole table, no epilogue) is an ordinary large bf16 GEMM
// (V x 2H x k_pad), the case a vendor-tuned kernel covers best; the plan's own grouped
// GEMM (gemm.hip) stays the fallback (INF_PROJECT_GEMM=own).  Per shape: the heuristic's
// 16 candidates (up to 256 MB of workspace, kept for the process) are timed once and the
// fastest is kept (400k x 512 x 1024: 0.47 ms for the heuristic's first pick, 0.51 ms for
// the best without workspace, 0.7-0.8 ms for gemm.hip).
#include "blaslt.hpp"

#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

namespace inf {
namespace {

struct LtPlan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  size_t ws = 0;
};

constexpr size_t WS_MAX = (size_t)256 << 20;  // workspace offered to the heuristic

// per device (a process may drive more than one): handle, tuned plans, workspace
struct DevState {
  hipblasLtHandle_t handle = nullptr;
  void* ws = nullptr;
  size_t ws_bytes = 0;
  std::map<std::tuple<int64_t, int64_t, int64_t, int64_t, int64_t, int64_t>, LtPlan> plans;
};
std::mutex g_mu;
std::map<int, DevState> g_dev;

#define LT_TRY(x)                                                     \
  do {                                                                \
    hipblasStatus_t s_ = (x);                                         \
    if (s_ != HIPBLAS_STATUS_SUCCESS) {                               \
      set_error(std::string("hipBLASLt: ") + #x + " failed");         \
      return INF_ERR_HIP;                                             \
    }                                                                 \
  } while (0)

}  // namespace

// Row-major C[M][N] = A[M][K] B[N][K]^T, bf16 in and out, fp32 accumulation.  Column-major
// for the library: C^T (N x M, ld ldc) = op_T(B as K x N, ld ldb) * (A^T as K x M, ld lda).
int blaslt_gemm_nt_bf16(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M,
                        int64_t N, int64_t K, hipStream_t stream) {
  std::lock_guard<std::mutex> lock(g_mu);
  int dev = 0;
  INF_HIP_TRY(hipGetDevice(&dev));
  DevState& ds = g_dev[dev];
  hipblasLtHandle_t& g_handle = ds.handle;
  if (g_handle == nullptr) LT_TRY(hipblasLtCreate(&g_handle));
  // the workspace is kept for the process (plans may be replayed from graphs)
  auto ensure_ws = [&](size_t need) -> int {
    if (need <= ds.ws_bytes) return INF_OK;
    if (ds.ws != nullptr) INF_HIP_TRY(hipFree(ds.ws));
    ds.ws = nullptr;
    ds.ws_bytes = 0;
    INF_HIP_TRY(hipMalloc(&ds.ws, need));
    ds.ws_bytes = need;
    return INF_OK;
  };
  const auto key = std::make_tuple(M, N, K, lda, ldb, ldc);
  auto it = ds.plans.find(key);
  if (it == ds.plans.end()) {
    LtPlan p;
    LT_TRY(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    const hipblasOperation_t opT = HIPBLAS_OP_T, opN = HIPBLAS_OP_N;
    LT_TRY(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opT, sizeof(opT)));
    LT_TRY(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opN, sizeof(opN)));
    LT_TRY(hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, (uint64_t)K, (uint64_t)N, ldb));
    LT_TRY(hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, (uint64_t)K, (uint64_t)M, lda));
    LT_TRY(hipblasLtMatrixLayoutCreate(&p.lc, HIP_R_16BF, (uint64_t)N, (uint64_t)M, ldc));
    hipblasLtMatmulPreference_t pref;
    LT_TRY(hipblasLtMatmulPreferenceCreate(&pref));
    const uint64_t ws = WS_MAX;
    LT_TRY(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws)));
    // the heuristic may rank algorithms that need more workspace than offered first (a
    // 400k-row problem came back with one): take the best that fits
#ifndef BLASLT_NREQ
#define BLASLT_NREQ 16
#endif
    constexpr int NREQ = BLASLT_NREQ;
    hipblasLtMatmulHeuristicResult_t res[NREQ] = {};
    int n = 0;
    const hipblasStatus_t hs =
        hipblasLtMatmulAlgoGetHeuristic(g_handle, p.desc, p.la, p.lb, p.lc, p.lc, pref, NREQ, res, &n);
    hipblasLtMatmulPreferenceDestroy(pref);
    int pick = -1;
    for (int i = 0; hs == HIPBLAS_STATUS_SUCCESS && i < n && pick < 0; ++i)
      if (res[i].state == HIPBLAS_STATUS_SUCCESS && res[i].workspaceSize <= WS_MAX) pick = i;
    // then time the candidates once on this shape (not while a graph is being captured)
    // and keep the fastest: the heuristic's order is a guess
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    INF_HIP_TRY(hipStreamIsCapturing(stream, &cap));
    if (pick >= 0 && cap == hipStreamCaptureStatusNone && std::getenv("INF_BLASLT_NO_TUNE") == nullptr) {
      size_t need = 0;
      for (int i = 0; i < n; ++i)
        if (res[i].state == HIPBLAS_STATUS_SUCCESS && res[i].workspaceSize <= WS_MAX)
          need = std::max(need, (size_t)res[i].workspaceSize);
      if (int rc = ensure_ws(need)) return rc;
      hipEvent_t e0, e1;
      INF_HIP_TRY(hipEventCreate(&e0));
      INF_HIP_TRY(hipEventCreate(&e1));
      const float alpha = 1.f, beta = 0.f;
      float best = 1e30f;
      for (int i = 0; i < n; ++i) {
        if (res[i].state != HIPBLAS_STATUS_SUCCESS || res[i].workspaceSize > WS_MAX) continue;
        float ms = 0.f;
        bool ok = true;
        for (int rep = 0; rep < 2 && ok; ++rep) {  // rep 0 warms up
          INF_HIP_TRY(hipEventRecord(e0, stream));
          ok = hipblasLtMatmul(g_handle, p.desc, &alpha, B, p.la, A, p.lb, &beta, C, p.lc, C, p.lc, &res[i].algo,
                               ds.ws, res[i].workspaceSize, stream) == HIPBLAS_STATUS_SUCCESS;
          INF_HIP_TRY(hipEventRecord(e1, stream));
          INF_HIP_TRY(hipEventSynchronize(e1));
          INF_HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
        }
        if (ok && ms < best) {
          best = ms;
          pick = i;
        }
      }
      INF_HIP_TRY(hipEventDestroy(e0));
      INF_HIP_TRY(hipEventDestroy(e1));
    }
    if (pick < 0) {
      set_error("hipBLASLt: no algorithm for the projection GEMM within " + std::to_string(WS_MAX >> 20) +
                " MB of workspace (" + std::to_string(n) + " candidates)");
      return INF_ERR_UNSUPPORTED;
    }
    p.algo = res[pick].algo;
    p.ws = res[pick].workspaceSize;
    if (std::getenv("INF_BLASLT_VERBOSE") != nullptr)
      for (int i = 0; i < n; ++i)
        std::fprintf(stderr, "hipBLASLt candidate %d: workspace %zu bytes%s\n", i, (size_t)res[i].workspaceSize,
                     i == pick ? " (picked)" : "");
    if (int rc = ensure_ws(p.ws)) return rc;
    it = ds.plans.emplace(key, p).first;
  }
  const LtPlan& p = it->second;
  const float alpha = 1.f, beta = 0.f;
  LT_TRY(hipblasLtMatmul(g_handle, p.desc, &alpha, B, p.la, A, p.lb, &beta, C, p.lc, C, p.lc, &p.algo,
                         p.ws > 0 ? ds.ws : nullptr, p.ws, stream));
  return INF_OK;
}

}  // namespace inf
