// Which hipBLASLt GELU-epilogue configurations have algorithms on this device (diagnostic).
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <stdio.h>

static int try_cfg(hipblasLtHandle_t h, int M, int N, int K, uint32_t epi, int auxType, int biasType, bool opT) {
  hipblasLtMatmulDesc_t d;
  int st = hipblasLtMatmulDescCreate(&d, HIPBLAS_COMPUTE_32F, HIP_R_32F);
  hipblasOperation_t opA = opT ? HIPBLAS_OP_T : HIPBLAS_OP_N, opB = HIPBLAS_OP_N;
  st |= hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_TRANSA, &opA, sizeof opA);
  st |= hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_TRANSB, &opB, sizeof opB);
  int s1 = hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof epi);
  int64_t ld = N;
  int s2 = 0, s3 = 0, s4 = 0;
  if (epi & 128) s2 = hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof ld);
  if (auxType >= 0) s3 = hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &auxType, sizeof auxType);
  if (biasType >= 0) s4 = hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &biasType, sizeof biasType);
  hipblasLtMatrixLayout_t la, lb, lc;
  if (opT) hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, K, N, K);
  else hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, N, K, N);
  hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, K, M, K);
  hipblasLtMatrixLayoutCreate(&lc, HIP_R_16BF, N, M, N);
  hipblasLtMatmulPreference_t pref;
  hipblasLtMatmulPreferenceCreate(&pref);
  uint64_t ws = 64ull << 20;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof ws);
  hipblasLtMatmulHeuristicResult_t res[4];
  int n = 0;
  int s5 = hipblasLtMatmulAlgoGetHeuristic(h, d, la, lb, lc, lc, pref, 4, res, &n);
  printf("M=%5d N=%5d K=%5d epi=%3u aux=%3d bias=%3d opT=%d | create=%d epi=%d auxld=%d auxT=%d biasT=%d heur=%d n=%d\n",
         M, N, K, epi, auxType, biasType, (int)opT, st, s1, s2, s3, s4, s5, n);
  return n;
}

int main() {
  hipblasLtHandle_t h;
  printf("create %d\n", hipblasLtCreate(&h));
  int shapes[][3] = {{25216, 1536, 384}, {64, 1536, 384}, {4096, 4096, 4096}};
  for (auto& s : shapes) {
    try_cfg(h, s[0], s[1], s[2], HIPBLASLT_EPILOGUE_DEFAULT, -1, -1, false);
    try_cfg(h, s[0], s[1], s[2], HIPBLASLT_EPILOGUE_BIAS, -1, HIP_R_16BF, false);
    try_cfg(h, s[0], s[1], s[2], HIPBLASLT_EPILOGUE_GELU, -1, -1, false);
    try_cfg(h, s[0], s[1], s[2], HIPBLASLT_EPILOGUE_GELU_BIAS, -1, HIP_R_16BF, false);
    try_cfg(h, s[0], s[1], s[2], HIPBLASLT_EPILOGUE_GELU_BIAS, -1, HIP_R_32F, false);
    try_cfg(h, s[0], s[1], s[2], HIPBLASLT_EPILOGUE_GELU_AUX, -1, -1, false);
    try_cfg(h, s[0], s[1], s[2], HIPBLASLT_EPILOGUE_GELU_AUX, HIP_R_16BF, -1, false);
    try_cfg(h, s[0], s[1], s[2], HIPBLASLT_EPILOGUE_GELU_AUX_BIAS, -1, HIP_R_16BF, false);
    try_cfg(h, s[0], s[1], s[2], HIPBLASLT_EPILOGUE_GELU_AUX_BIAS, HIP_R_16BF, HIP_R_16BF, false);
    try_cfg(h, s[0], s[1], s[2], HIPBLASLT_EPILOGUE_GELU_AUX_BIAS, HIP_R_32F, HIP_R_32F, false);
    try_cfg(h, s[0], s[1], s[2], HIPBLASLT_EPILOGUE_DGELU, -1, -1, true);
    try_cfg(h, s[0], s[1], s[2], HIPBLASLT_EPILOGUE_DGELU, HIP_R_16BF, -1, true);
    try_cfg(h, s[0], s[1], s[2], HIPBLASLT_EPILOGUE_DGELU, -1, -1, false);
  }
  return 0;
}
