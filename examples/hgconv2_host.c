/*
 * A plain-C host of the hgd C ABI (include/hgd.h): builds a small user × item incidence H on the
 * host, uploads it, derives the CSC / degree scales / edge weights with the library's structure
 * primitives, runs the HGNN two-hop Y = D_v^-1/2·H·D_e^-1·Hᵀ·D_v^-1/2·X (data/graph.py:28-42)
 * with two hgd_spmm calls, and checks Y against a float64 host computation.
 *
 * Build (see tests/test_gpu_native_host.py):
 *   gcc -std=c11 -D__HIP_PLATFORM_AMD__ -I include -I /opt/rocm/include examples/hgconv2_host.c \
 *       -L hypergraph_diffusion_for_recommendation_amd/_lib -lhgd -L /opt/rocm/lib -lamdhip64 \
 *       -Wl,-rpath,... -lm -o hgconv2_host
 * Exit status 0 and "hgconv2_host ok" on success.
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hgd.h"

#define CHECK_HGD(call)                                                              \
  do {                                                                               \
    hgd_status s_ = (call);                                                          \
    if (s_ != HGD_OK) {                                                              \
      fprintf(stderr, "%s failed (%d): %s\n", #call, (int)s_, hgd_get_last_error_string()); \
      return 1;                                                                      \
    }                                                                                \
  } while (0)
#define CHECK_HIP(call)                                                              \
  do {                                                                               \
    hipError_t e_ = (call);                                                          \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s failed: %s\n", #call, hipGetErrorString(e_));              \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

static uint64_t lcg = 0x9E3779B97F4A7C15ull;
static uint32_t next_u32(void) {
  lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
  return (uint32_t)(lcg >> 33);
}

int main(void) {
  const int64_t U = 2000, I = 300, per_user = 12;
  const int32_t d = 64;
  /* CSR of H on the host: each user picks per_user distinct items, ascending */
  int64_t* rowptr = malloc(sizeof(int64_t) * (U + 1));
  int32_t* col = malloc(sizeof(int32_t) * U * per_user);
  unsigned char* seen = calloc((size_t)I, 1);
  int64_t nnz = 0;
  rowptr[0] = 0;
  for (int64_t u = 0; u < U; ++u) {
    memset(seen, 0, (size_t)I);
    const int64_t k = 1 + next_u32() % per_user;
    for (int64_t j = 0; j < k; ++j) seen[next_u32() % I] = 1;
    for (int64_t i = 0; i < I; ++i)
      if (seen[i]) col[nnz++] = (int32_t)i;
    rowptr[u + 1] = nnz;
  }
  float* X = malloc(sizeof(float) * U * d);
  for (int64_t i = 0; i < U * d; ++i) X[i] = (float)((int32_t)(next_u32() % 2001) - 1000) / 1000.f;

  /* device copies */
  int64_t *d_rowptr, *d_colptr;
  int32_t *d_col, *d_rows, *d_keys, *d_perm, *d_rows_t;
  float *d_dv, *d_de, *d_ev, *d_X, *d_M, *d_Y;
  CHECK_HIP(hipMalloc((void**)&d_rowptr, sizeof(int64_t) * (U + 1)));
  CHECK_HIP(hipMalloc((void**)&d_colptr, sizeof(int64_t) * (I + 1)));
  CHECK_HIP(hipMalloc((void**)&d_col, sizeof(int32_t) * nnz));
  CHECK_HIP(hipMalloc((void**)&d_rows, sizeof(int32_t) * nnz));
  CHECK_HIP(hipMalloc((void**)&d_keys, sizeof(int32_t) * nnz));
  CHECK_HIP(hipMalloc((void**)&d_perm, sizeof(int32_t) * nnz));
  CHECK_HIP(hipMalloc((void**)&d_rows_t, sizeof(int32_t) * nnz));
  CHECK_HIP(hipMalloc((void**)&d_dv, sizeof(float) * U));
  CHECK_HIP(hipMalloc((void**)&d_de, sizeof(float) * I));
  CHECK_HIP(hipMalloc((void**)&d_ev, sizeof(float) * nnz));
  CHECK_HIP(hipMalloc((void**)&d_X, sizeof(float) * U * d));
  CHECK_HIP(hipMalloc((void**)&d_M, sizeof(float) * I * d));
  CHECK_HIP(hipMalloc((void**)&d_Y, sizeof(float) * U * d));
  CHECK_HIP(hipMemcpy(d_rowptr, rowptr, sizeof(int64_t) * (U + 1), hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_col, col, sizeof(int32_t) * nnz, hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_X, X, sizeof(float) * U * d, hipMemcpyHostToDevice));
  hipStream_t st;
  CHECK_HIP(hipStreamCreate(&st));

  /* CSC of H: expand the CSR rows, stable-sort by column, row pointer of the sorted columns */
  const size_t ws_bytes = hgd_sort_perm_workspace_size(nnz);
  void* ws;
  CHECK_HIP(hipMalloc(&ws, ws_bytes));
  CHECK_HGD(hgd_expand_rows(d_rowptr, U, nnz, d_rows, st));
  CHECK_HGD(hgd_sort_perm(d_col, nnz, I, d_keys, d_perm, ws, ws_bytes, st));
  CHECK_HGD(hgd_rowptr_from_sorted(d_keys, nnz, I, d_colptr, st));
  CHECK_HGD(hgd_gather32(d_rows, d_perm, nnz, d_rows_t, st));
  /* D_v^-1/2, D_e^-1 and the hop-1 weights D_v^-1/2[user] folded per CSC nonzero */
  CHECK_HGD(hgd_degree_scale(d_rowptr, NULL, U, -0.5, d_dv, st));
  CHECK_HGD(hgd_degree_scale(d_colptr, NULL, I, -1.0, d_de, st));
  CHECK_HGD(hgd_edge_values(NULL, NULL, d_dv, d_rows_t, nnz, d_ev, st));
  /* M = D_e^-1·Hᵀ·(D_v^-1/2·X), Y = D_v^-1/2·H·M (no long rows here: no split plan) */
  CHECK_HGD(hgd_spmm(d_colptr, d_rows_t, d_ev, d_de, I, U, 0, I, d_X, d, d_M, d, d,
                     HGD_EPI_NONE, 0.f, NULL, NULL, 0, st));
  CHECK_HGD(hgd_spmm(d_rowptr, d_col, NULL, d_dv, U, I, 0, U, d_M, d, d_Y, d, d,
                     HGD_EPI_NONE, 0.f, NULL, NULL, 0, st));
  float* Y = malloc(sizeof(float) * U * d);
  CHECK_HIP(hipStreamSynchronize(st));
  CHECK_HIP(hipMemcpy(Y, d_Y, sizeof(float) * U * d, hipMemcpyDeviceToHost));

  /* float64 host reference and the 1e-5 magnitude-relative bound */
  double* dv = malloc(sizeof(double) * U);
  double* de = calloc((size_t)I, sizeof(double));
  for (int64_t u = 0; u < U; ++u) {
    const double g = (double)(rowptr[u + 1] - rowptr[u]);
    dv[u] = g > 0 ? 1.0 / sqrt(g) : 0.0;
    for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e) de[col[e]] += 1.0;
  }
  for (int64_t i = 0; i < I; ++i) de[i] = de[i] > 0 ? 1.0 / de[i] : 0.0;
  double* M = calloc((size_t)(I * d), sizeof(double));
  double* Ma = calloc((size_t)(I * d), sizeof(double));
  for (int64_t u = 0; u < U; ++u)
    for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e)
      for (int32_t k = 0; k < d; ++k) {
        M[col[e] * d + k] += dv[u] * X[u * d + k] * de[col[e]];
        Ma[col[e] * d + k] += dv[u] * fabs(X[u * d + k]) * de[col[e]];
      }
  double worst = 0.0;
  for (int64_t u = 0; u < U; ++u)
    for (int32_t k = 0; k < d; ++k) {
      double ref = 0.0, mag = 0.0;
      for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e) {
        ref += dv[u] * M[col[e] * d + k];
        mag += dv[u] * Ma[col[e] * d + k];
      }
      const double r = fabs((double)Y[u * d + k] - ref) / (mag + 1e-30);
      if (r > worst) worst = r;
    }
  printf("nnz %lld, max |Y - ref| / magnitude = %.3e\n", (long long)nnz, worst);
  if (worst > 1e-5) {
    fprintf(stderr, "hgconv2_host: mismatch\n");
    return 1;
  }
  printf("hgconv2_host ok\n");
  return 0;
}
