/*
 * A plain-C host of the incidence-object ABI (include/hgd.h, "Incidence objects"): the HGNN
 * two-hop Y = D_v^-1/2·H·D_e^-1·Hᵀ·D_v^-1/2·X (data/graph.py:28-42) and its backward through
 * hgd_incidence_create + hgd_conv2hop_forward/backward, on user-row shards with the RCCL
 * exchange (hgd_comm_*) — what a native host would write in place of the reference's
 * torch.sparse.mm calls (HGNN_HD4.py:455-462).
 *
 * One process per GPU. WORLD_SIZE / RANK (default 1 / 0) pick this process's user shard;
 * with WORLD_SIZE > 1, rank 0 writes the RCCL id to $HGD_COMM_ID_FILE and the others read it.
 * Every rank builds the same deterministic graph, keeps its contiguous user range, runs the
 * sharded conv and checks its rows of Y and dX against a float64 host computation over the
 * whole graph (dX = the same operator applied to dY: the op is self-adjoint).
 * Exit status 0 and "conv2hop_objects ok" on success. Built by tests/_native_host.py.
 */
#define _POSIX_C_SOURCE 200809L
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

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

static uint64_t lcg = 0x243F6A8885A308D3ull;
static uint32_t next_u32(void) {
  lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
  return (uint32_t)(lcg >> 33);
}
static float next_f(void) { return (float)((int32_t)(next_u32() % 2001) - 1000) / 1000.f; }

static int exchange_id(int world, int rank, void* id) {
  const char* path = getenv("HGD_COMM_ID_FILE");
  if (world == 1) return hgd_comm_get_unique_id(id) == HGD_OK ? 0 : 1;
  if (!path) {
    fprintf(stderr, "WORLD_SIZE > 1 needs HGD_COMM_ID_FILE\n");
    return 1;
  }
  if (rank == 0) {
    if (hgd_comm_get_unique_id(id) != HGD_OK) return 1;
    char tmp[4096];
    snprintf(tmp, sizeof tmp, "%s.tmp", path);
    FILE* f = fopen(tmp, "wb");
    if (!f || fwrite(id, 1, HGD_COMM_ID_BYTES, f) != HGD_COMM_ID_BYTES) return 1;
    fclose(f);
    return rename(tmp, path) == 0 ? 0 : 1;
  }
  for (int tries = 0; tries < 6000; ++tries) {  /* up to 60 s */
    FILE* f = fopen(path, "rb");
    if (f) {
      size_t got = fread(id, 1, HGD_COMM_ID_BYTES, f);
      fclose(f);
      if (got == HGD_COMM_ID_BYTES) return 0;
    }
    struct timespec ts = {0, 10 * 1000 * 1000};
    nanosleep(&ts, NULL);
  }
  fprintf(stderr, "rank %d: no id in %s\n", rank, path);
  return 1;
}

int main(void) {
  const int world = getenv("WORLD_SIZE") ? atoi(getenv("WORLD_SIZE")) : 1;
  const int rank = getenv("RANK") ? atoi(getenv("RANK")) : 0;
  const int64_t U = 3000, I = 400;
  const int32_t d = 64;
  /* the whole graph on the host (CSR by user, columns ascending) */
  int64_t* rowptr = malloc(sizeof(int64_t) * (U + 1));
  int32_t* col = malloc(sizeof(int32_t) * U * 16);
  unsigned char* seen = calloc((size_t)I, 1);
  int64_t nnz = 0;
  rowptr[0] = 0;
  for (int64_t u = 0; u < U; ++u) {
    memset(seen, 0, (size_t)I);
    const int64_t k = u % 50 == 7 ? 0 : 1 + next_u32() % 16; /* some users without items */
    for (int64_t j = 0; j < k; ++j) seen[next_u32() % I] = 1;
    for (int64_t i = 0; i < I; ++i)
      if (seen[i]) col[nnz++] = (int32_t)i;
    rowptr[u + 1] = nnz;
  }
  float* X = malloc(sizeof(float) * U * d);
  float* dY = malloc(sizeof(float) * U * d);
  for (int64_t i = 0; i < U * d; ++i) X[i] = next_f();
  for (int64_t i = 0; i < U * d; ++i) dY[i] = next_f();

  /* this rank's user shard [u0, u1) */
  const int64_t u0 = U * rank / world, u1 = U * (rank + 1) / world, Us = u1 - u0;
  const int64_t e0 = rowptr[u0], e1 = rowptr[u1], nnz_s = e1 - e0;
  int64_t* rp_s = malloc(sizeof(int64_t) * (Us + 1));
  for (int64_t u = 0; u <= Us; ++u) rp_s[u] = rowptr[u0 + u] - e0;

  int64_t* d_rowptr;
  int32_t* d_col;
  float *d_X, *d_dY, *d_Y, *d_dX;
  CHECK_HIP(hipMalloc((void**)&d_rowptr, sizeof(int64_t) * (Us + 1)));
  CHECK_HIP(hipMalloc((void**)&d_col, sizeof(int32_t) * (nnz_s > 0 ? nnz_s : 1)));
  CHECK_HIP(hipMalloc((void**)&d_X, sizeof(float) * Us * d));
  CHECK_HIP(hipMalloc((void**)&d_dY, sizeof(float) * Us * d));
  CHECK_HIP(hipMalloc((void**)&d_Y, sizeof(float) * Us * d));
  CHECK_HIP(hipMalloc((void**)&d_dX, sizeof(float) * Us * d));
  CHECK_HIP(hipMemcpy(d_rowptr, rp_s, sizeof(int64_t) * (Us + 1), hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_col, col + e0, sizeof(int32_t) * nnz_s, hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_X, X + u0 * d, sizeof(float) * Us * d, hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_dY, dY + u0 * d, sizeof(float) * Us * d, hipMemcpyHostToDevice));
  hipStream_t st;
  CHECK_HIP(hipStreamCreate(&st));

  /* object + communicator; item scales made global before the conv */
  hgd_incidence* H = NULL;
  CHECK_HGD(hgd_incidence_create(d_rowptr, d_col, NULL, Us, I, nnz_s, &H, st));
  unsigned char id[HGD_COMM_ID_BYTES];
  if (exchange_id(world, rank, id)) return 1;
  hgd_comm* comm = NULL;
  CHECK_HGD(hgd_comm_create(id, world, rank, &comm));
  CHECK_HGD(hgd_incidence_globalize_columns(H, comm, st));
  CHECK_HGD(hgd_incidence_prepare(H, 1u << HGD_SCALE_SYM, st));
  const size_t wsb = hgd_conv2hop_workspace_size(H, d, HGD_EPI_NONE);
  void* ws;
  CHECK_HIP(hipMalloc(&ws, wsb));
  CHECK_HGD(hgd_conv2hop_forward(H, HGD_SCALE_SYM, HGD_SCALE_MEAN, HGD_SCALE_SYM, d_X, d, d, d_Y,
                                 d, HGD_EPI_NONE, 0.f, NULL, NULL, comm, ws, wsb, st));
  CHECK_HGD(hgd_conv2hop_backward(H, HGD_SCALE_SYM, HGD_SCALE_MEAN, HGD_SCALE_SYM, d_dY, d, d,
                                  NULL, HGD_EPI_NONE, 0.f, d_dX, d, comm, ws, wsb, st));
  CHECK_HIP(hipStreamSynchronize(st));
  float* Y = malloc(sizeof(float) * Us * d);
  float* dX = malloc(sizeof(float) * Us * d);
  CHECK_HIP(hipMemcpy(Y, d_Y, sizeof(float) * Us * d, hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(dX, d_dX, sizeof(float) * Us * d, hipMemcpyDeviceToHost));

  /* float64 host reference over the whole graph for this rank's rows */
  double* dv = malloc(sizeof(double) * U);
  double* de = calloc((size_t)I, sizeof(double));
  for (int64_t u = 0; u < U; ++u) {
    const double g = (double)(rowptr[u + 1] - rowptr[u]);
    dv[u] = g > 0 ? 1.0 / sqrt(g) : 0.0;
    for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e) de[col[e]] += 1.0;
  }
  for (int64_t i = 0; i < I; ++i) de[i] = de[i] > 0 ? 1.0 / de[i] : 0.0;
  double worst = 0.0;
  for (int pass = 0; pass < 2; ++pass) {
    const float* in = pass == 0 ? X : dY;
    const float* got = pass == 0 ? Y : dX;
    double* M = calloc((size_t)(I * d), sizeof(double));
    double* Ma = calloc((size_t)(I * d), sizeof(double));
    for (int64_t u = 0; u < U; ++u)
      for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e)
        for (int32_t k = 0; k < d; ++k) {
          M[col[e] * d + k] += dv[u] * in[u * d + k] * de[col[e]];
          Ma[col[e] * d + k] += dv[u] * fabs(in[u * d + k]) * de[col[e]];
        }
    for (int64_t u = u0; u < u1; ++u)
      for (int32_t k = 0; k < d; ++k) {
        double ref = 0.0, mag = 0.0;
        for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e) {
          ref += dv[u] * M[col[e] * d + k];
          mag += dv[u] * Ma[col[e] * d + k];
        }
        const double r = fabs((double)got[(u - u0) * d + k] - ref) / (mag + 1e-30);
        if (r > worst) worst = r;
      }
    free(M);
    free(Ma);
  }
  printf("rank %d/%d: users [%lld,%lld), nnz %lld, max |err| / magnitude = %.3e\n", rank, world,
         (long long)u0, (long long)u1, (long long)nnz_s, worst);
  hgd_comm_destroy(comm);
  hgd_incidence_destroy(H);
  if (worst > 1e-5) {
    fprintf(stderr, "conv2hop_objects: mismatch\n");
    return 1;
  }
  printf("conv2hop_objects ok\n");
  return 0;
}
