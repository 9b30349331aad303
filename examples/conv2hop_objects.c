/*
 * A plain-C host of the incidence-object ABI (include/hgd.h, "Incidence objects"): the HGNN
 * two-hop Y = D_v^-1/2·H·D_e^-1·Hᵀ·D_v^-1/2·X (data/graph.py:28-42) and its backward through
 * hgd_incidence_create + hgd_conv2hop_forward/backward, on user-row shards with the RCCL
 * exchange (hgd_comm_*) or the direct peer exchange (hgd_p2p_* + hgd_comm_create_p2p) — what a
 * native host would write in place of the reference's torch.sparse.mm calls
 * (HGNN_HD4.py:455-462).
 *
 * One process per GPU. WORLD_SIZE / RANK (default 1 / 0) pick this process's user shard;
 * HGD_TRANSPORT=p2p selects the peer exchange (default rccl). With WORLD_SIZE > 1 the setup
 * travels through files next to $HGD_COMM_ID_FILE: rank 0 writes the RCCL id there, or every
 * rank writes its hgd_p2p handle to $HGD_COMM_ID_FILE.<rank> and reads the others'.
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

static int read_file(const char* path, void* buf, size_t n) {
  for (int tries = 0; tries < 6000; ++tries) { /* up to 60 s */
    FILE* f = fopen(path, "rb");
    if (f) {
      size_t got = fread(buf, 1, n, f);
      fclose(f);
      if (got == n) return 0;
    }
    struct timespec ts = {0, 10 * 1000 * 1000};
    nanosleep(&ts, NULL);
  }
  return 1;
}

/* The peer exchange: create, export, all-gather the handles through files, open. */
static int open_p2p(int world, int rank, int64_t max_count, int32_t n_slots, hgd_p2p** out) {
  static unsigned char handles[8 * HGD_P2P_HANDLE_BYTES];
  if (world > 8) return 1;
  if (hgd_p2p_create(world, rank, max_count, n_slots, out) != HGD_OK) return 1;
  unsigned char* mine = handles + (size_t)rank * HGD_P2P_HANDLE_BYTES;
  if (hgd_p2p_export(*out, mine) != HGD_OK) return 1;
  if (world > 1) {
    const char* path = getenv("HGD_COMM_ID_FILE");
    if (!path) {
      fprintf(stderr, "WORLD_SIZE > 1 needs HGD_COMM_ID_FILE\n");
      return 1;
    }
    char name[4096], tmp[4200];
    snprintf(name, sizeof name, "%s.%d", path, rank);
    snprintf(tmp, sizeof tmp, "%s.tmp", name);
    FILE* f = fopen(tmp, "wb");
    if (!f || fwrite(mine, 1, HGD_P2P_HANDLE_BYTES, f) != HGD_P2P_HANDLE_BYTES) return 1;
    fclose(f);
    if (rename(tmp, name) != 0) return 1;
    for (int q = 0; q < world; ++q) {
      if (q == rank) continue;
      snprintf(name, sizeof name, "%s.%d", path, q);
      if (read_file(name, handles + (size_t)q * HGD_P2P_HANDLE_BYTES, HGD_P2P_HANDLE_BYTES)) {
        fprintf(stderr, "rank %d: no p2p handle in %s\n", rank, name);
        return 1;
      }
    }
  }
  return hgd_p2p_open(*out, handles) == HGD_OK ? 0 : 1;
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
  const char* transport = getenv("HGD_TRANSPORT");
  const int use_p2p = transport && strcmp(transport, "p2p") == 0;
  hgd_comm* comm = NULL;
  hgd_p2p* p2p = NULL;
  if (use_p2p) {
    /* two sets of ceil(d / 32) column slices of the [I, 32] item messages (d <= 128) */
    const int32_t n_slices = (d + 31) / 32;
    if (open_p2p(world, rank, I * 32, 2 * n_slices, &p2p)) {
      fprintf(stderr, "rank %d: peer exchange setup failed: %s\n", rank,
              hgd_get_last_error_string());
      return 1;
    }
    CHECK_HGD(hgd_comm_create_p2p(p2p, world, rank, &comm));
  } else {
    unsigned char id[HGD_COMM_ID_BYTES];
    if (exchange_id(world, rank, id)) return 1;
    CHECK_HGD(hgd_comm_create(id, world, rank, &comm));
  }
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
  printf("rank %d/%d (%s): users [%lld,%lld), nnz %lld, max |err| / magnitude = %.3e\n", rank,
         world, use_p2p ? "p2p" : "rccl", (long long)u0, (long long)u1, (long long)nnz_s, worst);
  hgd_comm_destroy(comm);
  if (p2p) {
    CHECK_HGD(hgd_p2p_check(p2p));
    if (world > 1) { /* the peers stop reading before the buffers go: a file barrier */
      const char* path = getenv("HGD_COMM_ID_FILE");
      char name[4096];
      snprintf(name, sizeof name, "%s.done.%d", path, rank);
      FILE* f = fopen(name, "wb");
      if (!f) return 1;
      fputc(1, f);
      fclose(f);
      for (int q = 0; q < world; ++q) {
        unsigned char b;
        snprintf(name, sizeof name, "%s.done.%d", path, q);
        if (read_file(name, &b, 1)) return 1;
      }
    }
    hgd_p2p_destroy(p2p);
  }
  hgd_incidence_destroy(H);
  if (worst > 1e-5) {
    fprintf(stderr, "conv2hop_objects: mismatch\n");
    return 1;
  }
  printf("conv2hop_objects ok\n");
  return 0;
}
