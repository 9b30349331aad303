// Incidence objects, the two-hop conv over them and the RCCL exchange (include/hgd.h, "Incidence
// objects"; SURVEY.md §8b C ABI, §8e multi-GPU).
//
// The object is the library-owned counterpart of the reference's torch.sparse COO adjacency
// (base/torch_interface.py:8-12): built once, it carries everything the hops need so that a
// forward/backward is two hgd_spmm launches each with no per-call structure work — where the
// reference's torch.sparse.mm re-coalesces and transposes `adj` inside every call
// (HGNN_HD4.py:455-462). The compute is the flat ABI's kernels (spmm.hip, structure.hip); this
// file only sequences them and owns memory.
//
// Multi-GPU: one process per GPU, users (rows of H) sharded, items replicated. Two transports
// for the all-reduce of hop 1's partial item sums, both on the communicator's side stream:
//  * RCCL (hgd_comm_create): item chunks, each chunk's ncclAllReduce queued behind the hop kernel
//    that produced it (event), so RCCL moves chunk k over xGMI while the CUs gather chunk k+1;
//  * the direct peer exchange (hgd_comm_create_p2p over an opened hgd_p2p): the embedding
//    COLUMNS are cut into slices (32 columns for d <= 128, else 64; hgd_comm_set_slice_width),
//    hop 1 of slice s writes straight into a send slot of the exchange, the slot's two-shot mesh
//    reduce runs on the side stream behind it, and hop 2 of slice s waits only for that slice —
//    the same pipeline, kernels and slot alternation as sharded.ShardedIncidence (transport
//    'p2p'), so the two give the same bits.

#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "hgd_internal.h"

namespace hgd {
namespace {

// Split-plan defaults, the same policy as incidence.auto_split (Python). A row walked by one
// lane group costs about 1.4 µs per 16 nonzeros of dependent index → gather round trips, so an
// unsplit row of T nonzeros ends the hop no sooner than ~T/11 µs: large structures split rows
// above pow2_floor(nnz / 8192) nonzeros (clamped to [128, 2048]) into chunks of half that (at most
// 512) — the longest walk stays a fraction of the whole hop's streaming time (a skewed catalogue's hop,
// scripts/bench_skewed_hop.py: 180 µs at 2048 / 512, 43 µs at 128 / 64); a structure with fewer
// rows than the lane-group tasks that fill the chip (256 CUs × 16 waves × 4 groups) is cut
// finer.
constexpr int64_t kSplitThreshold = 2048;
constexpr int32_t kSplitChunk = 512;
constexpr int64_t kSplitThresholdMin = 128;
constexpr int64_t kSplitNnzPerThreshold = 8192;
constexpr int64_t kTargetGroups = 16384;

void auto_split(int64_t n_rows, int64_t nnz, int64_t* threshold, int32_t* chunk) {
  if (n_rows >= kTargetGroups || nnz == 0) {
    int64_t t = kSplitThresholdMin;
    while (2 * t <= nnz / kSplitNnzPerThreshold && t < kSplitThreshold) t *= 2;
    *threshold = t;
    *chunk = static_cast<int32_t>(std::min<int64_t>(t / 2, kSplitChunk));
    return;
  }
  const int64_t want = std::max<int64_t>(1, nnz / kTargetGroups);
  int32_t c = 32;
  while (c < want && c < kSplitChunk) c *= 2;
  *threshold = 2 * static_cast<int64_t>(c);
  *chunk = c;
}

__global__ void k_validate_csr(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                               int64_t n_rows, int64_t n_cols, int64_t nnz,
                               unsigned long long* __restrict__ bad) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  unsigned long long local = 0;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
       i < std::max(n_rows + 1, nnz); i += stride) {
    if (i < n_rows && rowptr[i] > rowptr[i + 1]) ++local;
    if (i == 0 && rowptr[0] != 0) ++local;
    if (i == n_rows && rowptr[n_rows] != nnz) ++local;
    if (i < nnz) {
      const int32_t c = col[i];
      if (c < 0 || c >= n_cols) ++local;
    }
  }
  if (local) atomicAdd(bad, local);  // a count of violations: order does not matter
}

__global__ void k_fill(float* __restrict__ p, int64_t n, float v) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n; i += stride)
    p[i] = v;
}

__global__ void k_degree_f64(const int64_t* __restrict__ ptr, int64_t n, double* __restrict__ deg) {
  const int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (i < n) deg[i] = static_cast<double>(ptr[i + 1] - ptr[i]);
}

// Global column scales from the all-reduced degrees: 1/deg and 1/sqrt(deg) in float64 (both
// correctly rounded steps), 0 for an empty column, rounded to fp32 — the arithmetic of
// hgd_degree_scale and of sharded.ShardedIncidence._global_col_scale, so every path gives the
// same bits.
__global__ void k_scale_from_f64(const double* __restrict__ deg, int64_t n,
                                 float* __restrict__ mean, float* __restrict__ sym) {
  const int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (i >= n) return;
  const double g = deg[i];
  mean[i] = g > 0 ? static_cast<float>(1.0 / g) : 0.f;
  sym[i] = g > 0 ? static_cast<float>(1.0 / sqrt(g)) : 0.f;
}

// Integer degrees as three 16-bit limbs in fp32 (limb k of column i at k·n + i): a sum over <= 8
// ranks of limbs < 2^16 stays below 2^24, so the peer exchange's fp32 sum is exact.
__global__ void k_degree_limbs(const int64_t* __restrict__ ptr, int64_t n, int64_t count4,
                               float* __restrict__ out) {
  const int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (i < n) {
    const uint64_t g = static_cast<uint64_t>(ptr[i + 1] - ptr[i]);
    out[i] = static_cast<float>(g & 0xffff);
    out[n + i] = static_cast<float>((g >> 16) & 0xffff);
    out[2 * n + i] = static_cast<float>(g >> 32);
  } else if (i < count4 - 2 * n) {  // zero the padding to a multiple of 4 floats
    out[2 * n + i] = 0.f;
  }
}

__global__ void k_limbs_to_f64(const float* __restrict__ sum, int64_t n, double* __restrict__ deg) {
  const int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (i < n)
    deg[i] = static_cast<double>(sum[i]) + 65536.0 * static_cast<double>(sum[n + i]) +
             4294967296.0 * static_cast<double>(sum[2 * n + i]);
}

unsigned capped_grid(int64_t n) { return std::min<unsigned>(grid_for(n), 4096u); }

}  // namespace
}  // namespace hgd

// ---------------------------------------------------------------------------------------------
struct hgd_incidence {
  int64_t n_rows = 0, n_cols = 0, nnz = 0;
  int device = 0;
  bool weighted = false;
  bool global_cols = false;
  int64_t *rowptr = nullptr, *colptr = nullptr;
  int32_t *col = nullptr, *row_t = nullptr, *perm_t = nullptr;
  float *val = nullptr, *val_t = nullptr;
  float* scale[2][5] = {};  // [side][hgd_scale]; weighted kinds alias the plain ones when binary
  hgd_split_plan plan[2] = {};  // [0] CSR, [1] CSC
  // per-nonzero CSC weights val_t[e]·S[row_t[e]] for source kind S (lazily built)
  mutable std::mutex mu;
  mutable float* ev_csc[5] = {};
  // block-major copies of the CSC for the source-blocked hop (hgd_spmm_blocked), one per block
  // count in use, with the CSC weights of each source kind gathered into their order (lazily)
  struct BlockCopy {
    int32_t P = 0;
    int64_t* start = nullptr;
    int32_t* col = nullptr;
    int32_t* perm = nullptr;
    float* w[5] = {};  // [source kind]; HGD_SCALE_NONE = val_t (weighted objects only)
  };
  mutable BlockCopy blk[4];
  mutable std::vector<void*> owned;

  template <class T>
  hgd_status alloc(T** p, int64_t n) {
    *p = nullptr;
    if (n <= 0) return HGD_OK;
    void* q = nullptr;
    HGD_HIP(hipMalloc(&q, static_cast<size_t>(n) * sizeof(T)));
    owned.push_back(q);
    *p = static_cast<T*>(q);
    return HGD_OK;
  }
  ~hgd_incidence() {
    for (void* p : owned) (void)hipFree(p);
  }
};

struct hgd_comm {
  ncclComm_t comm = nullptr;  // RCCL transport (NULL for a peer-exchange communicator)
  hgd_p2p* p2p = nullptr;     // peer-exchange transport (not owned)
  int32_t nranks = 1, rank = 0, n_chunks = 4, slice_width = 0;
  int device = 0;
  uint64_t p2p_calls = 0;     // exchanges of conv hops issued: alternates the two slot sets
  hipStream_t side = nullptr;
  hipEvent_t ev[65] = {};
  hipEvent_t done[64] = {};
  ~hgd_comm() {
    for (hipEvent_t e : ev)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : done)
      if (e) (void)hipEventDestroy(e);
    if (side) (void)hipStreamDestroy(side);
    if (comm) (void)ncclCommDestroy(comm);
  }
};

namespace hgd {
namespace {

#define HGD_NCCL(call)                                                                  \
  do {                                                                                  \
    ncclResult_t _r = (call);                                                           \
    if (_r != ncclSuccess)                                                              \
      return ::hgd::fail(HGD_ERR_HIP, "%s failed: %s", #call, ncclGetErrorString(_r));  \
  } while (0)

hgd_status temp_alloc(void** p, size_t bytes, std::vector<void*>& temps) {
  *p = nullptr;
  if (bytes == 0) return HGD_OK;
  HGD_HIP(hipMalloc(p, bytes));
  temps.push_back(*p);
  return HGD_OK;
}

struct Temps {
  std::vector<void*> p;
  ~Temps() {
    for (void* q : p) (void)hipFree(q);
  }
};

// Degree scales of both sides (plain, and weighted when the object has values).
hgd_status build_scales(hgd_incidence* o, hipStream_t st) {
  const int64_t n[2] = {o->n_rows, o->n_cols};
  const int64_t* ptr[2] = {o->rowptr, o->colptr};
  const float* w[2] = {o->val, o->val_t};
  for (int s = 0; s < 2; ++s) {
    for (int k = HGD_SCALE_MEAN; k <= HGD_SCALE_WSYM; ++k) {
      const bool wk = k >= HGD_SCALE_WMEAN;
      if (wk && !o->weighted) {
        o->scale[s][k] = o->scale[s][k - 2];
        continue;
      }
      hgd_status r = o->alloc(&o->scale[s][k], n[s]);
      if (r != HGD_OK) return r;
      if (n[s] == 0) continue;
      const double p = (k == HGD_SCALE_MEAN || k == HGD_SCALE_WMEAN) ? -1.0 : -0.5;
      r = hgd_degree_scale(ptr[s], wk ? w[s] : nullptr, n[s], p, o->scale[s][k], st);
      if (r != HGD_OK) return r;
    }
  }
  return HGD_OK;
}

// Split plans of both orientations; `count` says whether a plan may be needed at all (a
// drop-edge child of a parent without split rows has none: degrees only shrink). One sync.
hgd_status build_plans(hgd_incidence* o, const bool count[2], hipStream_t st) {
  const int64_t n[2] = {o->n_rows, o->n_cols};
  const int64_t* ptr[2] = {o->rowptr, o->colptr};
  int64_t* dcounts = nullptr;
  int64_t hcounts[4] = {0, 0, 0, 0};
  bool any = false;
  Temps t;
  for (int s = 0; s < 2; ++s) {
    auto_split(n[s], o->nnz, &o->plan[s].threshold, &o->plan[s].chunk);
    o->plan[s].flags = 0;
    o->plan[s].n_heavy = 0;
    o->plan[s].n_chunks = 0;
  }
  for (int s = 0; s < 2; ++s) {
    if (!count[s] || n[s] == 0 || o->nnz <= o->plan[s].threshold) continue;
    if (!dcounts) {
      hgd_status r = temp_alloc(reinterpret_cast<void**>(&dcounts), 4 * sizeof(int64_t), t.p);
      if (r != HGD_OK) return r;
      HGD_HIP(hipMemsetAsync(dcounts, 0, 4 * sizeof(int64_t), st));
    }
    hgd_status r = hgd_split_plan_count(ptr[s], n[s], o->plan[s].threshold, o->plan[s].chunk,
                                        dcounts + 2 * s, st);
    if (r != HGD_OK) return r;
    any = true;
  }
  if (!any) return HGD_OK;
  HGD_HIP(hipMemcpyAsync(hcounts, dcounts, sizeof(hcounts), hipMemcpyDeviceToHost, st));
  HGD_HIP(hipStreamSynchronize(st));
  for (int s = 0; s < 2; ++s) {
    hgd_split_plan& p = o->plan[s];
    const int64_t n_heavy = hcounts[2 * s], n_chunks = hcounts[2 * s + 1];
    if (n_heavy == 0) continue;
    int32_t *rows = nullptr, *owner = nullptr;
    int64_t* cptr = nullptr;
    hgd_status r = o->alloc(&rows, n_heavy);
    if (r == HGD_OK) r = o->alloc(&cptr, n_heavy + 1);
    if (r == HGD_OK) r = o->alloc(&owner, n_chunks);
    if (r != HGD_OK) return r;
    void* ws = nullptr;
    const size_t wsb = hgd_split_plan_workspace_size(n[s]);
    r = temp_alloc(&ws, wsb, t.p);
    if (r != HGD_OK) return r;
    r = hgd_split_plan_build(ptr[s], n[s], p.threshold, p.chunk, rows, cptr, owner, n_heavy,
                             n_chunks, ws, wsb, st);
    if (r != HGD_OK) return r;
    p.n_heavy = n_heavy;
    p.n_chunks = n_chunks;
    p.heavy_rows = rows;
    p.heavy_cptr = cptr;
    p.chunk_heavy = owner;
  }
  HGD_HIP(hipStreamSynchronize(st));  // the plan workspaces are freed on return
  return HGD_OK;
}

// CSC (stable sort of the column ids: rows stay ascending inside a column), the CSC→CSR
// permutation, scales and plans of an object whose CSR arrays are in place.
hgd_status derive(hgd_incidence* o, hipStream_t st) {
  hgd_status r;
  if ((r = o->alloc(&o->colptr, o->n_cols + 1)) != HGD_OK) return r;
  if ((r = o->alloc(&o->row_t, o->nnz)) != HGD_OK) return r;
  if ((r = o->alloc(&o->perm_t, o->nnz)) != HGD_OK) return r;
  if (o->weighted && (r = o->alloc(&o->val_t, o->nnz)) != HGD_OK) return r;
  Temps t;
  if (o->nnz > 0) {
    int32_t *rows = nullptr, *keys = nullptr;
    void* ws = nullptr;
    const size_t wsb = hgd_sort_perm_workspace_size(o->nnz);
    if ((r = temp_alloc(reinterpret_cast<void**>(&rows), o->nnz * 4, t.p)) != HGD_OK) return r;
    if ((r = temp_alloc(reinterpret_cast<void**>(&keys), o->nnz * 4, t.p)) != HGD_OK) return r;
    if ((r = temp_alloc(&ws, wsb, t.p)) != HGD_OK) return r;
    if ((r = hgd_expand_rows(o->rowptr, o->n_rows, o->nnz, rows, st)) != HGD_OK) return r;
    if ((r = hgd_sort_perm(o->col, o->nnz, o->n_cols, keys, o->perm_t, ws, wsb, st)) != HGD_OK)
      return r;
    if ((r = hgd_rowptr_from_sorted(keys, o->nnz, o->n_cols, o->colptr, st)) != HGD_OK) return r;
    if ((r = hgd_gather32(rows, o->perm_t, o->nnz, o->row_t, st)) != HGD_OK) return r;
    if (o->weighted && (r = hgd_gather32(o->val, o->perm_t, o->nnz, o->val_t, st)) != HGD_OK)
      return r;
  } else {
    HGD_HIP(hipMemsetAsync(o->colptr, 0, (o->n_cols + 1) * sizeof(int64_t), st));
  }
  if ((r = build_scales(o, st)) != HGD_OK) return r;
  const bool count[2] = {true, true};
  if ((r = build_plans(o, count, st)) != HGD_OK) return r;
  HGD_HIP(hipStreamSynchronize(st));  // temporaries are freed on return
  return HGD_OK;
}

hgd_status check_sizes(int64_t n_rows, int64_t n_cols, int64_t nnz, const char* fn) {
  HGD_REQUIRE(n_rows >= 0 && n_cols >= 0 && nnz >= 0, "%s: negative sizes", fn);
  HGD_REQUIRE(n_rows < (int64_t(1) << 31) && n_cols < (int64_t(1) << 31),
              "%s: rows and columns must be < 2^31", fn);
  return HGD_OK;
}

// CSC weights for source-side kind k: val_t[e]·S_rows[k][row_t[e]] (NONE: val_t itself).
hgd_status csc_weights(const hgd_incidence* o, int k, const float** out, hipStream_t st) {
  *out = nullptr;
  if (k == HGD_SCALE_NONE) {
    *out = o->val_t;
    return HGD_OK;
  }
  std::lock_guard<std::mutex> g(o->mu);
  if (!o->ev_csc[k] && o->nnz > 0) {
    float* w = nullptr;
    void* q = nullptr;
    HGD_HIP(hipMalloc(&q, static_cast<size_t>(o->nnz) * 4));
    w = static_cast<float*>(q);
    hgd_status r = hgd_edge_values(o->val_t, nullptr, o->scale[HGD_SIDE_ROWS][k], o->row_t, o->nnz,
                                   w, st);
    if (r != HGD_OK) {
      (void)hipFree(q);
      return r;
    }
    o->owned.push_back(q);
    o->ev_csc[k] = w;
  }
  *out = o->ev_csc[k];
  return HGD_OK;
}

bool valid_kind(int32_t k) { return k >= HGD_SCALE_NONE && k <= HGD_SCALE_WSYM; }

// Source blocks of the hop over the CSC at width d: the structure and environment checks of
// incidence.spmm_blocks (the Python host) and the library's size rule hgd_spmm_blocks_for, so both
// hosts sum in the same order. 0 = one pass.
int32_t csc_blocks(const hgd_incidence* o, int32_t d) {
  const hgd_split_plan& pl = o->plan[1];
  if (o->nnz == 0 || (pl.threshold > 0 && pl.n_heavy > 0) || (pl.flags & HGD_PLAN_SEGMENTED))
    return 0;
  const char* env = std::getenv("HGD_SPMM_BLOCKS");
  if (env && *env && std::strcmp(env, "auto") != 0) {
    const long p = std::strtol(env, nullptr, 10);
    return (p > 1 && p <= 64) ? static_cast<int32_t>(p) : 0;
  }
  return hgd_spmm_blocks_for(o->n_rows, d);
}

// The block-major copy for P blocks and the CSC weights `w` of source kind k in its order.
hgd_status block_copy(const hgd_incidence* o, int32_t P, int32_t k, const float* w,
                      const hgd_incidence::BlockCopy** out, const float** out_w, hipStream_t st) {
  std::lock_guard<std::mutex> g(o->mu);
  hgd_incidence::BlockCopy* b = nullptr;
  for (auto& c : o->blk)
    if (c.P == P) b = &c;
  auto grab = [&](void** q, size_t bytes) -> hgd_status {
    HGD_HIP(hipMalloc(q, bytes));
    o->owned.push_back(*q);
    return HGD_OK;
  };
  if (!b) {
    for (auto& c : o->blk)
      if (c.P == 0 && !b) b = &c;
    HGD_REQUIRE(b, "hgd_incidence: more than 4 block counts in use");
    void *a = nullptr, *c = nullptr, *pm = nullptr, *ws = nullptr;
    const size_t wsb = hgd_spmm_col_blocks_workspace_size(o->n_cols, P);
    hgd_status r = grab(&a, (static_cast<size_t>(P) * o->n_cols + 1) * 8);
    if (r == HGD_OK) r = grab(&c, static_cast<size_t>(o->nnz) * 4);
    if (r == HGD_OK) r = grab(&pm, static_cast<size_t>(o->nnz) * 4);
    if (r != HGD_OK) return r;
    HGD_HIP(hipMalloc(&ws, wsb));
    r = hgd_spmm_col_blocks(o->colptr, o->row_t, o->n_cols, o->n_rows, P,
                            static_cast<int64_t*>(a), static_cast<int32_t*>(c),
                            static_cast<int32_t*>(pm), ws, wsb, st);
    const hipError_t e = hipStreamSynchronize(st);  // the workspace is freed here
    (void)hipFree(ws);
    if (r != HGD_OK) return r;
    if (e != hipSuccess)
      return fail(HGD_ERR_HIP, "hgd_incidence block copy: %s", hipGetErrorString(e));
    b->P = P;
    b->start = static_cast<int64_t*>(a);
    b->col = static_cast<int32_t*>(c);
    b->perm = static_cast<int32_t*>(pm);
  }
  if (w && !b->w[k]) {
    void* q = nullptr;
    hgd_status r = grab(&q, static_cast<size_t>(o->nnz) * 4);
    if (r != HGD_OK) return r;
    if ((r = hgd_gather32(w, b->perm, o->nnz, q, st)) != HGD_OK) return r;
    b->w[k] = static_cast<float*>(q);
  }
  *out = b;
  *out_w = w ? b->w[k] : nullptr;
  return HGD_OK;
}

// One hop over the CSC (rows [a, b) of Aᵀ) with the CSC weights w of source kind k: the
// source-blocked hop when csc_blocks says so, else hgd_spmm.
hgd_status csc_hop(const hgd_incidence* o, int32_t k, const float* w, const float* q, int64_t a,
                   int64_t b, const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t d,
                   int32_t epilogue, float slope, void* ws, size_t wsb, hipStream_t st) {
  const int32_t P = csc_blocks(o, d);
  if (P > 1) {
    const hgd_incidence::BlockCopy* bc = nullptr;
    const float* bw = nullptr;
    hgd_status r = block_copy(o, P, k, w, &bc, &bw, st);
    if (r != HGD_OK) return r;
    return hgd_spmm_blocked(bc->start, bc->col, bw, q, o->n_cols, o->n_rows, a, b, X, ldx, Y, ldy,
                            d, epilogue, slope, P, st);
  }
  return hgd_spmm(o->colptr, o->row_t, w, q, o->n_cols, o->n_rows, a, b, X, ldx, Y, ldy, d,
                  epilogue, slope, &o->plan[1], ws, wsb, st);
}

size_t spmm_ws(const hgd_incidence* o, int32_t d) {
  return std::max(hgd_spmm_workspace_size(&o->plan[0], d), hgd_spmm_workspace_size(&o->plan[1], d));
}

// Hop 1 of the conv: M = Q·Aᵀ·(S·X) over the CSC, all-reduced over `comm` in item chunks.
hgd_status hop_to_items(const hgd_incidence* o, int32_t Q, int32_t S, const float* X, int64_t ldx,
                        int32_t d, float* M, hgd_comm* comm, void* ws, size_t wsb,
                        hipStream_t st, const char* fn) {
  const float* w = nullptr;
  hgd_status r = csc_weights(o, S, &w, st);
  if (r != HGD_OK) return r;
  const float* q = Q == HGD_SCALE_NONE ? nullptr : o->scale[HGD_SIDE_COLS][Q];
  const int64_t n = o->n_cols;
  if (!comm) return csc_hop(o, S, w, q, 0, n, X, ldx, M, d, d, HGD_EPI_NONE, 0.f, ws, wsb, st);
  HGD_REQUIRE(comm->device == o->device, "%s: communicator and incidence on different devices",
              fn);
  const int64_t chunks = std::max<int64_t>(1, std::min<int64_t>(comm->n_chunks, n));
  const int64_t step = n ? (n + chunks - 1) / chunks : 0;
  int used = 0;
  for (int64_t a = 0; a < n; a += step) {
    const int64_t b = std::min(n, a + step);
    r = csc_hop(o, S, w, q, a, b, X, ldx, M, d, d, HGD_EPI_NONE, 0.f, ws, wsb, st);
    if (r != HGD_OK) return r;
    HGD_HIP(hipEventRecord(comm->ev[used], st));
    HGD_HIP(hipStreamWaitEvent(comm->side, comm->ev[used], 0));
    HGD_NCCL(ncclAllReduce(M + a * d, M + a * d, static_cast<size_t>((b - a) * d), ncclFloat32,
                           ncclSum, comm->comm, comm->side));
    ++used;
  }
  HGD_HIP(hipEventRecord(comm->ev[64], comm->side));
  HGD_HIP(hipStreamWaitEvent(st, comm->ev[64], 0));
  return HGD_OK;
}

hgd_status check_conv(const hgd_incidence* o, int32_t P, int32_t Q, int32_t R, int32_t d,
                      int32_t epilogue, hgd_comm* comm, const char* fn) {
  HGD_REQUIRE(o, "%s: null incidence", fn);
  HGD_REQUIRE(valid_kind(P) && valid_kind(Q) && valid_kind(R), "%s: bad scale kind", fn);
  HGD_REQUIRE(d > 0, "%s: d must be > 0", fn);
  HGD_REQUIRE(epilogue >= HGD_EPI_NONE && epilogue <= HGD_EPI_RELU, "%s: bad epilogue %d", fn,
              epilogue);
  if (comm) {
    HGD_REQUIRE(Q == HGD_SCALE_NONE || ((Q == HGD_SCALE_MEAN || Q == HGD_SCALE_SYM) &&
                                        o->global_cols),
                "%s: with a communicator Q must be NONE or a global MEAN/SYM "
                "(hgd_incidence_globalize_columns)", fn);
  }
  return HGD_OK;
}

// Column slice width of the peer-exchange pipeline (sharded.ShardedIncidence.slices).
int p2p_slice_width(const hgd_comm* c, int32_t d) {
  int w = c->slice_width > 0 ? c->slice_width : (d <= 128 ? 32 : 64);
  w = std::max(4, (w / 4) * 4);
  return std::min<int>(w, d);
}

// The two hops over the peer exchange, slice by slice (see the file header):
//   hop 1  slot = Q·Aᵀ·(S_src·X[:, c0:c1])   into send slot (parity·n_sl + s), compute stream
//          M_s  = Σ_ranks slot              hgd_p2p_allreduce on the side stream
//   hop 2  out[:, c0:c1] = epi(S_dst·A·M_s) after slice s's exchange only
// M holds the slices as contiguous [n_cols, w] blocks; saved_M (optional) gets them as [n_cols, d].
hgd_status two_hop_p2p(const hgd_incidence* o, int32_t Q, int32_t S_src, const float* X,
                       int64_t ldx, int32_t d, int32_t S_dst, float* out, int64_t ldo,
                       int32_t epilogue, float slope, float* saved_M, hgd_comm* c, float* M,
                       void* ws, size_t wsb, hipStream_t st, const char* fn) {
  HGD_REQUIRE(c->device == o->device, "%s: communicator and incidence on different devices", fn);
  HGD_REQUIRE(d % 4 == 0, "%s: the peer exchange needs d %% 4 == 0 (got %d)", fn, d);
  const int w = p2p_slice_width(c, d);
  const int n_sl = (d + w - 1) / w;
  const int64_t I = o->n_cols;
  HGD_REQUIRE(n_sl <= 64, "%s: %d column slices (at most 64)", fn, n_sl);
  HGD_REQUIRE(hgd_p2p_n_slots(c->p2p) >= 2 * n_sl && hgd_p2p_max_count(c->p2p) >= I * w,
              "%s: the exchange needs %d slots of %lld floats (has %d of %lld)", fn, 2 * n_sl,
              static_cast<long long>(I * w), hgd_p2p_n_slots(c->p2p),
              static_cast<long long>(hgd_p2p_max_count(c->p2p)));
  hgd_status r = hgd_p2p_poll(c->p2p);  // an earlier exchange timed out: stop here
  if (r != HGD_OK) return r;
  const float* wt = nullptr;
  if ((r = csc_weights(o, S_src, &wt, st)) != HGD_OK) return r;
  const float* q = Q == HGD_SCALE_NONE ? nullptr : o->scale[HGD_SIDE_COLS][Q];
  const float* p = S_dst == HGD_SCALE_NONE ? nullptr : o->scale[HGD_SIDE_ROWS][S_dst];
  const int parity = static_cast<int>(c->p2p_calls++ % 2);
  for (int s = 0; s < n_sl; ++s) {
    const int c0 = s * w, ws_ = std::min(w, d - c0);
    const int slot = parity * n_sl + s;
    float* send = hgd_p2p_slot(c->p2p, slot);
    // never source-blocked here: the send slot is uncached exchange memory (as sharded.py)
    if (I > 0 && (r = hgd_spmm(o->colptr, o->row_t, wt, q, I, o->n_rows, 0, I, X + c0, ldx, send,
                               ws_, ws_, HGD_EPI_NONE, 0.f, &o->plan[1], ws, wsb, st)) != HGD_OK)
      return r;
    HGD_HIP(hipEventRecord(c->ev[s], st));
    HGD_HIP(hipStreamWaitEvent(c->side, c->ev[s], 0));
    if ((r = hgd_p2p_allreduce(c->p2p, slot, I * ws_, M + I * c0, c->side)) != HGD_OK) return r;
    HGD_HIP(hipEventRecord(c->done[s], c->side));
  }
  for (int s = 0; s < n_sl; ++s) {
    const int c0 = s * w, ws_ = std::min(w, d - c0);
    const float* Ms = M + I * c0;
    HGD_HIP(hipStreamWaitEvent(st, c->done[s], 0));
    if (saved_M && I > 0)
      HGD_HIP(hipMemcpy2DAsync(saved_M + c0, static_cast<size_t>(d) * 4, Ms,
                               static_cast<size_t>(ws_) * 4, static_cast<size_t>(ws_) * 4, I,
                               hipMemcpyDeviceToDevice, st));
    if ((r = hgd_spmm(o->rowptr, o->col, o->val, p, o->n_rows, I, 0, o->n_rows, Ms, ws_,
                      out + c0, ldo, ws_, epilogue, slope, &o->plan[0], ws, wsb, st)) != HGD_OK)
      return r;
  }
  return HGD_OK;
}

size_t conv_ws(const hgd_incidence* o, int32_t d, int32_t epilogue) {
  size_t b = align_up(static_cast<size_t>(o->n_cols) * d * 4);
  if (epilogue != HGD_EPI_NONE) b += align_up(static_cast<size_t>(o->n_rows) * d * 4);
  return b + spmm_ws(o, d);
}

}  // namespace
}  // namespace hgd

using namespace hgd;

extern "C" hgd_status hgd_incidence_create(const int64_t* rowptr, const int32_t* col,
                                           const float* val, int64_t n_rows, int64_t n_cols,
                                           int64_t nnz, hgd_incidence** out, void* stream) {
  clear_error();
  HGD_REQUIRE(out, "hgd_incidence_create: null out");
  *out = nullptr;
  hgd_status r = check_sizes(n_rows, n_cols, nnz, "hgd_incidence_create");
  if (r != HGD_OK) return r;
  HGD_REQUIRE(rowptr && (nnz == 0 || col), "hgd_incidence_create: null rowptr/col");
  hipStream_t st = as_stream(stream);
  auto* o = new hgd_incidence();
  HGD_HIP(hipGetDevice(&o->device));
  o->n_rows = n_rows;
  o->n_cols = n_cols;
  o->nnz = nnz;
  o->weighted = val != nullptr;
  auto bail = [&](hgd_status s) {
    (void)hipStreamSynchronize(st);
    delete o;
    return s;
  };
  if ((r = o->alloc(&o->rowptr, n_rows + 1)) != HGD_OK) return bail(r);
  if ((r = o->alloc(&o->col, nnz)) != HGD_OK) return bail(r);
  if (o->weighted && (r = o->alloc(&o->val, nnz)) != HGD_OK) return bail(r);
  if (hipMemcpyAsync(o->rowptr, rowptr, (n_rows + 1) * sizeof(int64_t), hipMemcpyDeviceToDevice,
                     st) != hipSuccess ||
      (nnz && hipMemcpyAsync(o->col, col, nnz * 4, hipMemcpyDeviceToDevice, st) != hipSuccess) ||
      (nnz && o->weighted &&
       hipMemcpyAsync(o->val, val, nnz * 4, hipMemcpyDeviceToDevice, st) != hipSuccess))
    return bail(fail(HGD_ERR_HIP, "hgd_incidence_create: copy failed"));
  // validation (one sync): a bad structure would make the hops read out of bounds
  {
    Temps t;
    unsigned long long* dbad = nullptr;
    unsigned long long bad = 0;
    if ((r = temp_alloc(reinterpret_cast<void**>(&dbad), 8, t.p)) != HGD_OK) return bail(r);
    if (hipMemsetAsync(dbad, 0, 8, st) != hipSuccess)
      return bail(fail(HGD_ERR_HIP, "hgd_incidence_create: memset failed"));
    hipLaunchKernelGGL(k_validate_csr, dim3(capped_grid(std::max(n_rows + 1, nnz))),
                       dim3(kBlock), 0, st, o->rowptr, o->col, n_rows, n_cols, nnz, dbad);
    if ((r = check_launch("hgd_incidence_create: validate")) != HGD_OK) return bail(r);
    if (hipMemcpyAsync(&bad, dbad, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return bail(fail(HGD_ERR_HIP, "hgd_incidence_create: validation readback failed"));
    if (bad)
      return bail(fail(HGD_ERR_INVALID_ARG,
                       "hgd_incidence_create: malformed CSR (%llu violations: rowptr must rise "
                       "from 0 to nnz, 0 <= col < n_cols)", bad));
  }
  if ((r = derive(o, st)) != HGD_OK) return bail(r);
  *out = o;
  return HGD_OK;
}

extern "C" hgd_status hgd_incidence_from_dense(const float* H, int64_t n_rows, int64_t n_cols,
                                               int64_t ld, float thresh, int32_t mode,
                                               int32_t keep_values, hgd_incidence** out,
                                               void* stream) {
  clear_error();
  HGD_REQUIRE(out, "hgd_incidence_from_dense: null out");
  *out = nullptr;
  hgd_status r = check_sizes(n_rows, n_cols, 0, "hgd_incidence_from_dense");
  if (r != HGD_OK) return r;
  HGD_REQUIRE(H || n_rows * n_cols == 0, "hgd_incidence_from_dense: null H");
  hipStream_t st = as_stream(stream);
  auto* o = new hgd_incidence();
  HGD_HIP(hipGetDevice(&o->device));
  o->n_rows = n_rows;
  o->n_cols = n_cols;
  o->weighted = keep_values != 0;
  auto bail = [&](hgd_status s) {
    (void)hipStreamSynchronize(st);
    delete o;
    return s;
  };
  if ((r = o->alloc(&o->rowptr, n_rows + 1)) != HGD_OK) return bail(r);
  {
    Temps t;
    void* ws = nullptr;
    const size_t wsb = hgd_dense_threshold_workspace_size(n_rows);
    if ((r = temp_alloc(&ws, wsb, t.p)) != HGD_OK) return bail(r);
    r = hgd_dense_threshold_rowptr(H, n_rows, n_cols, ld, thresh, mode, o->rowptr, ws, wsb, st);
    if (r != HGD_OK) return bail(r);
    int64_t nnz = 0;
    if (hipMemcpyAsync(&nnz, o->rowptr + n_rows, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return bail(fail(HGD_ERR_HIP, "hgd_incidence_from_dense: count readback failed"));
    o->nnz = nnz;
  }
  if ((r = o->alloc(&o->col, o->nnz)) != HGD_OK) return bail(r);
  if (o->weighted && (r = o->alloc(&o->val, o->nnz)) != HGD_OK) return bail(r);
  if (o->nnz) {
    r = hgd_dense_threshold_fill(H, n_rows, n_cols, ld, thresh, mode, o->rowptr, o->col, o->val,
                                 st);
    if (r != HGD_OK) return bail(r);
  }
  if ((r = derive(o, st)) != HGD_OK) return bail(r);
  *out = o;
  return HGD_OK;
}

extern "C" hgd_status hgd_incidence_dropedge(const hgd_incidence* p, const uint8_t* keep_mask,
                                             float keep, hgd_incidence** out, void* stream) {
  clear_error();
  HGD_REQUIRE(out, "hgd_incidence_dropedge: null out");
  *out = nullptr;
  HGD_REQUIRE(p, "hgd_incidence_dropedge: null parent");
  HGD_REQUIRE(keep > 0.f, "hgd_incidence_dropedge: keep must be > 0");
  HGD_REQUIRE(p->nnz == 0 || keep_mask, "hgd_incidence_dropedge: null mask");
  if (p->nnz > 0 && !p->perm_t)
    return fail(HGD_ERR_UNSUPPORTED,
                "hgd_incidence_dropedge: a drop-edge child cannot be dropped again");
  hipStream_t st = as_stream(stream);
  auto* o = new hgd_incidence();
  o->device = p->device;
  o->n_rows = p->n_rows;
  o->n_cols = p->n_cols;
  o->weighted = true;  // values val/keep (1/keep for a binary parent), SpAdjDropEdge's newVals
  auto bail = [&](hgd_status s) {
    (void)hipStreamSynchronize(st);
    delete o;
    return s;
  };
  hgd_status r;
  const int64_t nnz = p->nnz;
  if ((r = o->alloc(&o->rowptr, p->n_rows + 1)) != HGD_OK) return bail(r);
  if ((r = o->alloc(&o->colptr, p->n_cols + 1)) != HGD_OK) return bail(r);
  if ((r = o->alloc(&o->col, nnz)) != HGD_OK) return bail(r);
  if ((r = o->alloc(&o->row_t, nnz)) != HGD_OK) return bail(r);
  if ((r = o->alloc(&o->val, nnz)) != HGD_OK) return bail(r);
  if ((r = o->alloc(&o->val_t, nnz)) != HGD_OK) return bail(r);
  {
    Temps t;
    void* ws = nullptr;
    const size_t wsb = hgd_dropedge_structure_workspace_size(nnz);
    if ((r = temp_alloc(&ws, wsb, t.p)) != HGD_OK) return bail(r);
    r = hgd_dropedge_structure(p->rowptr, p->col, p->val, p->colptr, p->row_t, p->val_t,
                               p->perm_t, p->n_rows, p->n_cols, nnz, keep_mask, keep, o->rowptr,
                               o->col, p->weighted ? o->val : nullptr, o->colptr, o->row_t,
                               p->weighted ? o->val_t : nullptr, ws, wsb, st);
    if (r != HGD_OK) return bail(r);
    int64_t kept = 0;
    if (hipMemcpyAsync(&kept, o->rowptr + p->n_rows, 8, hipMemcpyDeviceToHost, st) !=
            hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return bail(fail(HGD_ERR_HIP, "hgd_incidence_dropedge: count readback failed"));
    o->nnz = kept;
  }
  if (!p->weighted && o->nnz) {  // 1.0f / keep, the IEEE quotient the reference computes
    const float v = 1.0f / keep;
    hipLaunchKernelGGL(k_fill, dim3(capped_grid(o->nnz)), dim3(kBlock), 0, st, o->val, o->nnz, v);
    hipLaunchKernelGGL(k_fill, dim3(capped_grid(o->nnz)), dim3(kBlock), 0, st, o->val_t, o->nnz,
                       v);
    if ((r = check_launch("hgd_incidence_dropedge: fill")) != HGD_OK) return bail(r);
  }
  if ((r = build_scales(o, st)) != HGD_OK) return bail(r);
  const bool count[2] = {p->plan[0].n_heavy > 0, p->plan[1].n_heavy > 0};
  if ((r = build_plans(o, count, st)) != HGD_OK) return bail(r);
  *out = o;
  return HGD_OK;
}

extern "C" void hgd_incidence_destroy(hgd_incidence* inc) { delete inc; }

extern "C" hgd_status hgd_incidence_get_view(const hgd_incidence* o, hgd_incidence_view* v) {
  clear_error();
  HGD_REQUIRE(o && v, "hgd_incidence_get_view: null pointer");
  v->n_rows = o->n_rows;
  v->n_cols = o->n_cols;
  v->nnz = o->nnz;
  v->rowptr = o->rowptr;
  v->col = o->col;
  v->val = o->val;
  v->colptr = o->colptr;
  v->row_t = o->row_t;
  v->val_t = o->val_t;
  v->perm_t = o->perm_t;
  return HGD_OK;
}

extern "C" hgd_status hgd_incidence_scale(const hgd_incidence* o, int32_t side, int32_t kind,
                                          const float** out) {
  clear_error();
  HGD_REQUIRE(o && out, "hgd_incidence_scale: null pointer");
  HGD_REQUIRE(side == HGD_SIDE_ROWS || side == HGD_SIDE_COLS, "hgd_incidence_scale: bad side");
  HGD_REQUIRE(valid_kind(kind), "hgd_incidence_scale: bad kind %d", kind);
  *out = kind == HGD_SCALE_NONE ? nullptr : o->scale[side][kind];
  return HGD_OK;
}

extern "C" hgd_status hgd_incidence_prepare(const hgd_incidence* o, uint32_t kinds_mask,
                                            void* stream) {
  clear_error();
  HGD_REQUIRE(o, "hgd_incidence_prepare: null incidence");
  for (int k = HGD_SCALE_MEAN; k <= HGD_SCALE_WSYM; ++k) {
    if (!(kinds_mask & (1u << k))) continue;
    const float* w = nullptr;
    hgd_status r = csc_weights(o, k, &w, as_stream(stream));
    if (r != HGD_OK) return r;
  }
  return HGD_OK;
}

extern "C" size_t hgd_incidence_workspace_size(const hgd_incidence* o, int32_t d) {
  return o && d > 0 ? spmm_ws(o, d) : 0;
}

extern "C" hgd_status hgd_incidence_spmm(const hgd_incidence* o, int32_t transpose,
                                         const float* X, int64_t ldx, float* Y, int64_t ldy,
                                         int32_t d, const float* row_scale, int32_t epilogue,
                                         float slope, void* ws, size_t wsb, void* stream) {
  clear_error();
  HGD_REQUIRE(o, "hgd_incidence_spmm: null incidence");
  if (transpose)
    return csc_hop(o, HGD_SCALE_NONE, o->val_t, row_scale, 0, o->n_cols, X, ldx, Y, ldy, d,
                   epilogue, slope, ws, wsb, as_stream(stream));
  return hgd_spmm(o->rowptr, o->col, o->val, row_scale, o->n_rows, o->n_cols, 0, o->n_rows, X,
                  ldx, Y, ldy, d, epilogue, slope, &o->plan[0], ws, wsb, stream);
}

extern "C" size_t hgd_conv2hop_workspace_size(const hgd_incidence* o, int32_t d,
                                              int32_t epilogue) {
  return o && d > 0 ? conv_ws(o, d, epilogue) : 0;
}

extern "C" hgd_status hgd_conv2hop_forward(const hgd_incidence* o, int32_t P, int32_t Q,
                                           int32_t R, const float* X, int64_t ldx, int32_t d,
                                           float* Y, int64_t ldy, int32_t epilogue, float slope,
                                           float* saved_M, float* pre_act, hgd_comm* comm,
                                           void* ws, size_t wsb, void* stream) {
  clear_error();
  const char* fn = "hgd_conv2hop_forward";
  hgd_status r = check_conv(o, P, Q, R, d, epilogue, comm, fn);
  if (r != HGD_OK) return r;
  const bool fuse = epilogue == HGD_EPI_NONE || slope >= 0.f;
  HGD_REQUIRE(fuse || pre_act, "%s: an epilogue with slope < 0 needs pre_act", fn);
  HGD_REQUIRE(fuse || ldy == d, "%s: an epilogue with slope < 0 needs ldy == d", fn);
  const size_t need = conv_ws(o, d, epilogue);
  if (wsb < need || !ws)
    return fail(HGD_ERR_WORKSPACE, "%s: workspace %zu < required %zu", fn, wsb, need);
  hipStream_t st = as_stream(stream);
  float* M = static_cast<float*>(ws);
  char* sws = static_cast<char*>(ws) + (need - spmm_ws(o, d));
  const size_t swsb = spmm_ws(o, d);
  if (comm && comm->p2p) {
    if (fuse)
      return two_hop_p2p(o, Q, R, X, ldx, d, P, Y, ldy, epilogue, slope, saved_M, comm, M, sws,
                         swsb, st, fn);
    r = two_hop_p2p(o, Q, R, X, ldx, d, P, pre_act, d, HGD_EPI_NONE, 0.f, saved_M, comm, M, sws,
                    swsb, st, fn);
    if (r != HGD_OK) return r;
    return hgd_epilogue_apply(pre_act, o->n_rows * d, epilogue, slope, Y, st);
  }
  if ((r = hop_to_items(o, Q, R, X, ldx, d, M, comm, sws, swsb, st, fn)) != HGD_OK) return r;
  if (saved_M && o->n_cols)
    HGD_HIP(hipMemcpyAsync(saved_M, M, static_cast<size_t>(o->n_cols) * d * 4,
                           hipMemcpyDeviceToDevice, st));
  const float* p = P == HGD_SCALE_NONE ? nullptr : o->scale[HGD_SIDE_ROWS][P];
  if (fuse)
    return hgd_spmm(o->rowptr, o->col, o->val, p, o->n_rows, o->n_cols, 0, o->n_rows, M, d, Y,
                    ldy, d, epilogue, slope, &o->plan[0], sws, swsb, st);
  r = hgd_spmm(o->rowptr, o->col, o->val, p, o->n_rows, o->n_cols, 0, o->n_rows, M, d, pre_act, d,
               d, HGD_EPI_NONE, 0.f, &o->plan[0], sws, swsb, st);
  if (r != HGD_OK) return r;
  return hgd_epilogue_apply(pre_act, o->n_rows * d, epilogue, slope, Y, st);
}

extern "C" hgd_status hgd_conv2hop_backward(const hgd_incidence* o, int32_t P, int32_t Q,
                                            int32_t R, const float* dY, int64_t ldy, int32_t d,
                                            const float* act_ref, int32_t epilogue, float slope,
                                            float* dX, int64_t ldx, hgd_comm* comm, void* ws,
                                            size_t wsb, void* stream) {
  clear_error();
  const char* fn = "hgd_conv2hop_backward";
  hgd_status r = check_conv(o, P, Q, R, d, epilogue, comm, fn);
  if (r != HGD_OK) return r;
  const size_t need = conv_ws(o, d, epilogue);
  if (wsb < need || !ws)
    return fail(HGD_ERR_WORKSPACE, "%s: workspace %zu < required %zu", fn, wsb, need);
  hipStream_t st = as_stream(stream);
  float* dM = static_cast<float*>(ws);
  const size_t swsb = spmm_ws(o, d);
  char* sws = static_cast<char*>(ws) + (need - swsb);
  const float* g = dY;
  int64_t ldg = ldy;
  if (epilogue != HGD_EPI_NONE) {
    HGD_REQUIRE(act_ref, "%s: an epilogue needs act_ref (forward Y, or pre_act if slope < 0)", fn);
    HGD_REQUIRE(ldy == d, "%s: an epilogue needs ldy == d", fn);
    float* dZ = reinterpret_cast<float*>(static_cast<char*>(ws) +
                                         align_up(static_cast<size_t>(o->n_cols) * d * 4));
    if (o->n_rows && (r = hgd_epilogue_backward(act_ref, dY, o->n_rows * d, epilogue, slope, dZ,
                                                st)) != HGD_OK)
      return r;
    g = dZ;
    ldg = d;
  }
  if (comm && comm->p2p)
    return two_hop_p2p(o, Q, P, g, ldg, d, R, dX, ldx, HGD_EPI_NONE, 0.f, nullptr, comm, dM, sws,
                       swsb, st, fn);
  if ((r = hop_to_items(o, Q, P, g, ldg, d, dM, comm, sws, swsb, st, fn)) != HGD_OK) return r;
  const float* rs = R == HGD_SCALE_NONE ? nullptr : o->scale[HGD_SIDE_ROWS][R];
  return hgd_spmm(o->rowptr, o->col, o->val, rs, o->n_rows, o->n_cols, 0, o->n_rows, dM, d, dX,
                  ldx, d, HGD_EPI_NONE, 0.f, &o->plan[0], sws, swsb, st);
}

// ---------------------------------------------------------------------------------------------
extern "C" hgd_status hgd_comm_get_unique_id(void* id_out) {
  clear_error();
  HGD_REQUIRE(id_out, "hgd_comm_get_unique_id: null out");
  static_assert(sizeof(ncclUniqueId) == HGD_COMM_ID_BYTES, "RCCL id size");
  ncclUniqueId id;
  HGD_NCCL(ncclGetUniqueId(&id));
  memcpy(id_out, &id, sizeof(id));
  return HGD_OK;
}

extern "C" hgd_status hgd_comm_create(const void* id, int32_t nranks, int32_t rank,
                                      hgd_comm** out) {
  clear_error();
  HGD_REQUIRE(id && out, "hgd_comm_create: null pointer");
  HGD_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "hgd_comm_create: bad rank %d of %d",
              rank, nranks);
  *out = nullptr;
  auto* c = new hgd_comm();
  c->nranks = nranks;
  c->rank = rank;
  auto bail = [&](hgd_status s) {
    delete c;
    return s;
  };
  if (hipGetDevice(&c->device) != hipSuccess ||
      hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess)
    return bail(fail(HGD_ERR_HIP, "hgd_comm_create: stream creation failed"));
  for (hipEvent_t& e : c->ev)
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
      return bail(fail(HGD_ERR_HIP, "hgd_comm_create: event creation failed"));
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclResult_t nr = ncclCommInitRank(&c->comm, nranks, uid, rank);
  if (nr != ncclSuccess) {
    c->comm = nullptr;
    return bail(fail(HGD_ERR_HIP, "hgd_comm_create: ncclCommInitRank: %s", ncclGetErrorString(nr)));
  }
  *out = c;
  return HGD_OK;
}

extern "C" hgd_status hgd_comm_create_p2p(hgd_p2p* p2p, int32_t nranks, int32_t rank,
                                          hgd_comm** out) {
  clear_error();
  HGD_REQUIRE(p2p && out, "hgd_comm_create_p2p: null pointer");
  HGD_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "hgd_comm_create_p2p: bad rank %d of %d",
              rank, nranks);
  *out = nullptr;
  auto* c = new hgd_comm();
  c->p2p = p2p;
  c->nranks = nranks;
  c->rank = rank;
  auto bail = [&](hgd_status s) {
    delete c;
    return s;
  };
  // the exchange's waits run on the side stream at high priority, as in sharded.py: its few
  // workgroups are placed as soon as a CU frees instead of behind the queued hop grid
  int lo = 0, hi = 0;
  if (hipGetDevice(&c->device) != hipSuccess ||
      hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess ||
      hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, std::min(lo, hi)) != hipSuccess)
    return bail(fail(HGD_ERR_HIP, "hgd_comm_create_p2p: stream creation failed"));
  for (hipEvent_t& e : c->ev)
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
      return bail(fail(HGD_ERR_HIP, "hgd_comm_create_p2p: event creation failed"));
  for (hipEvent_t& e : c->done)
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
      return bail(fail(HGD_ERR_HIP, "hgd_comm_create_p2p: event creation failed"));
  *out = c;
  return HGD_OK;
}

extern "C" hgd_status hgd_comm_set_slice_width(hgd_comm* comm, int32_t width) {
  clear_error();
  HGD_REQUIRE(comm, "hgd_comm_set_slice_width: null comm");
  HGD_REQUIRE(width == 0 || (width >= 4 && width % 4 == 0),
              "hgd_comm_set_slice_width: width must be 0 (default) or a multiple of 4");
  comm->slice_width = width;
  return HGD_OK;
}

extern "C" void hgd_comm_destroy(hgd_comm* comm) {
  if (comm && comm->side) (void)hipStreamSynchronize(comm->side);
  delete comm;
}

extern "C" hgd_status hgd_comm_set_chunks(hgd_comm* comm, int32_t n_chunks) {
  clear_error();
  HGD_REQUIRE(comm, "hgd_comm_set_chunks: null comm");
  HGD_REQUIRE(n_chunks >= 1 && n_chunks <= 64, "hgd_comm_set_chunks: n_chunks in [1, 64]");
  comm->n_chunks = n_chunks;
  return HGD_OK;
}

extern "C" hgd_status hgd_exchange_allreduce(hgd_comm* comm, float* buf, int64_t count,
                                             void* stream) {
  clear_error();
  HGD_REQUIRE(comm, "hgd_exchange_allreduce: null comm");
  HGD_REQUIRE(count >= 0 && (count == 0 || buf), "hgd_exchange_allreduce: bad buffer");
  if (count == 0) return HGD_OK;
  if (comm->p2p) {  // through send slot 0 of the exchange (the conv hops alternate all slots)
    HGD_REQUIRE(count % 4 == 0 && reinterpret_cast<uintptr_t>(buf) % 16 == 0,
                "hgd_exchange_allreduce: over the peer exchange count must be a multiple of 4 "
                "and buf 16-byte aligned");
    HGD_REQUIRE(count <= hgd_p2p_max_count(comm->p2p),
                "hgd_exchange_allreduce: %lld floats exceed the exchange's slots",
                static_cast<long long>(count));
    HGD_HIP(hipMemcpyAsync(hgd_p2p_slot(comm->p2p, 0), buf, static_cast<size_t>(count) * 4,
                           hipMemcpyDeviceToDevice, as_stream(stream)));
    return hgd_p2p_allreduce(comm->p2p, 0, count, buf, stream);
  }
  HGD_NCCL(ncclAllReduce(buf, buf, static_cast<size_t>(count), ncclFloat32, ncclSum, comm->comm,
                         as_stream(stream)));
  return HGD_OK;
}

extern "C" hgd_status hgd_incidence_globalize_columns(hgd_incidence* o, hgd_comm* comm,
                                                      void* stream) {
  clear_error();
  HGD_REQUIRE(o && comm, "hgd_incidence_globalize_columns: null pointer");
  HGD_REQUIRE(!o->global_cols, "hgd_incidence_globalize_columns: already global");
  hipStream_t st = as_stream(stream);
  const int64_t n = o->n_cols;
  if (n == 0) {
    o->global_cols = true;
    return HGD_OK;
  }
  Temps t;
  double* deg = nullptr;
  hgd_status r = temp_alloc(reinterpret_cast<void**>(&deg), n * sizeof(double), t.p);
  if (r != HGD_OK) return r;
  if (comm->p2p) {
    // exact integer sums over the fp32 exchange: three 16-bit limbs per degree
    const int64_t count4 = (3 * n + 3) / 4 * 4;
    HGD_REQUIRE(count4 <= hgd_p2p_max_count(comm->p2p),
                "hgd_incidence_globalize_columns: %lld limbs exceed the exchange's slots",
                static_cast<long long>(count4));
    float* sum = nullptr;
    if ((r = temp_alloc(reinterpret_cast<void**>(&sum), count4 * sizeof(float), t.p)) != HGD_OK)
      return r;
    hipLaunchKernelGGL(k_degree_limbs, dim3(grid_for(count4 - 2 * n)), dim3(kBlock), 0, st,
                       o->colptr, n, count4, hgd_p2p_slot(comm->p2p, 0));
    if ((r = check_launch("hgd_incidence_globalize_columns")) != HGD_OK) return r;
    if ((r = hgd_p2p_allreduce(comm->p2p, 0, count4, sum, st)) != HGD_OK) return r;
    hipLaunchKernelGGL(k_limbs_to_f64, dim3(grid_for(n)), dim3(kBlock), 0, st, sum, n, deg);
    if ((r = check_launch("hgd_incidence_globalize_columns")) != HGD_OK) return r;
    HGD_HIP(hipStreamSynchronize(st));
    if ((r = hgd_p2p_check(comm->p2p)) != HGD_OK) return r;
  } else {
    hipLaunchKernelGGL(k_degree_f64, dim3(grid_for(n)), dim3(kBlock), 0, st, o->colptr, n, deg);
    if ((r = check_launch("hgd_incidence_globalize_columns")) != HGD_OK) return r;
    HGD_NCCL(ncclAllReduce(deg, deg, static_cast<size_t>(n), ncclFloat64, ncclSum, comm->comm,
                           st));
  }
  hipLaunchKernelGGL(k_scale_from_f64, dim3(grid_for(n)), dim3(kBlock), 0, st, deg, n,
                     o->scale[HGD_SIDE_COLS][HGD_SCALE_MEAN],
                     o->scale[HGD_SIDE_COLS][HGD_SCALE_SYM]);
  if ((r = check_launch("hgd_incidence_globalize_columns")) != HGD_OK) return r;
  HGD_HIP(hipStreamSynchronize(st));
  o->global_cols = true;
  return HGD_OK;
}
