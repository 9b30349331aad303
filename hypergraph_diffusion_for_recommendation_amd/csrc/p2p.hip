// Direct xGMI peer exchange: the all-reduce of the item messages without RCCL.
//
// Every rank exposes ONE uncached device allocation to its peers (hipIpcGetMemHandle, opened by
// the others with hipIpcOpenMemHandle):
//
//   [ flags: 2 kinds × 64 uint64 | send slots: n_slots × max_count f32 | reduced slots: same ]
//
// An exchange of `count` floats in send slot k is a two-shot all-reduce over the mesh:
//   1. signal/wait "sent":   this rank stores seq into flags[SENT][rank] of every peer, then
//                            waits until its own flags[SENT][q] >= seq for every q;
//   2. reduce:               rank r sums block r of the N send slots (own + N-1 peers, read over
//                            xGMI; q ascending, so every rank's result is the same bits) into its
//                            reduced slot k and into `out`;
//   3. signal/wait "reduced";
//   4. gather:               the other N-1 blocks are read from the peers' reduced slots into out.
// Each rank moves 2·(N-1)/N·count·4 bytes over its links, all N-1 at once (a ring moves the same
// volume one link at a time). Memory is uncached (hipDeviceMallocUncached) so a peer's reads
// see the owner's stores without cache maintenance; the flags are system-scope release /
// acquire atomics; every wait is bounded (wall clock) and a timeout sets a device error flag
// that turns the remaining exchanges into no-ops instead of hanging the GPU.
//
// Slot reuse: the buffers of an exchange i may be rewritten once any later exchange j > i has
// completed on this rank's stream — a peer signals "sent" for j only after its own stream has
// finished every read of i (exchanges are issued in the same order on every rank, on one
// stream per rank). The sharded hop alternates two sets of slots per call (sharded.py).
#include "hgd_internal.h"

#include <cstring>
#include <vector>

namespace {

constexpr int kMaxRanks = 8;
constexpr int kFlagSlots = 64;
constexpr size_t kFlagsBytes = 4096;  // 2 × 64 × 8 = 1 KiB, padded to a page
constexpr int kSent = 0, kReduced = 1;

struct Packed {  // the exported handle (HGD_P2P_HANDLE_BYTES)
  hipIpcMemHandle_t ipc;
  int64_t total_bytes;
  int64_t max_count;
  int32_t n_slots;
  int32_t rank;
  int32_t nranks;
  int32_t magic;
};
static_assert(sizeof(Packed) <= HGD_P2P_HANDLE_BYTES, "handle too large");
constexpr int32_t kMagic = 0x68676470;  // "hgdp"

__global__ void k_signal_wait(uint64_t* const* flags, int kind, int rank, int nranks,
                              uint64_t seq, uint64_t timeout_ticks, int* err) {
  const int t = threadIdx.x;
  if (t >= nranks) return;
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  // publish: peer t's slot for this rank (the previous kernels of this stream are complete, and
  // their stores to the uncached slots are in memory)
  __hip_atomic_store(flags[t] + kind * kFlagSlots + rank, seq, __ATOMIC_RELEASE,
                     __HIP_MEMORY_SCOPE_SYSTEM);
  // wait for peer t's store into this rank's slot
  const uint64_t* mine = flags[rank] + kind * kFlagSlots + t;
  const uint64_t t0 = static_cast<uint64_t>(wall_clock64());
  while (__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < seq) {
    __builtin_amdgcn_s_sleep(8);
    if (static_cast<uint64_t>(wall_clock64()) - t0 > timeout_ticks) {
      __hip_atomic_store(err, 1 + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
  }
}

// The block arithmetic of an exchange (host and device share it; hgd_p2p_block_range and
// hgd_p2p_gather_index expose it to the CPU tests): rank q reduces float4s [lo(q), hi(q)), the
// last blocks may be short or empty; gather element i < n4 - |own block| is float4 j of rank
// q's block, the own block skipped.
struct Blocks {
  int64_t n4, b4;  // float4s in the exchange, float4s per rank block
  __host__ __device__ static Blocks of(int64_t count, int nranks) {
    Blocks b;
    b.n4 = count / 4;
    b.b4 = (b.n4 + nranks - 1) / nranks;
    return b;
  }
  __host__ __device__ int64_t lo(int q) const { int64_t v = q * b4; return v < n4 ? v : n4; }
  __host__ __device__ int64_t hi(int q) const { int64_t v = (q + 1) * b4; return v < n4 ? v : n4; }
  __host__ __device__ int64_t gather_count(int rank) const { return n4 - (hi(rank) - lo(rank)); }
  __host__ __device__ int64_t gather_j(int rank, int64_t i) const {
    const int64_t own_lo = lo(rank), own_len = hi(rank) - own_lo;
    return i < own_lo ? i : i + own_len;
  }
  __host__ __device__ int gather_owner(int64_t j) const { return static_cast<int>(j / b4); }
};

// out[block r] = reduced_r[block r] = Σ_q send_q[block r], q ascending
__global__ void k_reduce(char* const* base, size_t send_off, size_t red_off, Blocks bl,
                         int rank, int nranks, float4* __restrict__ out, const int* err) {
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  const int64_t lo = bl.lo(rank), hi = bl.hi(rank);
  const float4* src[kMaxRanks];
#pragma unroll
  for (int q = 0; q < kMaxRanks; ++q)
    src[q] = reinterpret_cast<const float4*>(base[q < nranks ? q : 0] + send_off);
  float4* red = reinterpret_cast<float4*>(base[rank] + red_off);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = lo + blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < hi;
       i += stride) {
    float4 v[kMaxRanks];
#pragma unroll
    for (int q = 0; q < kMaxRanks; ++q)  // all loads in flight before the first add
      if (q < nranks) v[q] = src[q][i];
    float4 a = v[0];
#pragma unroll
    for (int q = 1; q < kMaxRanks; ++q)
      if (q < nranks) { a.x += v[q].x; a.y += v[q].y; a.z += v[q].z; a.w += v[q].w; }
    red[i] = a;
    out[i] = a;
  }
}

// out[block q] = reduced_q[block q] for every q != rank
__global__ void k_gather(char* const* base, size_t red_off, Blocks bl, int rank,
                         float4* __restrict__ out, const int* err) {
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  const int64_t n = bl.gather_count(rank);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += stride) {
    const int64_t j = bl.gather_j(rank, i);
    out[j] = reinterpret_cast<const float4*>(base[bl.gather_owner(j)] + red_off)[j];
  }
}

}  // namespace

struct hgd_p2p {
  int device = -1;
  int32_t nranks = 0, rank = 0, n_slots = 0;
  int64_t max_count = 0;
  size_t slot_bytes = 0, total_bytes = 0;
  char* base = nullptr;               // own exposed allocation
  std::vector<char*> bases;           // every rank's mapping (own = base), host copy
  char** d_bases = nullptr;           // the same on the device
  uint64_t** d_flags = nullptr;       // every rank's flag array on the device
  int* err = nullptr;                 // device error flag (0 = ok, q+1 = timed out on rank q)
  uint64_t seq = 0;                   // exchanges issued
  uint64_t ticks_per_s = 100000000;
  double timeout_s = 30.0;
  bool opened = false;

  size_t send_off(int slot) const { return kFlagsBytes + static_cast<size_t>(slot) * slot_bytes; }
  size_t red_off(int slot) const {
    return kFlagsBytes + static_cast<size_t>(n_slots + slot) * slot_bytes;
  }
  ~hgd_p2p() {
    if (device >= 0) (void)hipSetDevice(device);
    (void)hipDeviceSynchronize();
    for (int q = 0; q < static_cast<int>(bases.size()); ++q)
      if (q != rank && bases[q]) (void)hipIpcCloseMemHandle(bases[q]);
    if (d_bases) (void)hipFree(d_bases);
    if (d_flags) (void)hipFree(d_flags);
    if (err) (void)hipFree(err);
    if (base) (void)hipFree(base);
  }
};

using hgd::fail;

extern "C" hgd_status hgd_p2p_create(int32_t nranks, int32_t rank, int64_t max_count,
                                     int32_t n_slots, hgd_p2p** out) {
  hgd::clear_error();
  HGD_REQUIRE(out, "hgd_p2p_create: null out");
  *out = nullptr;
  HGD_REQUIRE(nranks >= 1 && nranks <= kMaxRanks && rank >= 0 && rank < nranks,
              "hgd_p2p_create: rank %d of %d (1..%d ranks)", rank, nranks, kMaxRanks);
  HGD_REQUIRE(max_count > 0 && max_count % 4 == 0,
              "hgd_p2p_create: max_count must be a positive multiple of 4, got %lld",
              static_cast<long long>(max_count));
  HGD_REQUIRE(n_slots >= 1 && n_slots <= 1024, "hgd_p2p_create: n_slots in [1, 1024]");
  auto* h = new hgd_p2p();
  auto bail = [&](hgd_status s) { delete h; return s; };
  if (hipGetDevice(&h->device) != hipSuccess) return bail(fail(HGD_ERR_HIP, "hgd_p2p_create: no device"));
  h->nranks = nranks;
  h->rank = rank;
  h->n_slots = n_slots;
  h->max_count = max_count;
  h->slot_bytes = hgd::align_up(static_cast<size_t>(max_count) * 4, 4096);
  h->total_bytes = kFlagsBytes + 2 * static_cast<size_t>(n_slots) * h->slot_bytes;
  void* p = nullptr;
  hipError_t e = hipExtMallocWithFlags(&p, h->total_bytes, hipDeviceMallocUncached);
  if (e != hipSuccess)
    return bail(fail(HGD_ERR_HIP, "hgd_p2p_create: uncached allocation of %zu bytes: %s",
                     h->total_bytes, hipGetErrorString(e)));
  h->base = static_cast<char*>(p);
  if (hipMemset(h->base, 0, kFlagsBytes) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&h->err), sizeof(int)) != hipSuccess ||
      hipMemset(h->err, 0, sizeof(int)) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&h->d_bases), kMaxRanks * sizeof(char*)) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&h->d_flags), kMaxRanks * sizeof(uint64_t*)) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess)
    return bail(fail(HGD_ERR_HIP, "hgd_p2p_create: setup failed"));
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, h->device) == hipSuccess &&
      khz > 0)
    h->ticks_per_s = static_cast<uint64_t>(khz) * 1000;
  h->bases.assign(nranks, nullptr);
  h->bases[rank] = h->base;
  *out = h;
  return HGD_OK;
}

extern "C" hgd_status hgd_p2p_export(const hgd_p2p* h, void* handle_out) {
  hgd::clear_error();
  HGD_REQUIRE(h && handle_out, "hgd_p2p_export: null pointer");
  Packed pk;
  std::memset(&pk, 0, sizeof(pk));
  HGD_HIP(hipSetDevice(h->device));
  HGD_HIP(hipIpcGetMemHandle(&pk.ipc, h->base));
  pk.total_bytes = static_cast<int64_t>(h->total_bytes);
  pk.max_count = h->max_count;
  pk.n_slots = h->n_slots;
  pk.rank = h->rank;
  pk.nranks = h->nranks;
  pk.magic = kMagic;
  std::memset(handle_out, 0, HGD_P2P_HANDLE_BYTES);
  std::memcpy(handle_out, &pk, sizeof(pk));
  return HGD_OK;
}

extern "C" hgd_status hgd_p2p_open(hgd_p2p* h, const void* handles) {
  hgd::clear_error();
  HGD_REQUIRE(h && handles, "hgd_p2p_open: null pointer");
  HGD_REQUIRE(!h->opened, "hgd_p2p_open: already open");
  HGD_HIP(hipSetDevice(h->device));
  const char* in = static_cast<const char*>(handles);
  for (int q = 0; q < h->nranks; ++q) {
    Packed pk;
    std::memcpy(&pk, in + static_cast<size_t>(q) * HGD_P2P_HANDLE_BYTES, sizeof(pk));
    HGD_REQUIRE(pk.magic == kMagic && pk.rank == q && pk.nranks == h->nranks &&
                    pk.total_bytes == static_cast<int64_t>(h->total_bytes) &&
                    pk.max_count == h->max_count && pk.n_slots == h->n_slots,
                "hgd_p2p_open: handle %d does not match this exchange (rank %d, %d ranks, "
                "%lld bytes)", q, pk.rank, pk.nranks, static_cast<long long>(pk.total_bytes));
    if (q == h->rank) continue;
    void* p = nullptr;
    HGD_HIP(hipIpcOpenMemHandle(&p, pk.ipc, hipIpcMemLazyEnablePeerAccess));
    h->bases[q] = static_cast<char*>(p);
  }
  std::vector<char*> b(kMaxRanks, h->base);
  std::vector<uint64_t*> f(kMaxRanks, reinterpret_cast<uint64_t*>(h->base));
  for (int q = 0; q < h->nranks; ++q) {
    b[q] = h->bases[q];
    f[q] = reinterpret_cast<uint64_t*>(h->bases[q]);
  }
  HGD_HIP(hipMemcpy(h->d_bases, b.data(), kMaxRanks * sizeof(char*), hipMemcpyHostToDevice));
  HGD_HIP(hipMemcpy(h->d_flags, f.data(), kMaxRanks * sizeof(uint64_t*), hipMemcpyHostToDevice));
  h->opened = true;
  return HGD_OK;
}

extern "C" float* hgd_p2p_slot(hgd_p2p* h, int32_t slot) {
  if (!h || slot < 0 || slot >= h->n_slots) return nullptr;
  return reinterpret_cast<float*>(h->base + h->send_off(slot));
}

extern "C" hgd_status hgd_p2p_set_timeout(hgd_p2p* h, double seconds) {
  hgd::clear_error();
  HGD_REQUIRE(h && seconds > 0.0, "hgd_p2p_set_timeout: null handle or non-positive timeout");
  h->timeout_s = seconds;
  return HGD_OK;
}

extern "C" hgd_status hgd_p2p_allreduce(hgd_p2p* h, int32_t slot, int64_t count, float* out,
                                        void* stream) {
  hgd::clear_error();
  HGD_REQUIRE(h && h->opened, "hgd_p2p_allreduce: handle not opened (hgd_p2p_open)");
  HGD_REQUIRE(slot >= 0 && slot < h->n_slots, "hgd_p2p_allreduce: slot %d of %d", slot,
              h->n_slots);
  HGD_REQUIRE(count >= 0 && count <= h->max_count && count % 4 == 0,
              "hgd_p2p_allreduce: count %lld (multiple of 4, <= %lld)",
              static_cast<long long>(count), static_cast<long long>(h->max_count));
  HGD_REQUIRE(out && reinterpret_cast<uintptr_t>(out) % 16 == 0,
              "hgd_p2p_allreduce: out must be a 16-byte aligned device pointer");
  if (count == 0) return HGD_OK;
  hipStream_t st = hgd::as_stream(stream);
  const uint64_t seq = ++h->seq;
  const uint64_t tmo = static_cast<uint64_t>(h->timeout_s * static_cast<double>(h->ticks_per_s));
  const Blocks bl = Blocks::of(count, h->nranks);
  float4* o = reinterpret_cast<float4*>(out);
  hipLaunchKernelGGL(k_signal_wait, dim3(1), dim3(64), 0, st, h->d_flags, kSent, h->rank,
                     h->nranks, seq, tmo, h->err);
  if (hgd_status r = hgd::check_launch("hgd_p2p_allreduce (signal)"); r != HGD_OK) return r;
  const unsigned g1 = std::min<unsigned>(1024, hgd::grid_for(std::max<int64_t>(bl.b4, 1)));
  hipLaunchKernelGGL(k_reduce, dim3(g1), dim3(hgd::kBlock), 0, st, h->d_bases,
                     h->send_off(slot), h->red_off(slot), bl, h->rank, h->nranks, o, h->err);
  if (hgd_status r = hgd::check_launch("hgd_p2p_allreduce (reduce)"); r != HGD_OK) return r;
  if (h->nranks > 1) {
    hipLaunchKernelGGL(k_signal_wait, dim3(1), dim3(64), 0, st, h->d_flags, kReduced, h->rank,
                       h->nranks, seq, tmo, h->err);
    if (hgd_status r = hgd::check_launch("hgd_p2p_allreduce (signal)"); r != HGD_OK) return r;
    const int64_t rest = bl.gather_count(h->rank);
    if (rest > 0) {
      const unsigned g2 = std::min<unsigned>(2048, hgd::grid_for(rest));
      hipLaunchKernelGGL(k_gather, dim3(g2), dim3(hgd::kBlock), 0, st, h->d_bases,
                         h->red_off(slot), bl, h->rank, o, h->err);
      if (hgd_status r = hgd::check_launch("hgd_p2p_allreduce (gather)"); r != HGD_OK) return r;
    }
  }
  return HGD_OK;
}

extern "C" hgd_status hgd_p2p_check(hgd_p2p* h) {
  hgd::clear_error();
  HGD_REQUIRE(h, "hgd_p2p_check: null handle");
  HGD_HIP(hipSetDevice(h->device));
  int e = 0;
  HGD_HIP(hipMemcpy(&e, h->err, sizeof(int), hipMemcpyDeviceToHost));
  if (e != 0)
    return fail(HGD_ERR_HIP, "hgd_p2p: an exchange timed out waiting for rank %d after %.1f s",
                e - 1, h->timeout_s);
  return HGD_OK;
}

extern "C" void hgd_p2p_destroy(hgd_p2p* h) { delete h; }

extern "C" hgd_status hgd_p2p_block_range(int64_t count, int32_t nranks, int32_t q, int64_t* lo,
                                          int64_t* hi) {
  hgd::clear_error();
  HGD_REQUIRE(count >= 0 && count % 4 == 0 && nranks >= 1 && nranks <= kMaxRanks && q >= 0 &&
                  q < nranks && lo && hi,
              "hgd_p2p_block_range: bad arguments");
  const Blocks b = Blocks::of(count, nranks);
  *lo = 4 * b.lo(q);
  *hi = 4 * b.hi(q);
  return HGD_OK;
}

extern "C" hgd_status hgd_p2p_gather_index(int64_t count, int32_t nranks, int32_t rank,
                                           int64_t i, int64_t* j, int32_t* owner) {
  hgd::clear_error();
  HGD_REQUIRE(count >= 0 && count % 4 == 0 && nranks >= 1 && nranks <= kMaxRanks && rank >= 0 &&
                  rank < nranks && j && owner,
              "hgd_p2p_gather_index: bad arguments");
  const Blocks b = Blocks::of(count, nranks);
  HGD_REQUIRE(i >= 0 && i < b.gather_count(rank), "hgd_p2p_gather_index: i out of range");
  *j = b.gather_j(rank, i);
  *owner = b.gather_owner(*j);
  return HGD_OK;
}
