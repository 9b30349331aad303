// Direct xGMI peer exchange: the all-reduce of the item messages without RCCL.
//
// Every rank exposes uncached device memory to its peers (hipIpcGetMemHandle, opened by the
// others with hipIpcOpenMemHandle): a 4 KiB flag page and 2·n_slots slots of max_count floats
// (n_slots send slots, then n_slots reduced slots), packed whole into SEGMENTS — separate
// allocations of at most 1 GiB each (HGD_TUNE_P2P_SEGMENT_MB). One allocation per rank is not
// possible at the configs[4] sizes: on the ROCm 7.2 box, hipIpcOpenMemHandle of a 3.5 GiB or
// 4 GiB uncached allocation never returns (every rank of a 4-process rehearsal blocked inside
// it for 100 s, profiles/r04_scale/p2p_stall/), while 1 GiB imports open in milliseconds.
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
// volume one link at a time).
//
// Memory ordering (the argument does not depend on how the importing GPU caches a peer's
// memory: whether the dmabuf import keeps the exporter's uncached MTYPE or maps it
// non-coherent-cacheable is the driver's choice, so both must be correct):
//   * writer side: the owner's slot stores (hop 1 into a send slot, k_reduce into a reduced
//     slot) go to uncached memory, and are complete when their kernel ends. k_reduce also ends
//     with a system-scope release per workgroup. The flag that announces them is stored by a
//     LATER kernel of the same stream with release semantics at system scope (L2 write-back,
//     then the store), so no announced byte can still sit in a cache of the writer;
//   * reader side: the flag is read with a system-scope acquire by the wait kernel, and every
//     workgroup of k_reduce / k_gather starts with a system-scope acquire fence, which
//     invalidates its CU's L1 and the non-coherent lines of its L2 before the first peer load.
//     A slot is reused every second exchange of a stream (sharded.py alternates two slot sets),
//     so without that fence a non-coherent L2 line of the previous exchange could be read back;
//   * flags are only touched by system-scope atomics (never cached).
// Every wait is bounded (wall clock). A timeout sets a device error flag and its host-visible
// copy (hgd_p2p_poll reads it without a sync): the remaining exchanges then write NaN into
// their output instead of summing, so a failed exchange never passes for data.
//
// Slot reuse: the buffers of an exchange i may be rewritten once any later exchange j > i has
// completed on this rank's stream — a peer signals "sent" for j only after its own stream has
// finished every read of i (exchanges are issued in the same order on every rank, on one
// stream per rank).
#include "hgd_internal.h"

#include <algorithm>
#include <cstring>
#include <vector>

namespace {

constexpr int kMaxRanks = 8;
constexpr int kFlagSlots = 64;
constexpr size_t kFlagsBytes = 4096;  // 2 × 64 × 8 = 1 KiB, padded to a page
constexpr int kSent = 0, kReduced = 1;
constexpr int kMaxSegments = 62;      // handles per rank record (HGD_P2P_HANDLE_BYTES)
size_t g_segment_bytes = size_t(1) << 30;  // HGD_TUNE_P2P_SEGMENT_MB
int g_cached = 0;                          // HGD_TUNE_P2P_CACHED
// Workgroups of k_reduce / k_gather (HGD_TUNE_P2P_GRID). They run beside the hop kernels on a
// high-priority stream; over xGMI the links, not the CUs, bound them (a phase moves one 16 MB
// block per link at N = 8), and 256 workgroups keep 256 × 256 threads × 2 float4 × N loads in
// flight — far more than the links' bandwidth-latency product — while leaving the CUs to the
// hops the exchange overlaps.
unsigned g_grid = 256;

struct Packed {  // one rank's record in the handle exchange (HGD_P2P_HANDLE_BYTES)
  int32_t magic, rank, nranks, n_slots;
  int64_t max_count, slot_bytes;
  int32_t n_segments, slots_per_segment;
  int32_t cached, pad;
  hipIpcMemHandle_t flags;
  hipIpcMemHandle_t seg[kMaxSegments];
};
static_assert(sizeof(Packed) <= HGD_P2P_HANDLE_BYTES, "handle too large");
constexpr int32_t kMagic = 0x68676471;  // "hgdq" (segmented layout)

// System-scope fences (see "Memory ordering" above): the acquire invalidates this CU's vector L1
// and the non-coherent lines of the L2, so the loads after it fetch peer memory afresh; the
// release waits for this wave's stores and writes dirty L2 lines back to memory.
__device__ __forceinline__ void acquire_system() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); }
__device__ __forceinline__ void release_system() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, ""); }

__device__ __forceinline__ bool failed(const int* err) {
  return __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}

__global__ void k_signal_wait(uint64_t* const* flags, int kind, int rank, int nranks,
                              uint64_t seq, uint64_t timeout_ticks, int* err, int* host_err) {
  const int t = threadIdx.x;
  if (t >= nranks) return;
  if (failed(err)) return;
  // publish: peer t's slot for this rank. The release orders every earlier kernel of this stream
  // (complete before this one started) before the flag: its stores are in memory.
  __hip_atomic_store(flags[t] + kind * kFlagSlots + rank, seq, __ATOMIC_RELEASE,
                     __HIP_MEMORY_SCOPE_SYSTEM);
  // wait for peer t's store into this rank's slot
  const uint64_t* mine = flags[rank] + kind * kFlagSlots + t;
  const uint64_t t0 = static_cast<uint64_t>(wall_clock64());
  while (__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < seq) {
    __builtin_amdgcn_s_sleep(8);
    if (static_cast<uint64_t>(wall_clock64()) - t0 > timeout_ticks) {
      __hip_atomic_store(err, 1 + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // the host-visible copy hgd_p2p_poll reads without synchronising
      __hip_atomic_store(host_err, 1 + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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

// Every rank's address of one slot (kernel argument, by value).
struct SlotPtrs {
  const float4* p[kMaxRanks];
};

// After a timed-out wait the exchange's output is NaN, never stale or uninitialised memory.
__device__ __forceinline__ float4 nan4() {
  const float n = __builtin_nanf("");
  return make_float4(n, n, n, n);
}

// out[block r] = reduced_r[block r] = Σ_q send_q[block r], q ascending
__device__ __forceinline__ float4 add4(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

__global__ void k_reduce(SlotPtrs send, float4* red, Blocks bl, int rank, int nranks,
                         float4* __restrict__ out, const int* err) {
  const int64_t hi = bl.hi(rank);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const int64_t first = bl.lo(rank) + blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (failed(err)) {
    for (int64_t i = first; i < hi; i += stride) out[i] = nan4();
    return;
  }
  // the "sent" flags were acquired by the wait kernel before this one: drop any copy of a
  // peer's slot a cache may still hold from an earlier exchange of the same slot
  acquire_system();
  // two float4 per thread per step, all 2·N loads in flight before the first add
  int64_t i = first;
  for (; i + stride < hi; i += 2 * stride) {
    float4 v[kMaxRanks], w[kMaxRanks];
#pragma unroll
    for (int q = 0; q < kMaxRanks; ++q)
      if (q < nranks) { v[q] = send.p[q][i]; w[q] = send.p[q][i + stride]; }
    float4 a = v[0], b = w[0];
#pragma unroll
    for (int q = 1; q < kMaxRanks; ++q)
      if (q < nranks) { a = add4(a, v[q]); b = add4(b, w[q]); }
    red[i] = a;
    out[i] = a;
    red[i + stride] = b;
    out[i + stride] = b;
  }
  if (i < hi) {
    float4 v[kMaxRanks];
#pragma unroll
    for (int q = 0; q < kMaxRanks; ++q)
      if (q < nranks) v[q] = send.p[q][i];
    float4 a = v[0];
#pragma unroll
    for (int q = 1; q < kMaxRanks; ++q)
      if (q < nranks) a = add4(a, v[q]);
    red[i] = a;
    out[i] = a;
  }
  // the peers read red[] after the "reduced" flag: this workgroup's stores are performed at
  // system scope before the kernel ends (one release per workgroup, after all its waves' stores)
  __syncthreads();
  if (threadIdx.x == 0) release_system();
}

// out[block q] = reduced_q[block q] for every q != rank
__global__ void k_gather(SlotPtrs red, Blocks bl, int rank, float4* __restrict__ out,
                         const int* err) {
  const int64_t n = bl.gather_count(rank);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const int64_t first = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (failed(err)) {
    for (int64_t i = first; i < n; i += stride) out[bl.gather_j(rank, i)] = nan4();
    return;
  }
  acquire_system();  // the "reduced" flags were acquired by the wait kernel before this one
  int64_t i = first;
  for (; i + 3 * stride < n; i += 4 * stride) {  // four loads in flight per thread
    float4 v[4];
    int64_t j[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      j[u] = bl.gather_j(rank, i + u * stride);
      v[u] = red.p[bl.gather_owner(j[u])][j[u]];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) out[j[u]] = v[u];
  }
  for (; i < n; i += stride) {
    const int64_t jj = bl.gather_j(rank, i);
    out[jj] = red.p[bl.gather_owner(jj)][jj];
  }
}

}  // namespace

struct hgd_p2p {
  int device = -1;
  int32_t nranks = 0, rank = 0, n_slots = 0;
  int64_t max_count = 0;
  size_t slot_bytes = 0;
  int n_segments = 0, per_segment = 0;  // slots per segment (2·n_slots slots in all)
  int cached = 0;
  char* flags_own = nullptr;
  std::vector<char*> segs_own;
  // every rank's mappings (own entries are the own allocations), host copies
  std::vector<char*> flags;                // [rank]
  std::vector<std::vector<char*>> segs;    // [rank][segment]
  uint64_t** d_flags = nullptr;       // every rank's flag page on the device
  int* err = nullptr;                 // device error flag (0 = ok, q+1 = timed out on rank q)
  int* host_err = nullptr;            // its host-visible copy (pinned, coherent), host address
  int* host_err_dev = nullptr;        // ... and its device address
  uint64_t seq = 0;                   // exchanges issued
  uint64_t ticks_per_s = 100000000;
  double timeout_s = 30.0;
  bool opened = false;

  // slot g of rank q: send slots are g = 0 .. n_slots-1, reduced slots n_slots .. 2·n_slots-1
  char* slot(int q, int g) const {
    return segs[q][g / per_segment] + static_cast<size_t>(g % per_segment) * slot_bytes;
  }
  size_t segment_bytes(int s) const {
    const int first = s * per_segment;
    return static_cast<size_t>(std::min(per_segment, 2 * n_slots - first)) * slot_bytes;
  }
  ~hgd_p2p() {
    if (device >= 0) (void)hipSetDevice(device);
    (void)hipDeviceSynchronize();
    for (int q = 0; q < static_cast<int>(flags.size()); ++q) {
      if (q == rank) continue;
      if (flags[q]) (void)hipIpcCloseMemHandle(flags[q]);
      for (char* p : segs[q])
        if (p) (void)hipIpcCloseMemHandle(p);
    }
    if (d_flags) (void)hipFree(d_flags);
    if (err) (void)hipFree(err);
    if (host_err) (void)hipHostFree(host_err);
    for (char* p : segs_own)
      if (p) (void)hipFree(p);
    if (flags_own) (void)hipFree(flags_own);
  }
};

namespace hgd {
void set_p2p_segment_mb(int mb) { g_segment_bytes = (mb > 0 ? size_t(mb) : 1024) << 20; }
void set_p2p_cached(int cached) { g_cached = cached; }
void set_p2p_grid(int grid) { g_grid = grid > 0 ? static_cast<unsigned>(grid) : 256u; }
}  // namespace hgd

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
  const size_t slot_bytes = hgd::align_up(static_cast<size_t>(max_count) * 4, 4096);
  HGD_REQUIRE(slot_bytes <= g_segment_bytes,
              "hgd_p2p_create: a slot of %lld floats exceeds the %zu MiB segment limit",
              static_cast<long long>(max_count), g_segment_bytes >> 20);
  const int per_segment =
      static_cast<int>(std::min<size_t>(g_segment_bytes / slot_bytes, 2 * size_t(n_slots)));
  const int n_segments = (2 * n_slots + per_segment - 1) / per_segment;
  HGD_REQUIRE(n_segments <= kMaxSegments,
              "hgd_p2p_create: %d slots of %zu bytes need %d segments (at most %d)", 2 * n_slots,
              slot_bytes, n_segments, kMaxSegments);
  auto* h = new hgd_p2p();
  auto bail = [&](hgd_status s) { delete h; return s; };
  if (hipGetDevice(&h->device) != hipSuccess) return bail(fail(HGD_ERR_HIP, "hgd_p2p_create: no device"));
  h->nranks = nranks;
  h->rank = rank;
  h->n_slots = n_slots;
  h->max_count = max_count;
  h->slot_bytes = slot_bytes;
  h->per_segment = per_segment;
  h->n_segments = n_segments;
  h->cached = g_cached;
  const unsigned flag = g_cached ? hipDeviceMallocDefault : hipDeviceMallocUncached;
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, kFlagsBytes, hipDeviceMallocUncached) != hipSuccess)
    return bail(fail(HGD_ERR_HIP, "hgd_p2p_create: flag page allocation failed"));
  h->flags_own = static_cast<char*>(p);
  h->segs_own.assign(n_segments, nullptr);
  for (int s = 0; s < n_segments; ++s) {
    p = nullptr;
    hipError_t e = hipExtMallocWithFlags(&p, h->segment_bytes(s), flag);
    if (e != hipSuccess)
      return bail(fail(HGD_ERR_HIP, "hgd_p2p_create: segment %d of %zu bytes: %s", s,
                       h->segment_bytes(s), hipGetErrorString(e)));
    h->segs_own[s] = static_cast<char*>(p);
  }
  if (hipMemset(h->flags_own, 0, kFlagsBytes) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&h->err), sizeof(int)) != hipSuccess ||
      hipMemset(h->err, 0, sizeof(int)) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&h->d_flags), kMaxRanks * sizeof(uint64_t*)) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&h->host_err), sizeof(int),
                    hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&h->host_err_dev), h->host_err, 0) !=
          hipSuccess ||
      hipDeviceSynchronize() != hipSuccess)
    return bail(fail(HGD_ERR_HIP, "hgd_p2p_create: setup failed"));
  *h->host_err = 0;
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, h->device) == hipSuccess &&
      khz > 0)
    h->ticks_per_s = static_cast<uint64_t>(khz) * 1000;
  h->flags.assign(nranks, nullptr);
  h->segs.assign(nranks, std::vector<char*>(n_segments, nullptr));
  h->flags[rank] = h->flags_own;
  h->segs[rank] = h->segs_own;
  *out = h;
  return HGD_OK;
}

extern "C" hgd_status hgd_p2p_export(const hgd_p2p* h, void* handle_out) {
  hgd::clear_error();
  HGD_REQUIRE(h && handle_out, "hgd_p2p_export: null pointer");
  Packed pk;
  std::memset(&pk, 0, sizeof(pk));
  HGD_HIP(hipSetDevice(h->device));
  HGD_HIP(hipIpcGetMemHandle(&pk.flags, h->flags_own));
  for (int s = 0; s < h->n_segments; ++s) HGD_HIP(hipIpcGetMemHandle(&pk.seg[s], h->segs_own[s]));
  pk.magic = kMagic;
  pk.rank = h->rank;
  pk.nranks = h->nranks;
  pk.n_slots = h->n_slots;
  pk.max_count = h->max_count;
  pk.slot_bytes = static_cast<int64_t>(h->slot_bytes);
  pk.n_segments = h->n_segments;
  pk.slots_per_segment = h->per_segment;
  pk.cached = h->cached;
  std::memset(handle_out, 0, HGD_P2P_HANDLE_BYTES);
  std::memcpy(handle_out, &pk, sizeof(pk));
  return HGD_OK;
}

namespace {
// Opens one peer allocation and checks that the mapping spans all of it (a short import would
// fault, or read another object, at the first slot past its end).
hgd_status open_one(const hipIpcMemHandle_t& ipc, size_t bytes, int q, char** out) {
  void* p = nullptr;
  HGD_HIP(hipIpcOpenMemHandle(&p, ipc, hipIpcMemLazyEnablePeerAccess));
  *out = static_cast<char*>(p);
  hipDeviceptr_t mb = nullptr;
  size_t msz = 0;
  if (hipMemGetAddressRange(&mb, &msz, p) == hipSuccess) {
    const char* lo = static_cast<const char*>(mb);
    const char* at = static_cast<const char*>(p);
    if (at < lo || static_cast<size_t>(lo + msz - at) < bytes)
      return fail(HGD_ERR_HIP, "hgd_p2p_open: rank %d's mapping covers %zu of %zu bytes", q,
                  at < lo ? size_t(0) : static_cast<size_t>(lo + msz - at), bytes);
  } else {
    (void)hipGetLastError();
  }
  return HGD_OK;
}
}  // namespace

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
                    pk.max_count == h->max_count && pk.n_slots == h->n_slots &&
                    pk.slot_bytes == static_cast<int64_t>(h->slot_bytes) &&
                    pk.n_segments == h->n_segments && pk.slots_per_segment == h->per_segment &&
                    pk.cached == h->cached,
                "hgd_p2p_open: handle %d does not match this exchange (rank %d, %d ranks, "
                "%lld floats x %d slots in %d segments)", q, pk.rank, pk.nranks,
                static_cast<long long>(pk.max_count), pk.n_slots, pk.n_segments);
    if (q == h->rank) continue;
    if (hgd_status r = open_one(pk.flags, kFlagsBytes, q, &h->flags[q]); r != HGD_OK) return r;
    for (int s = 0; s < h->n_segments; ++s)
      if (hgd_status r = open_one(pk.seg[s], h->segment_bytes(s), q, &h->segs[q][s]); r != HGD_OK)
        return r;
  }
  std::vector<uint64_t*> f(kMaxRanks, reinterpret_cast<uint64_t*>(h->flags_own));
  for (int q = 0; q < h->nranks; ++q) f[q] = reinterpret_cast<uint64_t*>(h->flags[q]);
  HGD_HIP(hipMemcpy(h->d_flags, f.data(), kMaxRanks * sizeof(uint64_t*), hipMemcpyHostToDevice));
  h->opened = true;
  return HGD_OK;
}

extern "C" float* hgd_p2p_slot(hgd_p2p* h, int32_t slot) {
  if (!h || slot < 0 || slot >= h->n_slots) return nullptr;
  return reinterpret_cast<float*>(h->slot(h->rank, slot));
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
  SlotPtrs send{}, red{};
  for (int q = 0; q < kMaxRanks; ++q) {
    const int qq = q < h->nranks ? q : h->rank;
    send.p[q] = reinterpret_cast<const float4*>(h->slot(qq, slot));
    red.p[q] = reinterpret_cast<const float4*>(h->slot(qq, h->n_slots + slot));
  }
  float4* o = reinterpret_cast<float4*>(out);
  hipLaunchKernelGGL(k_signal_wait, dim3(1), dim3(64), 0, st, h->d_flags, kSent, h->rank,
                     h->nranks, seq, tmo, h->err, h->host_err_dev);
  if (hgd_status r = hgd::check_launch("hgd_p2p_allreduce (signal)"); r != HGD_OK) return r;
  const unsigned g1 = std::min<unsigned>(g_grid, hgd::grid_for(std::max<int64_t>(bl.b4, 1)));
  hipLaunchKernelGGL(k_reduce, dim3(g1), dim3(hgd::kBlock), 0, st, send,
                     reinterpret_cast<float4*>(h->slot(h->rank, h->n_slots + slot)), bl, h->rank,
                     h->nranks, o, h->err);
  if (hgd_status r = hgd::check_launch("hgd_p2p_allreduce (reduce)"); r != HGD_OK) return r;
  if (h->nranks > 1) {
    hipLaunchKernelGGL(k_signal_wait, dim3(1), dim3(64), 0, st, h->d_flags, kReduced, h->rank,
                       h->nranks, seq, tmo, h->err, h->host_err_dev);
    if (hgd_status r = hgd::check_launch("hgd_p2p_allreduce (signal)"); r != HGD_OK) return r;
    const int64_t rest = bl.gather_count(h->rank);
    if (rest > 0) {
      const unsigned g2 = std::min<unsigned>(g_grid, hgd::grid_for(rest));
      hipLaunchKernelGGL(k_gather, dim3(g2), dim3(hgd::kBlock), 0, st, red, bl, h->rank, o,
                         h->err);
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

extern "C" hgd_status hgd_p2p_poll(const hgd_p2p* h) {
  hgd::clear_error();
  HGD_REQUIRE(h, "hgd_p2p_poll: null handle");
  const int e = __atomic_load_n(h->host_err, __ATOMIC_ACQUIRE);
  if (e != 0)
    return fail(HGD_ERR_HIP, "hgd_p2p: an exchange timed out waiting for rank %d after %.1f s",
                e - 1, h->timeout_s);
  return HGD_OK;
}

// Pricing hook (profiles/r04_scale): the exchange's two data kernels at the block sizes of an
// `nranks`-way exchange, with every "peer" slot a separate LOCAL allocation (uncached unless
// `cached`): k_reduce of rank 0's block over nranks sources, then k_gather of the other
// nranks - 1 blocks; mean ms per launch over `iters` launches each (HIP events on `stream`).
// Local HBM stands in for the xGMI peers, so this prices the kernels' own cost, not the links.
extern "C" hgd_status hgd_p2p_price_local(int32_t nranks, int64_t count, int32_t cached,
                                          int32_t iters, float* ms_reduce, float* ms_gather,
                                          void* stream) {
  hgd::clear_error();
  HGD_REQUIRE(nranks >= 1 && nranks <= kMaxRanks && count > 0 && count % 4 == 0 && iters >= 1 &&
                  ms_reduce && ms_gather,
              "hgd_p2p_price_local: bad arguments");
  hipStream_t st = hgd::as_stream(stream);
  const size_t bytes = static_cast<size_t>(count) * 4;
  std::vector<void*> send(nranks, nullptr), red(nranks, nullptr);
  void* out = nullptr;
  int* err = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  auto cleanup = [&] {
    for (void* p : send) if (p) (void)hipFree(p);
    for (void* p : red) if (p) (void)hipFree(p);
    if (out) (void)hipFree(out);
    if (err) (void)hipFree(err);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
  };
  const unsigned flag = cached ? hipDeviceMallocDefault : hipDeviceMallocUncached;
  bool ok = hipMalloc(&out, bytes) == hipSuccess && hipMalloc(reinterpret_cast<void**>(&err),
                                                              sizeof(int)) == hipSuccess &&
            hipMemsetAsync(err, 0, sizeof(int), st) == hipSuccess &&
            hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess;
  for (int q = 0; ok && q < nranks; ++q)
    ok = hipExtMallocWithFlags(&send[q], bytes, flag) == hipSuccess &&
         hipExtMallocWithFlags(&red[q], bytes, flag) == hipSuccess &&
         hipMemsetAsync(send[q], 0, bytes, st) == hipSuccess &&
         hipMemsetAsync(red[q], 0, bytes, st) == hipSuccess;
  if (!ok) {
    cleanup();
    return fail(HGD_ERR_HIP, "hgd_p2p_price_local: allocation of %d x 2 x %zu bytes failed",
                nranks, bytes);
  }
  SlotPtrs sp{}, rp{};
  for (int q = 0; q < kMaxRanks; ++q) {
    sp.p[q] = static_cast<const float4*>(send[q < nranks ? q : 0]);
    rp.p[q] = static_cast<const float4*>(red[q < nranks ? q : 0]);
  }
  const Blocks bl = Blocks::of(count, nranks);
  float4* o = static_cast<float4*>(out);
  const unsigned g1 = std::min<unsigned>(g_grid, hgd::grid_for(std::max<int64_t>(bl.b4, 1)));
  const int64_t rest = bl.gather_count(0);
  const unsigned g2 = std::min<unsigned>(g_grid, hgd::grid_for(std::max<int64_t>(rest, 1)));
  auto reduce = [&] {
    hipLaunchKernelGGL(k_reduce, dim3(g1), dim3(hgd::kBlock), 0, st, sp,
                       const_cast<float4*>(rp.p[0]), bl, 0, nranks, o, err);
  };
  auto gather = [&] {
    if (rest > 0) hipLaunchKernelGGL(k_gather, dim3(g2), dim3(hgd::kBlock), 0, st, rp, bl, 0, o, err);
  };
  float t = 0.f;
  reduce();
  gather();
  ok = hipEventRecord(e0, st) == hipSuccess;
  for (int i = 0; i < iters; ++i) reduce();
  ok = ok && hipEventRecord(e1, st) == hipSuccess && hipEventSynchronize(e1) == hipSuccess &&
       hipEventElapsedTime(&t, e0, e1) == hipSuccess;
  *ms_reduce = t / iters;
  ok = ok && hipEventRecord(e0, st) == hipSuccess;
  for (int i = 0; i < iters; ++i) gather();
  ok = ok && hipEventRecord(e1, st) == hipSuccess && hipEventSynchronize(e1) == hipSuccess &&
       hipEventElapsedTime(&t, e0, e1) == hipSuccess;
  *ms_gather = rest > 0 ? t / iters : 0.f;
  const hipError_t le = hipGetLastError();
  cleanup();
  if (!ok || le != hipSuccess)
    return fail(HGD_ERR_HIP, "hgd_p2p_price_local: timing failed: %s", hipGetErrorString(le));
  return HGD_OK;
}

extern "C" int32_t hgd_p2p_n_slots(const hgd_p2p* h) { return h ? h->n_slots : 0; }
extern "C" int64_t hgd_p2p_max_count(const hgd_p2p* h) { return h ? h->max_count : 0; }

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
