// SpAdjDropEdge's keep-mask from torch's CPU generator, bit for bit, without torch's four
// tensor passes.
//
// Reference (paths relative to /root/reference/HD_SELFRec): SpAdjDropEdge.forward
// (model/graph/HCCF.py:217-226 and its copies) draws
//     mask = ((torch.rand(edgeNum) + keepRate).floor()).type(torch.bool)
// on the default CPU generator every layer of every step — at Yelp2018 size 2.3 M draws per
// layer, ≈ 10-30 ms per layer in torch (rand, add, floor, cast, then a count), which bounds the
// whole training step. The same mask comes out of one pass here:
//   * torch's CPU generator is at::mt19937 (MT19937, 32-bit outputs; ATen/core/MT19937RNGEngine.h)
//     and torch.rand(float32) takes one output per element, serially, as
//     ((y & 0xFFFFFF) · 2^-24) (uniform_real_distribution<float>, ATen/core/TransformationHelper.h);
//   * `+ keepRate` adds the float32-rounded scalar in float32, floor(·) != 0  ⇔  sum >= 1.
// The generator state is torch.get_rng_state()'s byte layout (CPUGeneratorImplState: the legacy
// POD with the 624 MT words as uint64, then the float-normal cache), read and written in place
// so the caller hands it back with torch.set_rng_state; the Python side checks the layout once
// against torch.rand itself before using this path.
#include <algorithm>
#include <atomic>
#include <climits>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <immintrin.h>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "../../include/hgd.h"
#include "hgd_internal.h"

namespace hgd {
namespace {

constexpr int kN = 624;
constexpr int kM = 397;

// torch/csrc (aten/src/ATen/CPUGeneratorImpl.cpp) CPUGeneratorImplStateLegacy + State
struct TorchCpuStateLegacy {
  uint64_t the_initial_seed;
  int32_t left;
  int32_t seeded;
  uint64_t next;
  uint64_t state[kN];
  double normal_x;
  double normal_y;
  double normal_rho;
  int32_t normal_is_valid;
};
struct TorchCpuState {
  TorchCpuStateLegacy legacy_pod;
  float next_float_normal_sample;
  bool is_next_float_normal_sample_valid;
};
static_assert(sizeof(TorchCpuState) == 5056, "torch CPU generator state layout");

__attribute__((always_inline)) inline uint32_t twist(uint32_t u, uint32_t v) {
  return (((u & 0x80000000u) | (v & 0x7fffffffu)) >> 1) ^ ((v & 1u) ? 0x9908b0dfu : 0u);
}

// at::mt19937::next_state on a plain uint32 array
__attribute__((always_inline)) inline void next_state(uint32_t* s) {
  uint32_t* p = s;
  for (int j = kN - kM + 1; --j; ++p) *p = p[kM] ^ twist(p[0], p[1]);
  for (int j = kM; --j; ++p) *p = p[kM - kN] ^ twist(p[0], p[1]);
  *p = p[kM - kN] ^ twist(p[0], s[0]);
}

__attribute__((always_inline)) inline uint32_t temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

// The draw loop, shared by the AVX2 and the baseline build of it (selected at run time): the
// tempering / compare loop and both halves of the state refill auto-vectorise.
// One cache-line-aligned object per drawing thread: the split draw keeps the threads' states
// side by side, and an unpadded state's counters shared a line with its neighbour's first words
// (rewritten every refill) — a line bouncing between two cores every 624 draws.
struct alignas(64) Draws {
  uint32_t s[kN];
  int left;
  uint32_t next;
};

__attribute__((always_inline)) inline int64_t draw_mask(Draws& g, int64_t n, float keep,
                                                        uint8_t* mask) {
  int64_t cnt = 0;
  int64_t k = 0;
  int left = g.left;  // in registers: the byte stores below may not alias them
  uint32_t next = g.next;
  while (k < n) {
    // at::mt19937::operator(): if (--left == 0) next_state(); y = state[next++]
    if (--left == 0) {
      next_state(g.s);
      left = kN;
      next = 0;
    }
    // calls that succeed before the next refill: `left` of them (this one included), each
    // consuming s[next++]
    const int64_t run = std::min<int64_t>(n - k, left);
    const uint32_t* __restrict__ src = g.s + next;
    uint8_t* __restrict__ dst = mask + k;
    int64_t c = 0;
    for (int64_t t = 0; t < run; ++t) {
      const uint32_t y = temper(src[t]);
      const float r = static_cast<float>(y & 0xFFFFFFu) * (1.0f / 16777216.0f);
      const float v = r + keep;              // float32 add, as the tensor op
      const uint8_t m = v >= 1.0f ? 1 : 0;   // floor(v) != 0 for v in [keep, keep + 1)
      dst[t] = m;
      c += m;
    }
    cnt += c;
    next += static_cast<uint32_t>(run);
    left -= static_cast<int>(run - 1);  // the first call of the run already decremented
    k += run;
  }
  g.left = left;
  g.next = next;
  return cnt;
}

__attribute__((target("avx2"))) int64_t draw_mask_avx2(Draws& g, int64_t n, float keep,
                                                       uint8_t* mask) {
  return draw_mask(g, n, keep, mask);
}

int64_t draw_mask_base(Draws& g, int64_t n, float keep, uint8_t* mask) {
  return draw_mask(g, n, keep, mask);
}

int64_t draw_any(Draws& g, int64_t n, float keep, uint8_t* mask) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  if (n == 0) return 0;
  return avx2 ? draw_mask_avx2(g, n, keep, mask) : draw_mask_base(g, n, keep, mask);
}

// ---------------------------------------------------------------------------------------------
// Jump-ahead: the draws split over threads, each starting from the generator state T refills
// ahead, computed in GF(2) (no draws skipped by stepping).
//
// Let w_0, w_1, … be the raw (untempered) words in output order; the array after r refills holds
// w_{624r} … w_{624r+623} (r = 0: the current array). The generator's linear state is the upper
// bit of w_t plus w_{t+1} … w_{t+623} (19,937 bits), so every bit of u_t = w_{t+1} satisfies the
// recurrence with MT19937's characteristic polynomial φ (degree 19,937): with
// x^N mod φ = Σ c_i x^i, u_{t+N} = ⊕_{c_i = 1} u_{t+i} for all t >= 0. The array after R refills
// is then word j = w_{624R+j} = u_{624R-1+j} = ⊕_{c_i = 1} u_{i+j} (N = 624R - 1): a XOR of
// shifted windows of the next 19,937 + 623 words, which one thread generates by plain refills.
// φ comes from Berlekamp–Massey on one bit of a generated sequence (once per process); x^N mod φ
// by square-and-multiply, cached per N (the split of a draw depends only on its length).
// ---------------------------------------------------------------------------------------------
constexpr int kDeg = 19937;
constexpr int kPhiWords = (kDeg + 1 + 63) / 64;  // 312
using Poly = std::vector<uint64_t>;

inline bool bit(const Poly& p, int64_t i) { return (p[i >> 6] >> (i & 63)) & 1u; }
inline void flip(Poly& p, int64_t i) { p[i >> 6] ^= uint64_t(1) << (i & 63); }

struct Gf2 {
  Poly phi;                      // φ, kDeg + 1 coefficients
  std::vector<Poly> phi_sh;      // φ·x^s for s = 0..63 (kPhiWords + 1 words each)
  uint16_t spread[256];          // bit i of a byte → bit 2i
  bool ok = false;
};

// at::mt19937's seeding (init_genrand) of a plain array
void seed_array(uint32_t* s, uint32_t seed) {
  s[0] = seed;
  for (int i = 1; i < kN; ++i) s[i] = 1812433253u * (s[i - 1] ^ (s[i - 1] >> 30)) + i;
}

// Berlekamp–Massey over GF(2) on bit 0 of 2·kDeg + 64 generated words: returns φ (the
// reciprocal of the connection polynomial), degree L.
Poly berlekamp_massey(int* L_out) {
  const int n_bits = 2 * kDeg + 64;
  std::vector<uint8_t> seq(n_bits);
  uint32_t s[kN];
  seed_array(s, 5489u);
  for (int k = 0; k < n_bits; k += kN) {
    next_state(s);
    for (int i = 0; i < kN && k + i < n_bits; ++i) seq[k + i] = s[i] & 1u;
  }
  const int W = (n_bits + 63) / 64 + 1;
  Poly C(W, 0), B(W, 0), win(W, 0);  // win bit i = seq[n - i]
  C[0] = B[0] = 1;
  int L = 0, m = 1;
  auto xor_shifted = [&](Poly& dst, const Poly& src, int sh) {  // dst ^= src << sh
    const int ws = sh >> 6, bs = sh & 63;
    for (int i = W - 1; i >= ws; --i) {
      uint64_t v = src[i - ws] << bs;
      if (bs && i - ws - 1 >= 0) v |= src[i - ws - 1] >> (64 - bs);
      dst[i] ^= v;
    }
  };
  for (int n = 0; n < n_bits; ++n) {
    // window ← window·x + seq[n]
    for (int i = W - 1; i > 0; --i) win[i] = (win[i] << 1) | (win[i - 1] >> 63);
    win[0] = (win[0] << 1) | seq[n];
    int d = 0;
    const int lw = (L >> 6) + 1;
    for (int i = 0; i < lw && i < W; ++i) d ^= __builtin_parityll(C[i] & win[i]);
    if (d == 0) {
      ++m;
    } else if (2 * L <= n) {
      Poly T = C;
      xor_shifted(C, B, m);
      L = n + 1 - L;
      B.swap(T);
      m = 1;
    } else {
      xor_shifted(C, B, m);
      ++m;
    }
  }
  Poly phi(kPhiWords, 0);
  if (L <= kDeg)
    for (int i = 0; i <= L; ++i)
      if (bit(C, i)) flip(phi, L - i);
  *L_out = L;
  return phi;
}

const Gf2& gf2() {
  static Gf2 g;
  static std::once_flag once;
  std::call_once(once, [] {
    int L = 0;
    g.phi = berlekamp_massey(&L);
    g.ok = L == kDeg && bit(g.phi, kDeg) && bit(g.phi, 0);
    g.phi_sh.assign(64, Poly(kPhiWords + 1, 0));
    for (int s = 0; s < 64; ++s)
      for (int i = 0; i <= kDeg; ++i)
        if (bit(g.phi, i)) flip(g.phi_sh[s], i + s);
    for (int b = 0; b < 256; ++b) {
      uint16_t v = 0;
      for (int i = 0; i < 8; ++i) v |= static_cast<uint16_t>(((b >> i) & 1) << (2 * i));
      g.spread[b] = v;
    }
  });
  return g;
}

// a mod φ in place (a has at most 2·kDeg bits); returns kPhiWords words
void reduce(const Gf2& g, Poly& a) {
  for (int64_t p = static_cast<int64_t>(a.size()) * 64 - 1; p >= kDeg; --p) {
    if (!bit(a, p)) continue;
    const int64_t sh = p - kDeg;
    const Poly& f = g.phi_sh[sh & 63];
    const int64_t w0 = sh >> 6;
    for (int i = 0; i <= kPhiWords && w0 + i < static_cast<int64_t>(a.size()); ++i)
      a[w0 + i] ^= f[i];
  }
  a.resize(kPhiWords);
}

// x^N mod φ
Poly x_pow_mod(const Gf2& g, int64_t N) {
  Poly r(kPhiWords, 0);
  r[0] = 1;
  int top = 63;
  while (top > 0 && !((N >> top) & 1)) --top;
  for (int b = top; b >= 0; --b) {
    Poly sq(2 * kPhiWords + 1, 0);  // r², spread bits
    for (int i = 0; i < kPhiWords; ++i) {
      uint64_t lo = 0, hi = 0;
      for (int k = 0; k < 4; ++k) {
        lo |= static_cast<uint64_t>(g.spread[(r[i] >> (8 * k)) & 0xff]) << (16 * k);
        hi |= static_cast<uint64_t>(g.spread[(r[i] >> (8 * k + 32)) & 0xff]) << (16 * k);
      }
      sq[2 * i] = lo;
      sq[2 * i + 1] = hi;
    }
    if ((N >> b) & 1) {  // ·x
      for (int i = static_cast<int>(sq.size()) - 1; i > 0; --i)
        sq[i] = (sq[i] << 1) | (sq[i - 1] >> 63);
      sq[0] <<= 1;
    }
    reduce(g, sq);
    r.swap(sq);
  }
  return r;
}

// x^N mod φ as its nonzero 4-bit windows, (k << 4) | m for coefficient bits 4k + b, b in m
// (cached: a draw of a given length uses the same jumps).
const std::vector<int32_t>& jump_windows(int64_t N) {
  static std::mutex mu;
  static std::map<int64_t, std::vector<int32_t>> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(N);
  if (it != cache.end()) return it->second;
  if (cache.size() > 256) cache.clear();
  const Poly c = x_pow_mod(gf2(), N);
  std::vector<int32_t> win;
  for (int k = 0; 4 * k < kDeg; ++k) {
    const int m = static_cast<int>((c[(4 * k) >> 6] >> ((4 * k) & 63)) & 15);
    if (m) win.push_back((k << 4) | m);
  }
  return cache.emplace(N, std::move(win)).first->second;
}

// out[j0 .. j0 + 8·NR) ^= ⊕ over windows (k, m) in [wb, we) of V_m[4k + j0 ..]: NR ymm
// accumulators
template <int NR>
__attribute__((target("avx2"))) inline void xor_windows(const uint32_t* const* V,
                                                        const int32_t* wb, const int32_t* we,
                                                        int j0, uint32_t* out) {
  __m256i a[NR];
  for (int r = 0; r < NR; ++r)
    a[r] = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(out + j0) + r);
  for (const int32_t* p = wb; p < we; ++p) {
    const int32_t e = *p;
    const uint32_t* src = V[e & 15] + 4 * (e >> 4) + j0;
    for (int r = 0; r < NR; ++r)
      a[r] = _mm256_xor_si256(a[r], _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src) + r));
  }
  for (int r = 0; r < NR; ++r) _mm256_storeu_si256(reinterpret_cast<__m256i*>(out + j0) + r, a[r]);
}

// The array after R >= 1 refills of the array `cur` (w_0 … w_623) from the windows of
// x^(624R-1) mod φ: u_t = w_{t+1} for t < kDeg + 627 by plain refills, the 15 window tables
// V_m[t] = ⊕_{b in m} u_{t+b}, then word j = ⊕_{(k,m)} V_m[4k + j] (4-bit windows halve the XORs
// of the bit-by-bit sum; the accumulators stay in registers, 64 words at a time).
__attribute__((target("avx2"))) void jump_array_avx2(const uint32_t* cur,
                                                     const std::vector<int32_t>& win,
                                                     uint32_t* out) {
  constexpr int kV = kDeg + kN;  // V_m[t] for t < kV (4k + j <= 19,936 + 623)
  constexpr int kU = kV + 4;     // u_t for t < kV + 3
  thread_local std::vector<uint32_t> u, tab;
  u.resize(kU + kN);
  tab.resize(16 * static_cast<size_t>(kV));
  uint32_t work[kN];
  std::memcpy(work, cur, sizeof(work));
  std::memcpy(u.data(), cur + 1, (kN - 1) * sizeof(uint32_t));
  for (int k = kN - 1; k < kU; k += kN) {
    next_state(work);
    std::memcpy(u.data() + k, work, sizeof(work));
  }
  const uint32_t* V[16];
  for (int m = 1; m < 16; ++m) {
    uint32_t* v = tab.data() + static_cast<size_t>(m) * kV;
    const int b = __builtin_ctz(m);
    const uint32_t* sh = u.data() + b;
    if (m == (1 << b)) {
      std::memcpy(v, sh, kV * sizeof(uint32_t));
    } else {
      const uint32_t* prev = tab.data() + static_cast<size_t>(m & (m - 1)) * kV;
      for (int t = 0; t < kV; ++t) v[t] = prev[t] ^ sh[t];
    }
    V[m] = v;
  }
  V[0] = nullptr;
  static_assert(kN == 9 * 64 + 48, "block split of the 624 state words");
  // windows in chunks (ascending k), every word block per chunk: the table rows a chunk reads
  // (15 × ~6.6 KB) stay in the core's L2 across the ten blocks, where a block-outer sweep read
  // all 1.2 MB of tables ten times through the shared L3 — the cost that grew with the threads
  std::memset(out, 0, kN * sizeof(uint32_t));
  constexpr size_t kChunk = 256;
  const int32_t* w = win.data();
  for (size_t c = 0; c < win.size(); c += kChunk) {
    const int32_t* wb = w + c;
    const int32_t* we = w + std::min(win.size(), c + kChunk);
    for (int j0 = 0; j0 < 9 * 64; j0 += 64) xor_windows<8>(V, wb, we, j0, out);
    xor_windows<6>(V, wb, we, 9 * 64, out);
  }
}

// Futex waits on one 32-bit word (private to the process).
inline void futex_wait(std::atomic<uint32_t>* w, uint32_t seen) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAIT_PRIVATE, seen, nullptr, nullptr,
          0);
}
inline void futex_wake(std::atomic<uint32_t>* w, int n) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAKE_PRIVATE, n, nullptr, nullptr, 0);
}

// A small persistent pool for the split draws (one call at a time). A call bumps the wake word
// of each worker it needs (one futex wake per worker; the others sleep on), each of them runs
// its task and counts itself off, and the caller runs task 0 and then waits for the count to
// reach zero. No mutex on either path: a condition variable's notify_all woke every worker and
// made them re-take one mutex in turn on the way in and again on the way out — a convoy that
// cost more than the draws' jumps at 16 threads (scripts/diag/diag_cpu_mask_threads.py).
class Pool {
 public:
  static Pool& get() {  // never destroyed: its detached workers wait on it until the process ends
    static Pool* p = new Pool;
    return *p;
  }
  std::mutex call_mu;  // serialises whole calls
  void run(int n_tasks, const std::function<void(int)>& fn) {
    ensure(n_tasks - 1);
    fn_ = &fn;
    pending_.store(static_cast<uint32_t>(n_tasks - 1), std::memory_order_relaxed);
    for (int i = 1; i < n_tasks; ++i) {
      slots_[i].go.fetch_add(1, std::memory_order_release);  // publishes fn_ / pending_
      futex_wake(&slots_[i].go, 1);
    }
    fn(0);
    for (int spin = 0;; ++spin) {  // a short spin, then sleep on the count
      const uint32_t p = pending_.load(std::memory_order_acquire);
      if (p == 0) break;
      if (spin < 256)
        _mm_pause();
      else
        futex_wait(&pending_, p);
    }
    fn_ = nullptr;
  }

 private:
  static constexpr int kMaxWorkers = 64;
  struct alignas(64) Slot {
    std::atomic<uint32_t> go{0};
  };
  void ensure(int workers) {
    while (threads_ < workers && threads_ < kMaxWorkers - 1) {
      const int idx = ++threads_;
      std::thread([this, idx] { loop(idx); }).detach();
    }
  }
  void loop(int idx) {
    uint32_t seen = 0;  // the slot's word starts at 0 and only this worker's calls bump it
    for (;;) {
      uint32_t g;
      for (int spin = 0; (g = slots_[idx].go.load(std::memory_order_acquire)) == seen; ++spin) {
        if (spin < 256)
          _mm_pause();
        else
          futex_wait(&slots_[idx].go, seen);
      }
      seen = g;
      (*fn_)(idx);
      if (pending_.fetch_sub(1, std::memory_order_acq_rel) == 1) futex_wake(&pending_, 1);
    }
  }
  Slot slots_[kMaxWorkers];
  std::atomic<uint32_t> pending_{0};
  const std::function<void(int)>* fn_ = nullptr;
  int threads_ = 0;  // workers started (indices 1 .. threads_); only run() starts them
};

int g_rng_threads = 0;  // HGD_TUNE_CPU_RNG_THREADS: 0 = auto, 1 = serial

// default: up to 16 threads (0.36 ms for 2.47 M draws on the GPU box's EPYC 9575F, 1.16 ms on
// one; profiles/r04_hccf/cpu_mask.jsonl), no more than the hardware threads or OMP_NUM_THREADS
int rng_threads() {
  if (g_rng_threads > 0) return g_rng_threads;
  static const int auto_threads = [] {
    int t = static_cast<int>(std::min(16u, std::max(1u, std::thread::hardware_concurrency())));
    if (const char* e = std::getenv("OMP_NUM_THREADS"))
      if (std::atoi(e) > 0) t = std::min(t, std::atoi(e));
    return std::max(1, t);
  }();
  return auto_threads;
}

// The split draw: thread 0 continues the real state over the head of the current block and the
// first Q refills; thread t >= 1 starts at refill 1 + t·Q from a jumped array. The last thread
// with draws leaves the final state.
int64_t draw_split(Draws& g, int64_t n, float keep, uint8_t* mask, int T) {
  const int64_t Q = ((n + kN - 1) / kN + T - 1) / T;  // refills per thread (from n alone)
  const int64_t head = std::min<int64_t>(n, g.left - 1);
  const int64_t rest = n - head;
  const int64_t r_tot = (rest + kN - 1) / kN;
  const int used = static_cast<int>(std::max<int64_t>(1, (r_tot + Q - 1) / Q));
  std::vector<int64_t> counts(used, 0);
  std::vector<Draws> st(used);
  st[0] = g;
  std::vector<const std::vector<int32_t>*> wins(used, nullptr);
  for (int t = 1; t < used; ++t) wins[t] = &jump_windows(kN * (1 + t * Q) - 1);
  auto task = [&](int t) {
    if (t >= used) return;
    const int64_t lo = t == 0 ? 0 : head + t * Q * kN;
    const int64_t hi = std::min<int64_t>(n, head + (t + 1) * Q * kN);
    if (t > 0) {
      jump_array_avx2(g.s, *wins[t], st[t].s);
      st[t].left = kN + 1;
      st[t].next = 0;
    }
    counts[t] = draw_any(st[t], hi - lo, keep, mask + lo);
  };
  Pool::get().run(used, task);
  g = st[used - 1];
  int64_t cnt = 0;
  for (int64_t c : counts) cnt += c;
  return cnt;
}

}  // namespace

void set_cpu_rng_threads(int threads) { g_rng_threads = threads; }

// Self-check of the jump (tests): the array after R refills of the seeded state, by stepping
// and by the GF(2) jump, must be equal.
bool cpu_rng_jump_selfcheck(int64_t R) {
  if (!gf2().ok) return false;
  uint32_t s[kN], a[kN], b[kN];
  seed_array(s, 1234u);
  next_state(s);
  std::memcpy(a, s, sizeof(a));
  for (int64_t r = 0; r < R; ++r) next_state(a);
  jump_array_avx2(s, jump_windows(kN * R - 1), b);
  return std::memcmp(a, b, sizeof(a)) == 0;
}

}  // namespace hgd

extern "C" size_t hgd_torch_cpu_state_bytes(void) { return sizeof(hgd::TorchCpuState); }

extern "C" int32_t hgd_torch_cpu_jump_selfcheck(int64_t refills) {
  return refills >= 1 && hgd::cpu_rng_jump_selfcheck(refills) ? 1 : 0;
}

extern "C" hgd_status hgd_torch_cpu_keep_mask_threads(uint8_t* torch_state, int64_t state_bytes,
                                                      int64_t n, float keep, uint8_t* mask,
                                                      int64_t* kept, int32_t threads) {
  using namespace hgd;
  clear_error();
  HGD_REQUIRE(threads >= 0 && threads <= 64, "hgd_torch_cpu_keep_mask: threads in [0, 64]");
  HGD_REQUIRE(torch_state && state_bytes == static_cast<int64_t>(sizeof(TorchCpuState)),
              "hgd_torch_cpu_keep_mask: state must be the %zu bytes of torch.get_rng_state()",
              sizeof(TorchCpuState));
  HGD_REQUIRE(n >= 0 && (mask || n == 0), "hgd_torch_cpu_keep_mask: bad n / mask");
  TorchCpuState st;
  std::memcpy(&st, torch_state, sizeof(st));
  TorchCpuStateLegacy& L = st.legacy_pod;
  HGD_REQUIRE(L.left >= 1 && L.left <= kN && L.next <= static_cast<uint64_t>(kN),
              "hgd_torch_cpu_keep_mask: generator state out of range (left=%d next=%llu)",
              L.left, static_cast<unsigned long long>(L.next));
  Draws g;
  for (int i = 0; i < kN; ++i) g.s[i] = static_cast<uint32_t>(L.state[i]);
  g.left = L.left;
  g.next = static_cast<uint32_t>(L.next);
  // long draws split over threads from jumped states (bitwise the serial draw); short ones, a
  // serial tuning or a CPU without AVX2 run the one-thread loop
  static const bool avx2 = __builtin_cpu_supports("avx2");
  const int T = threads > 0 ? threads : rng_threads();
  int64_t cnt;
  if (T > 1 && avx2 && n >= static_cast<int64_t>(T) * 64 * kN && gf2().ok) {
    std::lock_guard<std::mutex> lk(Pool::get().call_mu);
    cnt = draw_split(g, n, keep, mask, T);
  } else {
    cnt = draw_any(g, n, keep, mask);
  }
  for (int i = 0; i < kN; ++i) L.state[i] = g.s[i];
  L.left = g.left;
  L.next = g.next;
  std::memcpy(torch_state, &st, sizeof(st));
  if (kept) *kept = cnt;
  return HGD_OK;
}

extern "C" hgd_status hgd_torch_cpu_keep_mask(uint8_t* torch_state, int64_t state_bytes,
                                              int64_t n, float keep, uint8_t* mask,
                                              int64_t* kept) {
  return hgd_torch_cpu_keep_mask_threads(torch_state, state_bytes, n, keep, mask, kept, 0);
}
