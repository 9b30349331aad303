// Host-side pairwise sampler, bit-identical to the reference's Python one.
//
// Reference (paths relative to /root/reference/HD_SELFRec): next_batch_pairwise
// (util/sampler.py:237-264) shuffles data.training_data IN PLACE with random.shuffle, then for
// every record of a batch draws n_negs negatives with random.choice(item_list), redrawing while
// the item is in the user's training items. Every training epoch of every plugin runs this
// Python loop (≈ 3 µs per record: seconds per epoch at Yelp2018 size, more than the device
// step it feeds).
//
// This file restates CPython's generator exactly — MT19937 (Modules/_randommodule.c
// genrand_uint32), getrandbits(k) = genrand_uint32() >> (32 - k) for k <= 32, and
// Random._randbelow_with_getrandbits(n) (k = n.bit_length(), redraw while r >= n), which both
// shuffle (j = randbelow(i + 1), i = n-1 .. 1) and choice (seq[randbelow(len(seq))]) use — on the
// state random.getstate() exposes (624 words + position), so the caller can hand the state in
// and back (random.setstate) and the Python random stream continues exactly as if the reference
// loop had run. item_list = list(data.item.keys()) is the dense item order, so the choice index
// IS the dense id; membership is a binary search in the user's sorted training items.
#include <cstdint>
#include <cstring>

#include "../../include/hgd.h"
#include "hgd_internal.h"

namespace hgd {
namespace {

constexpr int kMtN = 624;
constexpr int kMtM = 397;

struct Mt {
  uint32_t* mt;  // 624 words
  uint32_t index;

  uint32_t next() {
    static const uint32_t mag01[2] = {0x0u, 0x9908b0dfu};
    if (index >= static_cast<uint32_t>(kMtN)) {
      int kk;
      uint32_t y;
      for (kk = 0; kk < kMtN - kMtM; ++kk) {
        y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
        mt[kk] = mt[kk + kMtM] ^ (y >> 1) ^ mag01[y & 1u];
      }
      for (; kk < kMtN - 1; ++kk) {
        y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
        mt[kk] = mt[kk + (kMtM - kMtN)] ^ (y >> 1) ^ mag01[y & 1u];
      }
      y = (mt[kMtN - 1] & 0x80000000u) | (mt[0] & 0x7fffffffu);
      mt[kMtN - 1] = mt[kMtM - 1] ^ (y >> 1) ^ mag01[y & 1u];
      index = 0;
    }
    uint32_t y = mt[index++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }

  // Random._randbelow_with_getrandbits(n), 1 <= n < 2^32
  uint32_t below(uint64_t n) {
    int k = 0;
    while ((n >> k) != 0) ++k;  // n.bit_length()
    uint64_t r = k >= 32 ? next() : (next() >> (32 - k));
    while (r >= n) r = k >= 32 ? next() : (next() >> (32 - k));
    return static_cast<uint32_t>(r);
  }
};

bool sorted_contains(const int32_t* a, int64_t lo, int64_t hi, int32_t v) {
  while (lo < hi) {
    const int64_t mid = lo + ((hi - lo) >> 1);
    if (a[mid] == v) return true;
    if (a[mid] < v)
      lo = mid + 1;
    else
      hi = mid;
  }
  return false;
}

hgd_status check_state(const uint32_t* state) {
  if (!state) return fail(HGD_ERR_INVALID_ARG, "null MT19937 state");
  if (state[kMtN] > static_cast<uint32_t>(kMtN))
    return fail(HGD_ERR_INVALID_ARG, "MT19937 position %u > 624", state[kMtN]);
  return HGD_OK;
}

}  // namespace
}  // namespace hgd

extern "C" hgd_status hgd_py_shuffle(uint32_t* mt_state, int64_t* order, int64_t n) {
  using namespace hgd;
  clear_error();
  hgd_status s = check_state(mt_state);
  if (s != HGD_OK) return s;
  HGD_REQUIRE(n >= 0 && n < (int64_t{1} << 32), "hgd_py_shuffle: n out of range");
  HGD_REQUIRE(order || n == 0, "hgd_py_shuffle: null order");
  Mt g{mt_state, mt_state[kMtN]};
  for (int64_t i = n - 1; i >= 1; --i) {  // random.shuffle: reversed(range(1, len(x)))
    const int64_t j = g.below(static_cast<uint64_t>(i) + 1);
    const int64_t t = order[i];
    order[i] = order[j];
    order[j] = t;
  }
  mt_state[kMtN] = g.index;
  return HGD_OK;
}

extern "C" hgd_status hgd_sample_pairwise(uint32_t* mt_state, const int64_t* order, int64_t begin,
                                          int64_t end, const int32_t* rec_user,
                                          const int32_t* rec_item, const int64_t* user_rowptr,
                                          const int32_t* user_items, int64_t n_users,
                                          int64_t n_items, int32_t n_negs, int32_t* out_u,
                                          int32_t* out_i, int32_t* out_j) {
  using namespace hgd;
  clear_error();
  hgd_status s = check_state(mt_state);
  if (s != HGD_OK) return s;
  HGD_REQUIRE(begin >= 0 && begin <= end, "hgd_sample_pairwise: bad record range");
  HGD_REQUIRE(n_items >= 1 && n_items < (int64_t{1} << 32), "hgd_sample_pairwise: n_items");
  HGD_REQUIRE(n_negs >= 0, "hgd_sample_pairwise: n_negs < 0");
  if (begin == end) return HGD_OK;
  HGD_REQUIRE(order && rec_user && rec_item && user_rowptr && out_u && out_i &&
                  (out_j || n_negs == 0),
              "hgd_sample_pairwise: null pointer");
  Mt g{mt_state, mt_state[kMtN]};
  for (int64_t k = begin; k < end; ++k) {
    const int64_t rec = order[k];
    const int32_t u = rec_user[rec];
    if (u < 0 || u >= n_users) {
      mt_state[kMtN] = g.index;
      return fail(HGD_ERR_INVALID_ARG, "hgd_sample_pairwise: user id %d out of range", u);
    }
    out_u[k - begin] = u;
    out_i[k - begin] = rec_item[rec];
    const int64_t lo = user_rowptr[u], hi = user_rowptr[u + 1];
    if (hi - lo >= n_items && n_negs > 0) {  // the reference would loop forever
      mt_state[kMtN] = g.index;
      return fail(HGD_ERR_INVALID_ARG,
                  "hgd_sample_pairwise: user %d has interacted with every item", u);
    }
    for (int32_t m = 0; m < n_negs; ++m) {
      int32_t neg = static_cast<int32_t>(g.below(static_cast<uint64_t>(n_items)));
      while (sorted_contains(user_items, lo, hi, neg))
        neg = static_cast<int32_t>(g.below(static_cast<uint64_t>(n_items)));
      out_j[(k - begin) * n_negs + m] = neg;
    }
  }
  mt_state[kMtN] = g.index;
  return HGD_OK;
}
