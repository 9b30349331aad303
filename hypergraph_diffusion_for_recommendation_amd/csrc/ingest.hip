// Ingest and graph build: the data path that produces the
// hot path's input matrices, re-built native instead of Python/scipy
// (paths relative to /root/reference/HD_SELFRec):
//
//  * hgd_ingest_read / _count / _copy / _free — FileIO.load_data_set (data/loader.py:24-38) as a
//    host parser: the file is mapped once, cut into n_threads chunks at line boundaries and parsed
//    in parallel (each chunk into its own arrays, concatenated in file order). Line semantics
//    follow the reference exactly: the first line is skipped (next(f)); a line containing a tab
//    is split on tabs, otherwise on commas, after stripping surrounding whitespace; fields 0 and 1
//    are parsed like Python int() (surrounding whitespace, optional sign, '_' between digits);
//    anything else in the line is ignored. Lines end at "\n", "\r\n" or "\r" (universal
//    newlines). Where the reference would raise (empty line, non-integer field, < 2 fields), the
//    call fails with the 1-based line number.
//  * hgd_remap_first_appearance — the user / item dictionaries of Interaction.__generate_set
//    (data/ui_graph.py:43-56): ids in order of first appearance, on the device by sorting
//    (key, position) pairs: a stable radix sort, segment heads give each key's first position,
//    a second sort of those positions ranks the keys. Bit-exact with the dict loop.
//  * hgd_coo_coalesce — scipy csr_matrix((ones, (row, col))) with duplicates summed, canonical
//    (data/ui_graph.py:70-84, :95-112): a 64-bit radix sort of row·n_cols + col, run-length
//    encode, counts as float32 values.
//  * hgd_normalize_values — Graph.normalize_graph_mat (data/graph.py:11-25) given the degree
//    scales of hgd_degree_scale: val·d_r, then ·d_c for the square case, in that float32 order.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <hipcub/hipcub.hpp>
#include <string>
#include <thread>
#include <vector>

#include "hgd_internal.h"

struct hgd_ingest {
  std::vector<int64_t> users;
  std::vector<int64_t> items;
};

namespace hgd {
namespace {

// ---------------------------------------------------------------- host parser
inline bool py_space(unsigned char c) {
  // str.strip() / int() whitespace for ASCII: \t \n \v \f \r, space, and \x1c-\x1f
  return c == ' ' || (c >= 0x09 && c <= 0x0d) || (c >= 0x1c && c <= 0x1f);
}

// Python int() of bytes [b, e): whitespace, sign, digits with single '_' between digits.
bool parse_int(const char* b, const char* e, int64_t& out) {
  while (b < e && py_space(static_cast<unsigned char>(*b))) ++b;
  while (e > b && py_space(static_cast<unsigned char>(e[-1]))) --e;
  if (b == e) return false;
  bool neg = false;
  if (*b == '+' || *b == '-') {
    neg = *b == '-';
    ++b;
  }
  if (b == e || *b < '0' || *b > '9') return false;
  unsigned long long v = 0;
  bool prev_digit = false;
  for (; b < e; ++b) {
    const char c = *b;
    if (c >= '0' && c <= '9') {
      const unsigned long long nv = v * 10ULL + static_cast<unsigned long long>(c - '0');
      if (nv / 10ULL != v) return false;  // overflow
      v = nv;
      prev_digit = true;
    } else if (c == '_' && prev_digit && b + 1 < e && b[1] >= '0' && b[1] <= '9') {
      prev_digit = false;
    } else {
      return false;
    }
  }
  if (!neg && v > 0x7fffffffffffffffULL) return false;
  if (neg && v > 0x8000000000000000ULL) return false;
  out = neg ? static_cast<int64_t>(0ULL - v) : static_cast<int64_t>(v);
  return true;
}

// Next line [b, e) starting at p; returns the position after its terminator.
inline const char* next_line(const char* p, const char* end, const char*& le) {
  const char* q = p;
  while (q < end && *q != '\n' && *q != '\r') ++q;
  le = q;
  if (q < end) {
    if (*q == '\r' && q + 1 < end && q[1] == '\n') return q + 2;
    return q + 1;
  }
  return q;
}

struct Chunk {
  const char* begin;
  const char* end;
  int64_t first_line;  // 1-based line number of the chunk's first line (filled after a count)
  std::vector<int64_t> users, items;
  int64_t bad_line = 0;  // first offending line (0 = none)
  std::string why;
};

void parse_chunk(Chunk& c) {
  const char* p = c.begin;
  int64_t line = c.first_line;
  while (p < c.end) {
    const char* le;
    const char* nx = next_line(p, c.end, le);
    // the reference tests for '\t' on the raw line (terminator included: a '\t' only appears in
    // [p, le) since the terminator is \n / \r)
    bool has_tab = false;
    for (const char* q = p; q < le; ++q)
      if (*q == '\t') {
        has_tab = true;
        break;
      }
    const char sep = has_tab ? '\t' : ',';
    // strip, then split on sep
    const char* b = p;
    const char* e = le;
    while (b < e && py_space(static_cast<unsigned char>(*b))) ++b;
    while (e > b && py_space(static_cast<unsigned char>(e[-1]))) --e;
    const char* f0e = b;
    while (f0e < e && *f0e != sep) ++f0e;
    int64_t u = 0, it = 0;
    if (f0e == e) {
      c.bad_line = line;
      c.why = (b == e) ? "empty line" : "fewer than 2 fields";
      return;
    }
    const char* f1b = f0e + 1;
    const char* f1e = f1b;
    while (f1e < e && *f1e != sep) ++f1e;
    if (!parse_int(b, f0e, u) || !parse_int(f1b, f1e, it)) {
      c.bad_line = line;
      c.why = "field is not an integer";
      return;
    }
    c.users.push_back(u);
    c.items.push_back(it);
    ++line;
    p = nx;
  }
}

// ---------------------------------------------------------------- device kernels
__global__ void k_iota64(int64_t* out, int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) out[i] = i;
}

__global__ void k_head_flags(const int64_t* __restrict__ sorted_keys, int64_t n,
                             int64_t* __restrict__ flags) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) flags[i] = (i == 0 || sorted_keys[i] != sorted_keys[i - 1]) ? 1 : 0;
}

// seg = inclusive_scan(flags) - 1; at heads: first_pos[seg] = sorted_pos[i], head_idx[seg] = i
__global__ void k_heads(const int64_t* __restrict__ flags_incl, const int64_t* __restrict__ sorted_pos,
                        int64_t n, int64_t* __restrict__ first_pos, int64_t* __restrict__ head_idx) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  const bool head = i == 0 || flags_incl[i] != flags_incl[i - 1];
  if (head) {
    const int64_t seg = flags_incl[i] - 1;
    first_pos[seg] = sorted_pos[i];
    head_idx[seg] = i;
  }
}

// unused segment slots (i >= n_seg) get first-position keys n + i, after every real one
__global__ void k_pad_segments(const int64_t* __restrict__ n_seg_p, int64_t n,
                               int64_t* __restrict__ first_pos, int64_t* __restrict__ seg_iota) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  seg_iota[i] = i;
  if (i >= *n_seg_p) first_pos[i] = n + i;
}

// order[r] = segment with the r-th smallest first position → new_id[order[r]] = r, uniq[r] = key
__global__ void k_rank(const int64_t* __restrict__ order, const int64_t* __restrict__ n_seg_p,
                       const int64_t* __restrict__ head_idx, const int64_t* __restrict__ sorted_keys,
                       int32_t* __restrict__ new_id, int64_t* __restrict__ uniq) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (r >= *n_seg_p) return;  // r < n_seg ⇒ order[r] is a real segment
  const int64_t seg = order[r];
  new_id[seg] = static_cast<int32_t>(r);
  uniq[r] = sorted_keys[head_idx[seg]];
}

__global__ void k_scatter_ids(const int64_t* __restrict__ flags_incl,
                              const int64_t* __restrict__ sorted_pos, int64_t n,
                              const int32_t* __restrict__ new_id, int32_t* __restrict__ ids) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) ids[sorted_pos[i]] = new_id[flags_incl[i] - 1];
}

__global__ void k_keys2(const int32_t* __restrict__ rows, const int32_t* __restrict__ cols,
                        int64_t n, int64_t n_cols, int64_t* __restrict__ keys) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) keys[i] = static_cast<int64_t>(rows[i]) * n_cols + cols[i];
}

__global__ void k_split_keys(const int64_t* __restrict__ uniq, const int32_t* __restrict__ counts,
                             const int64_t* __restrict__ n_runs, int64_t n_cols,
                             int32_t* __restrict__ rows, int32_t* __restrict__ cols,
                             float* __restrict__ vals) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= *n_runs) return;
  rows[i] = static_cast<int32_t>(uniq[i] / n_cols);
  cols[i] = static_cast<int32_t>(uniq[i] % n_cols);
  vals[i] = static_cast<float>(counts[i]);
}

// rowptr[r] = first run with row >= r, searching only the *nnz valid runs
__global__ void k_rowptr_runs(const int32_t* __restrict__ rr, const int64_t* __restrict__ nnz,
                              int64_t n_rows, int64_t* __restrict__ rowptr) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (r > n_rows) return;
  int64_t lo = 0, hi = *nnz;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (rr[mid] < r)
      lo = mid + 1;
    else
      hi = mid;
  }
  rowptr[r] = lo;
}

__global__ void k_normalize_values(const int64_t* __restrict__ rowptr,
                                   const int32_t* __restrict__ col, const float* __restrict__ val,
                                   int64_t n_rows, const float* __restrict__ row_scale,
                                   const float* __restrict__ col_scale, float* __restrict__ out) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (r >= n_rows) return;
  const float dr = row_scale[r];
  for (int64_t e = rowptr[r]; e < rowptr[r + 1]; ++e) {
    float v = dr * val[e];                    // d_mat_inv.dot(adj_mat)
    if (col_scale) v = v * col_scale[col[e]];  // .dot(d_mat_inv)
    out[e] = v;
  }
}

int bits_for(int64_t n) {
  int b = 1;
  while (b < 63 && (1LL << b) < n) ++b;
  return b;
}

template <typename K, typename V>
size_t sort_pairs_bytes(int64_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, static_cast<const K*>(nullptr),
                                     static_cast<K*>(nullptr), static_cast<const V*>(nullptr),
                                     static_cast<V*>(nullptr), static_cast<int>(n));
  return bytes;
}

size_t scan_bytes(int64_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceScan::InclusiveSum(nullptr, bytes, static_cast<const int64_t*>(nullptr),
                                   static_cast<int64_t*>(nullptr), static_cast<int>(n));
  return bytes;
}

size_t rle_bytes(int64_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceRunLengthEncode::Encode(nullptr, bytes, static_cast<const int64_t*>(nullptr),
                                        static_cast<int64_t*>(nullptr),
                                        static_cast<int32_t*>(nullptr),
                                        static_cast<int64_t*>(nullptr), static_cast<int>(n));
  return bytes;
}

}  // namespace
}  // namespace hgd

// ------------------------------------------------------------------------ host ABI
extern "C" hgd_status hgd_ingest_read(const char* path, int32_t skip_header, int32_t n_threads,
                                      hgd_ingest** out) {
  using namespace hgd;
  clear_error();
  HGD_REQUIRE(path && out, "hgd_ingest_read: null path/out");
  *out = nullptr;
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return fail(HGD_ERR_INVALID_ARG, "hgd_ingest_read: cannot open %s", path);
  struct stat sb;
  if (fstat(fd, &sb) != 0) {
    close(fd);
    return fail(HGD_ERR_INVALID_ARG, "hgd_ingest_read: cannot stat %s", path);
  }
  const size_t size = static_cast<size_t>(sb.st_size);
  const char* data = nullptr;
  void* map = nullptr;
  if (size > 0) {
    map = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
    if (map == MAP_FAILED) {
      close(fd);
      return fail(HGD_ERR_INVALID_ARG, "hgd_ingest_read: mmap of %s failed", path);
    }
    data = static_cast<const char*>(map);
  }
  close(fd);
  const char* end = data + size;
  const char* p = data;
  int64_t line0 = 1;
  if (skip_header) {
    if (size == 0) {
      return fail(HGD_ERR_INVALID_ARG, "hgd_ingest_read: %s is empty (no header line)", path);
    }
    const char* le;
    p = next_line(p, end, le);
    line0 = 2;
  }
  int T = n_threads > 0 ? n_threads : static_cast<int>(std::thread::hardware_concurrency());
  if (T < 1) T = 1;
  if (T > 64) T = 64;
  const size_t body = static_cast<size_t>(end - p);
  if (body < (1u << 20)) T = 1;  // small files: one chunk
  std::vector<Chunk> chunks(T);
  const char* cb = p;
  for (int t = 0; t < T; ++t) {
    const char* ce = (t == T - 1) ? end : p + body / T * (t + 1);
    if (ce < cb) ce = cb;
    // move the cut to just after a line terminator
    while (ce < end && ce > cb && ce[-1] != '\n' && ce[-1] != '\r') ++ce;
    if (ce < end && ce > cb && ce[-1] == '\r' && *ce == '\n') ++ce;
    chunks[t].begin = cb;
    chunks[t].end = ce;
    cb = ce;
  }
  // line numbers: count the lines of every chunk (cheap, parallel), then prefix
  std::vector<int64_t> nlines(T, 0);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        const char* q = chunks[t].begin;
        int64_t k = 0;
        while (q < chunks[t].end) {
          const char* le;
          q = next_line(q, chunks[t].end, le);
          ++k;
        }
        nlines[t] = k;
      });
    for (auto& x : th) x.join();
  }
  int64_t acc = line0;
  for (int t = 0; t < T; ++t) {
    chunks[t].first_line = acc;
    acc += nlines[t];
    chunks[t].users.reserve(static_cast<size_t>(nlines[t]));
    chunks[t].items.reserve(static_cast<size_t>(nlines[t]));
  }
  {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back([&, t] { parse_chunk(chunks[t]); });
    for (auto& x : th) x.join();
  }
  if (map) munmap(map, size);
  for (int t = 0; t < T; ++t)
    if (chunks[t].bad_line)
      return fail(HGD_ERR_INVALID_ARG, "hgd_ingest_read: %s line %lld: %s", path,
                  static_cast<long long>(chunks[t].bad_line), chunks[t].why.c_str());
  hgd_ingest* h = new hgd_ingest;
  const size_t total = static_cast<size_t>(acc - line0);
  h->users.reserve(total);
  h->items.reserve(total);
  for (int t = 0; t < T; ++t) {
    h->users.insert(h->users.end(), chunks[t].users.begin(), chunks[t].users.end());
    h->items.insert(h->items.end(), chunks[t].items.begin(), chunks[t].items.end());
  }
  *out = h;
  return HGD_OK;
}

extern "C" int64_t hgd_ingest_count(const hgd_ingest* h) {
  return h ? static_cast<int64_t>(h->users.size()) : -1;
}

extern "C" hgd_status hgd_ingest_copy(const hgd_ingest* h, int64_t* user_raw, int64_t* item_raw) {
  hgd::clear_error();
  HGD_REQUIRE(h, "hgd_ingest_copy: null handle");
  const size_t n = h->users.size();
  if (n == 0) return HGD_OK;
  HGD_REQUIRE(user_raw && item_raw, "hgd_ingest_copy: null output");
  std::copy(h->users.begin(), h->users.end(), user_raw);
  std::copy(h->items.begin(), h->items.end(), item_raw);
  return HGD_OK;
}

extern "C" void hgd_ingest_free(hgd_ingest* h) { delete h; }

// ------------------------------------------------------------------------ device ABI
extern "C" size_t hgd_remap_workspace_size(int64_t n) {
  using namespace hgd;
  if (n <= 0) return 0;
  const size_t arr = align_up(static_cast<size_t>(n) * 8);
  // pos, sorted_keys, sorted_pos, flags, first_pos, head_idx, order_key, order (8 int64 arrays)
  // + new_id int32 + max(sort temp, scan temp)
  size_t tmp = sort_pairs_bytes<int64_t, int64_t>(n);
  const size_t sb = scan_bytes(n);
  if (sb > tmp) tmp = sb;
  return 8 * arr + align_up(static_cast<size_t>(n) * 4) + align_up(tmp);
}

extern "C" hgd_status hgd_remap_first_appearance(const int64_t* keys, int64_t n, int32_t* ids,
                                                 int64_t* uniq, int64_t* n_unique,
                                                 void* workspace, size_t workspace_bytes,
                                                 void* stream) {
  using namespace hgd;
  clear_error();
  HGD_REQUIRE(n >= 0 && n < 0x7fffffffLL, "hgd_remap_first_appearance: n out of range");
  HGD_REQUIRE(n_unique, "hgd_remap_first_appearance: null n_unique");
  hipStream_t st = as_stream(stream);
  if (n == 0) {
    HGD_HIP(hipMemsetAsync(n_unique, 0, sizeof(int64_t), st));
    return HGD_OK;
  }
  HGD_REQUIRE(keys && ids && uniq, "hgd_remap_first_appearance: null pointer");
  const size_t need = hgd_remap_workspace_size(n);
  if (workspace_bytes < need || !workspace)
    return fail(HGD_ERR_WORKSPACE, "hgd_remap_first_appearance: workspace %zu < %zu",
                workspace_bytes, need);
  char* ws = static_cast<char*>(workspace);
  const size_t arr = align_up(static_cast<size_t>(n) * 8);
  int64_t* pos = reinterpret_cast<int64_t*>(ws);
  int64_t* skeys = reinterpret_cast<int64_t*>(ws + arr);
  int64_t* spos = reinterpret_cast<int64_t*>(ws + 2 * arr);
  int64_t* flags = reinterpret_cast<int64_t*>(ws + 3 * arr);
  int64_t* first_pos = reinterpret_cast<int64_t*>(ws + 4 * arr);
  int64_t* head_idx = reinterpret_cast<int64_t*>(ws + 5 * arr);
  int64_t* order_key = reinterpret_cast<int64_t*>(ws + 6 * arr);
  int64_t* order = reinterpret_cast<int64_t*>(ws + 7 * arr);
  int32_t* new_id = reinterpret_cast<int32_t*>(ws + 8 * arr);
  char* tmp = ws + 8 * arr + align_up(static_cast<size_t>(n) * 4);
  size_t tb = workspace_bytes - (8 * arr + align_up(static_cast<size_t>(n) * 4));
  const dim3 g(grid_for(n));
  const int N = static_cast<int>(n);
  hipLaunchKernelGGL(k_iota64, g, dim3(kBlock), 0, st, pos, n);
  // 1. stable sort of (key, position): equal keys keep ascending positions
  HGD_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tb, keys, skeys, pos, spos, N, 0, 64, st));
  // 2. segments of equal keys; first position and head index per segment
  hipLaunchKernelGGL(k_head_flags, g, dim3(kBlock), 0, st, skeys, n, flags);
  size_t sb = workspace_bytes - (8 * arr + align_up(static_cast<size_t>(n) * 4));
  HGD_HIP(hipcub::DeviceScan::InclusiveSum(tmp, sb, flags, flags, N, st));
  hipLaunchKernelGGL(k_heads, g, dim3(kBlock), 0, st, flags, spos, n, first_pos, head_idx);
  HGD_HIP(hipMemcpyAsync(n_unique, flags + (n - 1), sizeof(int64_t), hipMemcpyDeviceToDevice, st));
  // 3. rank segments by first position (segments past the count hold stale values; they are
  //    given keys above every position so they sort last)
  //    — the segment count is only known on the device: all n slots are sorted, the unused
  //    ones keyed n + i (k_pad_segments) so that they come after every real first position
  hgd_status s = check_launch("hgd_remap_first_appearance heads");
  if (s != HGD_OK) return s;
  hipLaunchKernelGGL(k_pad_segments, g, dim3(kBlock), 0, st, flags + (n - 1), n, first_pos, pos);
  tb = workspace_bytes - (8 * arr + align_up(static_cast<size_t>(n) * 4));
  HGD_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tb, first_pos, order_key, pos, order, N, 0,
                                             bits_for(2 * n), st));
  // 4. new ids and unique keys in id order, then ids in file order
  hipLaunchKernelGGL(k_rank, g, dim3(kBlock), 0, st, order, flags + (n - 1), head_idx, skeys,
                     new_id, uniq);
  s = check_launch("hgd_remap_first_appearance rank");
  if (s != HGD_OK) return s;
  hipLaunchKernelGGL(k_scatter_ids, g, dim3(kBlock), 0, st, flags, spos, n, new_id, ids);
  return check_launch("hgd_remap_first_appearance scatter");
}

extern "C" size_t hgd_coo_coalesce_workspace_size(int64_t n) {
  using namespace hgd;
  if (n <= 0) return 0;
  const size_t arr = align_up(static_cast<size_t>(n) * 8);
  size_t tmp = 0;
  {
    size_t b = 0;
    (void)hipcub::DeviceRadixSort::SortKeys(nullptr, b, static_cast<const int64_t*>(nullptr),
                                      static_cast<int64_t*>(nullptr), static_cast<int>(n));
    tmp = b;
  }
  const size_t rb = rle_bytes(n);
  if (rb > tmp) tmp = rb;
  // keys, sorted keys, unique keys (int64) + counts (int32) + run count + temp
  return 3 * arr + align_up(static_cast<size_t>(n) * 4) + align_up(8) + align_up(tmp);
}

extern "C" hgd_status hgd_coo_coalesce(const int32_t* rows, const int32_t* cols, int64_t n,
                                       int64_t n_rows, int64_t n_cols, int64_t* rowptr,
                                       int32_t* col_out, float* val_out, int64_t* nnz_out,
                                       void* workspace, size_t workspace_bytes, void* stream) {
  using namespace hgd;
  clear_error();
  HGD_REQUIRE(n >= 0 && n < 0x7fffffffLL, "hgd_coo_coalesce: n out of range");
  HGD_REQUIRE(n_rows > 0 && n_cols > 0 && n_rows < 0x7fffffffLL && n_cols < 0x7fffffffLL,
              "hgd_coo_coalesce: bad shape");
  HGD_REQUIRE(rowptr && nnz_out, "hgd_coo_coalesce: null rowptr/nnz_out");
  hipStream_t st = as_stream(stream);
  if (n == 0) {
    HGD_HIP(hipMemsetAsync(rowptr, 0, static_cast<size_t>(n_rows + 1) * 8, st));
    HGD_HIP(hipMemsetAsync(nnz_out, 0, 8, st));
    return HGD_OK;
  }
  HGD_REQUIRE(rows && cols && col_out && val_out, "hgd_coo_coalesce: null pointer");
  const size_t need = hgd_coo_coalesce_workspace_size(n);
  if (workspace_bytes < need || !workspace)
    return fail(HGD_ERR_WORKSPACE, "hgd_coo_coalesce: workspace %zu < %zu", workspace_bytes, need);
  char* ws = static_cast<char*>(workspace);
  const size_t arr = align_up(static_cast<size_t>(n) * 8);
  int64_t* keys = reinterpret_cast<int64_t*>(ws);
  int64_t* skeys = reinterpret_cast<int64_t*>(ws + arr);
  int64_t* ukeys = reinterpret_cast<int64_t*>(ws + 2 * arr);
  int32_t* counts = reinterpret_cast<int32_t*>(ws + 3 * arr);
  char* tmp = ws + 3 * arr + align_up(static_cast<size_t>(n) * 4) + align_up(8);
  size_t tb = workspace_bytes - (3 * arr + align_up(static_cast<size_t>(n) * 4) + align_up(8));
  const dim3 g(grid_for(n));
  const int N = static_cast<int>(n);
  hipLaunchKernelGGL(k_keys2, g, dim3(kBlock), 0, st, rows, cols, n, n_cols, keys);
  HGD_HIP(hipcub::DeviceRadixSort::SortKeys(tmp, tb, keys, skeys, N, 0, bits_for(n_rows * n_cols),
                                            st));
  tb = workspace_bytes - (3 * arr + align_up(static_cast<size_t>(n) * 4) + align_up(8));
  HGD_HIP(hipcub::DeviceRunLengthEncode::Encode(tmp, tb, skeys, ukeys, counts, nnz_out, N, st));
  // rows of the runs go to the (caller's) col_out scratch first: rowptr needs them sorted
  int32_t* run_rows = reinterpret_cast<int32_t*>(keys);  // keys no longer needed
  hipLaunchKernelGGL(k_split_keys, g, dim3(kBlock), 0, st, ukeys, counts, nnz_out, n_cols,
                     run_rows, col_out, val_out);
  hgd_status s = check_launch("hgd_coo_coalesce split");
  if (s != HGD_OK) return s;
  // rowptr: binary search over the run rows; runs past *nnz_out hold stale data, so the search
  // range must be the true count — done on the device by the rowptr kernel below
  hipLaunchKernelGGL(k_rowptr_runs, dim3(grid_for(n_rows + 1)), dim3(kBlock), 0, st, run_rows,
                     nnz_out, n_rows, rowptr);
  return check_launch("hgd_coo_coalesce rowptr");
}

extern "C" hgd_status hgd_normalize_values(const int64_t* rowptr, const int32_t* col,
                                           const float* val, int64_t n_rows,
                                           const float* row_scale, const float* col_scale,
                                           float* out, void* stream) {
  using namespace hgd;
  clear_error();
  HGD_REQUIRE(n_rows >= 0, "hgd_normalize_values: n_rows < 0");
  if (n_rows == 0) return HGD_OK;
  HGD_REQUIRE(rowptr && val && row_scale && out && (!col_scale || col),
              "hgd_normalize_values: null pointer");
  hipLaunchKernelGGL(k_normalize_values, dim3(grid_for(n_rows)), dim3(kBlock), 0,
                     as_stream(stream), rowptr, col, val, n_rows, row_scale, col_scale, out);
  return check_launch("hgd_normalize_values");
}
