/*
 * hgd.h — C ABI of libhgd, the MI355X (gfx950) hypergraph-propagation library.
 *
 * This is the drop-in boundary for the hot path named by BASELINE.json `north_star`:
 * the incidence SpMM hops (Hᵀ·X then H·M, with degree normalisation) that sit under
 * SELFRec's model/graph plugins, plus the per-step structure work feeding them.
 * Every entry point replaces one implicit device-op call site of the reference
 * (paths relative to /root/reference/HD_SELFRec):
 *
 *   hgd_spmm                 torch.sparse.mm(adj, X)            model/graph/HCCF.py:199,
 *                            torch.sparse.mm(adj.t(), X)        model/graph/HGNN_HD4.py:459-462,
 *                                                               model/graph/HGCN.py:173-175,
 *                            torch_scatter.scatter(.., 'mean')  model/layers/layers2/EquivSetConv2.py:88-93
 *                            (row_scale = 1/count is the scatter-mean; val = per-nonzero weight)
 *   hgd_spmm_blocked         the same torch.sparse.mm(adj.t(), X) hop for a gathered table larger
 *                            than the Infinity Cache (source-blocked; hgd_spmm_col_blocks builds
 *                            its block-major copy of the CSC)
 *   hgd_sort_perm            COO→CSR / CSR→CSC ordering that cuSPARSE re-derives per call
 *                            (`adj.t()` in HGCNConv.forward, HGNN_HD4.py:459; coalesce in torch.sparse.mm)
 *   hgd_rowptr_from_sorted   row pointer of a row-sorted COO  base/torch_interface.py:8-12
 *   hgd_degree_scale         D^-1/2 and D^-1 of data/graph.py:11-25 (inf→0) and data/graph.py:28-42
 *   hgd_edge_values          per-nonzero weights with a source-side diagonal folded in
 *   hgd_dropedge_compact     SpAdjDropEdge.forward, model/graph/HCCF.py:213-226 (vals[mask]/keep, idxs[:,mask])
 *   hgd_dense_threshold_*    torch.nonzero(hypergraph > 0), model/layers/layers2/EquivSetGNN2.py:105-133
 *                            (row-major order identical to torch.nonzero)
 *
 * Conventions:
 *   - All pointers are DEVICE pointers unless a parameter says "host".
 *   - The caller owns every buffer; the library never allocates or frees caller memory.
 *     Scratch comes from a caller-provided workspace sized by the matching *_workspace_size.
 *   - Every call is stream-ordered on `stream` (a hipStream_t passed as void*; NULL = legacy
 *     default stream) and performs no host synchronisation, so it can be graph-captured.
 *   - Errors come back as hgd_status; hgd_get_last_error_string() describes the last failure
 *     on the calling thread. No C++ exception crosses the ABI.
 *   - Indices: row pointers are int64, column/row indices are int32 (rows, cols < 2^31).
 *   - Floating point is fp32 in and out; sums run in fp32 in edge order (deterministic).
 */
#ifndef HGD_H
#define HGD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum hgd_status {
  HGD_OK = 0,
  HGD_ERR_INVALID_ARG = 1,
  HGD_ERR_HIP = 2,
  HGD_ERR_UNSUPPORTED = 3,
  HGD_ERR_WORKSPACE = 4
} hgd_status;

typedef enum hgd_epilogue {
  HGD_EPI_NONE = 0,
  HGD_EPI_LEAKY_RELU = 1, /* nn.LeakyReLU(negative_slope=slope): HGCNConv act=True */
  HGD_EPI_RELU = 2
} hgd_epilogue;

/* Tuning knobs of the SpMM hop (process-wide; defaults are the measured best on MI355X).
 *   HGD_TUNE_SPMM_UNROLL: independent row gathers in flight per lane (8 or 16)
 *   HGD_TUNE_SPMM_POLICY: 0 plain, 1 non-temporal Y stores, 8 software-pipelined index
 *                         batches (default), 9 both, 10 prefetch + non-temporal index/weight
 *                         loads, 11 all three (d = 64 float4 path only)
 *   HGD_TUNE_SPMM_PASS_COLS: widest column pass of a hop without a fused row epilogue
 *                         (64, 128 or 256 fp32 columns; wider rows run as several passes;
 *                         0 = auto, the default: one pass up to 128 columns, else 64)
 *   HGD_TUNE_ROWGEMM_BLOCKS: most workgroups of a row-GEMM launch (hgd_gemm_rows, hgd_linear_*;
 *                         0 = default 512, else 64..8192; each wave takes 16-row tiles at a
 *                         stride of 4·blocks)
 *   HGD_TUNE_SPLITK_ROWS: rows per slice of the split-K products (hgd_gemm_tn,
 *                         hgd_linear_backward_weight; 0 = default sizing, else a multiple of 64
 *                         in [64, 65536]; the workspace size follows it)
 *   HGD_TUNE_GEMM_EXACT:  0 (default) = the dense products with K (row GEMM) or the row count's
 *                         reduction (split-K) eligible run as split-bf16 MFMAs (every f32
 *                         operand cut exactly into three bf16 terms, six products: error
 *                         ≈ 1e-7·Σ|a·b| like the f32 fmaf chain, not bitwise equal to it);
 *                         1 = the exact f32-input MFMA kernels only (bitwise k-ordered fmaf)
 *   HGD_TUNE_X3_COLS:     output columns per workgroup of the split-bf16 row GEMM (64 or 128;
 *                         0 = default)
 *   HGD_TUNE_X3_SPLITK:   weight-gradient (split-K) kernel when HGD_TUNE_GEMM_EXACT is 0:
 *                         2 (default) = by shape: the producer-wave split-bf16 kernel for
 *                         64 × 64 and 128 × 128 outputs (16-byte aligned rows, ≥ 4,096 rows),
 *                         the one-wave-per-tile split-bf16 kernel for other outputs ≤ 64 × 64
 *                         over ≥ 49,152 rows, else the f32-MFMA kernel; 1 = always the
 *                         one-wave-per-tile split-bf16 kernel; 0 = always f32 MFMA
 *   HGD_TUNE_X3S_TILES:   form of the staged split-bf16 row GEMM at N > 32: 1 or 2 16-column
 *                         tiles per wave (1: half the W registers, two workgroups per CU), 3 =
 *                         two tiles + 4 producer waves that load and split the rows while the
 *                         others multiply; 0 = default (1 for masked products, else 3)
 *   HGD_TUNE_P2P_SEGMENT_MB: largest allocation hgd_p2p_create exposes to its peers, in MiB
 *                         (0 = default 1024; slots are packed whole into segments of at most
 *                         this size, each imported separately: a single 3.5 GiB import never
 *                         returned on the ROCm 7.2 box); applies to later hgd_p2p_create calls
 *   HGD_TUNE_P2P_CACHED:  0 (default) = uncached segments (hipDeviceMallocUncached); 1 = plain
 *                         device memory (the exchange's fences keep it correct either way; the
 *                         knob prices what uncached hop-1 stores cost)
 *   HGD_TUNE_CPU_RNG_THREADS: host threads of hgd_torch_cpu_keep_mask's split draw (0 = default
 *                         min(16, hardware threads, OMP_NUM_THREADS); 1 = one thread)
 *   HGD_TUNE_X3P_QUEUE:   form of the producer-wave weight gradient: 0 (default) = one workgroup
 *                         barrier per 32-row stage, 1 = three LDS buffers with full / empty
 *                         counters (measured slower: 45.1 vs 41.5 µs at 144,242 x 128); a
 *                         counter wait that runs out (≈ 0.1 s) writes the workgroup's partial
 *                         sums as NaN instead of reading an unfilled buffer
 *   HGD_TUNE_P2P_GRID:    workgroups of the peer exchange's reduce / gather kernels (0 = default
 *                         256: the links bound them, the hops they overlap need the CUs)
 *   HGD_TUNE_MASK_PAIR:   the masked hop (hgd_spmm_masked*) walks two index batches per step,
 *                         their kept entries packed by forward permutes (2, default) or by
 *                         set-bit searches and pulls (1), or one batch per step (0); the sums
 *                         are the same bits every way
 *   HGD_TUNE_MASK_DIV:    the masked hop's kept weights val / keep: 0 (default) = one multiply by
 *                         1 / keep when keep is a power of two (the same bits: one real value,
 *                         rounded once), else the IEEE division; 1 = always the division
 *   HGD_TUNE_SPMM_PASS_INTERLEAVE: rows wider than one column pass (d > 128 by default, unfused,
 *                         no split rows): 0 = one launch per pass; 1 = all passes in one launch,
 *                         a row block's passes on consecutive workgroups of one XCD (the same
 *                         bits either way)
 *   HGD_TUNE_SPMM_BLOCKED_SEG: hgd_spmm_blocked walks each source block's (short) rows with
 *                         0 = a lane group per row (default), 1 = the segmented kernel (a group
 *                         owns G consecutive rows as one nonzero stream; the same bits) */
typedef enum hgd_tune_key {
  HGD_TUNE_SPMM_UNROLL = 1,
  HGD_TUNE_SPMM_POLICY = 2,
  HGD_TUNE_SPMM_PASS_COLS = 3,
  HGD_TUNE_ROWGEMM_BLOCKS = 4,
  HGD_TUNE_SPLITK_ROWS = 5,
  HGD_TUNE_GEMM_EXACT = 6,
  HGD_TUNE_X3_COLS = 7,
  HGD_TUNE_X3_SPLITK = 8,
  HGD_TUNE_X3S_TILES = 9,
  HGD_TUNE_P2P_SEGMENT_MB = 10,
  HGD_TUNE_P2P_CACHED = 11,
  HGD_TUNE_CPU_RNG_THREADS = 12,
  HGD_TUNE_X3P_QUEUE = 13,
  HGD_TUNE_P2P_GRID = 14,
  HGD_TUNE_MASK_PAIR = 15,
  HGD_TUNE_MASK_DIV = 16,
  HGD_TUNE_SPMM_PASS_INTERLEAVE = 17,
  HGD_TUNE_SPMM_BLOCKED_SEG = 18
} hgd_tune_key;
hgd_status hgd_set_tuning(int32_t key, int32_t value);

/* Library ABI version (major*10000 + minor*100 + patch). */
int hgd_version(void);
/* Human-readable description of the last error on this thread ("" if none). */
const char* hgd_get_last_error_string(void);

/* ------------------------------------------------------------------------------------------
 * Split plan for long rows. Rows whose degree exceeds `threshold` are cut into chunks of
 * `chunk` nonzeros, summed by separate wavefront groups into a workspace, then combined in
 * chunk order (deterministic, no atomics). All arrays are device arrays built by
 * hgd_split_plan_build; a NULL plan or n_heavy == 0 means no row is split.
 * ---------------------------------------------------------------------------------------- */
typedef struct hgd_split_plan {
  int64_t threshold;           /* rows with degree > threshold are split (<=0: none)   */
  int32_t chunk;               /* nonzeros per chunk                                    */
  int32_t flags;               /* HGD_PLAN_SEGMENTED: short rows, use the segmented kernel */
  int64_t n_heavy;             /* number of split rows                                  */
  int64_t n_chunks;            /* total chunks over all split rows                      */
  const int32_t* heavy_rows;   /* [n_heavy]   split row ids, ascending                  */
  const int64_t* heavy_cptr;   /* [n_heavy+1] chunk range of each split row             */
  const int32_t* chunk_heavy;  /* [n_chunks]  split-row index owning each chunk         */
} hgd_split_plan;

/* plan.flags bit: the structure has short rows (average degree ≲ 32) and no split rows —
 * hgd_spmm then walks groups of consecutive rows as one nonzero stream (segmented kernel). */
#define HGD_PLAN_SEGMENTED 1

/* Counts (n_heavy, n_chunks) for a plan into device int64[2] `counts`. */
hgd_status hgd_split_plan_count(const int64_t* rowptr, int64_t n_rows, int64_t threshold,
                                int32_t chunk, int64_t* counts, void* stream);
size_t hgd_split_plan_workspace_size(int64_t n_rows);
/* Fills plan->heavy_rows / heavy_cptr / chunk_heavy (caller-allocated, sized from counts). */
hgd_status hgd_split_plan_build(const int64_t* rowptr, int64_t n_rows, int64_t threshold,
                                int32_t chunk, int32_t* heavy_rows, int64_t* heavy_cptr,
                                int32_t* chunk_heavy, int64_t n_heavy, int64_t n_chunks,
                                void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * One SpMM hop over a CSR structure (the CSC of H is the CSR of Hᵀ):
 *   for r in [row_begin, row_end):
 *     Y[r, 0:d] = epi( row_scale[r] * Σ_{e=rowptr[r]}^{rowptr[r+1]-1} val[e] * X[col[e], 0:d] )
 * val == NULL means all ones; row_scale == NULL means 1. X rows are n_src_rows × ldx floats.
 * Rows outside [row_begin,row_end) are not written. Workspace: hgd_spmm_workspace_size.
 * ---------------------------------------------------------------------------------------- */
size_t hgd_spmm_workspace_size(const hgd_split_plan* plan, int32_t d);
hgd_status hgd_spmm(const int64_t* rowptr, const int32_t* col, const float* val,
                    const float* row_scale, int64_t n_rows, int64_t n_src_rows,
                    int64_t row_begin, int64_t row_end, const float* X, int64_t ldx, float* Y,
                    int64_t ldy, int32_t d, int32_t epilogue, float slope,
                    const hgd_split_plan* plan, void* workspace, size_t workspace_bytes,
                    void* stream);

/* ------------------------------------------------------------------------------------------
 * The same hop (rows [row_begin,row_end), no split plan) run in n_blocks passes over SOURCE-ROW
 * ranges [⌊n_src_rows·k/n_blocks⌋, ⌊n_src_rows·(k+1)/n_blocks⌋): pass k sums only a row's
 * nonzeros whose column lies in block k and adds that partial to Y (pass 0 writes it; the
 * activation runs after the last). Replaces the same call sites as hgd_spmm
 * (torch.sparse.mm(adj.t(), X), model/graph/HGNN_HD4.py:459-462) when the gathered table is too
 * large for the 256 MB Infinity Cache: each pass gathers from a 1/n_blocks slice of X, for
 * (n_blocks−1) extra read+write passes over Y. The sum is a different fp32 association of the same
 * terms (blockwise partials, each scaled by row_scale), so it is not bitwise hgd_spmm's.
 *
 * hgd_spmm_col_blocks builds the BLOCK-MAJOR copy of a structure whose rows' columns ascend (the
 * CSC of an incidence): all rows' block-0 nonzeros, then all rows' block-1 nonzeros, …
 *   blk_start: int64 [n_blocks·n_rows + 1], row r's block-k nonzeros are
 *              [blk_start[k·n_rows + r], blk_start[k·n_rows + r + 1]) of
 *   blk_col:   int32 [nnz], their columns, and
 *   blk_perm:  int32 [nnz] (may be NULL), their positions in the source structure — gather any
 *              per-nonzero weights through it (hgd_gather32) to get hgd_spmm_blocked's blk_val
 *              (int32 positions: nnz < 2^31, the library's limit for permutations, as perm_t).
 * Workspace: hgd_spmm_col_blocks_workspace_size.
 * ---------------------------------------------------------------------------------------- */
/* The size rule both hosts use (measured on MI355X): the number of source
 * blocks for a hop gathering n_src_rows rows at width d (a pass of at most 128 columns):
 * 0 (one pass) under 512 MiB, 2 under 1 GiB, else about one per 640 MiB, 4..16. */
int32_t hgd_spmm_blocks_for(int64_t n_src_rows, int32_t d);
size_t hgd_spmm_col_blocks_workspace_size(int64_t n_rows, int32_t n_blocks);
hgd_status hgd_spmm_col_blocks(const int64_t* rowptr, const int32_t* col, int64_t n_rows,
                               int64_t n_cols, int32_t n_blocks, int64_t* blk_start,
                               int32_t* blk_col, int32_t* blk_perm, void* workspace,
                               size_t workspace_bytes, void* stream);
hgd_status hgd_spmm_blocked(const int64_t* blk_start, const int32_t* blk_col,
                            const float* blk_val, const float* row_scale, int64_t n_rows,
                            int64_t n_src_rows, int64_t row_begin, int64_t row_end,
                            const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t d,
                            int32_t epilogue, float slope, int32_t n_blocks, void* stream);

/* The same hop over the EDGE-DROPPED matrix of SpAdjDropEdge (model/graph/HCCF.py:213-226:
 * mask = floor(rand + keepRate), idxs[:, mask], vals[mask] / keepRate) without building it: the
 * structure is the parent's, `mask` (uint8, this orientation's edge order; for the CSC of the
 * parent that is mask_csr[perm_t]) selects the kept edges, each weighted by val[e] / keep (IEEE
 * fp32 division, as the dropped COO's values; val == NULL keeps all-ones weights, like
 * hgd_dropedge_structure). Kept edges are summed in edge order, so a row's sum equals the hop
 * over the compacted matrix of hgd_dropedge_structure whenever the split plan covers the same
 * rows (no split rows: bit-identical). Replaces the per-step compaction (count, scan, compact,
 * row pointers for the CSR and the CSC) of a training step's drop-edge. */
hgd_status hgd_spmm_masked(const int64_t* rowptr, const int32_t* col, const float* val,
                           const uint8_t* mask, float keep, const float* row_scale,
                           int64_t n_rows, int64_t n_src_rows, int64_t row_begin,
                           int64_t row_end, const float* X, int64_t ldx, float* Y, int64_t ldy,
                           int32_t d, int32_t epilogue, float slope, const hgd_split_plan* plan,
                           void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * Fused row epilogue of an ED-HNN / HGCN layer. Replaces the torch ops
 * the reference runs on the hop output, each an extra [N,d] HBM round trip and launch:
 *   LayerNorm + residual     Xe = LN0(HGCNConv(adj, Xve)) + Xve   model/layers/EquivSetConv.py:86-107,
 *                                                                 model/graph/HGNN_HD3.py:705-720
 *   restart blend            X = (1-α)·Xv + α·X0                   model/layers/layers2/EquivSetConv2.py:96
 * For every row r written by the hop (z = row_scale[r]·Σ of hgd_spmm):
 *   a = act(z)                         (act_out[r] = a when act_out != NULL)
 *   b = layer_norm ? (a - μ_r)·rstd_r·γ + β : a      (biased variance, rstd = 1/sqrt(var+eps);
 *                                                      stats[2r] = μ_r, stats[2r+1] = rstd_r)
 *   Y[r] = out_scale·b + res1_scale·res1[r] + res2_scale·res2[r]    (NULL residuals skipped)
 *   sum_out[r] = Y[r] + sum_res[r]                                    (when sum_out != NULL)
 * layer_norm needs the whole row in one lane group: d <= 256 with 16-byte aligned rows (X, Y,
 * residuals, act_out, leading dims % 4 == 0), or d <= 64 otherwise (HGD_ERR_UNSUPPORTED beyond).
 * act must be NONE or have slope >= 0, so that act'(z) can be read from the sign of a.
 * ---------------------------------------------------------------------------------------- */
typedef struct hgd_row_epilogue {
  int32_t act;            /* hgd_epilogue */
  float slope;
  int32_t layer_norm;     /* 0 / 1 */
  float ln_eps;
  const float* ln_gamma;  /* [d] or NULL (= 1) */
  const float* ln_beta;   /* [d] or NULL (= 0) */
  float out_scale;
  const float* res1;      /* [n_rows, ld_res1] or NULL */
  int64_t ld_res1;
  float res1_scale;
  const float* res2;
  int64_t ld_res2;
  float res2_scale;
  float* act_out;         /* [n_rows, ld_act] or NULL */
  int64_t ld_act;
  float* stats;           /* [n_rows, 2] or NULL */
  /* optional second output after the residuals: sum_out[r] = Y[r] + sum_res[r] (HCCF's
   * backward: the layer gradient dh and dh + the InfoNCE gradient of the layer below in one
   * store); both NULL or both set. res1 / res2 may alias Y (each row is read before it is
   * written, by the same lanes). */
  const float* sum_res;
  int64_t ld_sum_res;
  float* sum_out;
  int64_t ld_sum_out;
} hgd_row_epilogue;

/* hgd_spmm with the fused row epilogue `epi` (which replaces hgd_spmm's epilogue/slope). */
hgd_status hgd_spmm_fused(const int64_t* rowptr, const int32_t* col, const float* val,
                          const float* row_scale, int64_t n_rows, int64_t n_src_rows,
                          int64_t row_begin, int64_t row_end, const float* X, int64_t ldx,
                          float* Y, int64_t ldy, int32_t d, const hgd_row_epilogue* epi,
                          const hgd_split_plan* plan, void* workspace, size_t workspace_bytes,
                          void* stream);

/* hgd_spmm_masked (the edge-dropped view) with the fused row epilogue `epi`. HCCF's layer
 * (model/graph/HCCF.py:182-187): gcn = A_drop·h stored through act_out while the row store adds
 * the layer's hypergraph term as res1, so hidden[k+1] = gcn + hgnn needs no separate add; the
 * backward hop adds the layer-sum gradient the same way. */
hgd_status hgd_spmm_masked_fused(const int64_t* rowptr, const int32_t* col, const float* val,
                                 const uint8_t* mask, float keep, const float* row_scale,
                                 int64_t n_rows, int64_t n_src_rows, int64_t row_begin,
                                 int64_t row_end, const float* X, int64_t ldx, float* Y,
                                 int64_t ldy, int32_t d, const hgd_row_epilogue* epi,
                                 const hgd_split_plan* plan, void* workspace,
                                 size_t workspace_bytes, void* stream);

/* The same row epilogue applied to an existing matrix Z [n_rows, ldz] (z = Z[r], no hop): the
 * LayerNorms that do not follow a hop, e.g. the MLP InputNorm of model/layers/MLP.py:65-71,109-110.
 * Needs d <= 256 with 16-byte aligned rows, or d <= 64. Y may alias Z. */
hgd_status hgd_row_epilogue_forward(const float* Z, int64_t ldz, int64_t n_rows, int32_t d,
                                    const hgd_row_epilogue* epi, float* Y, int64_t ldy,
                                    void* stream);

/* Backward of the row epilogue up to z (the residual gradients are res_scale·dY, left to the
 * caller): dZ = act'(a) ⊙ LN_bwd(out_scale·dY), with LN_bwd the LayerNorm input gradient
 * rstd·(ĝ - mean(ĝ) - â·mean(ĝ⊙â)), ĝ = γ⊙dy, â = (a-μ)·rstd recomputed from act_out and stats.
 * dgamma = Σ_r dy⊙â, dbeta = Σ_r dy (written, not accumulated; summed in a fixed order, so the
 * result is deterministic). act_out is required when act != NONE or layer_norm. */
size_t hgd_row_epilogue_backward_workspace_size(int64_t n_rows, int32_t d);
hgd_status hgd_row_epilogue_backward(const float* dY, int64_t ldy, const float* act_out,
                                     int64_t ld_act, const float* stats, const float* ln_gamma,
                                     int64_t n_rows, int32_t d, int32_t act, float slope,
                                     int32_t layer_norm, float out_scale, float* dZ, int64_t ldz,
                                     float* dgamma, float* dbeta, void* workspace,
                                     size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * Skinny Linear layers on the f32 MFMA: nn.Linear(in, out) over
 * n_rows ≫ in, out — lin_in of model/layers/EquivSetGNN.py:88-89 /
 * layers2/EquivSetGNN2.py:93-94 (with its F.relu) and the MLP layers of
 * model/layers/MLP.py:109-117. W is [out_features, ldw] row-major (nn.Linear.weight); features
 * are multiples of 16, rows 16-byte aligned. Forward: in_features <= 128; backward-data:
 * out_features <= 128. Exact f32 products and sums (order differs from a library GEMM).
 *   forward          Y = relu?(X·Wᵀ + bias)
 *   backward_data    dX = (dY ⊙ [relu_out > 0])·W        (relu_out = the forward Y, or NULL)
 *   backward_weight  dW = (dY ⊙ [relu_out > 0])ᵀ·X, db = Σ_rows dY ⊙ [relu_out > 0]
 *                    (dW written contiguous [out, in]; split-K partials summed in a fixed order)
 * ---------------------------------------------------------------------------------------- */
hgd_status hgd_linear_forward(const float* X, int64_t ldx, int64_t n_rows, int32_t in_features,
                              const float* W, int64_t ldw, int32_t out_features,
                              const float* bias, int32_t relu, float* Y, int64_t ldy,
                              void* stream);
hgd_status hgd_linear_backward_data(const float* dY, int64_t ldy, const float* relu_out,
                                    int64_t ldr, int64_t n_rows, int32_t out_features,
                                    const float* W, int64_t ldw, int32_t in_features, float* dX,
                                    int64_t ldx, void* stream);
size_t hgd_linear_backward_weight_workspace_size(int64_t n_rows, int32_t out_features,
                                                 int32_t in_features);
hgd_status hgd_linear_backward_weight(const float* dY, int64_t ldy, const float* relu_out,
                                      int64_t ldr, const float* X, int64_t ldx, int64_t n_rows,
                                      int32_t out_features, int32_t in_features, float* dW,
                                      float* db, void* workspace, size_t workspace_bytes,
                                      void* stream);

/* Grouped forms of the skinny products above (HCCF's learned hypergraph HCCF.py:201-211 runs
 * every product once for the users and once for the items): one launch for one or two
 * independent products of equal shape class, which is what bounds these ~10 MB products.
 *   hgd_gemm_rows: Y = relu?((A ⊙ [relu_mask > 0])·B + bias) (+ Y when accumulate), A [rows, K]
 *     (16-byte aligned rows), B[k][n] = B[k·bsk + n·bsn]; K a multiple of 16 in [16, 128], N a
 *     multiple of 16; the two products must share K, N and mask presence. The masked form
 *     (relu_mask set: the backward-data product) takes none of the drop / res / row_inv /
 *     binarize_a epilogues below (HGD_ERR_INVALID_ARG).
 *   hgd_gemm_tn: C [M, N] = (A ⊙ [relu_mask > 0])ᵀ·B over `rows` rows (split-K, partials summed
 *     in slice order: deterministic), colsum_A [M] = Σ_rows A ⊙ mask when non-NULL; the two
 *     products must share M, N and mask presence. Workspace: hgd_gemm_tn_workspace_size. */
typedef struct hgd_gemm_rows_desc {
  const float* A;
  int64_t lda;
  const float* relu_mask; /* [rows, K] or NULL */
  int64_t ldm;
  const float* B;
  int64_t bsk;
  int64_t bsn;
  const float* bias;      /* [N] or NULL */
  int32_t relu;
  int32_t accumulate;
  float* Y;
  int64_t ldy;
  int64_t rows;
  int32_t K;
  int32_t N;
  /* forward epilogue after bias / ReLU (NULL / 0 = off): nn.Dropout — element (row, col) kept as
   * hgd_dropout_apply keeps element row·N + col (rows·N < 2^32) for seed *drop_seed (a device
   * value: a captured step draws it inside the graph), kept values × drop_scale (1 / (1 - p));
   * then the second store Y2 = Y + res (res and Y2 both NULL or both set) — the "+ res" after
   * an ED-HNN block (HGNN_HD4.py:399) */
  const uint64_t* drop_seed;
  float drop_keep;
  float drop_scale;
  const float* res;
  int64_t ldres;
  float* Y2;
  int64_t ldy2;
  /* row_inv (NULL = off): the product's rows scaled by 1 / max(Σ_k A'[r, k], 1) before bias /
   * ReLU and that factor stored to row_inv[r] — with binarize_a, the scatter mean over a vertex's
   * hyperedges of a dense learned hypergraph (EquivSetConv2.py:93 on nonzero(H > 0),
   * EquivSetGNN2.py:105-133); binarize_a: A' = (A > 0 ? 1 : 0) instead of A */
  float* row_inv;
  int32_t binarize_a;
  /* b_row_count (NULL = off): row k of B scaled by 1 / max(b_row_count[k], 1) as it is staged —
   * the hyperedge means D_e^-1·Xe of the mean two-hop from the raw column counts colsum_A of the
   * split-K product that made Xe (same product as scaling B beforehand) */
  const float* b_row_count;
  float b_scale;          /* 0 = off: B × b_scale as it is staged (a Dropout's 1/(1-p) in dX) */
  /* a_drop_seed (NULL = off): nn.Dropout on A as it is loaded — element (row, k) kept as
   * hgd_dropout_apply keeps element row·K + k (rows·K < 2^32) for seed *a_drop_seed, kept values
   * × a_drop_scale, before relu_mask / binarize_a: the ED-HNN block's input dropout inside
   * lin_in (EquivSetGNN2.py:91-92). With relu_mask set, drop_seed is the backward of such an
   * input dropout: the masked product's output × its keep-bits × drop_scale. */
  const uint64_t* a_drop_seed;
  float a_drop_keep;
  float a_drop_scale;
} hgd_gemm_rows_desc;
hgd_status hgd_gemm_rows(const hgd_gemm_rows_desc* descs, int32_t count, void* stream);

typedef struct hgd_gemm_tn_desc {
  const float* A;
  int64_t lda;
  const float* relu_mask; /* [rows, M] or NULL */
  int64_t ldm;
  const float* B;
  int64_t ldb;
  int64_t rows;
  int32_t M;
  int32_t N;
  float* C;               /* [M, N] */
  float* colsum_A;        /* [M] or NULL */
  int32_t binarize_a;     /* A' = (A > 0 ? 1 : 0) instead of A (colsum_A then counts nonzeros) */
  const float* b_row_scale; /* [rows] or NULL: B's row r × b_row_scale[r] as it is loaded (the
                             * vertex means D_v^-1 of the mean two-hop's backward) */
  float c_scale;          /* 0 = off: C and colsum_A × c_scale as they are stored */
  /* b_drop_seed (NULL = off): nn.Dropout on B as it is loaded (element row·N + n kept as
   * hgd_dropout_apply keeps it, rows·N < 2^32, kept × b_drop_scale; before b_row_scale) — the
   * weight gradient of a Linear whose input dropout ran inside its forward */
  const uint64_t* b_drop_seed;
  float b_drop_keep;
  float b_drop_scale;
} hgd_gemm_tn_desc;
size_t hgd_gemm_tn_workspace_size(const hgd_gemm_tn_desc* descs, int32_t count);
hgd_status hgd_gemm_tn(const hgd_gemm_tn_desc* descs, int32_t count, void* workspace,
                       size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * Fused InfoNCE, contrastLoss of util/loss_torch.py:103-110:
 *   p1 = normalize(E1[nodes] + 1e-8), p2 = normalize(E2[nodes] + 1e-8)   (eps 1e-12)
 *   loss = -(1/B) Σ_b log( exp(<p1_b,p2_b>/τ) / (Σ_j exp(<p1_b,p2_j>/τ) + 1e-8) )
 * Only the B batch rows are gathered and normalised; the [B, B] exp-sum is never materialised.
 * nodes follow torch indexing: negative ids count from the end of the table (HCCF.py:65-66 passes
 * torch.unique(emb.long())); ids outside [-n_rows, n_rows) are the caller's error (clamped here).
 * Forward writes P1, P2 [B, d] (contiguous), inv_norm1/2 [B], pos_logit [B], deno [2, B] and
 * the scalar loss (all device): deno[b] = Σ_j exp(<p1_b,p2_j>/τ) + 1e-8 and deno[B + b] = its
 * off-diagonal part (Σ_{j≠b} … + 1e-8), from which the loss term and the diagonal gradient
 * weight 1 − p_bb are formed without cancellation (p_bb rounds to 1 in fp32 for a one-node list;
 * the reference's fp32 autograd returns rounding noise there). B is the capacity for the _n
 * forms. Backward recomputes the logits and writes dX1, dX2 [B, d] =
 * dloss/d(E1[nodes]), dloss/d(E2[nodes]) scaled by the device scalar *grad_loss; scattering
 * them into the [N, d] table gradients (duplicate nodes add) is the caller's. d: multiple of 16
 * in [16, 256]. Deterministic (fixed-order reductions). Workspace: hgd_infonce_workspace_size.
 * ---------------------------------------------------------------------------------------- */
size_t hgd_infonce_workspace_size(int64_t batch, int32_t d);
hgd_status hgd_infonce_forward(const float* E1, int64_t ld1, const float* E2, int64_t ld2,
                               int64_t n_rows, const int64_t* nodes, int64_t batch, int32_t d,
                               float temp, float* P1, float* P2, float* inv_norm1,
                               float* inv_norm2, float* pos_logit, float* deno, float* loss,
                               void* workspace, size_t workspace_bytes, void* stream);
hgd_status hgd_infonce_backward(const float* P1, const float* P2, const float* inv_norm1,
                                const float* inv_norm2, const float* deno, int64_t batch,
                                int32_t d, float temp, const float* grad_loss, float* dX1,
                                float* dX2, void* workspace, size_t workspace_bytes,
                                void* stream);
/* The same with the batch size held on the device (*batch_count <= capacity; the node list
 * is capacity-sized, e.g. a device-side unique whose count is never read back): grids and
 * strides use `capacity`, the kernels read the live count, rows past it come out as zeros
 * (P1/P2/dX1/dX2) and the mean divides by the live count. Nothing is read to the host, so a
 * training step using them can be captured in a HIP graph. Workspace:
 * hgd_infonce_workspace_size(capacity, d). */
hgd_status hgd_infonce_forward_n(const float* E1, int64_t ld1, const float* E2, int64_t ld2,
                                 int64_t n_rows, const int64_t* nodes, int64_t capacity,
                                 const int64_t* batch_count, int32_t d, float temp, float* P1,
                                 float* P2, float* inv_norm1, float* inv_norm2, float* pos_logit,
                                 float* deno, float* loss, void* workspace,
                                 size_t workspace_bytes, void* stream);
/* Backward with the scatter fused: the gradient rows are added straight into the [n_rows, d]
 * table gradients dE1 / dE2 (zero-filled by the caller; either may be NULL: that side is not
 * computed) at
 * the batch rows' nodes (torch indexing, negative ids wrap), rows past *batch_count add nothing.
 * Atomic adds, but at most two batch rows meet on one table row, so the result is
 * deterministic. */
hgd_status hgd_infonce_backward_n(const float* P1, const float* P2, const float* inv_norm1,
                                  const float* inv_norm2, const float* deno, int64_t capacity,
                                  const int64_t* batch_count, int32_t d, float temp,
                                  const float* grad_loss, const int64_t* nodes, int64_t n_rows,
                                  float* dE1, int64_t ldE1, float* dE2, int64_t ldE2,
                                  void* workspace, size_t workspace_bytes, void* stream);

/* Several InfoNCE terms in ONE launch per kernel (HCCF's user and item terms of a layer,
 * HCCF.py:65-66): each term as hgd_infonce_forward_n / hgd_infonce_backward_n would take it
 * (batch_count NULL = all `capacity` rows live), with its own workspace
 * (hgd_infonce_workspace_size(capacity, d)). Backward outputs: dX1 / dX2 compact [capacity, d]
 * rows, or dE1 / dE2 scatter-adds into [n_rows, ld] tables (nodes required); a side without an
 * output is skipped. count is 1 to 8 (HCCF: the user and item terms of up to four layers, one
 * launch per kernel for the whole step's InfoNCE); all terms share d, temp and — backward —
 * grad_loss (the group's loss is the sum of its terms' losses). */
typedef struct hgd_infonce_term {
  const float* E1;
  int64_t ld1;
  const float* E2;
  int64_t ld2;
  int64_t n_rows;
  const int64_t* nodes;
  int64_t capacity;
  const int64_t* batch_count;
  float* P1;
  float* P2;
  float* inv_norm1;
  float* inv_norm2;
  float* pos_logit;
  float* deno;
  float* loss;
  float* dX1;
  float* dX2;
  float* dE1;
  int64_t ldE1;
  float* dE2;
  int64_t ldE2;
  void* workspace;
  size_t workspace_bytes;
} hgd_infonce_term;
hgd_status hgd_infonce_forward_group(const hgd_infonce_term* terms, int32_t count, int32_t d,
                                     float temp, void* stream);
hgd_status hgd_infonce_backward_group(const hgd_infonce_term* terms, int32_t count, int32_t d,
                                      float temp, const float* grad_loss, void* stream);

/* ------------------------------------------------------------------------------------------
 * Ingest and graph build — the data path producing the hot path's
 * input matrices (data/loader.py:24-38, data/ui_graph.py:43-112, data/graph.py:11-25).
 *
 * Host (no GPU needed): hgd_ingest_read parses a "user<sep>item[<sep>…]" file exactly like
 * FileIO.load_data_set — first line skipped; a line with a tab splits on tabs, else on commas,
 * after stripping; fields 0/1 parsed like Python int(); other fields ignored; "\n", "\r\n" and
 * "\r" end lines — with n_threads parser threads (<= 0: all cores). Lines the reference would
 * reject fail the call (the message names the line). The handle owns the parsed arrays.
 * ---------------------------------------------------------------------------------------- */
typedef struct hgd_ingest hgd_ingest;
hgd_status hgd_ingest_read(const char* path, int32_t skip_header, int32_t n_threads,
                           hgd_ingest** out);
int64_t hgd_ingest_count(const hgd_ingest* h);  /* records, -1 for NULL */
/* Copies the raw user / item ids (host int64 arrays of hgd_ingest_count entries, file order). */
hgd_status hgd_ingest_copy(const hgd_ingest* h, int64_t* user_raw, int64_t* item_raw);
void hgd_ingest_free(hgd_ingest* h);

/* Device: ids[i] = rank of keys[i] among the distinct keys ordered by first appearance (the
 * `if user not in self.user: self.user[user] = len(self.user)` loop, data/ui_graph.py:43-56);
 * uniq[r] = the key with id r (first *n_unique entries); *n_unique on the device. */
size_t hgd_remap_workspace_size(int64_t n);
hgd_status hgd_remap_first_appearance(const int64_t* keys, int64_t n, int32_t* ids,
                                      int64_t* uniq, int64_t* n_unique, void* workspace,
                                      size_t workspace_bytes, void* stream);

/* Device: canonical CSR (rows ascending, columns ascending, duplicates summed into float32
 * counts) of the COO (rows, cols) [n] — scipy csr_matrix((ones, (row, col))), ui_graph.py:70-84.
 * col_out / val_out need n entries; the nonzero count lands in device *nnz_out. */
size_t hgd_coo_coalesce_workspace_size(int64_t n);
hgd_status hgd_coo_coalesce(const int32_t* rows, const int32_t* cols, int64_t n, int64_t n_rows,
                            int64_t n_cols, int64_t* rowptr, int32_t* col_out, float* val_out,
                            int64_t* nnz_out, void* workspace, size_t workspace_bytes,
                            void* stream);

/* Device: out[e] = (row_scale[r]·val[e])·col_scale[col[e]] (col_scale NULL: no second factor) —
 * d_mat_inv.dot(adj).dot(d_mat_inv) of Graph.normalize_graph_mat with the scales of
 * hgd_degree_scale (power -0.5 square, -1 rectangular). */
hgd_status hgd_normalize_values(const int64_t* rowptr, const int32_t* col, const float* val,
                                int64_t n_rows, const float* row_scale, const float* col_scale,
                                float* out, void* stream);

/* ------------------------------------------------------------------------------------------
 * Structure primitives (all deterministic; indices bit-exact with the CPU restatement).
 * ---------------------------------------------------------------------------------------- */
/* int64 indices → int32, checking 0 <= v < upper; err_count (device int64) += #violations. */
hgd_status hgd_index_narrow(const int64_t* in, int64_t n, int64_t upper, int32_t* out,
                            int64_t* err_count, void* stream);
/* Stable sort of int32 keys in [0, n_keys): keys_out = sorted keys, perm_out[i] = source position. */
size_t hgd_sort_perm_workspace_size(int64_t n);
hgd_status hgd_sort_perm(const int32_t* keys, int64_t n, int64_t n_keys, int32_t* keys_out,
                         int32_t* perm_out, void* workspace, size_t workspace_bytes,
                         void* stream);
/* rowptr[r] = first position p with sorted_rows[p] >= r, r in [0, n_rows]. */
hgd_status hgd_rowptr_from_sorted(const int32_t* sorted_rows, int64_t nnz, int64_t n_rows,
                                  int64_t* rowptr, void* stream);
/* Counts positions where sorted_rows decreases or leaves [0,n_rows) into device int64 *bad. */
hgd_status hgd_check_sorted(const int32_t* rows, int64_t nnz, int64_t n_rows, int64_t* bad,
                            void* stream);
/* rows_out[e] = r for e in [rowptr[r], rowptr[r+1]), nnz = rowptr[n_rows]. */
hgd_status hgd_expand_rows(const int64_t* rowptr, int64_t n_rows, int64_t nnz, int32_t* rows_out,
                           void* stream);
/* out[i] = src[perm[i]] (4-byte elements: int32 or fp32 bit patterns). */
hgd_status hgd_gather32(const void* src, const int32_t* perm, int64_t n, void* out,
                        void* stream);
/* out[i] = src[perm[i]] for bytes: a CSR-order keep-mask into CSC order through perm_t
 * (hgd_spmm_masked's backward hop). perm 16-byte aligned, out 4-byte aligned. */
hgd_status hgd_gather_u8(const uint8_t* src, const int32_t* perm, int64_t n, uint8_t* out,
                         void* stream);
/* s[r] = deg(r)^power with deg = rowptr diff (val == NULL) or Σ val over the row; deg == 0 → 0.
 * power is -1.0 (D^-1) or -0.5 (D^-1/2) or any other exponent. */
hgd_status hgd_degree_scale(const int64_t* rowptr, const float* val, int64_t n_rows,
                            double power, float* scale_out, void* stream);
/* out[e] = (base ? base[perm ? perm[e] : e] : 1) * (src_scale ? src_scale[src_idx[e]] : 1). */
hgd_status hgd_edge_values(const float* base, const int32_t* perm, const float* src_scale,
                           const int32_t* src_idx, int64_t n, float* out, void* stream);

/* Drop-edge compaction (SpAdjDropEdge): keeps entries with mask[e] != 0 in order,
 * out_val = val[e] / keep. Writes the kept count to device int64 *out_count. */
size_t hgd_dropedge_workspace_size(int64_t nnz);
hgd_status hgd_dropedge_compact(const int64_t* rows, const int64_t* cols, const float* val,
                                const uint8_t* mask, int64_t nnz, float keep,
                                int64_t* out_rows, int64_t* out_cols, float* out_val,
                                int64_t* out_count, void* workspace, size_t workspace_bytes,
                                void* stream);

/* Device keep-mask for drop-edge: mask[i] = floor(u_i + keep) != 0 with u_i a 24-bit uniform
 * from a counter-based hash of (seed, i) — the SpAdjDropEdge expression (HCCF.py:223) without
 * the host RNG round trip (statistically, not bitwise, equal to torch's CPU stream). */
hgd_status hgd_bernoulli_mask(uint64_t seed, int64_t n, float keep, uint8_t* mask, void* stream);
/* The same draw with the 64-bit seed read from device memory (seed[0]): a captured training step
 * advances the counter on the device, so every graph replay draws a fresh mask. */
hgd_status hgd_bernoulli_mask_dev(const uint64_t* seed, int64_t n, float keep, uint8_t* mask,
                                  void* stream);
/* The same draw for both orientations of a structure (hgd_spmm_masked's forward and backward
 * hops): mask[i] as hgd_bernoulli_mask_dev, mask_t[j] = mask[perm_t[j]] computed from the hash
 * of perm_t[j] (perm_t: CSC position → CSR position) instead of a byte gather. */
hgd_status hgd_bernoulli_mask_dev_pair(const uint64_t* seed, const int32_t* perm_t, int64_t n,
                                       float keep, uint8_t* mask, uint8_t* mask_t, void* stream);
/* Zeroes entries [*count, capacity) of the capacity-sized outputs of hgd_dropedge_structure
 * (count = rowptr_out + n_rows, on the device): a dropped structure whose kept count is never read
 * back keeps full-size arrays with a defined tail (index 0, weight 0). Null arrays are skipped. */
hgd_status hgd_dropedge_fill_tail(const int64_t* count, int64_t capacity, int32_t* col,
                                  float* val, int32_t* row_t, float* val_t, void* stream);

/* Sort-free rebuild of a drop-edge'd structure from its parent: compacts the parent CSR with the
 * mask (CSR order) and the parent CSC with mask[perm_t[e']] (perm_t: CSC position → CSR
 * position), dividing values by keep; row pointers are remapped through the prefix sums.
 * Outputs are sized for nnz (upper bound); the kept count is rowptr_out[n_rows]. No host sync. */
size_t hgd_dropedge_structure_workspace_size(int64_t nnz);
hgd_status hgd_dropedge_structure(const int64_t* rowptr, const int32_t* col, const float* val,
                                  const int64_t* colptr, const int32_t* row_t, const float* val_t,
                                  const int32_t* perm_t, int64_t n_rows, int64_t n_cols,
                                  int64_t nnz, const uint8_t* mask, float keep,
                                  int64_t* rowptr_out, int32_t* col_out, float* val_out,
                                  int64_t* colptr_out, int32_t* row_t_out, float* val_t_out,
                                  void* workspace, size_t workspace_bytes, void* stream);

/* torch.nonzero(H > thresh) (mode HGD_DENSE_GREATER) or torch.nonzero(H) (HGD_DENSE_NONZERO)
 * of a dense row-major [n_rows, n_cols] fp32 matrix (leading dim ld), in two passes: rowptr
 * (n_rows+1, int64), then the column list (rowptr[n_rows] int32 entries) and, if vals != NULL,
 * the kept values in the same order. */
#define HGD_DENSE_GREATER 0
#define HGD_DENSE_NONZERO 1
size_t hgd_dense_threshold_workspace_size(int64_t n_rows);
hgd_status hgd_dense_threshold_rowptr(const float* H, int64_t n_rows, int64_t n_cols, int64_t ld,
                                      float thresh, int32_t mode, int64_t* rowptr,
                                      void* workspace, size_t workspace_bytes, void* stream);
hgd_status hgd_dense_threshold_fill(const float* H, int64_t n_rows, int64_t n_cols, int64_t ld,
                                    float thresh, int32_t mode, const int64_t* rowptr,
                                    int32_t* cols, float* vals, void* stream);

/* ------------------------------------------------------------------------------------------
 * Evaluation (GraphRecommender.test, base/graph_recommender.py:61-92).
 *   hgd_mask_scores: scores[r, cols[rowptr[m]:rowptr[m+1]]] = value, m = row_map ? row_map[r] : r
 *                    (rated items → -10e8, :79-80).
 *   hgd_topk_rows:   per row, the K entries find_k_largest (util/algorithm.py:143-173) returns —
 *                    first K of {(c_j, j): j < K} ∪ {(c_i, i)} by score desc, seed first, index
 *                    asc (so top items among the first K appear twice, as in the reference).
 *                    1 <= k <= 256, n_cols >= k; out_ids int32 [n_rows, k], out_scores fp32.
 * ---------------------------------------------------------------------------------------- */
hgd_status hgd_mask_scores(float* scores, int64_t n_rows, int64_t ld, const int64_t* rowptr,
                           const int32_t* cols, const int32_t* row_map, float value,
                           void* stream);
hgd_status hgd_topk_rows(const float* scores, int64_t n_rows, int64_t n_cols, int64_t ld,
                         int32_t k, int32_t* out_ids, float* out_scores, void* stream);

/* Per-user inputs of ranking_evaluation (util/evaluation.py:169-196) for the lists above:
 *   hits[r, c] = |set(test items of r) ∩ set(ids[r, :N_c])|        (Metric.hits, :8-15)
 *   dcg[r, c]  = Σ_{n < N_c, ids[r, n] in test} discount[n], in n order (Metric.NDCG, :84-97)
 * ids int32 [n_rows, ld] (device, k <= 256 used per row, negative = never a hit); the test items
 * of row r are test_cols[test_rowptr[r] : test_rowptr[r+1]] (device, ascending, distinct
 * internal item ids); discount float64 [k] (device) = 1.0/math.log(n+2, 2) computed by the host
 * so DCG is bit-identical to the reference; cutoffs = the N values (HOST array, ascending, in
 * [1, k], at most 16). Outputs hits int32 / dcg float64 [n_rows, n_cutoffs]. */
hgd_status hgd_rank_metrics(const int32_t* ids, int64_t n_rows, int64_t ld, int32_t k,
                            const int64_t* test_rowptr, const int32_t* test_cols,
                            const int32_t* cutoffs, int32_t n_cutoffs, const double* discount,
                            int32_t* hits, double* dcg, void* stream);

/* ------------------------------------------------------------------------------------------
 * Pairwise training sampler (HOST functions, host pointers): next_batch_pairwise
 * (util/sampler.py:237-264) with CPython's random module bit for bit. mt_state = the 625 words
 * of random.getstate()[1] (624 MT19937 words + position), read and advanced in place — the
 * caller hands it back with random.setstate, so the Python stream continues exactly as if the
 * reference loop had run.
 *   hgd_py_shuffle:      random.shuffle(x) applied to order[0..n) (x[k] = record order[k]).
 *   hgd_sample_pairwise: records order[begin..end): out_u / out_i = rec_user / rec_item of the
 *                        record, then n_negs draws choice(item_list) per record (dense id =
 *                        _randbelow(n_items)), redrawn while in the user's training items
 *                        user_items[user_rowptr[u] : user_rowptr[u+1]] (ascending);
 *                        out_j [(end-begin) * n_negs]. Fails (instead of looping forever like the
 *                        reference) for a user who has every item.
 * ---------------------------------------------------------------------------------------- */
hgd_status hgd_py_shuffle(uint32_t* mt_state, int64_t* order, int64_t n);
hgd_status hgd_sample_pairwise(uint32_t* mt_state, const int64_t* order, int64_t begin,
                               int64_t end, const int32_t* rec_user, const int32_t* rec_item,
                               const int64_t* user_rowptr, const int32_t* user_items,
                               int64_t n_users, int64_t n_items, int32_t n_negs, int32_t* out_u,
                               int32_t* out_i, int32_t* out_j);

/* SpAdjDropEdge's CPU keep-mask (HCCF.py:223: floor(torch.rand(nnz) + keepRate).bool()) from
 * torch's default CPU generator, bit for bit, in one host pass (HOST function). torch_state =
 * the bytes of torch.get_rng_state() (hgd_torch_cpu_state_bytes(), 5056 on x86-64), advanced in
 * place by n draws for torch.set_rng_state; mask uint8 [n] (host); *kept = number of ones.
 * Long draws are split over host threads (HGD_TUNE_CPU_RNG_THREADS), each starting from the
 * MT19937 state its first draw sees, computed by a GF(2) jump-ahead: the same bits as one thread. */
size_t hgd_torch_cpu_state_bytes(void);
hgd_status hgd_torch_cpu_keep_mask(uint8_t* torch_state, int64_t state_bytes, int64_t n,
                                   float keep, uint8_t* mask, int64_t* kept);
/* The same with an explicit host thread count (0 = HGD_TUNE_CPU_RNG_THREADS' default): a draw
 * that runs beside a host-bound eager step should leave cores to it. */
hgd_status hgd_torch_cpu_keep_mask_threads(uint8_t* torch_state, int64_t state_bytes, int64_t n,
                                           float keep, uint8_t* mask, int64_t* kept,
                                           int32_t threads);
/* Test hook: 1 if the jump-ahead reproduces `refills` MT19937 refills of a seeded state. */
int32_t hgd_torch_cpu_jump_selfcheck(int64_t refills);

/* ------------------------------------------------------------------------------------------
 * Sorted unique of integer keys — torch.unique(t.long()) as HCCF's loss calls it every step on
 * [batch, d] embedding blocks: contrastLoss(..., torch.unique(ancs.long()), ...),
 * model/graph/HCCF.py:65-66 (the truncated embedding values become the node list).
 *   hgd_unique_i64 / hgd_unique_trunc_f32: range-bitmap path, no host sync. out [n] receives the
 *     distinct keys ascending (the trunc variant truncates floats toward zero like Tensor.long();
 *     NaN / ±inf / |x| >= 2^63 become INT64_MIN), device *n_out their count — or -1 when the
 *     key range exceeds 2^24, in which case the caller runs the matching hgd_unique_sort_* (device
 *     radix sort + unique, same output). n < 2^31. Workspace: hgd_unique_workspace_size(n).
 * ---------------------------------------------------------------------------------------- */
size_t hgd_unique_workspace_size(int64_t n);
hgd_status hgd_unique_i64(const int64_t* keys, int64_t n, int64_t* out, int64_t* n_out,
                          void* workspace, size_t workspace_bytes, void* stream);
hgd_status hgd_unique_trunc_f32(const float* x, int64_t n, int64_t* out, int64_t* n_out,
                                void* workspace, size_t workspace_bytes, void* stream);
hgd_status hgd_unique_sort_i64(const int64_t* keys, int64_t n, int64_t* out, int64_t* n_out,
                               void* workspace, size_t workspace_bytes, void* stream);
hgd_status hgd_unique_sort_trunc_f32(const float* x, int64_t n, int64_t* out, int64_t* n_out,
                                     void* workspace, size_t workspace_bytes, void* stream);
/* Device-complete form (a captured training step cannot take the host-side fallback): the
 * bitmap window is [min, min + 2^24); keys beyond it are collected and sorted by one workgroup
 * (in LDS up to 4,096 of them, else a bitonic network over the workspace) and appended — they
 * are all larger. *n_out is always the unique count. Same output as the forms above. */
hgd_status hgd_unique_dev_i64(const int64_t* keys, int64_t n, int64_t* out, int64_t* n_out,
                              void* workspace, size_t workspace_bytes, void* stream);
hgd_status hgd_unique_dev_trunc_f32(const float* x, int64_t n, int64_t* out, int64_t* n_out,
                                    void* workspace, size_t workspace_bytes, void* stream);

/* Several lists through the device-complete path at once (HCCF's anchor and positive node
 * lists, HCCF.py:65-66): one launch per kernel for all of them, each list's out / n_out exactly
 * as hgd_unique_dev_i64 / hgd_unique_dev_trunc_f32 give it. Per list: exactly one of x_f32
 * (truncated like Tensor.long()) and x_i64, and its own workspace of
 * hgd_unique_workspace_size(n) bytes. `capacity` (0 = n): *n_out is clamped to it and
 * out[*n_out, capacity) zeroed — a fixed-size list whose live count stays on the device (the
 * capacity-sized node lists HCCF's InfoNCE reads). count is 1 to 4. */
typedef struct hgd_unique_job {
  const float* x_f32;
  const int64_t* x_i64;
  int64_t n;
  int64_t capacity;
  int64_t* out;
  int64_t* n_out;
  void* workspace;
  size_t workspace_bytes;
} hgd_unique_job;
hgd_status hgd_unique_dev_group(const hgd_unique_job* jobs, int32_t count, void* stream);

/* ------------------------------------------------------------------------------------------
 * BPR loss from the embedding table (util/loss_torch.py:5-9 over the rows HCCF.py:84-86
 * gathers): E [n_users + n_items, lde] (users first, 16-byte aligned rows, d % 4 == 0,
 * d <= 256); anc = E[uid], pos = E[n_users + pid], neg = E[n_users + nid] (int64 ids, torch
 * indexing semantics; out-of-range ids are clamped, never dereferenced, and the forward adds
 * the number of batch rows holding one to *bad_index when it is non-NULL — a device word the
 * caller zeroes and reads when it chooses: the reference's gather raises on such an id);
 *   loss = mean_k −log(1e-5 + σ(⟨anc_k,pos_k⟩ − ⟨anc_k,neg_k⟩)), coef_k = σ(1−σ)/(1e-5+σ).
 * anc_out / pos_out ([batch, d], optional) receive the gathered rows (HCCF's InfoNCE node lists
 * are taken from them). Backward: dE = ∂(grad·loss)/∂E written in full (zero rows included;
 * `grad` a device scalar), every touched row summed over its positions in a fixed order
 * (position order for rows with at most 8 positions; rows with more — a skewed catalogue's
 * popular items — by one workgroup in fixed contiguous ranges of their ascending positions,
 * combined in range order): deterministic, integer atomics only.
 * Workspace: hgd_bpr_workspace_size(batch, n_rows). */
size_t hgd_bpr_workspace_size(int64_t batch, int64_t n_rows);
hgd_status hgd_bpr_forward(const float* E, int64_t lde, int64_t n_users, int64_t n_items,
                           int32_t d, const int64_t* uid, const int64_t* pid, const int64_t* nid,
                           int64_t batch, float* anc_out, float* pos_out, float* coef,
                           float* loss, int32_t* bad_index, void* workspace,
                           size_t workspace_bytes, void* stream);
hgd_status hgd_bpr_backward(const float* E, int64_t lde, int64_t n_users, int64_t n_items,
                            int32_t d, const int64_t* uid, const int64_t* pid,
                            const int64_t* nid, int64_t batch, const float* coef,
                            const float* grad, float* dE, int64_t ldd, void* workspace,
                            size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * Elementwise epilogues around the hops (contiguous fp32, 16-byte aligned).
 *   apply:    y = epi(z)                                   (nn.LeakyReLU / nn.ReLU forward)
 *   backward: dz = dy * (ref > 0 ? 1 : slope) for LEAKY, dy * (ref > 0) for RELU, where ref is
 *             the pre-activation (or the output when slope >= 0, which has the same sign).
 * ---------------------------------------------------------------------------------------- */
hgd_status hgd_epilogue_apply(const float* z, int64_t n, int32_t epilogue, float slope, float* y,
                              void* stream);
hgd_status hgd_epilogue_backward(const float* ref, const float* dy, int64_t n, int32_t epilogue,
                                 float slope, float* dz, void* stream);
/* nn.Dropout(p) on the library's counter-based RNG (the ED-HNN block's dropouts,
 * layers2/EquivSetGNN2.py:91-101, when they run in its Linear stores or alone): y[i] = x[i]·scale
 * if element i (< 2^32) is kept, else 0. Elements 4c .. 4c + 3 share one draw:
 * h1 = lowbias32(lowbias32(c + lo32(s)) ^ hi32(s)), h2 = lowbias32(h1 ^ 0x9E3779B9), s = *seed
 * (a device value); element 4c + j is kept iff the j-th 16-bit half of (h1, h2), low half
 * first, is below floor(keep·65536 + 0.5) (f32). keep = 1 - p, scale = 1 / (1 - p). The
 * backward is the same call on the gradient with the same seed (no mask is stored). x, y
 * 16-byte aligned; y may alias x. */
/* The backward of `count` nn.Dropout calls on one tensor (torch's native_dropout_backward per
 * call, g_k = ((float)mask_k · dy_k) · scale, then autograd's accumulation of the calls'
 * gradients as they arrive, the last call's first): out = ((g_{count-1} + g_{count-2}) + …) + g_0
 * in one pass, products and sums rounded separately (bitwise torch's kernels). Up to 8 calls per
 * job, up to 4 jobs (tensors) per launch; dy / out 16-byte aligned, masks (bool bytes) 4-byte
 * aligned. HCCF's hypergraph dropouts (HCCF.py:182-186, one per layer on each of E_u·W_u and
 * E_i·W_i) are two such jobs. */
typedef struct hgd_masked_sum {
  const float* dy[8];
  const uint8_t* mask[8];
  float* out;
  int64_t n;
  int32_t count;
  float scale;
} hgd_masked_sum;
hgd_status hgd_masked_scale_sum(const hgd_masked_sum* jobs, int32_t n_jobs, void* stream);
hgd_status hgd_dropout_apply(const float* x, int64_t n, const uint64_t* seed, float keep,
                             float scale, float* y, void* stream);
/* out[i] = Σ_s P[s·slice_stride + i] over s = 0..n_slices-1, summed in slice order (bitwise the
 * chain ((P_0 + P_1) + P_2) + …): HCCF's `sum(hidden)` (model/graph/HCCF.py:188) over the layer
 * tables kept as slices of one buffer. P, out 16-byte aligned, slice_stride % 4 == 0. */
hgd_status hgd_sum_slices(const float* P, int64_t n_slices, int64_t slice_stride, int64_t n,
                          float* out, void* stream);
/* out[i] = ((a_0[i] + a_1[i]) + a_2[i]) + … over n_arrays (1..8) separate device arrays of
 * `count` floats, in array order, one pass: the gradient of a table used by several layers
 * (HGNN_HD4.py:390-405's residual `res`, read by every layer) as one sum instead of a chain of
 * binary accumulations. `arrays` is a HOST array of device pointers; all 16-byte aligned; out
 * may alias a_0. */
hgd_status hgd_sum_arrays(const float* const* arrays, int32_t n_arrays, int64_t count,
                          float* out, void* stream);

/* The reference's optimizer step, torch.optim.Adam(params, lr=…) (model/graph/HCCF.py:33; the
 * multi-tensor non-capturable form torch runs on the device, no weight decay / amsgrad), as ONE
 * kernel over up to 16 tensors — capturable, since its per-step scalars are read from the device
 * table `scalars` ([rows, count, 6] floats: 1 − β1, β2, 1 − β2, sqrt(1 − β2^t), eps,
 * −lr / (1 − β1^t), each the float of the double torch computes on the host, one row per step):
 * row *step_row is used and then step_row is advanced on the device (a second, one-thread
 * launch on the same stream), so a graph holding the call steps through the table by itself;
 * step_row NULL reads row 0 and advances nothing. Per element, in torch's op order and rounding:
 * m ← m + w·(g − m); v ← v·β2; v ← v + value·(g·g); d ← sqrt(v)/c2 + eps; p ← p + s·(m/d).
 * `variant` (0..31) selects the fused multiply-adds (bits 0–2: lerp, addcmul, addcdiv) and the
 * approximate sqrt / division (bits 3, 4) the torch build on the image matches bit for bit
 * (tests/test_gpu_adam.py). `tensors` is a HOST array. */
typedef struct hgd_adam_tensor {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t n;
} hgd_adam_tensor;
hgd_status hgd_adam_step(const hgd_adam_tensor* tensors, int32_t count, const float* scalars,
                         int32_t* step_row, int32_t variant, void* stream);

/* ------------------------------------------------------------------------------------------
 * Incidence objects (SURVEY.md §8b "C ABI libhgd"): the library-owned form of the structure the
 * flat calls above take as loose arrays. One object holds H's CSR (rows = vertices / users,
 * columns = hyperedges / items), its CSC, the CSC→CSR permutation, the degree scales of both
 * sides and the split plans — what the reference's torch.sparse COO `adj` plus cuSPARSE's
 * per-call coalesce/transpose stand for (base/torch_interface.py:8-12, HGNN_HD4.py:455-462).
 *
 *   hgd_incidence_create      convert_sparse_mat_to_tensor + the per-call adj.t() / coalesce
 *   hgd_incidence_from_dense  torch.nonzero(H > 0) of EquivSetGNN2.generate_V_E
 *                             (layers2/EquivSetGNN2.py:105-133) and DHCF's dense adjacency
 *   hgd_incidence_dropedge    SpAdjDropEdge.forward (HCCF.py:213-226) without a sort
 *   hgd_incidence_spmm        torch.sparse.mm(adj, X) / torch.sparse.mm(adj.t(), X)
 *   hgd_conv2hop_forward/     HGCNConv.forward (HGNN_HD4.py:455-462), the ED-HNN scatter-mean
 *   hgd_conv2hop_backward     pair (layers2/EquivSetConv2.py:88-93), HGNN normalisation
 *                             (data/graph.py:28-42) and their autograd backward
 *
 * Creation and drop-edge are setup calls: they allocate device memory (hipMalloc) and
 * synchronise `stream` once (split-plan and kept counts). The object is then immutable apart
 * from lazily built per-nonzero weights (guarded by an internal mutex; hgd_incidence_prepare
 * builds them ahead of graph capture), so it may be used from several threads and streams
 * at once. The object owns its arrays; callers' buffers are only read.
 * ---------------------------------------------------------------------------------------- */
typedef struct hgd_incidence hgd_incidence;

/* Degree scales of one side of H (torch_scatter 'mean' = 1/deg, data/graph.py:11-25 and :28-42
 * D^-1/2 / D^-1 with inf→0; the W-variants use the weighted degree Σ val). */
typedef enum hgd_scale {
  HGD_SCALE_NONE = 0,
  HGD_SCALE_MEAN = 1,  /* deg^-1   */
  HGD_SCALE_SYM = 2,   /* deg^-1/2 */
  HGD_SCALE_WMEAN = 3, /* (Σ val)^-1   */
  HGD_SCALE_WSYM = 4   /* (Σ val)^-1/2 */
} hgd_scale;
#define HGD_SIDE_ROWS 0
#define HGD_SIDE_COLS 1

/* Copies the CSR (rowptr [n_rows+1] int64, col [nnz] int32, val [nnz] or NULL = binary; device
 * pointers) into a new object, validates it (rowptr monotone from 0 to nnz, 0 <= col < n_cols;
 * columns need not be sorted within a row) and derives the CSC (stable: rows ascending within a
 * column), scales and split plans. */
hgd_status hgd_incidence_create(const int64_t* rowptr, const int32_t* col, const float* val,
                                int64_t n_rows, int64_t n_cols, int64_t nnz,
                                hgd_incidence** out, void* stream);
/* The object of torch.nonzero(H > thresh) (HGD_DENSE_GREATER) or torch.nonzero(H)
 * (HGD_DENSE_NONZERO) of a dense [n_rows, n_cols] matrix (leading dim ld); keep_values != 0
 * keeps H's entries as values, otherwise the incidence is binary. */
hgd_status hgd_incidence_from_dense(const float* H, int64_t n_rows, int64_t n_cols, int64_t ld,
                                    float thresh, int32_t mode, int32_t keep_values,
                                    hgd_incidence** out, void* stream);
/* SpAdjDropEdge: the child keeps the nonzeros with keep_mask[e] != 0 (CSR order, nnz bytes) and
 * carries values val[e]/keep (a binary parent's values are 1, so the child's are 1/keep).
 * Built by compaction of the parent's CSR and CSC (no sort). A child cannot be dropped again
 * (the reference always drops the base adjacency). */
hgd_status hgd_incidence_dropedge(const hgd_incidence* parent, const uint8_t* keep_mask,
                                  float keep, hgd_incidence** out, void* stream);
void hgd_incidence_destroy(hgd_incidence* inc);

/* Read-only view of the object's device arrays (valid until destroy). */
typedef struct hgd_incidence_view {
  int64_t n_rows, n_cols, nnz;
  const int64_t* rowptr;  /* CSR */
  const int32_t* col;
  const float* val;       /* NULL: binary */
  const int64_t* colptr;  /* CSC */
  const int32_t* row_t;
  const float* val_t;
  const int32_t* perm_t;  /* CSC position → CSR position (NULL for a drop-edge child) */
} hgd_incidence_view;
hgd_status hgd_incidence_get_view(const hgd_incidence* inc, hgd_incidence_view* out);
/* Device pointer to the object's degree scale of one side (HGD_SIDE_ROWS / HGD_SIDE_COLS);
 * NULL for HGD_SCALE_NONE. The column scales are the global ones after
 * hgd_incidence_globalize_columns. */
hgd_status hgd_incidence_scale(const hgd_incidence* inc, int32_t side, int32_t kind,
                               const float** out);
/* Builds the per-nonzero weights conv2hop needs for source-side scales `kinds_mask`
 * (bit k = hgd_scale k) now, so that later calls allocate nothing (graph capture). */
hgd_status hgd_incidence_prepare(const hgd_incidence* inc, uint32_t kinds_mask, void* stream);

/* Workspace of hgd_incidence_spmm for width d (the split-plan partials). */
size_t hgd_incidence_workspace_size(const hgd_incidence* inc, int32_t d);
/* Y = epi(row_scale ⊙ (A·X)) (transpose = 0, Y has n_rows rows) or epi(row_scale ⊙ (Aᵀ·X))
 * (transpose = 1, served by the CSC, Y has n_cols rows); values are A's. row_scale: NULL or a
 * device array over Y's rows (e.g. from hgd_incidence_scale). */
hgd_status hgd_incidence_spmm(const hgd_incidence* inc, int32_t transpose, const float* X,
                              int64_t ldx, float* Y, int64_t ldy, int32_t d,
                              const float* row_scale, int32_t epilogue, float slope,
                              void* workspace, size_t workspace_bytes, void* stream);

/* Multi-GPU exchange: one process per GPU, users (rows of H) sharded in
 * contiguous ranges, items (columns) replicated; RCCL over xGMI. The communicator owns a side
 * stream for the chunked, overlapped all-reduce of the item sums. */
typedef struct hgd_comm hgd_comm;
#define HGD_COMM_ID_BYTES 128
/* Rank 0 creates the id (host buffer of HGD_COMM_ID_BYTES) and distributes it out of band. */
hgd_status hgd_comm_get_unique_id(void* id_out);
/* Collective over the nranks processes; binds the communicator to the current HIP device. */
hgd_status hgd_comm_create(const void* id, int32_t nranks, int32_t rank, hgd_comm** out);
void hgd_comm_destroy(hgd_comm* comm);
/* Item chunks per exchange for the overlapped hop (default 4, 1..64; RCCL transport). */
hgd_status hgd_comm_set_chunks(hgd_comm* comm, int32_t n_chunks);
/* In-place sum of a device fp32 buffer over the ranks, ordered on `stream` (over the peer
 * exchange: count a multiple of 4 <= its max_count, buf 16-byte aligned; uses send slot 0). */
hgd_status hgd_exchange_allreduce(hgd_comm* comm, float* buf, int64_t count, void* stream);
/* Replaces the object's column degrees by their sum over the ranks (each rank holds a user
 * shard of the same item set), so column scales — the Q of conv2hop — are global. Collective;
 * synchronises `stream`. */
hgd_status hgd_incidence_globalize_columns(hgd_incidence* inc, hgd_comm* comm, void* stream);

/* Direct xGMI peer exchange (SURVEY.md §8e "mesh … direct hipIpc peer kernel"), an alternative
 * transport to RCCL for the same all-reduce of the item messages: a two-shot reduce over the
 * mesh — rank r sums block r of every rank's send slot (reading the N-1 peers over their own
 * xGMI links at once, ranks summed in ascending order), then gathers the other blocks from the
 * peers' reduced slots. Every rank exposes a flag page and 2·n_slots slots of max_count floats
 * (send, then reduced) in uncached segments of at most 1 GiB (HGD_TUNE_P2P_SEGMENT_MB), each
 * through hipIpcGetMemHandle. Setup is collective out of band: create, export, exchange the
 * handles (e.g. all_gather), open. Peer reads follow a system-scope acquire and announced
 * stores a system-scope release, so correctness does not depend on how the importing device
 * caches peer memory (csrc/p2p.hip, "Memory ordering").
 * Waits are bounded (hgd_p2p_set_timeout, default 30 s): a timeout sets a device error flag
 * and a host-visible copy; hgd_p2p_poll reports it without synchronising, hgd_p2p_check after
 * a sync, and every later exchange writes NaN into its output instead of summing.
 * A slot used by exchange i may be rewritten once any later exchange j > i has completed on
 * this rank's stream; every rank must issue the same exchanges in the same order.
 * Replaces: nothing in the reference (no distributed code, HCCF.py:24); the design's own. */
typedef struct hgd_p2p hgd_p2p;
#define HGD_P2P_HANDLE_BYTES 4096
/* A communicator whose exchanges run over an OPENED peer exchange instead of RCCL (no RCCL
 * communicator; `p2p` must outlive it and is not destroyed with it). conv2hop over it pipelines
 * column slices: hop 1 of a slice writes straight into a send slot, the slot's mesh reduce runs
 * on the communicator's high-priority side stream, hop 2 of the slice waits only for it (the
 * same slices, slots and kernels as sharded.ShardedIncidence with transport 'p2p'). Needs
 * d % 4 == 0 and 2·ceil(d / width) slots of n_cols·width floats. hgd_incidence_globalize_columns
 * over it sums the degrees exactly (16-bit limbs). */
hgd_status hgd_comm_create_p2p(hgd_p2p* p2p, int32_t nranks, int32_t rank, hgd_comm** out);
/* Column-slice width of the peer-exchange pipeline: 0 = default (32 for d <= 128, else 64),
 * else a multiple of 4. */
hgd_status hgd_comm_set_slice_width(hgd_comm* comm, int32_t width);
/* nranks 1..8; max_count a positive multiple of 4 (floats per slot, at most one segment);
 * n_slots 1..1024 (at most 62 segments in all). */
hgd_status hgd_p2p_create(int32_t nranks, int32_t rank, int64_t max_count, int32_t n_slots,
                          hgd_p2p** out);
void hgd_p2p_destroy(hgd_p2p* p2p);
/* This rank's handle (HGD_P2P_HANDLE_BYTES host bytes) for its peers. */
hgd_status hgd_p2p_export(const hgd_p2p* p2p, void* handle_out);
/* `handles`: nranks × HGD_P2P_HANDLE_BYTES in rank order (this rank's own entry included).
 * Checks that every imported mapping spans the peer's whole allocation. */
hgd_status hgd_p2p_open(hgd_p2p* p2p, const void* handles);
/* Device pointer of this rank's send slot (max_count floats; write the partial sums here). */
float* hgd_p2p_slot(hgd_p2p* p2p, int32_t slot);
int32_t hgd_p2p_n_slots(const hgd_p2p* p2p);
int64_t hgd_p2p_max_count(const hgd_p2p* p2p);
hgd_status hgd_p2p_set_timeout(hgd_p2p* p2p, double seconds);
/* out[0:count) = Σ_ranks send_slot[0:count), ordered on `stream`; count a multiple of 4 and
 * out 16-byte aligned. */
hgd_status hgd_p2p_allreduce(hgd_p2p* p2p, int32_t slot, int64_t count, float* out,
                             void* stream);
/* Synchronous: HGD_OK, or HGD_ERR_HIP if any exchange timed out. */
hgd_status hgd_p2p_check(hgd_p2p* p2p);
/* Non-blocking: HGD_ERR_HIP if a wait that has already run timed out (host-visible flag). */
hgd_status hgd_p2p_poll(const hgd_p2p* p2p);
/* Pricing hook: k_reduce (rank 0's block over nranks sources) and k_gather (the other blocks) of
 * a `count`-float exchange with every peer slot a separate LOCAL allocation (uncached unless
 * `cached`), mean ms per launch over `iters` launches; synchronises `stream`. Prices the
 * kernels, not xGMI (profiles/r04_scale). */
hgd_status hgd_p2p_price_local(int32_t nranks, int64_t count, int32_t cached, int32_t iters,
                               float* ms_reduce, float* ms_gather, void* stream);
/* The block arithmetic of hgd_p2p_allreduce (host only, no device calls): rank q reduces floats
 * [*lo, *hi) of a `count`-float exchange over `nranks` ranks; gather step i of `rank` copies
 * float4 *j from rank *owner's reduced block (its own block is skipped). */
hgd_status hgd_p2p_block_range(int64_t count, int32_t nranks, int32_t q, int64_t* lo,
                               int64_t* hi);
hgd_status hgd_p2p_gather_index(int64_t count, int32_t nranks, int32_t rank, int64_t i,
                                int64_t* j, int32_t* owner);

/* The two-hop conv over the object, Y = epi(P·A·Q·Aᵀ·R·X) with P, R row scales and Q a column
 * scale (hgd_scale each):
 *   HGCNConv (HGNN_HD4.py:455-462)        P = Q = R = NONE on the weighted norm_adj
 *   ED-HNN mean pair (EquivSetConv2:88-93) P = MEAN, Q = MEAN, R = NONE on the binary V/E incidence
 *   HGNN normalisation (graph.py:28-42)    P = SYM, Q = MEAN, R = SYM (the benchmarked op)
 * Forward: hop 1 M = Q·Aᵀ·(R·X) over the CSC into the workspace (copied to saved_M when not
 * NULL), hop 2 Y = epi(P·A·M) over the CSR. An activation with slope >= 0 is fused into hop 2;
 * with slope < 0, pre_act [n_rows, d] (contiguous) receives P·A·M and Y = epi(pre_act).
 * Backward: dZ = epi'(dY) (act_ref = the forward Y when slope >= 0, else pre_act; NULL without
 * an epilogue), dM = Q·Aᵀ·(P·dZ), dX = R·A·dM — the same hops with P and R swapped.
 * comm != NULL: this rank's A is a user shard; hop 1's item sums are all-reduced (chunked and
 * overlapped on the communicator's stream over RCCL, or column-sliced over the peer exchange of
 * hgd_comm_create_p2p) before hop 2; Q must be NONE or the global
 * MEAN / SYM of hgd_incidence_globalize_columns. Epilogues with slope < 0 or dY with ldy != d
 * need contiguous rows. Workspace: hgd_conv2hop_workspace_size. */
size_t hgd_conv2hop_workspace_size(const hgd_incidence* inc, int32_t d, int32_t epilogue);
hgd_status hgd_conv2hop_forward(const hgd_incidence* inc, int32_t P, int32_t Q, int32_t R,
                                const float* X, int64_t ldx, int32_t d, float* Y, int64_t ldy,
                                int32_t epilogue, float slope, float* saved_M, float* pre_act,
                                hgd_comm* comm, void* workspace, size_t workspace_bytes,
                                void* stream);
hgd_status hgd_conv2hop_backward(const hgd_incidence* inc, int32_t P, int32_t Q, int32_t R,
                                 const float* dY, int64_t ldy, int32_t d, const float* act_ref,
                                 int32_t epilogue, float slope, float* dX, int64_t ldx,
                                 hgd_comm* comm, void* workspace, size_t workspace_bytes,
                                 void* stream);

#ifdef __cplusplus
}
#endif

#endif /* HGD_H */
