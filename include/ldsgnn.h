/*
 * ldsgnn.h — C-ABI of the MI355X-native LDS bilevel hot path.
 *
 * The reference (andreas-grafberger/lds-gnn) is pure Python/PyTorch and has no
 * FFI: its "interface" for this path is a handful of Python functions whose
 * dense ATen calls these entry points replace.  Each entry point below names
 * the reference function (file:line under /root/reference) it stands in for.
 *
 * Conventions (every function):
 *   - all array arguments are DEVICE pointers owned by the caller (PyTorch);
 *     nothing is allocated inside, workspaces are passed in explicitly;
 *   - `stream` is a hipStream_t passed as void*; NULL = the legacy stream;
 *     every launch is asynchronous and graph-capturable (no host sync, no
 *     hipMalloc, no memcpy to host);
 *   - the return value is a hipError_t cast to int (0 = hipSuccess);
 *     argument errors return hipErrorInvalidValue (1) before any launch;
 *     lds_error_string() turns a code into text.
 *   - θ ("theta") is the reference's BernoulliGraphModel.probs: the row-major
 *     upper triangle INCLUDING the diagonal of an n×n matrix, n(n+1)/2 fp32
 *     values (torch.triu_indices(n, n) order, src/utils/graph.py:41-45).
 *     Index of (i, j), i <= j:  i*(2n - i + 1)/2 + (j - i).
 *   - sampled graphs are exchanged as a symmetric bit matrix (`bits`,
 *     n rows × `words` uint64, bit j%64 of word j/64 of row i = edge (i, j),
 *     diagonal = self-loop set) and as CSR (row_ptr[n+1], col[nnz], int32,
 *     columns ascending, self-loop included) plus s = deg^-1/2 (fp32).
 */
#ifndef LDSGNN_H
#define LDSGNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LDS_ABI_VERSION 18

/* ABI version of the loaded library (== LDS_ABI_VERSION). */
int lds_abi_version(void);

/* Text for a return code (hipGetErrorString). Never NULL. */
const char* lds_error_string(int err);

/* Device error word (ABI 12).  Kernels that meet an input they cannot use
 * faithfully set bits in a caller-provided uint32 (the `err` arguments; the
 * engine's is EngineScalars.error) instead of reading through it, and the
 * host raises when it reads a non-zero word:
 *   LDS_DEVERR_FILL_DEGREE — a CSR fill (lds_sample_fill_csr,
 *     lds_sample_graphs_multi, lds_engine_fill_x_linear) found a row whose
 *     drawn bits hold a different number of entries than its degree count in
 *     deg_ws (a workspace that was not zero on entry, or counts of another
 *     draw).  row_ptr follows the counts, so the row's slots past its drawn
 *     entries are written with the row's own index (valid, never outside the
 *     graph) instead of being left as whatever col held. */
#define LDS_DEVERR_FILL_DEGREE 1u
/*   LDS_DEVERR_CSR_COLUMNS (ABI 14) — lds_spmm_norm_dense's spill-pass kernel
 *     (grid >= 0) met a row whose column order it could not aggregate
 *     faithfully (a column that belongs to a column pass it had already
 *     multiplied: the row's columns are not ascending) or a column outside
 *     [0, n).  The result is then wrong and must not be used; rows out of
 *     order only within the window the kernel places exactly give exact
 *     results without the flag. */
#define LDS_DEVERR_CSR_COLUMNS 2u
/*   LDS_DEVERR_SGD_TILE_COUNTER (round 6) — lds_sgd_sample_graphs with its
 *     samples split over several blocks per tile found a per-tile counter
 *     (tile_ctr) that was not zero on entry: a block counted past the tile's
 *     block count.  That block does not write θ; the tile's update may have
 *     been written early or not at all, so θ and the draws must not be used.
 *     The word is the engine's EngineScalars.error (the `scalars` argument). */
#define LDS_DEVERR_SGD_TILE_COUNTER 4u

/* Number of uint64 words per bitmask row for n nodes (ceil(n/64) rounded up
 * to an even count so every row starts 16-byte aligned). Host-only. */
int lds_bitmask_words(int n);

/* ---------------------------------------------------------------------------
 * RNG contract.  All randomness on the path is counter-based Philox4x32-10:
 *   key  = (seed & 0xffffffff, seed >> 32)
 *   ctr  = (column, row >> 2, tag, counter)
 *   u(row, column) = ((out[row & 3] >> 8) * 2^-24)        in [0, 1), exact fp32
 * `tag` names the consumer (graph sample, dropout site, replica), `counter`
 * the draw index.  The CPU oracle (oracle/philox.py) implements the same map.
 * Writes u for a rows×cols row-major block (ld = cols).  Test hook.
 * ------------------------------------------------------------------------- */
int lds_philox_uniform(uint64_t seed, uint32_t tag, uint32_t counter,
                       int rows, int cols, float* out, void* stream);

/* ---------------------------------------------------------------------------
 * Graph sampling.  Replaces
 *   BernoulliGraphModel.forward -> triu_values_to_symmetric_matrix
 *       (src/models/graph.py:66-67, src/utils/graph.py:166-181)
 *   Sampler.sample -> sample_graph(undirected=True, NONE, dense=False)
 *       (src/models/sampling.py:106-138, 47-79): Bernoulli(P).sample() over
 *       the upper triangle, to_undirected(from_triu_only=True)
 *       (src/utils/graph.py:27-38)
 *   add_self_loops (src/utils/graph.py:123-133) — diagonal SET to 1.
 * Edge (i, j), i < j, iff u(i, j) < clamp(theta_ij, 0, 1).  With `u_inject`
 * non-NULL, u(i, j) = u_inject[i*n + j] (an n×n row-major fp32 array, e.g.
 * torch.rand(n, n) — reproduces torch.bernoulli(P) bit-exactly).
 * Writes the full symmetric `bits` (n × words); no memset needed.
 * ------------------------------------------------------------------------- */
int lds_sample_bitmask(const float* theta, int n, uint64_t seed, uint32_t tag,
                       uint32_t counter, const float* u_inject,
                       uint64_t* bits, int words, void* stream);

/* Degree of every row of `bits` (self-loop included) and s = 1/sqrt(deg),
 * i.e. the degree half of normalize_adjacency_matrix
 * (src/utils/graph.py:146-149).  deg has n entries. */
int lds_bitmask_degree(const uint64_t* bits, int n, int words, int* deg,
                       float* s, void* stream);

/* row_ptr[0] = 0, row_ptr[i+1] = row_ptr[i] + deg[i] (n+1 entries).
 * Single-workgroup scan; n <= 2^24. */
int lds_exclusive_scan(const int* deg, int n, int* row_ptr, void* stream);

/* Column indices of every row of `bits`, ascending, at col[row_ptr[i]...].
 * `col_capacity` bounds the writes (entries past it are dropped and
 * *overflow is set to 1 when overflow != NULL). */
int lds_bitmask_fill_csr(const uint64_t* bits, int n, int words,
                         const int* row_ptr, int* col, int64_t col_capacity,
                         int* overflow, void* stream);

/* deg[i] = row_ptr[i+1] - row_ptr[i] and s = 1/sqrt(deg) for a CSR built
 * elsewhere (e.g. a fixed dataset graph, src/scripts/gcn.py:78).  deg may be
 * NULL. */
int lds_csr_degree_scale(const int* row_ptr, int n, int* deg, float* s,
                         void* stream);

/* ELL head of a graph (the engine's aggregation layout): for every row its
 * first 64 CSR entries as {j, bits of s_j} int pairs (n × 64 × 2 ints),
 * padded with {row, 0}.  lds_bitmask_fill_csr plus the ELL head (s from
 * lds_bitmask_degree). */
int lds_bitmask_fill_csr_ell(const uint64_t* bits, int n, int words,
                             const int* row_ptr, int* col, int64_t col_capacity,
                             int* overflow, const float* s, int* ell, void* stream);

/* Workspace ints per graph of lds_sample_graphs_multi (the row degrees). */
int lds_sample_ws_ints(int n);
/* The outer SGD step + clamp of lds_engine_sgd_clamp fused with the NEXT
 * window's draw from the θ it writes (`count` graphs × `samples` replicas,
 * counters / tags as lds_sample_graphs_multi, the graph counter and the f64
 * lr read from the engine's `scalars`); bits and degree counts as
 * lds_sample_graphs_multi's tile kernel (deg_ws zero on entry), no fill.
 * tile_ctr (NULL or lds_sgd_tile_ints(n) ints, zero on entry and left zero):
 * per-tile counters that let the replica samples split over more blocks
 * (the tile's last block writes the new θ); same θ and draws either way.
 * Replaces, fused: src/trainers/outer.py:78-81 (SGD + clamp after the
 * all-reduce) and the next window's src/models/sampling.py:68 draws. */
int lds_sgd_sample_graphs(float* theta, const float* grad, const void* scalars, int n, uint64_t seed,
                          uint32_t tag, uint32_t tag_step, uint32_t counter_offset, int count,
                          int samples, uint64_t* bits, int words, int* deg_ws, int* tile_ctr, void* stream);
/* Ints of lds_sgd_sample_graphs' tile counters: the triangle's 64×64 tiles. */
int lds_sgd_tile_ints(int n);

/* ----- band-sharded replicas (BASELINE config 5 at N > 1, ABI 17) -----
 * Rank b of N owns the rows [row0_b, row1_b) of the packed triangle: it
 * assembles dθ of that band from EVERY rank's factors (all-gathered), applies
 * SGD + clamp there, and draws the band's upper-triangle words of every
 * replica's next graphs; the row bands go to their owners (all-to-all), which
 * complete the lower triangle.  Replaces, sharded across ranks:
 * src/trainers/outer.py:77-84 (dθ, SGD, clamp) and src/models/sampling.py:68
 * (the next window's draws); the reference runs one replica per job
 * (configs/seml/final/lds.yaml:1-13).
 *
 * lds_sample_band_bits: the draws of the tiles of 64-row blocks row0/64 …
 * (row0 a multiple of 64, row1 too or n) for count graphs × samples
 * replicas, counters / tags / storage as lds_sample_graphs_multi; writes the
 * band's rows' words only (no transposed words below the band, no degree
 * counts).  Every bit it writes equals lds_sample_graphs_multi's. */
int lds_sample_band_bits(const float* theta, int n, uint64_t seed, uint32_t tag, uint32_t tag_step,
                         const uint32_t* counter_base, uint32_t counter_offset, int count, int samples,
                         int row0, int row1, uint64_t* bits, int words, void* stream);
/* The strict lower triangle of `graphs` bitmasks from their upper triangle
 * (diagonal words included), then degrees into deg_ws (lds_sample_ws_ints(n)
 * ints per graph) and s = deg^-1/2 ([graphs][n]): the state
 * lds_sample_graphs_multi leaves with col = NULL. */
int lds_bitmask_mirror_degree(uint64_t* bits, int n, int words, int graphs, int* deg_ws, float* s,
                              void* stream);

/* The fill launch of lds_sample_graphs_multi alone (CSR, s, ELL head of
 * `graphs` graphs whose bits and degree counts are already drawn, e.g. by
 * lds_theta_grad_sgd_draw); deg_ws as lds_sample_graphs_multi's.  col == NULL:
 * s only (graphs aggregated from their bits, lds_aggregate_bitmask; row_ptr
 * and ell may be NULL). */
int lds_sample_fill_csr(const uint64_t* bits, int n, int words, const int* deg_ws, int graphs,
                        int* row_ptr, int* col, int64_t col_stride, float* s, int* ell,
                        const uint8_t* node_flags, uint32_t* err, void* stream);

/* lds_sample_graphs for `samples` replicas at once: graph (g, b), g < count,
 * b < samples, is draw counter *counter_base + counter_offset + g with tag
 * tag + b·tag_step, stored as graph g·samples + b of the batch arrays (one
 * θ tile load per block serves all samples).  Two launches: the tile kernel
 * draws the bits and counts them (integer atomics into deg_ws: per graph
 * lds_sample_ws_ints(n) ints, the row degrees), the fill takes each row's
 * CSR offset from those counts (no scan launch) and writes row_ptr, col, s
 * and the ELL head.  deg_ws must be zero on entry: ws_zeroed = 1 promises it
 * (lds_engine_end_window clears it), 0 makes this call clear it first.
 * col == NULL: bitmask, degrees and s only — no CSR / ELL (dense graphs
 * aggregated by lds_aggregate_bitmask), degrees by a popcount pass, deg_ws
 * need not be zero; row_ptr and ell may then be NULL.  node_flags (n bytes,
 * may be NULL): each ELL entry's j field carries the neighbour's flag byte in
 * bits 24-31 (index = j & 0xFFFFFF; the engine's bit 0 = train mask, bit 1 =
 * opt mask, read by the two-hop kernels).  err (may be NULL): device error
 * word, LDS_DEVERR_FILL_DEGREE when a row's degree count (ws_zeroed = 1 with a
 * workspace that was not zero) does not match its drawn bits. */
int lds_sample_graphs_multi(const float* theta, int n, uint64_t seed, uint32_t tag,
                            uint32_t tag_step, const uint32_t* counter_base,
                            uint32_t counter_offset, int count, int samples, uint64_t* bits,
                            int words, int* deg_ws, int* row_ptr, int* col, int64_t col_stride,
                            float* s, int* ell, const uint8_t* node_flags, int ws_zeroed,
                            uint32_t* err, void* stream);
/* Batched form for a window of graphs drawn from the same θ: graph g
 * (0 <= g < count) uses draw counter *counter_base + counter_offset + g and
 * writes bits + g·n·words, deg_ws + g·lds_sample_ws_ints(n),
 * row_ptr + g·(n+1), col + g·col_stride, s + g·n and (ell != NULL)
 * ell + g·n·128.  lds_sample_graphs_multi with samples = 1, ws_zeroed = 0. */
int lds_sample_graphs(const float* theta, int n, uint64_t seed, uint32_t tag,
                      const uint32_t* counter_base, uint32_t counter_offset, int count,
                      uint64_t* bits, int words, int* deg_ws, int* row_ptr, int* col,
                      int64_t col_stride, float* s, int* ell, void* stream);

/* The four launches above in order: sample -> degree/s -> scan -> fill.
 * deg_ws: n ints of workspace. */
int lds_sample_graph(const float* theta, int n, uint64_t seed, uint32_t tag,
                     uint32_t counter, const float* u_inject, uint64_t* bits,
                     int words, int* deg_ws, int* row_ptr, int* col,
                     int64_t col_capacity, int* overflow, float* s,
                     void* stream);

/* ---------------------------------------------------------------------------
 * Normalised aggregation (the north-star kernel).  Replaces
 *   torch.mm(normalize_adjacency_matrix(A), Z)
 *       (src/models/layers.py:44 with src/utils/graph.py:136-153)
 * Y[i, :f] = s_i * sum_{j in row i} s_j * Z[j, :f]   (beta = 0)
 * Y[i, :f] += ...                                     (beta = 1)
 * Â = diag(s)·Ã·diag(s) is symmetric, so the same call gives the backward
 * dZ = Â·dY.  f <= 64.  z/y row strides ldz/ldy in elements.
 * ------------------------------------------------------------------------- */
int lds_spmm_norm(const int* row_ptr, const int* col, const float* s, int n,
                  const float* z, int f, int ldz, float* y, int ldy, int beta,
                  void* stream);

/* Long-row form of lds_spmm_norm (dense sampled graphs, ~10^4 neighbours per
 * row: BASELINE config 5), F = 16 only.  The columns are cut into
 * lds_spmm_block_count(n) blocks of 512; a workgroup stages one block of
 * s⊙Z in LDS and aggregates its rows' segments in that block; the partials
 * (part_ws: block_count × n × 16 floats, 16-B aligned) are summed in block
 * order and scaled by s_i.  bptr: n × (block_count + 1) segment starts from
 * lds_csr_block_ptr (a property of the graph: compute once per sample).
 * fp32 parity with lds_spmm_norm (different summation order). */
int lds_spmm_block_count(int n);
int lds_csr_block_ptr(const int* row_ptr, const int* col, int n, int* bptr, void* stream);
int lds_spmm_norm_blocked(const int* bptr, const int* col, const float* s, int n,
                          const float* z, int ldz, float* y, int ldy, int beta,
                          float* part_ws, void* stream);

/* Bitmask aggregation for dense sampled graphs (config 5): the same
 *   y = diag(s)·Ã·diag(s)·z  (+ y if beta)
 * as lds_spmm_norm, reading Ã as the sampler's bitmask (bits: n rows ×
 * `words` uint64, self-loops set, as lds_sample_bitmask writes it) instead of
 * CSR.  F = 16 features.  s⊙z is quantised per feature column to 32-bit fixed
 * point against its column maximum (2^-31 relative) and summed exactly on the
 * int8 matrix cores (csrc/bitagg.hip).  Replaces the same reference code as
 * lds_spmm_norm (src/models/layers.py:44, src/utils/graph.py:136-153).
 * ws: lds_bitmask_agg_ws_bytes(n) bytes of device memory. */
int64_t lds_bitmask_agg_ws_bytes(int n);
/* lds_aggregate_bitmask without its final pass: the lds_bitmask_agg_splits(n)
 * partial sums Σ_{j in split p} Ã_ij s_j z_j (n × 16 each) are left at byte
 * offset lds_bitmask_agg_part_offset(n) of ws, for a consumer that forms
 * y_i = s_i · Σ_p part_p[i] in split order (LdsBatch.agg_splits): the same
 * bits as lds_aggregate_bitmask's y with beta = 0. */
/* CSR-SpMM for dense sampled graphs (long rows, e.g. BASELINE config 5):
 * y (= or +=) diag(s)·A·diag(s)·z for the 0/1 matrix A given as CSR
 * (row_ptr, col: distinct columns per row), F = 16 features — the operator
 * of lds_spmm_norm.  The column-index stream is read once; a workgroup's
 * rows become bit rows that the int8 matrix cores multiply with the
 * fixed-point digits of s⊙z (lds_aggregate_bitmask's
 * quantisation: exact integer sums, one rounding per digit at 2^-31 of the
 * column maximum).  n <= lds_spmm_dense_max_n(); col 16-byte aligned; ws:
 * lds_spmm_dense_ws_bytes(n) bytes, 16-byte aligned.
 *   grid >= 0: the spill-pass kernel (a workgroup's rows, at most 96, swept
 *     in column passes with their bit rows in LDS: 12 waves stream 2-KB steps
 *     of col through registers and set the bits, entries past a pass go
 *     straight into the next pass's bits, 4 waves multiply the previous
 *     pass), one workgroup per CU (0) or `grid` workgroups.  Columns must be
 *     ASCENDING within each row (canonical CSR, as every sampler and fill of
 *     this library writes it).  err != NULL (the checked form): the device
 *     error word; a row whose column order the kernel cannot aggregate
 *     faithfully, or a column outside [0, n), sets LDS_DEVERR_CSR_COLUMNS
 *     there (the result is then wrong; ABI 14 — ABI 13 dropped such entries
 *     silently).  err == NULL: the caller guarantees canonical columns (the
 *     unchecked form, ~4 % faster at config 5: the fast paths test a lane's
 *     first and last column only).
 *   grid < 0: the round-3 tile kernel on -grid persistent workgroups, columns
 *     in any order (err unused, may be NULL).
 * Three launches (column maxima, digits, the product); quantize = 0 skips
 * the first two (ws holds the digits of this s, z from an earlier call).
 * Replaces torch.mm(normalize_adjacency_matrix(A), Z) (src/models/layers.py:44,
 * src/utils/graph.py:136-153).  (The non-product forms rounds 3-4 measured
 * live in the tools-only tools/variants/libldsgnn_variants.so.) */
int64_t lds_spmm_dense_ws_bytes(int n);
int lds_spmm_dense_max_n(void);
int lds_spmm_norm_dense(const int* row_ptr, const int* col, const float* s, int n, const float* z, int ldz,
                        float* y, int ldy, int beta, void* ws, int grid, int quantize, uint32_t* err,
                        void* stream);
int lds_bitmask_agg_splits(int n);
int64_t lds_bitmask_agg_part_offset(int n);
int lds_aggregate_bitmask_partials(const uint64_t* bits, int words, const float* s, int n, const float* z,
                                   int ldz, void* ws, void* stream);
int lds_aggregate_bitmask(const uint64_t* bits, int words, const float* s, int n,
                          const float* z, int ldz, float* y, int ldy, int beta,
                          void* ws, void* stream);

/* ---------------------------------------------------------------------------
 * Hypergradient assembly.  Replaces the autograd of
 *   normalize_adjacency_matrix -> straight_through_estimator ->
 *   triu_values_to_symmetric_matrix w.r.t. BernoulliGraphModel.probs
 *       (src/utils/graph.py:136-153, src/models/sampling.py:82-85,
 *        src/utils/graph.py:166-181)
 * For a cotangent dL/dÂ = sum_c G_c Z_cᵀ on one sampled graph, with
 * U = s⊙[G_1|G_2|..], V = s⊙[Z_1|Z_2|..] (n×k, row stride ld) and
 * R_i = sum_{c} r[i, c] (r: n×nr, row stride ldr; r_c,i = -½ s_i² (G_i·(ÂZ)_i + Z_i·(ÂG)_i)):
 *   g_ij = mask_ij * ( U_i·V_j + V_i·U_j + R_i + R_j )   for i < j
 *   g_ii = 0                                             (fill_diagonal_)
 * mask_ij = (0 <= theta_ij <= 1) (clamp backward) when theta != NULL, else 1.
 * accumulate = 0: grad = g;  accumulate = 1: grad += g.
 * ------------------------------------------------------------------------- */
int lds_theta_grad(const float* u, const float* v, int ld, int k,
                   const float* r, int ldr, int nr, const float* theta, int n,
                   float* grad, int accumulate, int form, void* stream);

/* The same update on the fp32 VALU (the MFMA form above is the default);
 * kept for A/B timing. */
int lds_theta_grad_valu(const float* u, const float* v, int ld, int k,
                        const float* r, int ldr, int nr, const float* theta, int n,
                        float* grad, int accumulate, void* stream);

/* lds_theta_grad fused with the outer update (single replica):
 *   θ_ij = clamp(θ_ij - lr·g_ij, 0, 1),  lr = the engine scalars' outer_lr
 * (`scalars`: EngineScalars, see "Fused engine" below); grad = g when
 * grad != NULL.  Replaces loss.backward → SGD.step → clamp_
 * (src/trainers/outer.py:77-83) for one hyper step. */
int lds_theta_grad_sgd(const float* u, const float* v, int ld, int k,
                       const float* r, int ldr, int nr, float* theta, int n,
                       float* grad, const void* scalars, int form, void* stream);

/* lds_theta_grad_sgd for the last column chunk of a split assembly: grad
 * holds the sum of the earlier chunks (lds_theta_grad with accumulate, no R,
 * theta NULL); g = grad + this chunk + R_i + R_j (clamp mask on θ), grad = g,
 * θ = clamp(θ - lr·g, 0, 1).  Lets the chunks of finished graphs run on a side
 * stream while the reverse pass continues. */
int lds_theta_grad_sgd_accum(const float* u, const float* v, int ld, int k,
                             const float* r, int ldr, int nr, float* theta, int n,
                             float* grad, const void* scalars, int form, void* stream);

/* lds_theta_grad_sgd (split-bf16; see `form` below) that also draws
 * the NEXT window's `graphs` graphs from the θ it writes: graph g takes draw
 * counter counter_offset + g (+ *counter_base when non-NULL), bits and degree
 * accumulators as lds_sample_graphs_multi's tile kernel (deg_ws zero on
 * entry, lds_sample_ws_ints(n) ints per graph); the CSR fill is left to the
 * caller.  Requires ld % 4 == 0, k % 8 == 0 and 16-byte aligned u, v.
 * Replaces, fused: src/trainers/outer.py:77-81 (backward + SGD + clamp) and the
 * next window's src/models/sampling.py:68 draws. */
int lds_theta_grad_sgd_draw(const float* u, const float* v, int ld, int k,
                            const float* r, int ldr, int nr, float* theta, int n,
                            float* grad, const void* scalars, uint64_t seed, uint32_t tag,
                            const uint32_t* counter_base, uint32_t counter_offset, int graphs,
                            uint64_t* bits, int words, int* deg_ws, int form, void* stream);

/* General form of the assembly, for S replica samples per GPU (their factor
 * blocks side by side in U, V: k = S·ldk columns):
 *   g_ij = gscale · (Σ_c U_ic V_jc + V_ic U_jc + R_i + R_j),  i < j,
 *   R_i  = Σ_{c<nr} r[i·ldr_row + c·ldr_col]   (ldr_col = n: S stacked rows)
 * gscale = 1/S makes g the mean of the S replica hypergradients (the mean
 * OuterProblemTrainer.train_step's loss over S samples would give).
 * mode 0 grad = g; 1 grad += g; 2 θ = clamp(θ - lr·g, 0, 1) (+ grad = g when
 * grad != NULL); 3 as 2 with g += grad first.  lr from `scalars` (modes 2, 3). */
int lds_theta_grad_ex(const float* u, const float* v, int ld, int k, const float* r,
                      int ldr_row, int ldr_col, int nr, float* theta, int n, float* grad,
                      int mode, const void* scalars, float gscale, int form, void* stream);
/* lds_theta_grad_ex over the packed triangle's rows [row0, row1) only (the
 * band-sharded exchange, ABI 17): their 128-row block tiles, every column
 * block from the diagonal on, in the plain split-bf16 128-tile form; row0 a
 * multiple of 128, row1 too or n; mode 0 (dθ of the band) or 2 (fused SGD +
 * clamp of the band).  Each entry gets the bits the full launch gives it. */
int lds_theta_grad_band(const float* u, const float* v, int ld, int k, const float* r, int ldr_row,
                        int ldr_col, int nr, float* theta, int n, float* grad, int mode,
                        const void* scalars, float gscale, int row0, int row1, void* stream);
/* lds_theta_grad_ex on pre-split operands: every fp32 value x of U and V as
 * its three truncation-split bf16 words x = hi + mid + lo (lds_split_planes
 * makes them from fp32; the engine's factor producers write them directly),
 * so the staging copies instead of splitting.  Chunk-major layout: columns
 * 16c .. 16c+15 of row i are [hi ×16 | mid ×16 | lo ×16] (uint16) at offset
 * (c·n + i)·48.  Same arithmetic and result bits as the fp32-operand form.
 * k a multiple of 8 (columns past k in its last chunk are ignored), ld >= k
 * bounds the chunks, up / vp 16-byte aligned. */
int lds_theta_grad_planes(const uint16_t* up, const uint16_t* vp, int ld, int k, const float* r,
                          int ldr_row, int ldr_col, int nr, float* theta, int n, float* grad, int mode,
                          const void* scalars, float gscale, int form, void* stream);
/* The chunk-major split words of the first k columns of x (rows × ld fp32)
 * into planes (ceil(k/16) chunks of rows × 48 uint16). */
int lds_split_planes(const float* x, int rows, int ld, int k, uint16_t* planes, void* stream);
/* Form 10 of the assembly (round 3): the eight-wave 128 × 128 tile staged by
 * direct global -> LDS loads of pre-split operands, three stage buffers in
 * flight.  up / vp: the split words of U and V in the 128-row-tile layout of
 * lds_split_planes_t128 (made for these n rows and k columns).  Modes and
 * arguments as lds_theta_grad_ex; graphs > 0 (mode 2 only) also draws the
 * next window's graphs from the θ it writes, as lds_theta_grad_sgd_draw
 * (words even, >= 2·ceil(n/128)).  Same result bits as every split-bf16 form.
 * Replaces, fused: src/trainers/outer.py:77-81 and src/models/sampling.py:68. */
int lds_theta_grad_direct(const uint16_t* up, const uint16_t* vp, int k, const float* r, int ldr_row,
                          int ldr_col, int nr, float* theta, int n, float* grad, int mode,
                          const void* scalars, float gscale, uint64_t seed, uint32_t tag,
                          const uint32_t* counter_base, uint32_t counter_offset, int graphs,
                          uint64_t* bits, int words, int* deg_ws, void* stream);
/* uint16 count of the form-10 planes of `rows` rows × k columns:
 * ceil(k/16) · ceil(rows/128) · 6144.  Host-only. */
int64_t lds_planes_t128_elems(int rows, int k);
/* x (rows × ld fp32, first k columns) -> its form-10 planes: value x(i, kk),
 * word s (0 hi, 1 mid, 2 lo) at uint16 offset
 *   (((c·nt + T)·3 + s)·128 + r)·16 + 8·(h ^ ((r >> 3) & 1)) + (kk & 7),
 * c = kk >> 4, T = i >> 7, r = i & 127, h = (kk >> 3) & 1, nt = ceil(rows/128);
 * rows and columns past the ends are written as zeros.  planes 16-byte aligned. */
int lds_split_planes_t128(const float* x, int rows, int ld, int k, uint16_t* planes, void* stream);
/* `form`: the arithmetic form of every θ-gradient assembly above, chosen per
 * call (no process-wide state; a captured HIP graph holds the form it was
 * captured with in its launch):
 *   0 fp32 MFMA (v_mfma_f32_32x32x2_f32, exact fp32 FMA chains);
 *   1 split-bf16 MFMA, tile shape by problem size (the default): each fp32
 *     operand as three bf16 words, six v_mfma_f32_32x32x16_bf16 per product
 *     (fp32 accuracy, |error| <= ~2^-22 |U||V| per term, fp32 accumulation);
 *   2 split-bf16, 64 × 64 tiles, 16-wide k chunks;  3 the same, 32-wide;
 *   4 split-bf16, 128 × 128 tiles;  5 the same in XCD-grouped tile order;
 *   6 form 2 in XCD-grouped tile order;
 *   7 form 5 with 64-bit packed-index arithmetic at every n (the path n > 46 340
 *     takes; for testing);
 *   8 the software-pipelined 128 × 128 form (double-buffered stage);
 *   9 the eight-wave pipelined 128 × 128 form (64 × 32 wave tiles).
 * Every split-bf16 form gives bit-identical results.  lds_theta_grad_sgd_draw
 * runs form 9 when asked for it and the 64-tile form (6) otherwise. */

/* Slot factors for lds_theta_grad from one aggregation Y = ÂZ and its
 * cotangent G (dZ = ÂG):  U = s⊙G, V = s⊙Z, r = -½ s² (G·Y + Z·dZ) rowwise.
 * Columns [f, fpad) of U and V are zero-filled. */
int lds_slot_factors(const float* g, int ldg, const float* z, int ldz,
                     const float* y, int ldy, const float* dz, int lddz,
                     const float* s, int n, int f, int fpad, float* u, int ldu,
                     float* v, int ldv, float* r, int ldr, void* stream);

/* ---------------------------------------------------------------------------
 * Outer update.  Replaces SGD.step (no momentum) + ParameterClamper
 *   (src/trainers/outer.py:78-83, src/models/graph.py:16-20, 63-64):
 *   theta = clamp(theta - lr * grad, 0, 1)
 * ------------------------------------------------------------------------- */
int lds_sgd_clamp(float* theta, const float* grad, float lr, int64_t count,
                  void* stream);

/* ---------------------------------------------------------------------------
 * Keyed dropout.  Replaces F.dropout (src/models/gcn.py:27,29):
 *   y = x * (u(i, j) < 1 - p ? 1/(1-p) : 0)     element (i, j) of a rows×cols
 * block (row strides ldx, ldy).  Linear in x, so the same call with the same
 * key is its own backward.  `scale` = float(1) / float(1 - p).
 * ------------------------------------------------------------------------- */
int lds_dropout(const float* x, int ldx, float* y, int ldy, int rows, int cols,
                float keep_prob, float scale, uint64_t seed, uint32_t tag,
                uint32_t counter, void* stream);

/* ---------------------------------------------------------------------------
 * θ pre-training (Pretrainer.train_step, src/trainers/pretrainer.py:68-81, used
 * when OuterProblemTrainer(pretrain=True), src/trainers/outer.py:54-55,107-109):
 * one epoch of weighted BCE between P = triu_values_to_symmetric_matrix(θ)
 * and the training adjacency T (train_bits: n × words uint64 bitmask, the
 * sampler's layout), W = 1 + T·(pos_weight - 1), mean over n², followed by
 * torch.optim.Adam (lr, betas, eps; no weight decay) on the packed θ, in one
 * pass.  `step` = the Adam step count after this update (>= 1).
 * loss_rows[i] receives row i's Σ w·bce terms (loss = Σ_i loss_rows[i] / n²).
 * ------------------------------------------------------------------------- */
int lds_pretrain_step(float* theta, int n, const uint64_t* train_bits, int words, float pos_weight,
                      float* exp_avg, float* exp_avg_sq, int step, double lr, double beta1,
                      double beta2, double eps, float* loss_rows, void* stream);

/* ---------------------------------------------------------------------------
 * Fused engine (lds-gnn_amd/csrc/engine.hip; orchestrated by
 * lds-gnn_amd/ldsgnn/engine.py).  Replaces, for the LDS configuration, the
 * autograd work of
 *   InnerProblemTrainer.train_step + higher.DifferentiableAdam.step
 *       (src/trainers/inner.py:55-74, create_graph=True)
 *   OuterProblemTrainer.train_step's loss.backward through the unrolled
 *       window (src/trainers/outer.py:57-87) and the SGD/StepLR/clamp that
 *       follow (src/trainers/outer.py:78-83, src/models/graph.py:63-64)
 * with hand-derived forward / backward / reverse kernels.
 * Per-node arrays are n × 16 fp32 (hidden width 16; c <= 16 classes padded to
 * 16 columns).  `scalars` points to the engine's device-resident
 * EngineScalars {u32 graph_ctr, u32 fwd_ctr, i32 adam_step, i32 hyper_steps,
 * f64 outer_lr, f64 lr_decay, u32 error, u32 pad} (lds_engine_scalars_size()
 * bytes; `error` is the engine's device error word, LDS_DEVERR_*); kernels read
 * the RNG counters / Adam step / lr from it so one captured HIP graph of a
 * whole τ-window replays with advancing state.  `fwd_off`, `step_off` are
 * offsets added to those counters.  Factor outputs (U, V, R) feed
 * lds_theta_grad with ld = ldk.
 * ------------------------------------------------------------------------- */
int lds_engine_scalars_size(void);

/* Replica-sample batching (config "S Monte-Carlo samples per GPU"): the
 * engine entries taking `const LdsBatch* batch` run `samples` independent
 * replicas in one launch (grid.y = sample).  Sample b reads / writes every
 * per-sample array at base + b·stride (strides in elements of the array's
 * type; 0 = shared by all samples) and draws its dropout masks with the
 * replica tags tag_x / tag_h + b·tag_step.  Shared: X, labels, masks, θ, the
 * scalars (every replica advances them identically) and the Adam table.
 * batch == NULL (or samples == 1) is the single-replica launch.
 *
 * `agg` (the aggregating entry points: fwd_layer1/2, bwd_layer2, bwd1_reduce,
 * rev_a..c, rev_d_reduce): NULL = aggregate Â·Z from the CSR inside the
 * kernel (short rows); non-NULL = read the precomputed Â·Z (n × 16, same
 * batching as the activations) — long rows (config 5), where
 * lds_spmm_norm_blocked runs as a pre-pass.
 *   act : n×16 activation / adjoint arrays      row : n-vectors (s, R, loss rows)
 *   rp  : row_ptr (n+1)   col : CSR capacity     ell : ELL head (n·128 int32)
 *   par : flat parameter vectors (w, m, v, g', adjoints)
 *   xval: the X-values argument (0 when it is the shared X, else the Xd stride)
 *   xd  : stored Xd arrays (CSR / CSC order)
 *   uv  : factor COLUMN offset per sample (U, V are n × (samples·ldk); the
 *         ldk argument is then the row stride samples·ldk)
 *   part: reduction partials   met: metrics rows (2 floats) */
typedef struct LdsBatch {
    int32_t samples;
    uint32_t tag_step;
    int64_t act, row, rp, col, ell, par, xval, xd, uv, part, met;
    /* Row plan of the aggregating entry points (may be empty: n_heavy = 0).
     * Every row gets one wave, except the n_heavy rows listed in heavy_rows
     * (heavy_flag[row] = 1; rows expected to have more than 64 entries), which
     * run on a block of their own appended after the one-wave-per-row blocks,
     * all the block's waves splitting the row's entries.  The plan changes
     * speed only: any row is aggregated correctly either way.  With a plan the
     * fused reductions write ceil(n / 16) + n_heavy partials. */
    const int32_t* heavy_rows;
    const uint8_t* heavy_flag;
    int32_t n_heavy;
    /* > 0: the precomputed aggregation `agg` an entry point is given holds
     * agg_splits partial arrays (n × 16 each, consecutive): the kernel takes
     * Â·Z[i] = s_i · Σ_p agg_p[i] (p in order) — lds_aggregate_bitmask_partials
     * output, its final pass folded into the consumer.  0: agg is Â·Z. */
    int32_t agg_splits;
    /* ABI 11: lds_engine_xt_adam over pairs of samples (two per wave sharing
     * one walk of X's column indices; same sums): 0 by shape, 1 off, 2 on
     * (needs an even sample count, no heavy columns, column heads, no
     * xt_part, train == 0). */
    int32_t xt_pair;
} LdsBatch;

/* lds_sample_bitmask with the draw counter read from device memory:
 * counter = *counter_base + counter_offset. */
int lds_sample_bitmask_dev(const float* theta, int n, uint64_t seed, uint32_t tag,
                           const uint32_t* counter_base, uint32_t counter_offset,
                           uint64_t* bits, int words, void* stream);

/* H0 = dropout(X) W0ᵀ + b0 (X in CSR; wt = W0ᵀ as [fin][16]).  When
 * xd_csr != NULL the dropped values are also stored in CSR order, and when
 * xd_csc != NULL scattered to CSC order via csr2csc (position of each CSR entry
 * in the CSC arrays) — later products of the same step read them with
 * train = 0 instead of redrawing the mask.  xhead != NULL: the rows' heads
 * (built once per X) replace the row-pointer load: xinfo[row] = {p0, nnz}
 * (int pairs), xhead[row] = the row's first 64 entries as {column, value bits}
 * int pairs (zero-padded); head_vals = 1 takes the values from the head (X
 * itself), 0 from xval[p0 + e] (e.g. the stored Xd); entries past 64 come
 * from xcol / xval. */
int lds_engine_x_linear(const int* xrp, const int* xcol, const float* xval, int n,
                        const float* wt, const float* bias, float* out, uint64_t seed,
                        uint32_t tag_x, const void* scalars, int fwd_off, int train,
                        float keep, float scale, float* xd_csr, float* xd_csc,
                        const int* csr2csc, const int* xhead, const int* xinfo, int head_vals,
                        const LdsBatch* batch, void* stream);
/* lds_sample_fill_csr (CSR, s, ELL head of `graphs` drawn graphs) and
 * lds_engine_x_linear (every replica sample of `batch`) in ONE launch: the first inner
 * step's X product does not read the window's graphs, so a window that starts
 * from prefetched draws runs both halves side by side (blocks split by role)
 * with one dependent boundary instead of two.  Arguments as the two calls;
 * the fill reports into the scalars' error word. */
int lds_engine_fill_x_linear(const uint64_t* bits, int words, const int* deg_ws, int graphs,
                             int* row_ptr, int* col, int64_t col_stride, float* s, int* ell,
                             const uint8_t* node_flags, const int* xrp, const int* xcol,
                             const float* xval, int n, const float* wt, const float* bias, float* out,
                             uint64_t seed, uint32_t tag_x, const void* scalars, int fwd_off, int train,
                             float keep, float scale, float* xd_csr, float* xd_csc, const int* csr2csc,
                             const int* xhead, const int* xinfo, int head_vals, const LdsBatch* batch,
                             void* stream);
/* out[f][:] (+)= Σ_i dropout(X)[i][f] · d[i][:]  (+ wd · w)   (X in CSC). */
int lds_engine_xt_linear(const int* xcp, const int* xrow, const float* xval, int fin,
                         const float* d, float* out, const float* w, float wd,
                         int accumulate, uint64_t seed, uint32_t tag_x,
                         const void* scalars, int fwd_off, int train, float keep,
                         float scale, void* stream);
/* Y0 = ÂH0; H1d = dropout(relu(Y0)); H2 = H1d W1ᵀ + b1.  dmask (may be
 * NULL) receives D1 ⊙ [Y0 > 0] / keep, the Jacobian mask of relu + dropout,
 * which lds_engine_bwd_layer2 / rev_a / rev_c read instead of y0 + RNG. */
int lds_engine_fwd_layer1(const int* rp, const int* col, const float* s, const int* ell, int n,
                          const float* h0, float* y0, float* h1d, float* h2,
                          const float* w1, const float* b1, int c, uint64_t seed,
                          uint32_t tag_h, const void* scalars, int fwd_off, int train,
                          float keep, float scale, float* dmask, const float* agg, const LdsBatch* batch, void* stream);
/* O = ÂH2; P = softmax(O); dO = (P - onehot) ⊙ mask · inv_count; per-row
 * NLL and correctness where mask. */
int lds_engine_fwd_layer2(const int* rp, const int* col, const float* s, const int* ell, int n,
                          const float* h2, float* o, float* p, float* d_o,
                          const int* label, const uint8_t* mask, float inv_count,
                          float* lossrow, float* corrrow, int c, const float* agg, const LdsBatch* batch, void* stream);
/* dH2 = ÂdO; dY0 = (dH2 W1) ⊙ dropout' ⊙ relu'.  U != NULL: emit the outer
 * graph's factor (dO, H2) at columns [foff, foff + fwidth); r_assign != 0
 * writes R (first emitter of a window) instead of accumulating into it. */
int lds_engine_bwd_layer2(const int* rp, const int* col, const float* s, const int* ell, int n,
                          const float* d_o, const float* y0, float* dh2, float* dy0,
                          const float* w1, int c, uint64_t seed, uint32_t tag_h,
                          const void* scalars, int fwd_off, int train, float keep,
                          float scale, const float* o, const float* h2, float* U,
                          float* V, int ldk, float* R, int foff, int fwidth,
                          int r_assign, const float* dmask, const float* agg, const LdsBatch* batch, void* stream);
/* dH0 = ÂdY0.  U != NULL: emit the outer graph's factor (dY0, H0). */
int lds_engine_bwd_layer1(const int* rp, const int* col, const float* s, const int* ell, int n,
                          const float* dy0, float* dh0, const float* y0,
                          const float* h0, float* U, float* V, int ldk, float* R,
                          int foff, void* stream);
/* Deterministic two-stage column reductions over nodes (see engine.hip). */
int lds_engine_colreduce(int n, int c_n, const float* a1, const float* b1,
                         const float* a2, const float* b2, const float* x1,
                         const float* x2, const float* l, const float* q,
                         float* partials, int nblocks, float* dst_a, float* dst_v1,
                         int v1_width, float* dst_v2, int v2_width, float* dst_l,
                         int accumulate, void* stream);
/* higher's differentiable-Adam step, forward and reverse, per parameter.
 * hyper = {lr, beta1, beta2, eps, weight_decay} (host doubles); betas_dev =
 * {beta1, beta2, lr} (device doubles); params [0, n_wd) carry weight decay. */
int lds_engine_adam(int np, const float* w0, const float* g, const float* m0,
                    const float* v0, float* w1, float* m1, float* v1, float* gp_out,
                    const double* hyper, const double* betas_dev, int n_wd,
                    const void* scalars, int step_off, void* stream);
int lds_engine_adam_reverse(int np, float* wbar, float* mbar, float* vbar,
                            const float* m1, const float* v1, const float* gp,
                            float* gbar, const double* hyper, const double* betas_dev,
                            int n_wd, const void* scalars, int step_off, void* stream);
/* Reverse of the inner backward (Hessian-vector part): aggregation kernels
 * a (dY0bar = ÂdH0bar), b (dObar = ÂdH2bar), c (H2bar = ÂObar),
 * d (H0bar = ÂY0bar), each emitting its use's factor pair. */
int lds_engine_rev_a(const int* rp, const int* col, const float* s, const int* ell, int n,
                     const float* dh0bar, const float* dy0, const float* dh0,
                     const float* y0, const float* h1d, const float* dh2, const float* w1,
                     const float* gw1bar, const float* gb1bar, int c, float* dh1dbar,
                     float* dh2bar, float* h1dbar, uint64_t seed, uint32_t tag_h,
                     const void* scalars, int fwd_off, int train, float keep, float scale,
                     float* U, float* V, int ldk, float* R, int foff, const float* dmask,
                     const float* agg, const LdsBatch* batch, void* stream);
int lds_engine_rev_b(const int* rp, const int* col, const float* s, const int* ell, int n,
                     const float* dh2bar, const float* d_o, const float* dh2,
                     const float* p, const uint8_t* mask, float inv_count, int c,
                     float* obar, float* U, float* V, int ldk, float* R, int foff,
                     int cw, const float* agg, const LdsBatch* batch, void* stream);
int lds_engine_rev_c(const int* rp, const int* col, const float* s, const int* ell, int n,
                     const float* obar, const float* h2, const float* o,
                     const float* h1dbar_part, const float* y0, const float* w1, int c,
                     float* h2bar, float* y0bar, uint64_t seed, uint32_t tag_h,
                     const void* scalars, int fwd_off, int train, float keep, float scale,
                     float* U, float* V, int ldk, float* R, int foff, int cw,
                     const float* dmask, const float* agg, const LdsBatch* batch, void* stream);
int lds_engine_rev_d(const int* rp, const int* col, const float* s, const int* ell, int n,
                     const float* y0bar, const float* h0, const float* y0,
                     float* h0bar, float* U, float* V, int ldk, float* R, int foff,
                     void* stream);
/* Two-hop loss layer (the forward's last aggregation and the backward's
 * first, one launch; src/models/gcn.py:33-34 + F.nll_loss over the mask,
 * src/trainers/inner.py:65): the loss rows are the nodes whose flag byte
 * (the ELL j field's bits 24-31, lds_sample_graphs_multi node_flags) has
 * mask_bit set.  O, P, dO, loss and correctness at those rows (zeros
 * elsewhere), dH2 = Â dO computed from the masked neighbours only (their O
 * recomputed in-kernel), dY0 as lds_engine_bwd_layer2, and (U != NULL) factor
 * use 2.  Needs the ELL head (short rows). */
int lds_engine_fwd2_bwd2(const int* rp, const int* col, const float* s, const int* ell, int n,
                         const uint8_t* node_flags, int mask_bit, const float* h2, float* o, float* p,
                         float* d_o, const int* label, float inv_count, float* lossrow, float* corrrow,
                         int c, const float* y0, float* dh2, float* dy0, const float* w1, uint64_t seed,
                         uint32_t tag_h, const void* scalars, int fwd_off, int train, float keep,
                         float scale, float* U, float* V, int ldk, float* R, int foff, int fwidth,
                         int r_assign, const float* dmask, const LdsBatch* batch, void* stream);
/* lds_engine_rev_b + lds_engine_rev_c in one launch (the masked neighbours'
 * dŌ / Ōbar recomputed in-kernel): factor uses 3 (columns foff_b) and 2
 * (foff_c), R += r3 then += r2, H2bar, Y0bar. */
int lds_engine_rev_bc(const int* rp, const int* col, const float* s, const int* ell, int n,
                      const uint8_t* node_flags, int mask_bit, const float* dh2bar, const float* d_o,
                      const float* dh2, const float* p, const float* h2, const float* o, float inv_count,
                      int c, const float* h1dbar_part, const float* y0, const float* w1, float* h2bar,
                      float* y0bar, uint64_t seed, uint32_t tag_h, const void* scalars, int fwd_off,
                      int train, float keep, float scale, float* U, float* V, int ldk, float* R,
                      int foff_b, int foff_c, int cw, const float* dmask, const LdsBatch* batch,
                      void* stream);
/* θ = clamp(θ - lr·grad, 0, 1) with lr = scalars->outer_lr. */
int lds_engine_sgd_clamp(float* theta, const float* grad, int64_t count,
                         const void* scalars, void* stream);
/* Advance the scalars: counters += (graphs, forwards), adam_step +=
 * adam_steps, and `hypers` times {hyper_steps += 1; outer_lr *= lr_decay}. */
int lds_engine_advance(void* scalars, int graphs, int forwards, int adam_steps,
                       int hypers, void* stream);

/* ----- fused engine forms (fewer launches per τ-window) -----
 * Replaces, per inner step, the reference's loss.backward(create_graph=True)
 * + DifferentiableAdam.step (src/trainers/inner.py:64-72) and, per reversed
 * step, the corresponding part of the outer loss.backward through the unrolled
 * window (src/trainers/outer.py:70-80).
 *
 * Adam arguments common to lds_engine_final / lds_engine_xt_adam
 * (adam_mode 0 none, 1 forward, 2 reverse; pointers are whole flat parameter
 * vectors):
 *   mode 1: w0, m0, v0 -> w1, m1, v1 and g' (= g + wd·w) into gp;
 *   mode 2: reverse of the step with post-state m1, v1 and g' gp: the
 *           completed entry is the adjoint of w1; writes gbar, mbar, vbar
 *           (read as 0 when `first`), wbar (+ wd·ḡ in the decayed group).
 * The step's bias-corrected constants come from the Adam table (adam_tab,
 * 2 floats per step offset: {lr/(1-β1^k), sqrt(1-β2^k)}, k = adam_step + 1 +
 * step_off), written by lds_engine_adam_table / lds_engine_end_window;
 * step_off < 256. */

/* dH0 = ÂdY0 (+ outer factor (dY0, H0) when U != NULL) fused with the first
 * stage of {gW1 = dH2ᵀH1d, gb0 = ΣdH0, gb1 = ΣdH2, Σloss, Σcorrect}:
 * ceil(n/64) partials of 304 floats. */
int lds_engine_bwd1_reduce(const int* rp, const int* col, const float* s, const int* ell, int n,
                           const float* dy0, float* dh0, const float* y0, const float* h0,
                           float* U, float* V, int ldk, float* R, int foff,
                           const float* dh2, const float* h1d, const float* lossrow,
                           const float* corrrow, int c, float* partials, const float* agg, const LdsBatch* batch, void* stream);
/* H0bar = ÂY0bar (+ factor use 1) fused with the first stage of
 * {W̄1 += dH2ᵀdH1dbar + H2barᵀH1d, b̄0 += ΣH0bar, b̄1 += ΣH2bar}. */
int lds_engine_rev_d_reduce(const int* rp, const int* col, const float* s, const int* ell, int n,
                            const float* y0bar, const float* h0, const float* y0,
                            float* h0bar, float* U, float* V, int ldk, float* R, int foff,
                            const float* dh2, const float* dh1dbar, const float* h2bar,
                            const float* h1d, int c, float* partials, const float* agg, const LdsBatch* batch, void* stream);
/* Final stage: partials -> dst (flat parameter layout; = or +=), metrics[0..1]
 * (may be NULL), then Adam (mode) on b0 / W1 / b1. */
int lds_engine_final(const float* partials, int nblocks, int c, float* dst, int off_b0,
                     int off_w1, int off_b1, int accumulate, float* metrics, int adam_mode,
                     int first, const float* w0, const float* m0, const float* v0, float* w1,
                     float* m1, float* v1, float* gp, float* wbar, float* mbar, float* vbar,
                     float* gbar, const double* hyper, const float* adam_tab, int n_wd,
                     const void* scalars, int step_off, void* stream);
/* out: flat parameter-shaped buffer.  Its W0ᵀ part (= or +=) Xdᵀ d (the W0
 * gradient / adjoint), then Adam (mode) on it.  With partials != NULL the same
 * launch also runs the final stage of the fused reduction (as lds_engine_final
 * with dst = out), so one launch completes every parameter.  xt_part != NULL:
 * Xdᵀ d is read as the xt_splits partials of lds_engine_xt_partials (summed in
 * range order) instead of running the column products.  `order` (fin ints) is
 * the column plan: the first n_heavy entries are the columns with more than
 * 128 entries, each run by a whole 1024-thread block (16 waves over its entry
 * range, partials summed in wave order), then every other column, one wave
 * each (n_heavy = 0 with xt_part).  xtinfo != NULL: per plan slot s,
 * xtinfo[s] = {column, p0, nnz, 0} (int4) replaces order[s] -> xcp loads,
 * and xthead[s] (128 ints since ABI 18, NULL allowed) holds the column's
 * first 128 row indices, zero past its end (values from xval[p0 + e]).  ABI 15: after the heavy slots,
 * n_single slots run one column per wave, the next n_pair (columns of at most
 * 32 entries) two per wave and the rest (at most 16 entries) four per wave —
 * the same sums; n_single = fin - n_heavy, n_pair = 0 is the one-per-wave
 * plan, the only one allowed without xthead, with xt_part or with train. */
int lds_engine_xt_adam(const int* xcp, const int* xrow, const float* xval, int fin,
                       const float* d, float* out, int accumulate, uint64_t seed,
                       uint32_t tag_x, const void* scalars, int fwd_off, int train, float keep,
                       float scale, const float* partials, int nblocks, int c, int off_b0,
                       int off_w1, int off_b1, float* metrics, int adam_mode, int first,
                       const float* w0, const float* m0, const float* v0, float* w1, float* m1,
                       float* v1, float* gp, float* wbar, float* mbar, float* vbar, float* gbar,
                       const double* hyper, const float* adam_tab, int n_wd, int step_off,
                       const float* xt_part, int xt_splits, const int* order, int n_heavy,
                       const int* xtinfo, const int* xthead, int n_single, int n_pair,
                       const LdsBatch* batch, void* stream);
/* Long X columns (dense X, config 5): Xdᵀ d over `splits` entry ranges of every
 * column, one wave each; part[s][p][f][16] per replica sample s (stride
 * splits·fin·16).  Feeds lds_engine_xt_adam's xt_part. */
int lds_engine_xt_partials(const int* xcp, const int* xrow, const float* xval, int fin,
                           const float* d, uint64_t seed, uint32_t tag_x, const void* scalars,
                           int fwd_off, int train, float keep, float scale, int splits, float* part,
                           const LdsBatch* batch, void* stream);
/* Window end (both trainers' detach, src/trainers/bilevel.py:109-114): copy
 * w/m/v of slot T to slot 0 (skipped when wT == NULL), advance the scalars
 * as lds_engine_advance, (adam_tab != NULL) refresh the first tab_count
 * entries of the Adam table for the new adam_step, and zero ws_count ints at
 * ws (the next window's sampler workspace, lds_sample_graphs_multi
 * ws_zeroed = 1; ws may be NULL). */
int lds_engine_end_window(int np, const float* wT, const float* mT, const float* vT,
                          float* w0, float* m0, float* v0, void* scalars, int graphs,
                          int forwards, int adam_steps, int hypers, const double* betas_dev,
                          float* adam_tab, int tab_count, int* ws, int* ws_src, int64_t ws_count,
                          const LdsBatch* batch, void* stream);
/* Adam table for the current scalars->adam_step (betas_dev = {β1, β2, lr}
 * doubles): entry k = {lr/(1-β1^(s+1+k)), sqrt(1-β2^(s+1+k))}, k < tab_count
 * <= 256; the constants of torch/higher's Adam, computed in double. */
int lds_engine_adam_table(const void* scalars, const double* betas_dev, float* adam_tab,
                          int tab_count, void* stream);

/* ---------------------------------------------------------------------------
 * Captured-graph check (host only).  counts[t] = the number of nodes of HIP
 * graph type t (hipGraphNodeType: 0 kernel, 1 memcpy, 2 memset, 5 empty, …)
 * in `graph` (a hipGraph_t, e.g. torch.cuda.CUDAGraph(keep_graph=True)
 * .raw_cuda_graph()), t < ncounts - 1; the last slot counts the types past
 * the array.  The engine refuses a captured step or window that holds
 * anything but kernel and empty nodes.
 * ------------------------------------------------------------------------- */
int lds_graph_node_census(void* graph, int* counts, int ncounts);
/* Upload an instantiated graph's executable (hipGraphUpload) on `stream`, so
 * its first replay does not pay the one-time upload: the engine uploads every
 * sealed capture before the first replay.  Host only. */
int lds_graph_upload(void* graph_exec, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* LDSGNN_H */
