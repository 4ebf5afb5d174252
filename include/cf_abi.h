/*
 * cf_abi.h -- C ABI of libcf_mi355x.so, the MI355X-native hot path of
 * Dhole/collaborative_filtering (per-user local-graph Laplacian eigendecomposition,
 * graph-signal rating prediction, kNN item similarity).
 *
 * Conventions
 *   - Every entry point returns CF_OK (0) or a negative CF_E* code; a message is
 *     available from cf_last_error(ctx).  No C++ exception crosses this boundary.
 *   - Plain pointers and sizes only.  Functions without a suffix take HOST pointers
 *     (caller-owned, copied in/out, synchronous).  *_run functions take DEVICE
 *     pointers and a hipStream_t passed as void* (NULL = default stream) and are
 *     asynchronous on that stream.
 *   - One cf_ctx per GPU; a context is not thread-safe (callers serialise).
 *   - Item ids at this boundary are COMPACT indices 0..n_items-1 into the uploaded
 *     item graph; the host layer maps the reference's movie ids onto them.
 *
 * Reference interfaces replaced (file:line in /root/reference):
 *   cf_item_graph_upload[_dense] : the dense `weights` matrix load of
 *                                  precompute_local_threads.cpp:253-293 and the
 *                                  out_fin_ graph_loader of local_calc_precomp.cpp:122-136
 *   cf_eigen_batch / cf_eigen_run : compute_eigens(), precompute_local_threads.cpp:100-213
 *                                  (scheduled per user at :306-314)
 *   cf_predict_precomp / cf_predict_run : neigh_program::apply,
 *                                  local_calc_precomp.cpp:217-380 (per (movie,user) rating)
 *   cf_item_cosine               : weights_calc() via graph.transform_edges, knn2.cpp:127-146,206
 *                                  plus the w > 0.01 writer filter knn2.cpp:155-163
 *   cf_local_calc                : vertex_program::apply of local_calc.cpp:262-526 (per
 *                                  movie local graph, eigensolve, per-user w_lim, predict)
 *   cf_knn_predict               : knn_program gather/apply + error_vertex_data,
 *                                  knn3.cpp:185-256
 */
#ifndef CF_ABI_H
#define CF_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CF_OK 0
#define CF_EINVAL (-1)  /* bad argument / size */
#define CF_ENOMEM (-2)  /* device or host allocation failed */
#define CF_EHIP (-3)    /* HIP runtime or kernel launch error */
#define CF_ERANGE (-4)  /* problem size outside the supported buckets */
#define CF_ESTATE (-5)  /* missing prerequisite (e.g. no item graph uploaded) */

#define CF_MAX_K 192    /* largest per-user item count handled by the LDS eigen path */
#define CF_SPILL_MAX_K 5000  /* largest k of the spill paths' LDS layouts (fp64, HBM workspace);
                                larger k (no cap, as the reference) takes their HUGE layouts, every
                                k-long vector in HBM, bounded by HBM only (CF_ENOMEM) */

typedef struct cf_ctx cf_ctx;
typedef struct cf_plan cf_plan;

/* ---- context --------------------------------------------------------------- */
int cf_version(void);
/* Number of visible GPUs (0 when none or on error). */
int cf_device_count(void);
int cf_create(int device, cf_ctx** out);
void cf_destroy(cf_ctx* ctx);
/* Waits for the context's device, then frees its cached HBM workspaces (eigen and predictor
 * spill paths, the tridiagonal path, the predictor scratch, the knn2 planes); each is
 * allocated again, at the size its next call plans, when that call runs.  The spill paths
 * size their workspaces from the device's free HBM, so a workspace the predictor left behind
 * shrinks the next eigen call's and costs it waves: call this between stages of a long-lived
 * context (bench.py's config-5 legs).  No reference counterpart (one call per process there). */
int cf_release_workspaces(cf_ctx* ctx);
const char* cf_last_error(const cf_ctx* ctx);
/* Eigensolver of the k <= CF_MAX_K users: CF_EIGEN_JACOBI (default; one-sided Jacobi in
 * LDS, cf_eigen.hip) or CF_EIGEN_TRIDIAG (Householder + batched QL, cf_eigen_tri.hip). */
#define CF_EIGEN_TRIDIAG 0
#define CF_EIGEN_JACOBI 1
int cf_set_eigen_method(cf_ctx* ctx, int method);
/* Jacobi off-diagonal tolerance scale (default 1.0) and sweep cap (default 30). */
int cf_set_jacobi(cf_ctx* ctx, float tol_scale, int max_sweeps);
/* compute_eigens (precompute_local_threads.cpp:164-166) on the LDS Jacobi path: sweeps until
 * one rotates no pair by more than stop_rel (relative off-diagonal |b_p.b_q| / |b_p||b_q|),
 * then one first-order Gram refinement on the matrix cores for every pair whose eigenvalues
 * are more than delta apart.  Defaults: enable 1, stop_rel 1e-3, delta 1e-2; pairs closer than delta sweep to 8 tol.
 * enable 0 restores the sweeps-only rule (stop after a sweep with no rotation above 16 tol). */
int cf_set_eigen_refine(cf_ctx* ctx, int enable, float stop_rel, float delta);
/* LDS Jacobi, split layout: the sweeps of the users in buckets emax >= the minimum run
 * with the fixed column of every pair in registers and only the traveling half in LDS, several users
 * per CU, and the refinement and epilogue in the full-LDS kernel.  enable: 0 off (everything in the
 * full-LDS kernel), 1 the default minimum bucket (9: k > 128), 5..12 an explicit minimum; env
 * CF_EIGEN_SPLIT sets the same.  Same algorithm, same outputs up to the rotation order inside odd
 * segments.  Same call site as cf_eigen_run. */
int cf_set_eigen_split(cf_ctx* ctx, int enable);
/* Host only (no device): builds and verifies the split layout's sweep schedule for k columns in
 * LDS bucket emax (every pair of columns meets once per sweep, no two lane groups touch one LDS
 * slot in a level change, register groups and slots within capacity).  Returns CF_OK and the
 * steps per sweep, levels, and the largest register-group and slot counts of any level, or
 * CF_ERANGE when the split layout does not take k (those users keep the full-LDS kernel). */
int cf_debug_split_schedule(int emax, int k, int* steps, int* levels, int* max_groups, int* max_slots);
/* Complement-mask handoff (default on): an eigen run over a plan (cf_eigen_run, cf_step_run)
 * also writes, per rating, the 3 x 64-bit mask of the user's items that are NOT out-neighbours
 * (w <= 0.1) of that item, from the graph entries it gathers anyway (24 B per rating of HBM,
 * owned by the context); a later cf_predict_run* over the same plan, the same item arrays and the
 * same graph reads them instead of re-gathering k^2 graph entries per user.  Outputs are
 * bit-identical either way.  enable 0 frees nothing but makes every predictor run gather.
 * Replaces the per-rating neighbour scan of local_calc_precomp.cpp:254-265. */
int cf_set_step_masks(cf_ctx* ctx, int enable);
/* cf_local_calc, units with n > CF_MAX_K: bisect != 0 (default) computes the w_lim of a
 * (movie, test user) pair with c <= 184 rated rows from the eigenpairs of the movie's
 * B = L2 L2^T, shared by all its pairs (Haynsworth inertia count, bisection);
 * bisect 0 tridiagonalises each pair's L2_h L2_h^T as local_calc.cpp:425-436 spells it out.
 * Both return sqrt(lambda_min(L2_h L2_h^T)). */
int cf_set_local_wlim(cf_ctx* ctx, int bisect);
/* Diagnostics: enable != 0 allocates device counters that the eigen kernel fills;
 * out8 (optional) receives and resets {sum of sweeps, users, max sweeps, users that
 * hit the sweep cap, assembly cycles, Jacobi cycles, epilogue cycles, tournament
 * steps} (cycles: s_memtime of thread 0).  enable == 0 frees them. */
int cf_debug_stats(cf_ctx* ctx, int enable, uint64_t* out8);
/* Diagnostics of the eigen spill path (k > CF_MAX_K): enable != 0 makes its kernel sum
 * s_memtime cycles of thread 0 per phase; out8 (optional) receives and resets {users,
 * assembly, tridiagonalisation, Q accumulation, QL (total), QL rotation generation
 * (serial part), QL iterations, output} cycles. */
int cf_debug_spill(cf_ctx* ctx, int enable, uint64_t* out8);
/* Diagnostics of the tridiagonal eigen path: enable != 0 makes its kernels count;
 * out8 (optional) receives and resets {rotations, QL iterations, record overflows (users
 * recomputed by Jacobi), users, then thread-0 s_memtime cycles of the reduction kernel:
 * assembly, Householder steps, Q accumulation, and the sum of k}. */
int cf_debug_tri(cf_ctx* ctx, int enable, uint64_t* out8);
/* Diagnostics: predictor phase totals in s_memtime cycles.  out16[0..7], thread 0 of
 * each block: {per-user setup, basis, fast-path ratings, block-wide ratings} cycles,
 * the number of ratings taken by the fast path and by the block-wide paths, then the
 * cycles of the per-user Gbar GEMM and of the block-wide K path (a subset of the
 * block-wide cycles).  out16[8..15], summed over every wave: fast-path cycles in
 * {P/PG/PH gathers and border rows, LDL^T of K, the whole fast phase}, the cycles of
 * completed fast-path ratings with nc <= 4, 5..16 and > 16, and the counts of the first
 * two classes. */
int cf_debug_phases(cf_ctx* ctx, int enable, uint64_t* out16);
/* The predictor's fast-path system bound (rows min(nc, d)) in a k-bucket whose
 * Gram bound is lmax = 16 ceil(k / 16): ratings above it take the block-wide path.  -1 if
 * lmax is out of range.  (Test / diagnostics helper.) */
int cf_debug_predict_nmax(int lmax);
/* Per-bucket device time of compute_eigens (cf_eigen_run / cf_eigen_batch, Jacobi path):
 * enable != 0 records a HIP event pair around every LDS k-bucket launch on the stream it is
 * launched on (bucket e holds 16(e-1) < k <= 16e; e = 12 is eigen_kernel<12, narrow>, the
 * dominant kernel of the C4 step).  ms13 (optional) receives, after the recorded work has
 * finished, the mean milliseconds of each bucket's launch over the eigen runs since the last
 * read (at most the last 16; -1: not launched; [0] unused: the spill bucket runs on its own
 * streams) and clears the record.  Launches of
 * other buckets may co-run on the second stream, so these are the kernels' in-step
 * durations, as a profiler's per-dispatch trace shows them. */
int cf_eigen_bucket_timing(cf_ctx* ctx, int enable, float* ms13);
/* As cf_eigen_bucket_timing; sweeps_ms13[e] (optional) also receives, for buckets that ran in the
 * split layout, the mean ms from the bucket's start to the end of its sweep kernel
 * (split_sweep_kernel<e>; the rest of the bucket is eigen_kernel<e, .., RESUME>), else -1. */
int cf_eigen_bucket_timing_split(cf_ctx* ctx, int enable, float* ms13, float* sweeps_ms13);

/* ---- item graph (out_fin_) ---------------------------------------------------
 * Directed weighted graph exactly as parsed: w(a,b) and w(b,a) are independent.
 * HBM-resident in one of two layouts (cf_set_graph_layout, applies to the next upload):
 *   CF_GRAPH_DENSE (default) n_items x n_items fp32, direct indexing (the reference's own
 *                  dense `weights`, precompute_local_threads.cpp:255; ~250k items per GPU);
 *   CF_GRAPH_CSR   row pointers (u64), ascending columns (u32), weights (f32); every lookup
 *                  is a binary search of the row (the GraphLab out-edge lists,
 *                  local_calc_precomp.cpp:122-136): catalogues whose dense matrix does not fit.
 * Every kernel reads the same floats from either layout, so results are bit-identical.
 * A duplicate (a, b) keeps its LAST weight in input order (precompute_local_threads.cpp:284). */
#define CF_GRAPH_DENSE 0
#define CF_GRAPH_CSR 1
int cf_set_graph_layout(cf_ctx* ctx, int layout);
/* Layout, size and (CSR) stored edges of the resident graph. */
int cf_graph_info(const cf_ctx* ctx, int* layout, uint32_t* n_items, uint64_t* nnz);
int cf_item_graph_upload(cf_ctx* ctx, uint32_t n_items, const uint64_t* row_ptr,
                         const uint32_t* col, const float* w);
/* w_dense: n_items*n_items row-major; on_device != 0 means w_dense is a device
 * pointer that the context adopts by copy. */
int cf_item_graph_upload_dense(cf_ctx* ctx, uint32_t n_items, const float* w_dense,
                               int on_device);
/* Device pointer of the resident dense graph (for *_run callers), or NULL (none, or CSR). */
const float* cf_item_graph_device(const cf_ctx* ctx, uint32_t* n_items);

/* ---- user batch plan -----------------------------------------------------------
 * Buckets users by item count k (host item_off[n_users+1]); reused by eigen and
 * predict runs over the same user batch. */
int cf_plan_create(cf_ctx* ctx, uint32_t n_users, const uint64_t* item_off, cf_plan** out);
void cf_plan_destroy(cf_plan* plan);
/* Eigenvector slot size of a user with k items: k*max(k,2) floats. */
uint64_t cf_evec_slots(uint32_t k);
/* Fills evec_off[n_users] (prefix sum of cf_evec_slots) and returns the total. */
uint64_t cf_evec_offsets(uint32_t n_users, const uint64_t* item_off, uint64_t* evec_off);

/* ---- eigen stage: compute_eigens (precompute_local_threads.cpp:100-213) --------
 * Per user u with k = item_off[u+1]-item_off[u] items (sorted ascending compact ids;
 * that order is the row order of the user's block):
 *   sigs [item_off[u] + i]   i < k  : (float)(sig_min_i + 0.01)             (:169-177)
 *   evals[item_off[u] + j]   j < m  : eigenvalues of L2, ascending          (:164-166,193)
 *   evecs[evec_off[u] + i*m + j]    : eigenvector j, row i (k x m row-major) (:194,205-209)
 *   m_out[u]                        : lim, the stored eigenpair count       (:185-191)
 * k == 1 gives m == 2 with zero padding (reference: uninitialised, :193-194).
 * Device memory is bounded: the users run as the chunks of cf_eigen_batch_stream (below), each
 * chunk's blocks copied into the caller's arrays; only the host arrays scale with n_users. */
int cf_eigen_batch(cf_ctx* ctx, uint32_t n_users, const uint64_t* item_off,
                   const uint32_t* items, const uint64_t* evec_off, int32_t* m_out,
                   float* sigs, float* evals, float* evecs);
int cf_eigen_run(cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off,
                 const uint32_t* d_items, const uint64_t* d_evec_off, int32_t* d_m,
                 float* d_sigs, float* d_evals, float* d_evecs, void* stream);

/* ---- compute_eigens over any number of users at bounded memory ------------------
 * The reference runs one compute_eigens task per user and appends each record to out_eigen_
 * as it completes (precompute_local_threads.cpp:89-98, 306-314), so its memory does not grow
 * with the user count.  cf_eigen_batch_stream cuts users 0..n_users-1 (input order) into
 * contiguous chunks whose eigenvector slots (cf_evec_slots) fit chunk_bytes (0: a fifth of
 * the first context's HBM share, at most a quarter of host RAM (<= 64 GB) over the staging
 * sets), solves each chunk on the next free context (one per GPU, each with the graph
 * uploaded), packs its k x m blocks on the device and calls sink(sink_user, chunk) once per
 * chunk, in user order, from the calling thread, while the devices solve the next chunks.
 * The chunk's arrays live until the sink returns:
 *   item_off[count + 1]    chunk-local (item_off[0] = 0): user first+u has k = item_off[u+1] -
 *                          item_off[u] items, its sigs / evals at item_off[u] (as cf_eigen_batch)
 *   m[count], sigs, evals  as cf_eigen_batch
 *   packed_off[count + 1]  user first+u's k x m row-major block at evecs + packed_off[u]
 * A nonzero sink return stops the call (returned if negative, else CF_EINVAL).  The records
 * equal one cf_eigen_batch over all users bit for bit, for every chunk size and device count.
 * The contexts' eigen workspaces are released at the end (one-shot call).  stats (optional):
 * chunk count, the budget used, the largest chunk's slot bytes, and the peaks of the call's
 * own device bytes (its buffers + the contexts' workspaces) and of the device-wide bytes in
 * use (hipMemGetInfo, after each chunk's solve). */
typedef struct cf_eigen_chunk {
    uint32_t first;
    uint32_t count;
    const uint64_t* item_off;
    const int32_t* m;
    const float* sigs;
    const float* evals;
    const uint64_t* packed_off;
    const float* evecs;
} cf_eigen_chunk;
typedef int (*cf_eigen_sink)(void* sink_user, const cf_eigen_chunk* chunk);
typedef struct cf_eigen_stream_stats {
    uint32_t chunks;
    uint64_t chunk_slot_bytes;
    uint64_t max_chunk_slot_bytes;
    uint64_t own_peak_bytes;
    uint64_t device_peak_bytes;
} cf_eigen_stream_stats;
int cf_eigen_batch_stream(cf_ctx* const* ctxs, int n_dev, uint32_t n_users, const uint64_t* item_off,
                          const uint32_t* items, uint64_t chunk_bytes, cf_eigen_sink sink, void* sink_user,
                          cf_eigen_stream_stats* stats);

/* ---- multi-GPU eigen stage and the out_eigen_ gather ----------
 * Replaces the thread pool of precompute_local_threads.cpp:300-314 and the single shared
 * out_eigen_ (:196-211, read whole by every rank at local_calc_precomp.cpp:485-486,509).
 *
 * cf_cost_split: contiguous split points split[0..n_parts] of users 0..n_users-1 balancing
 * sum(k^3): split[p] = first user whose prefix cost reaches p/n_parts of the total.
 *
 * cf_pack_eigen_run: packs the k x m blocks of users 0..n_users-1 (stored in their
 * cf_evec_slots slots at d_evec_off by cf_eigen_run) into one contiguous run:
 *   d_packed_off[u] = sum_{v<u} k_v m_v  (n_users + 1 entries, u64, device)
 *   d_packed[d_packed_off[u] + i*m_u + j] = d_evecs[d_evec_off[u] + i*m_u + j]
 * With d_packed == NULL only the offsets are written (size the buffer from entry n_users).
 *
 * cf_eigen_batch_multi: cf_eigen_batch over ONE global user set on n_dev contexts (one per
 * GPU, each with the item graph uploaded; several contexts may share a device).  Users are
 * split by cf_cost_split, every context computes and packs its range concurrently, and the
 * ranges are gathered to ctxs[0]'s device by peer copies over xGMI.  Outputs as
 * cf_eigen_batch (m_out, sigs, evals at item_off) except the eigenvectors, which arrive
 * packed: packed_off[n_users + 1] as above and packed_evecs (capacity packed_cap floats;
 * the slot total of cf_evec_offsets always suffices).  split_out (optional, n_dev + 1)
 * receives the ranges.  The records are identical to the one-device run's. */
int cf_cost_split(uint32_t n_users, const uint64_t* item_off, int n_parts, uint32_t* split);
int cf_pack_eigen_run(cf_ctx* ctx, uint32_t n_users, const uint64_t* d_item_off, const int32_t* d_m,
                      const uint64_t* d_evec_off, const float* d_evecs, uint64_t* d_packed_off,
                      float* d_packed, void* stream);
int cf_eigen_batch_multi(cf_ctx* const* ctxs, int n_dev, uint32_t n_users, const uint64_t* item_off,
                         const uint32_t* items, int32_t* m_out, float* sigs, float* evals,
                         uint64_t* packed_off, float* packed_evecs, uint64_t packed_cap,
                         uint32_t* split_out);

/* ---- prediction stage: neigh_program::apply (local_calc_precomp.cpp:217-380) ----
 * For every user u and every row r < k of the user's block (test movie items[r] with
 * test rating ratings[item_off[u]+r]):
 *   mse[item_off[u]+r]  = (float)(rating - clamp(pred,1,5))^2     (:307-327,358)
 *   kk [item_off[u]+r]  = number of the user's items that are out-neighbours of the
 *                         movie with w > 0.1 (:132,254-265,359)
 *   pred[item_off[u]+r] = clamp(pred,1,5) (optional, may be NULL)
 * w_lim for row r:
 *   sig_mode CF_SIGS_COMPAT: sigtab[r]  -- the reference's accumulating sigs_min
 *                            vector (:414,437,440,271) reduces to the global
 *                            concatenation of all records' sigs in file order;
 *   sig_mode CF_SIGS_OWN:    sigtab[item_off[u]+r] -- the user's own sigs.
 * evecs are fp64 (parsed out_eigen_) or fp32 (device-resident eigen output). */
#define CF_SIGS_OWN 0
#define CF_SIGS_COMPAT 1
int cf_predict_precomp(cf_ctx* ctx, uint32_t n_users, const uint64_t* item_off,
                       const uint32_t* items, const float* ratings, const int32_t* m,
                       const double* evals, const uint64_t* evec_off, const double* evecs,
                       const double* sigtab, uint64_t sigtab_len, int sig_mode,
                       float* mse, int32_t* kk, double* pred);
/* cf_predict_precomp over the rows with row_sel[item_off[u] + r] != 0 only (row_sel NULL =
 * every row); the other rows' mse / kk / pred keep the values the caller passed in.  This is
 * the per-vertex sampling of local_calc_precomp --pct (rand() % 100 < pct before apply,
 * local_calc_precomp.cpp:221): unsampled movies cost no per-rating work. */
int cf_predict_precomp_sel(cf_ctx* ctx, uint32_t n_users, const uint64_t* item_off,
                           const uint32_t* items, const float* ratings, const int32_t* m,
                           const double* evals, const uint64_t* evec_off, const double* evecs,
                           const double* sigtab, uint64_t sigtab_len, int sig_mode,
                           const uint8_t* row_sel, float* mse, int32_t* kk, double* pred);
/* cf_predict_precomp_sel over ONE user set on n_dev contexts (one per GPU, each with the item
 * graph uploaded; several may share a device), for local_calc_precomp on several GPUs
 * (local_calc_precomp.cpp:485-486,509: every rank holds the whole out_eigen_).  Users are split
 * by cf_cost_split; each context predicts its range concurrently.  In CF_SIGS_COMPAT mode every
 * range reads the same global sig table, so the outputs are bit-identical to the one-context
 * call.  split_out (optional, n_dev + 1) receives the ranges. */
int cf_predict_precomp_multi(cf_ctx* const* ctxs, int n_dev, uint32_t n_users, const uint64_t* item_off,
                             const uint32_t* items, const float* ratings, const int32_t* m, const double* evals,
                             const uint64_t* evec_off, const double* evecs, const double* sigtab,
                             uint64_t sigtab_len, int sig_mode, const uint8_t* row_sel, float* mse, int32_t* kk,
                             double* pred, uint32_t* split_out);
/* The same two entry points with fp32 eigenvector blocks: the binary out_eigen_ stores fp32
 * values, and keeping them fp32 halves the host copy and the upload.  evals and sigtab are
 * taken as fp32 values (the binary file's own; they are narrowed back exactly).  The kernels
 * widen every value to fp64 on load, so results equal the fp64 entry points' on the widened
 * arrays bit for bit. */
int cf_predict_precomp_sel_f32(cf_ctx* ctx, uint32_t n_users, const uint64_t* item_off,
                               const uint32_t* items, const float* ratings, const int32_t* m,
                               const double* evals, const uint64_t* evec_off, const float* evecs,
                               const double* sigtab, uint64_t sigtab_len, int sig_mode,
                               const uint8_t* row_sel, float* mse, int32_t* kk, double* pred);
int cf_predict_precomp_multi_f32(cf_ctx* const* ctxs, int n_dev, uint32_t n_users, const uint64_t* item_off,
                                 const uint32_t* items, const float* ratings, const int32_t* m, const double* evals,
                                 const uint64_t* evec_off, const float* evecs, const double* sigtab,
                                 uint64_t sigtab_len, int sig_mode, const uint8_t* row_sel, float* mse, int32_t* kk,
                                 double* pred, uint32_t* split_out);
int cf_predict_run_f64(cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off,
                       const uint32_t* d_items, const float* d_ratings, const int32_t* d_m,
                       const double* d_evals, const uint64_t* d_evec_off,
                       const double* d_evecs, const double* d_sigtab, int sig_mode,
                       float* d_mse, int32_t* d_kk, double* d_pred, void* stream);
int cf_predict_run_f32(cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off,
                       const uint32_t* d_items, const float* d_ratings, const int32_t* d_m,
                       const float* d_evals, const uint64_t* d_evec_off,
                       const float* d_evecs, const float* d_sigtab, int sig_mode,
                       float* d_mse, int32_t* d_kk, double* d_pred, void* stream);

/* ---- fused step ------------------------------------------------------------------
 * cf_eigen_run followed by cf_predict_run_f32 on the SAME outputs (sigtab = d_sigs), with the
 * predictor of every k-bucket started as soon as that bucket's eigenpairs exist, on streams of
 * its own, so prediction overlaps the remaining eigen buckets.  Outputs are identical to the
 * two calls in sequence.  Ordered on `stream` like the *_run calls.  cf_step_timing: device
 * time of the last cf_step_run from its start to the last eigen bucket and to its end. */
int cf_step_run(cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off, const uint32_t* d_items,
                const float* d_ratings, const uint64_t* d_evec_off, int32_t* d_m, float* d_sigs,
                float* d_evals, float* d_evecs, int sig_mode, float* d_mse, int32_t* d_kk,
                double* d_pred, void* stream);
int cf_step_timing(cf_ctx* ctx, float* eigen_ms, float* total_ms);

/* ---- kNN stage ------------------------------------------------------------------
 * knn2 weights_calc (knn2.cpp:127-164): for every item pair a != b over the users
 * present in both train lists, cnt > cnt_min ? w = num/(sqrtf(den1)*sqrtf(den2)) : 0,
 * kept iff w > w_min (the reference writes w > 0.01, cnt > 5).  Output is the dense
 * n_items x n_items weight matrix (0 = no out_fin_ edge); symmetric for integer
 * ratings.  user_off/item/rating: per-user train ratings (CSR over users).
 * Integer ratings in [-11, 11] run on int8 MFMA (exact), others on fp32 MFMA.
 * adopt_as_graph != 0 also installs the result as the context's item graph. */
int cf_item_cosine(cf_ctx* ctx, uint32_t n_users, uint32_t n_items, const uint64_t* user_off,
                   const uint32_t* item, const float* rating, float w_min, int cnt_min,
                   int adopt_as_graph, float* w_out);
/* knn2 with the reference's output form: the compacted edge list "a b w" for w > w_min
 * (knn2.cpp:151-164), as CSR over compact source ids: edge_off[n_items + 1], targets ascending
 * in edge_col / edge_w (capacity edge_cap).  The dense similarity matrix is compacted on the
 * device; only the edges cross PCIe.  *n_edges = the edge count; edge_cap too small gives
 * CF_ERANGE with edge_off and *n_edges filled (retry with edge_cap = *n_edges).
 * adopt_as_graph != 0 installs the result as the context's item graph (its layout). */
int cf_item_cosine_edges(cf_ctx* ctx, uint32_t n_users, uint32_t n_items, const uint64_t* user_off,
                         const uint32_t* item, const float* rating, float w_min, int cnt_min, int adopt_as_graph,
                         uint64_t* edge_off, uint32_t* edge_col, float* edge_w, uint64_t edge_cap, uint64_t* n_edges);
/* Optional top-K cap on cf_item_cosine_edges' list (0 = off, the default: the reference has
 * no top-k, its neighbourhoods are thresholds, knn2.cpp:142,157): per source item only the K
 * largest weights are returned (ties at the K-th value: the lower target ids), still in
 * ascending target order; adopt_as_graph installs the capped list.  Selection is a per-row
 * radix select on the device over the exact weights, so the indices are bit-exact. */
int cf_set_knn2_topk(cf_ctx* ctx, uint32_t topk);
int cf_item_cosine_run(cf_ctx* ctx, uint32_t n_users, uint32_t n_items,
                       const uint64_t* d_user_off, const uint32_t* d_item, const float* d_rating,
                       int integer_ratings, float w_min, int cnt_min, float* d_w_out,
                       void* stream);
/* Durations of the last cf_item_cosine(_run) on its stream (HIP events): plane build
 * (rating scan, memset, scatter) and the MFMA similarity kernel; path = 1 one code
 * plane (<= 7 distinct integer ratings), 2 three int8 planes, 3 fp32 planes.
 * Waits for the launch to finish. */
int cf_knn2_timing(cf_ctx* ctx, float* plane_ms, float* gemm_ms, int* path);
/* The 2^24 guard of the last cf_item_cosine(_run) (SURVEY hard part 7): the reference sums
 * num, den1, den2 and cnt in float (knn2.cpp:129-140), which is exact for integer ratings
 * only while every partial sum stays <= 2^24.  max_accumulator = the largest such sum (the
 * per-item sum of r^2 or rater count, which bounds every pair's); exact = 1 when the
 * reference's floats are exact, so its weights equal this kernel's integer-accumulated
 * ones bit for bit, 0 otherwise (always 0 on the fp32 path of real-valued ratings, whose
 * reference sums are in hash order).  Waits for the launch to finish. */
int cf_knn2_exactness(cf_ctx* ctx, double* max_accumulator, int* exact);
/* K-chunk streaming of the one-code-plane knn2 path: when the int8 code
 * plane of all users (n_items x n_users bytes) exceeds ~60% of free HBM, users are processed
 * in chunks with the four int32 products carried per 128 x 128 tile in HBM between chunks
 * (256 KB per tile) and the epilogue on the last chunk: the weights are identical.
 * cf_set_knn2_chunk forces users_per_chunk (rounded down to a multiple of 128; 0 = automatic);
 * cf_knn2_chunks reports the chunk count of the last launch. */
int cf_set_knn2_chunk(cf_ctx* ctx, uint32_t users_per_chunk);
int cf_knn2_chunks(cf_ctx* ctx, int* n_chunks);
/* local_calc vertex_program::apply (local_calc.cpp:262-526) on the uploaded graph (raw
 * out_fin_ weights; edges count iff w > 0.1, graph_loader :113).  Movie unit v lists
 * movie_items[movie_off[v] .. movie_off[v+1]) = [m, the out-neighbours of m with w > 0.1]
 * (compact ids, any order: results are permutation-equivariant).  Units with fewer than 2
 * out-neighbours are skipped (:271-272); up to 191 run on the LDS kernels, more on the fp64
 * spill kernels (HBM workspace; above CF_SPILL_MAX_K - 1 in their HUGE layout).  There is no
 * neighbourhood cap, as in the reference: a unit whose n x n blocks and 2 n^2 fp64 solver slot
 * do not fit in HBM returns CF_ENOMEM.
 * Test ratings: CSR over all n_items compact ids, test_off[n_items + 1], users ascending
 * within an item.  For every test entry t of a processed movie m (test_off[m] <= t <
 * test_off[m+1]): mse[t] (float, :499), kk[t] (rated rows of the local graph), and when
 * non-null pred[t] (clamped), wlim[t] (= sqrt(lambda_min(L2_h L2_h^T)), :436) and lim[t].
 * Entries of movies not processed are left untouched. */
int cf_local_calc(cf_ctx* ctx, uint32_t n_movies, const uint64_t* movie_off,
                  const uint32_t* movie_items, const uint64_t* test_off, const uint32_t* test_user,
                  const float* test_rating, float* mse, int32_t* kk, double* pred, float* wlim,
                  int32_t* lim);
/* knn3 knn_program + error_vertex_data (knn3.cpp:185-256) on the uploaded graph:
 * per test rating (user u, movie items[e]) pred[e] = sum w*r / sum w over u's test
 * items j with w(movie, j) > 0.1 (0 when none); per movie (compact id)
 * movie_mse[i] = (sum over its test ratings of (r - round(pred))^2, 0 if pred < 0.1)
 * / count, and 0 for movies without test ratings.  The "Knn Average MSE" is
 * sum(movie_mse) / num_vertices (computed by the caller, knn3.cpp:263). */
int cf_knn_predict(cf_ctx* ctx, uint32_t n_users, const uint64_t* user_off,
                   const uint32_t* items, const float* ratings, double* pred,
                   float* movie_mse, uint32_t* movie_count);

/* ---- data prep: knn regroup and k-fold split on the GPU --------
 * cf_knn_regroup replaces the three GraphLab programs of knn.cpp (vertex_program :160-205,
 * vertex2/3_program :212-298) and feeds its writers (:303-357).  Input: n ratings in read
 * order with compact ids user[i] < n_users (in the order of the reference's remapped ids,
 * uimax - id, :103) and movie[i] < n_movies (ascending movie id), rating[i], and
 * validate[i] != 0 for the .validate role (NULL = all train, :88-92).  Output per movie m:
 *   train_user/train_rating[train_off[m] .. train_off[m+1]) : its train ratings, users
 *       ascending, one per user (the last one read wins: map assignment, :183-187);
 *   test_*  likewise for the validate role (ratings_test);
 *   edg_movie[edg_off[m] .. edg_off[m+1]) : the sorted unique movies co-rated with m by any
 *       of its raters, both roles, m itself excluded (:224-227, 271-274, 342-351).
 * train_* / test_* need room for n entries, edg_movie for edg_cap; when the co-rated lists
 * need more than edg_cap entries edg_off is still complete and the call returns CF_ERANGE
 * (the device variant drops the excess writes: check d_edg_off[n_movies] <= edg_cap). */
int cf_knn_regroup(cf_ctx* ctx, uint64_t n, uint32_t n_users, uint32_t n_movies, const uint32_t* user,
                   const uint32_t* movie, const float* rating, const uint8_t* validate, uint64_t* train_off,
                   uint32_t* train_user, float* train_rating, uint64_t* test_off, uint32_t* test_user,
                   float* test_rating, uint64_t* edg_off, uint32_t* edg_movie, uint64_t edg_cap);
int cf_knn_regroup_run(cf_ctx* ctx, uint64_t n, uint32_t n_users, uint32_t n_movies, const uint32_t* d_user,
                       const uint32_t* d_movie, const float* d_rating, const uint8_t* d_validate,
                       uint64_t* d_train_off, uint32_t* d_train_user, float* d_train_rating,
                       uint64_t* d_test_off, uint32_t* d_test_user, float* d_test_rating, uint64_t* d_edg_off,
                       uint32_t* d_edg_movie, uint64_t edg_cap, void* stream);
/* User-disjoint k-fold split (fold_cross_validation.py:31-57): rank[u] is user u's position
 * in the shuffled key list (a permutation of 0..n_users-1); order receives the rating indices
 * sorted by (rank[user[i]], i), i.e. the concatenation u0.test, u1.test, ... of the script
 * (each user's lines in read order).  The fold boundaries are rank ranges (host). */
int cf_fold_order(cf_ctx* ctx, uint64_t n, uint32_t n_users, const uint32_t* user, const uint32_t* rank,
                  uint32_t* order);
int cf_fold_order_run(cf_ctx* ctx, uint64_t n, uint32_t n_users, const uint32_t* d_user, const uint32_t* d_rank,
                      uint32_t* d_order, void* stream);
/* Device time (HIP events) of the last cf_knn_regroup(_run) / cf_fold_order(_run); waits. */
int cf_prep_timing(cf_ctx* ctx, float* ms);

/* ---- graph-signal polynomial filters ------------------------ */
#define CF_FILTER_CHEBY 0     /* cheby.cpp:152-274 (Chebyshev recurrence on [0, 2]) */
#define CF_FILTER_BINOMIAL 1  /* binomials.cpp:145-253 (quadratic factors, overlapping windows) */
/* Replaces the degree / init_values / cheby programs (cheby.cpp:152-245) and the degree /
 * binomial_a / binomial_b programs (binomials.cpp:145-250) with their sync-engine loops
 * (cheby.cpp:296-366, binomials.cpp:296-358).  Vertices are compact indices 0..n_vertices-1;
 * topology line l is (va[l], vb[l], w[l]): when w > 0.1 it adds va -> vb and vb -> va
 * (graph_loader, cheby.cpp:88-92), parallel edges kept, self-edges dropped.  signal[i] is
 * the graph_signal value of vertex i (0 where the file has none).  coeff holds n_coeff >= 3
 * values (both programs read coeff[2]).  out[i] = the filtered signal (fp64).  Synchronous:
 * returns after the copy-out. */
int cf_graph_filter(cf_ctx* ctx, int kind, uint32_t n_vertices, uint64_t n_lines, const uint32_t* va,
                    const uint32_t* vb, const double* w, const double* signal, const double* coeff,
                    uint32_t n_coeff, double* out);
/* Device time of the last cf_graph_filter's supersteps (HIP events) and its directed edges. */
int cf_graph_filter_timing(cf_ctx* ctx, float* device_ms, uint64_t* n_edges);

#ifdef __cplusplus
}
#endif
#endif /* CF_ABI_H */
