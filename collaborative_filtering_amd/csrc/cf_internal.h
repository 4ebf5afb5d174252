// cf_internal.h -- shared definitions of libcf_mi355x (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

#include "cf_abi.h"

// The resident item graph as the kernels see it: dense n x n fp32 row-major (direct
// indexing), or CSR (row_ptr, columns ascending per row, weights) for catalogues whose dense
// matrix does not fit, looked up by a binary search of the row.  Every kernel reads the graph
// through row(a)[b] = w(a -> b), 0 where there is no edge; both layouts give the same floats.
struct GraphRow {
    const float* dense;    // this row of the dense matrix, or null
    const uint32_t* col;   // CSR: the row's columns (ascending) and weights
    const float* w;
    uint32_t len;
    __device__ __forceinline__ float operator[](uint32_t b) const {
        if (dense) return dense[b];
        uint32_t lo = 0, hi = len;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (col[mid] < b) lo = mid + 1;
            else hi = mid;
        }
        return (lo < len && col[lo] == b) ? w[lo] : 0.0f;
    }
};
struct GraphDev {
    const float* dense = nullptr;   // dense layout
    uint64_t n = 0;
    const uint64_t* rp = nullptr;   // CSR layout
    const uint32_t* col = nullptr;
    const float* w = nullptr;
    __device__ __forceinline__ GraphRow row(uint32_t a) const {
        if (dense) return GraphRow{dense + (size_t)a * n, nullptr, nullptr, 0};
        const uint64_t b = rp[a];
        return GraphRow{nullptr, col + b, w + b, (uint32_t)(rp[a + 1] - b)};
    }
};

struct cf_ctx {
    int device = 0;
    std::string last_error;
    // Item graph, HBM-resident: dense fp32 n_items x n_items row-major (d_graph), or CSR
    // (d_grp / d_gcol / d_gw, graph_layout == CF_GRAPH_CSR).
    float* d_graph = nullptr;
    uint32_t n_items = 0;
    int graph_layout = CF_GRAPH_DENSE;   // layout of the next upload (cf_set_graph_layout)
    bool graph_csr = false;              // layout of the resident graph
    uint64_t* d_grp = nullptr;
    uint32_t* d_gcol = nullptr;
    float* d_gw = nullptr;
    uint64_t g_nnz = 0;
    // Jacobi controls
    float tol_scale = 1.0f;
    int max_sweeps = 30;
    // compute_eigens: Jacobi sweeps to stop_rel, then the first-order Gram refinement
    // (cf_set_eigen_refine; refine = 0 keeps the r03 rule: sweeps to 16 * tol)
    int eigen_refine = 1;
    float stop_rel = 1e-3f;
    float refine_delta = 1e-2f;
    float close_sigrot = 8.0f;    // pairs closer than refine_delta: sweeps to close_sigrot * tol
    int eigen_sort = 2;           // LDS Jacobi: norm-sorted sweeps, 2 ascending / 1 descending / 0 off (CF_EIGEN_SORT)
    // Optional device counters: [0] sum of sweeps, [1] users, [2] max sweeps, [3] capped users.
    unsigned long long* d_stats = nullptr;
    // Optional predictor phase-cycle counters (16 slots), see cf_debug_phases.
    unsigned long long* d_phase = nullptr;
    // Device scratch owned by the context (predictor per-block U^T U), grown on demand.
    void* d_scratch = nullptr;
    size_t scratch_bytes = 0;
    // fused predictor: one user counter per predictor stream (zeroed before each launch)
    uint32_t* d_pred_next = nullptr;
    // block-wide rating queue per predictor stream and the dense workgroups' factorisation
    // regions (pred_dense_kernel, cf_predict.hip), grown on demand
    uint32_t* d_dense_q = nullptr;
    size_t dense_q_words = 0;   // per stream (kAuxStreams copies are allocated)
    double* d_dense_ws = nullptr;
    size_t dense_ws_doubles = 0;   // per stream (kAuxStreams copies are allocated)
    // the complement masks the eigen kernel hands to the predictor (24 B per rating), valid for
    // the plan / item arrays / graph generation of the eigen run that wrote them (cf_cmask_*)
    void* d_cmask = nullptr;            // 3 words per rating at 3 * item_off[u]
    size_t cmask_bytes = 0;
    uint64_t* d_cmask_fp = nullptr;     // one item-list fingerprint per user (cf_items_fp)
    uint32_t cmask_users = 0;           // its capacity
    uint64_t cmask_plan = 0;                            // cf_plan::id of that run
    const void* cmask_key[2] = {nullptr, nullptr};      // its item_off, items
    uint64_t cmask_gen = ~0ull;
    uint64_t graph_gen = 0;   // bumped by every graph (re)load (free_graph)
    int step_masks = 1;       // cf_set_step_masks (env CF_STEP_MASKS=0 for A/B runs)
    int local_wlim_bisect = 1;   // cf_set_local_wlim: spill pairs' w_lim by bisection (cf_local.hip)
    // knn2 rating planes (R, S, B), grown on demand.
    void* d_knn = nullptr;
    size_t knn_bytes = 0;
    // eigen spill-path workspace (counter + per-workgroup fp64 k x k), grown on demand.
    void* d_spill = nullptr;
    size_t spill_bytes = 0;
    bool spill_debug = false;   // cf_debug_spill: phase counters (d_dbg[0..7])
    // debug counters of cf_debug_spill ([0..7]) and cf_debug_tri ([8..15]): a buffer of their own,
    // so releasing or evicting a workspace neither loses nor re-seeds them
    unsigned long long* d_dbg = nullptr;
    // the spill bucket's k > 3072 range runs on its own stream beside the smaller ranges:
    // fork / done events; spill_side_pending = its done event still has to be joined
    hipStream_t spill_side = nullptr;
    // staged spill users' slot offsets (per-user slot sizes): pinned staging, device copy, and
    // the event of the last copy out of the staging buffer
    uint64_t* h_spill_off = nullptr;
    uint64_t* d_spill_off = nullptr;
    size_t spill_off_bytes = 0;
    hipEvent_t spill_off_ev = nullptr;
    hipEvent_t spill_side_ev[2] = {};
    bool spill_side_pending = false;
    // predictor spill-path workspace (per-user Q / Gbar slots, per-workgroup LDL^T), grown on demand.
    void* d_pspill = nullptr;
    size_t pspill_bytes = 0;
    // its per-chunk slot tables: pinned host staging buffer and the event of the last copy
    void* h_pspill_meta = nullptr;
    size_t pspill_meta_bytes = 0;
    hipEvent_t pspill_meta_ev = nullptr;
    // tridiagonal eigen path scratch (T, QL records), grown on demand; eigen method
    void* d_tri = nullptr;
    size_t tri_bytes = 0;
    int eigen_method = CF_EIGEN_JACOBI;
    bool tri_debug = false;
    // knn2 stage events (plane build start, GEMM start, GEMM end) of the last launch.
    hipEvent_t knn_ev[3] = {nullptr, nullptr, nullptr};
    int knn_path = 0;   // 1 code plane, 2 three int8 planes, 3 fp32 planes
    unsigned int* d_knn_acc = nullptr;
    // knn2 K-chunk streaming: tile partial sums, forced chunk size (0 = by free HBM), chunks used
    void* d_knn_part = nullptr;
    size_t knn_part_bytes = 0;
    uint32_t knn_chunk_users = 0;
    uint32_t knn2_topk = 0;   // cf_set_knn2_topk: K largest weights per source in the edge list (0: all)
    int knn_chunks = 0;   // knn2: largest accumulator of the last launch (float bits)
    // data prep (cf_prep.hip): sort / bitmap scratch, grown on demand; events of the last call
    void* d_prep = nullptr;
    size_t prep_bytes = 0;
    hipEvent_t prep_ev[2] = {nullptr, nullptr};
    // bucket overlap (eigen, predict): kAuxStreams non-blocking streams, a join event per
    // stream and one fork event (cf_eigen.hip, cf_predict.hip)
    static constexpr int kAuxStreams = 2;   // measured: 3 streams no faster at C2
    hipStream_t aux_stream[kAuxStreams] = {};
    hipEvent_t aux_event[kAuxStreams + 1] = {};
    // fused step (cf_step_run): two predictor streams beside the two aux (eigen) streams, an
    // event per eigen bucket, and timing events {start, eigen done, end}
    // per-bucket timing of the eigen launches (cf_eigen_bucket_timing): an event pair per
    // k-bucket and eigen run, for the last kBucketRuns runs (a ring), read and cleared together
    static constexpr int kBucketRuns = 16;
    bool bucket_timing = false;
    hipEvent_t bucket_ev[kBucketRuns][13][3] = {};   // start, end, and (split layout) after the sweeps
    bool bucket_recorded[kBucketRuns][13] = {};
    bool bucket_mid[kBucketRuns][13] = {};
    hipEvent_t split_mid_ev = nullptr;   // set around one timed bucket launch: recorded after kernel A
    bool split_mid_recorded = false;
    int bucket_run = 0;   // runs recorded since the last read
    hipStream_t step_stream[2] = {};
    hipEvent_t step_bucket_ev[16] = {};
    hipEvent_t step_sync_ev[4] = {};
    hipEvent_t step_time_ev[3] = {};
    // split-storage Jacobi (cf_eigen_split.hip): per LDS bucket emax, the device copy of the
    // sweep schedule tables of every k the bucket's split kernel takes (built on first use)
    uint32_t* d_split_sched[13] = {};
    int eigen_split = -1;   // -1: not read yet (CF_EIGEN_SPLIT, default on); cf_set_eigen_split
    int split_finish = -1;  // -1: not read yet (CF_EIGEN_SPLIT_FINISH); 1 / 0 / 2 = refinement + epilogue in the split kernel always / never / buckets <= 8
    // graph filter (cf_graph_filter): device time of the last call's supersteps, its edges
    float filter_ms = 0.0f;
    uint64_t filter_nnz = 0;
};

// One launch of the eigen / predict kernels covers the users of one k-bucket.
constexpr int kSpillBucket = -1;   // cf_bucket::emax of the k > CF_MAX_K users (the spill paths)

struct cf_bucket {
    int emax = 0;              // elements per lane of a column (k <= 16*emax); kSpillBucket

    uint32_t count = 0;        // users in the bucket
    uint32_t first = 0;        // offset into the plan's user order
    uint32_t kmax = 0;         // largest k in the bucket
};

struct cf_tri_chunk {   // a group's sub-range inside one LDS bucket
    int emax;
    uint32_t first;
    uint32_t count;
    uint32_t kmax;
    uint32_t group;
};
struct cf_tri_group {   // plan-order range sharing one QL-record buffer and one kernel-B launch
    uint32_t first;
    uint32_t count;
    uint32_t kmax;
};

struct cf_plan {
    uint64_t id = 0;   // unique per process (cf_plan_create), never reused
    uint32_t n_users = 0;
    uint64_t n_entries = 0;
    // tridiagonal eigen path (cf_eigen_tri.hip): chunks and per-user QL record offsets
    std::vector<cf_tri_chunk> tri_chunks;
    std::vector<cf_tri_group> tri_groups;
    uint64_t tri_rot_max = 0, tri_hdr_max = 0;
    uint32_t tri_users_max = 0;
    uint64_t* d_tri_roff = nullptr;
    uint64_t* d_tri_hoff = nullptr;
    std::vector<uint32_t> h_order;   // user ids, grouped by bucket, largest k first
    uint32_t* d_order = nullptr;     // device copy
    std::vector<cf_bucket> buckets;
    uint32_t kmax = 0;
    std::vector<uint64_t> h_item_off;   // host copy of the user offsets (cf_step_run's compat prefix)
    cf_plan* prefix = nullptr;          // cf_step_run: plan of the users whose sigs form the compat table
};

int cf_set_error(cf_ctx* ctx, int code, const std::string& msg);

// Fingerprint of a user's (item_off[u], k, items) for the eigen -> predictor complement-mask
// handoff (cf_cmask_*): the eigen kernel stores it per user beside the masks, the predictor's
// basis kernel recomputes it from the arrays it is given and takes the masks only on a match
// (else it gathers the graph rows itself), so rewritten or reallocated item arrays cannot
// reach stale masks.  Wave-wide: every lane of the calling wave gets the value.
__device__ __forceinline__ uint64_t cf_fp_mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}
__device__ inline uint64_t cf_items_fp(const uint32_t* items, int k, uint64_t base, int lane) {
    uint64_t h = 0;
    for (int i = lane; i < k; i += 64) h += cf_fp_mix(((uint64_t)items[i] << 32) | (uint32_t)i);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) h += (uint64_t)__shfl_xor((unsigned long long)h, o);
    return cf_fp_mix(h ^ cf_fp_mix(base * 0x9e3779b97f4a7c15ull + (uint64_t)k)) | 1ull;   // never 0
}
// cf_plan_create with another largest k: local_calc's movie units and pairs (cf_local.hip) are
// not capped at CF_SPILL_MAX_K (their spill launches take the HUGE layout above it)
int cf_plan_create_cap(cf_ctx* ctx, uint32_t n_users, const uint64_t* item_off, uint64_t kcap, cf_plan** out);

inline bool has_graph(const cf_ctx* ctx) { return ctx->d_graph || ctx->graph_csr; }
inline GraphDev graph_dev(const cf_ctx* ctx) {
    GraphDev g;
    g.n = ctx->n_items;
    if (ctx->graph_csr) {
        g.rp = ctx->d_grp;
        g.col = ctx->d_gcol;
        g.w = ctx->d_gw;
    } else {
        g.dense = ctx->d_graph;
    }
    return g;
}

#define CF_HIP_CHECK(ctx, expr)                                                          \
    do {                                                                                 \
        hipError_t _e = (expr);                                                          \
        if (_e != hipSuccess)                                                            \
            return cf_set_error((ctx), CF_EHIP,                                          \
                                std::string(#expr) + ": " + hipGetErrorString(_e));      \
    } while (0)

// RAII device buffer used by the host-pointer wrappers.
struct DevBuf {
    void* p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

// Drop the context's cached eigen-side workspaces (the spill solver's and the tridiagonal
// path's; every launch that needs them sizes them again) after the device is idle.  Returns the
// bytes released.  The spill workspace may hold most of the context's HBM share (its budget is
// 0.75 of it), so every allocation below falls back on this before it reports CF_ENOMEM.
size_t cf_evict_workspaces(cf_ctx* ctx);
// hipMalloc that evicts the cached workspaces and retries once on failure; CF_ENOMEM (with
// `what` in the message) if the retry fails too.
int cf_malloc_evict(cf_ctx* ctx, void** p, size_t bytes, const char* what);
// the 16 debug counter words (ctx->d_dbg), allocated zeroed on first use
int cf_debug_counters(cf_ctx* ctx);

inline int dev_alloc(cf_ctx* ctx, DevBuf& b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    return cf_malloc_evict(ctx, &b.p, bytes, "device buffer");
}

inline int set_device(cf_ctx* ctx) {
    CF_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    return CF_OK;
}

// Live contexts per device (cf_create / cf_destroy): contexts sharing a GPU size their
// workspaces from the same free-HBM figure, so each takes 1/n of it.
int cf_contexts_on_device(int device);

// Workspace budget of one context: `frac` of (free HBM + the bytes the caller's own buffer
// already holds) / (contexts on the device), at least `floor` bytes but never more than half
// of that share -- a floor above the share would only turn into CF_ENOMEM.
inline size_t cf_hbm_budget(const cf_ctx* ctx, size_t own_bytes, double frac, size_t floor) {
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
    const size_t share = (free_b + own_bytes) / (size_t)std::max(1, cf_contexts_on_device(ctx->device));
    const size_t b = (size_t)((double)share * frac);
    return std::max(b, std::min(floor, share / 2));
}

#define CF_TRY(expr)              \
    do {                          \
        int _rc = (expr);         \
        if (_rc != CF_OK) return _rc; \
    } while (0)

// Launchers implemented in the .hip translation units.
// a8 (local_calc): kLocal / kSigma modes of the eigen kernel (cf_eigen.hip).
int cf_launch_local_eigen(cf_ctx* ctx, const cf_plan* movie_plan, const uint64_t* d_item_off,
                          const uint32_t* d_items, const uint64_t* d_evec_off, float* d_evals,
                          float* d_evecs, float* d_l2, const uint64_t* d_l2_off, int32_t* d_n_out,
                          hipStream_t stream);
int cf_launch_local_sigma(cf_ctx* ctx, const cf_plan* pair_plan, const uint64_t* d_item_off,
                          const uint32_t* d_items, const uint32_t* d_pair_movie,
                          const uint32_t* d_pair_user, const float* d_l2, const uint64_t* d_l2_off,
                          const uint64_t* d_test_off, const uint32_t* d_test_user,
                          const float* d_test_rating, float* d_wlim, hipStream_t stream,
                          const uint8_t* d_solved = nullptr, bool skip_spill = false);

// a8 (local_calc) modes of the spill eigen kernel for units with n > CF_MAX_K.
struct cf_spill_local {
    int mode;                      // 1: the movie's local graph (all n eigenpairs, L2 kept);
                                   // 2: w_lim of a (movie, test user) pair (eigenvalue only);
                                   // 3: all n eigenpairs of B = L2 L2^T of the movie
    float* l2;                     // per movie n x n row-major L2 (mode 1 writes, mode 2 reads)
    const uint64_t* l2_off;
    const uint32_t* pair_movie;    // mode 2: unit -> movie unit, test user
    const uint32_t* pair_user;
    const uint64_t* test_off;      // mode 2: test ratings, CSR over compact item ids
    const uint32_t* test_user;
    const float* test_rating;
    float* wlim;                   // mode 2 output per pair
    const uint8_t* solved;         // mode 2, optional: pairs whose w_lim is already written
};
// defer_join: the k > 3072 range's stream is left running (ctx->spill_side_pending); the caller
// joins it with cf_spill_join before the results are read.  Otherwise it is joined into `stream`.
int cf_launch_eigen_spill(cf_ctx* ctx, const cf_plan* plan, const cf_bucket& b, const uint64_t* d_item_off,
                          const uint32_t* d_items, const uint64_t* d_evec_off, int32_t* d_m, float* d_sigs,
                          float* d_evals, float* d_evecs, hipStream_t stream, const cf_spill_local* loc = nullptr,
                          bool defer_join = false);
int cf_spill_join(cf_ctx* ctx, hipStream_t stream);
// a8 predictor for (movie, test user) pairs of units with n > CF_MAX_K (cf_predict_spill.hip).
int cf_launch_local_predict_spill(cf_ctx* ctx, uint32_t n_pairs, int nmax, const uint32_t* d_pair_movie,
                                  const uint32_t* d_pair_user, const uint64_t* d_pair_out, const uint64_t* d_item_off,
                                  const uint32_t* d_items, const float* d_evals, const uint64_t* d_evec_off,
                                  const float* d_evecs, const float* d_wlim, const uint64_t* d_test_off,
                                  const uint32_t* d_test_user, const float* d_test_rating, float* d_mse,
                                  int32_t* d_kk, double* d_pred, int32_t* d_lim, hipStream_t stream);
int cf_tri_prepare(cf_ctx* ctx, cf_plan* plan, const uint64_t* item_off);
// emax_min: only the LDS buckets with emax >= emax_min (1: all; the hybrid method: 12)
int cf_launch_eigen_tri(cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off, const uint32_t* d_items,
                        const uint64_t* d_evec_off, int32_t* d_m, float* d_sigs, float* d_evals, float* d_evecs,
                        hipStream_t stream, int emax_min = 1);
// Jacobi kernel over plan order [first, first + count) of LDS bucket emax, only for users
// with flag[j - first] != 0 (fallback of the tridiagonal path); d_cmask (optional) receives
// the predictor's complement masks, 3 words per rating at 3 * item_off[u] (the fused step).
int cf_launch_eigen_flagged(cf_ctx* ctx, const cf_plan* plan, int emax, uint32_t first, uint32_t count,
                            const int* flag, const uint64_t* d_item_off, const uint32_t* d_items,
                            const uint64_t* d_evec_off, int32_t* d_m, float* d_sigs, float* d_evals,
                            float* d_evecs, hipStream_t stream, uint64_t* d_cmask = nullptr);
// Complement masks of the LDS-bucket users (cf_predict.hip): the buffer an eigen run over `plan`
// writes (null: disabled by CF_STEP_MASKS=0 or no HBM), marked valid once launched, and looked
// up by a predictor run over the same plan, item arrays and graph.
uint64_t* cf_cmask_buffer(cf_ctx* ctx, const cf_plan* plan);
void cf_cmask_mark(cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off, const uint32_t* d_items, bool valid);
const uint64_t* cf_cmask_lookup(const cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off,
                                const uint32_t* d_items);
int cf_launch_eigen(cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off,
                    const uint32_t* d_items, const uint64_t* d_evec_off, int32_t* d_m,
                    float* d_sigs, float* d_evals, float* d_evecs, hipStream_t stream);

template <typename T>
int cf_launch_predict(cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off,
                      const uint32_t* d_items, const float* d_ratings, const int32_t* d_m,
                      const T* d_evals, const uint64_t* d_evec_off, const T* d_evecs,
                      const T* d_sigtab, int sig_mode, float* d_mse, int32_t* d_kk,
                      double* d_pred, const uint8_t* d_row_sel, hipStream_t stream);

// Predictor for the spill bucket (CF_MAX_K < k <= CF_SPILL_MAX_K), cf_predict_spill.hip.
// cf_eigen_run + cf_predict_run_f32 with the predictor of each k-bucket started as soon as that
// bucket's eigenpairs exist (cf_predict.hip).
int cf_launch_step(cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off, const uint32_t* d_items,
                   const float* d_ratings, const uint64_t* d_evec_off, int32_t* d_m, float* d_sigs, float* d_evals,
                   float* d_evecs, int sig_mode, float* d_mse, int32_t* d_kk, double* d_pred, hipStream_t stream);

template <typename T>
int cf_launch_predict_spill(cf_ctx* ctx, const cf_plan* plan, const cf_bucket& b, const uint64_t* d_item_off,
                            const uint32_t* d_items, const float* d_ratings, const int32_t* d_m,
                            const T* d_evals, const uint64_t* d_evec_off, const T* d_evecs, const T* d_sigtab,
                            int sig_mode, float* d_mse, int32_t* d_kk, double* d_pred, const uint8_t* d_row_sel,
                            hipStream_t stream);

int cf_launch_knn2(cf_ctx* ctx, uint32_t n_users, uint32_t n_items, const uint64_t* d_user_off,
                   const uint32_t* d_item, const float* d_rating, int integer_ratings, float w_min,
                   int cnt_min, float* d_w_out, hipStream_t stream);
int cf_launch_knn3(cf_ctx* ctx, uint32_t n_users, const uint64_t* d_user_off, const uint32_t* d_items,
                   const float* d_ratings, double* d_pred, unsigned long long* d_sq, double* d_sq_real,
                   unsigned int* d_cnt, hipStream_t stream);

// cf_graph.hip: a device dense matrix as CSR (new buffers), and a device dense matrix
// installed as the context's graph in its upload layout (adopted, or compacted and freed).
int cf_dense_to_csr(cf_ctx* ctx, uint32_t n, const float* d_dense, uint64_t** d_rp, uint32_t** d_col, float** d_w,
                    uint64_t* nnz, hipStream_t stream, uint32_t topk = 0);
int cf_adopt_dense_graph(cf_ctx* ctx, uint32_t n, float* d_dense);

int cf_launch_dense_scatter(cf_ctx* ctx, uint32_t n_items, const uint64_t* d_row_ptr,
                            const uint32_t* d_col, const float* d_w, float* d_dense,
                            hipStream_t stream);
