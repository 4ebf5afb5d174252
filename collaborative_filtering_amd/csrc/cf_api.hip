// cf_api.hip -- the extern "C" boundary of libcf_mi355x.so (declared in include/cf_abi.h).
//
// Host-pointer entry points copy in, run the device path on the context's stream and
// copy out; *_run entry points take device pointers and an explicit stream.

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <new>

#include <type_traits>

#include "cf_internal.h"

int cf_set_error(cf_ctx* ctx, int code, const std::string& msg) {
    if (ctx) ctx->last_error = msg;
    return code;
}

namespace {
constexpr int kMaxDevices = 64;
std::atomic<int> g_ctx_per_device[kMaxDevices];
}  // namespace

int cf_contexts_on_device(int device) {
    return (device >= 0 && device < kMaxDevices) ? g_ctx_per_device[device].load() : 1;
}

namespace {

// Scatter a CSR graph into the dense matrix.  Duplicate (a,b) keep the LAST
// occurrence in CSR order, like repeated `weights(m1,m2) = w` assignments
// (precompute_local_threads.cpp:284): one thread per row walks its edges in order.
__global__ void dense_scatter_kernel(uint32_t n_items, const uint64_t* row_ptr, const uint32_t* col,
                                     const float* w, float* dense) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_items) return;
    float* row = dense + (size_t)r * n_items;
    for (uint64_t e = row_ptr[r]; e < row_ptr[r + 1]; ++e) {
        const uint32_t c = col[e];
        if (c < n_items) row[c] = w[e];
    }
}

}  // namespace

size_t cf_evict_workspaces(cf_ctx* ctx) {
    if (!ctx->d_spill && !ctx->d_tri) return 0;
    if (hipDeviceSynchronize() != hipSuccess) return 0;   // every stream of the context is done with them
    const size_t bytes = ctx->spill_bytes + ctx->tri_bytes;
    if (ctx->d_spill) (void)hipFree(ctx->d_spill);
    if (ctx->d_tri) (void)hipFree(ctx->d_tri);
    ctx->d_spill = ctx->d_tri = nullptr;
    ctx->spill_bytes = ctx->tri_bytes = 0;
    return bytes;
}

int cf_malloc_evict(cf_ctx* ctx, void** p, size_t bytes, const char* what) {
    *p = nullptr;
    if (hipMalloc(p, bytes) == hipSuccess) return CF_OK;
    (void)hipGetLastError();
    *p = nullptr;
    if (cf_evict_workspaces(ctx) > 0 && hipMalloc(p, bytes) == hipSuccess) return CF_OK;
    (void)hipGetLastError();
    *p = nullptr;
    return cf_set_error(ctx, CF_ENOMEM, std::string(what) + " (" + std::to_string(bytes) + " bytes)");
}

int cf_debug_counters(cf_ctx* ctx) {
    if (ctx->d_dbg) return CF_OK;
    void* p = nullptr;
    if (hipMalloc(&p, 16 * sizeof(unsigned long long)) != hipSuccess)
        return cf_set_error(ctx, CF_ENOMEM, "debug counters");
    ctx->d_dbg = static_cast<unsigned long long*>(p);
    CF_HIP_CHECK(ctx, hipMemset(ctx->d_dbg, 0, 16 * sizeof(unsigned long long)));
    return CF_OK;
}

int cf_launch_dense_scatter(cf_ctx* ctx, uint32_t n_items, const uint64_t* d_row_ptr,
                            const uint32_t* d_col, const float* d_w, float* d_dense,
                            hipStream_t stream) {
    const int threads = 256;
    const int blocks = (int)((n_items + threads - 1) / threads);
    if (blocks > 0) {
        hipLaunchKernelGGL(dense_scatter_kernel, dim3(blocks), dim3(threads), 0, stream, n_items,
                           d_row_ptr, d_col, d_w, d_dense);
        CF_HIP_CHECK(ctx, hipGetLastError());
    }
    return CF_OK;
}

extern "C" {

int cf_version(void) { return 2; }

int cf_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int cf_create(int device, cf_ctx** out) {
    if (!out) return CF_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return CF_EHIP;
    if (device < 0 || device >= n || device >= kMaxDevices) return CF_EINVAL;
    cf_ctx* ctx = new (std::nothrow) cf_ctx();
    if (!ctx) return CF_ENOMEM;
    ctx->device = device;
    if (const char* e = getenv("CF_EIGEN_REFINE")) ctx->eigen_refine = e[0] != '0';   // A/B switches
    if (const char* e = getenv("CF_EIGEN_CLOSE")) ctx->close_sigrot = (float)atof(e);
    if (const char* e = getenv("CF_EIGEN_SORT")) ctx->eigen_sort = atoi(e);   // 0 off, 1 descending, 2 ascending
    if (const char* e = getenv("CF_STEP_MASKS")) ctx->step_masks = e[0] != '0';
    if (hipSetDevice(device) != hipSuccess) {
        delete ctx;
        return CF_EHIP;
    }
    g_ctx_per_device[device].fetch_add(1);
    *out = ctx;
    return CF_OK;
}

int cf_release_workspaces(cf_ctx* ctx) {
    if (!ctx) return CF_EINVAL;
    CF_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    CF_HIP_CHECK(ctx, hipDeviceSynchronize());   // every stream of the context is done with them
    const auto drop = [](void*& p, size_t& bytes) {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    };
    drop(ctx->d_spill, ctx->spill_bytes);
    drop(ctx->d_pspill, ctx->pspill_bytes);
    drop(ctx->d_tri, ctx->tri_bytes);
    drop(ctx->d_scratch, ctx->scratch_bytes);
    drop(ctx->d_knn, ctx->knn_bytes);
    return CF_OK;
}

void cf_destroy(cf_ctx* ctx) {
    if (!ctx) return;
    g_ctx_per_device[ctx->device].fetch_sub(1);
    (void)hipSetDevice(ctx->device);
    if (ctx->d_graph) (void)hipFree(ctx->d_graph);
    if (ctx->d_grp) (void)hipFree(ctx->d_grp);
    if (ctx->d_gcol) (void)hipFree(ctx->d_gcol);
    if (ctx->d_gw) (void)hipFree(ctx->d_gw);
    if (ctx->d_stats) (void)hipFree(ctx->d_stats);
    if (ctx->d_dbg) (void)hipFree(ctx->d_dbg);
    if (ctx->d_phase) (void)hipFree(ctx->d_phase);
    if (ctx->d_scratch) (void)hipFree(ctx->d_scratch);
    if (ctx->d_pred_next) (void)hipFree(ctx->d_pred_next);
    if (ctx->d_dense_q) (void)hipFree(ctx->d_dense_q);
    if (ctx->d_dense_ws) (void)hipFree(ctx->d_dense_ws);
    if (ctx->d_cmask) (void)hipFree(ctx->d_cmask);
    if (ctx->d_cmask_fp) (void)hipFree(ctx->d_cmask_fp);
    if (ctx->d_knn) (void)hipFree(ctx->d_knn);
    if (ctx->d_knn_acc) (void)hipFree(ctx->d_knn_acc);
    if (ctx->d_knn_part) (void)hipFree(ctx->d_knn_part);
    if (ctx->d_prep) (void)hipFree(ctx->d_prep);
    for (hipEvent_t& e : ctx->prep_ev)
        if (e) (void)hipEventDestroy(e);
    for (auto& run : ctx->bucket_ev)
        for (auto& pr : run)
            for (hipEvent_t& e : pr)
                if (e) (void)hipEventDestroy(e);
    if (ctx->d_spill) (void)hipFree(ctx->d_spill);
    if (ctx->d_spill_off) (void)hipFree(ctx->d_spill_off);
    if (ctx->h_spill_off) (void)hipHostFree(ctx->h_spill_off);
    if (ctx->spill_off_ev) (void)hipEventDestroy(ctx->spill_off_ev);
    for (hipEvent_t& e : ctx->spill_side_ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->spill_side) (void)hipStreamDestroy(ctx->spill_side);
    if (ctx->d_pspill) (void)hipFree(ctx->d_pspill);
    if (ctx->pspill_meta_ev) {
        (void)hipEventSynchronize(ctx->pspill_meta_ev);
        (void)hipEventDestroy(ctx->pspill_meta_ev);
    }
    if (ctx->h_pspill_meta) (void)hipHostFree(ctx->h_pspill_meta);
    if (ctx->d_tri) (void)hipFree(ctx->d_tri);
    for (uint32_t* p : ctx->d_split_sched)
        if (p) (void)hipFree(p);
    for (hipEvent_t& e : ctx->knn_ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t& e : ctx->aux_event)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t* arr : {ctx->step_bucket_ev, ctx->step_sync_ev, ctx->step_time_ev})
        for (int i = 0; i < (arr == ctx->step_bucket_ev ? 16 : arr == ctx->step_sync_ev ? 4 : 3); ++i)
            if (arr[i]) (void)hipEventDestroy(arr[i]);
    for (hipStream_t& st : ctx->step_stream)
        if (st) (void)hipStreamDestroy(st);
    for (hipStream_t& st : ctx->aux_stream)
        if (st) (void)hipStreamDestroy(st);
    delete ctx;
}

int cf_debug_phases(cf_ctx* ctx, int enable, uint64_t* out16) {
    if (!ctx) return CF_EINVAL;
    CF_TRY(set_device(ctx));
    if (enable && !ctx->d_phase) {
        if (hipMalloc(&ctx->d_phase, 16 * sizeof(unsigned long long)) != hipSuccess)
            return cf_set_error(ctx, CF_ENOMEM, "phase counters");
        CF_HIP_CHECK(ctx, hipMemset(ctx->d_phase, 0, 16 * sizeof(unsigned long long)));
    }
    if (out16 && ctx->d_phase) {
        CF_HIP_CHECK(ctx, hipDeviceSynchronize());
        CF_HIP_CHECK(ctx, hipMemcpy(out16, ctx->d_phase, 16 * sizeof(uint64_t), hipMemcpyDeviceToHost));
        CF_HIP_CHECK(ctx, hipMemset(ctx->d_phase, 0, 16 * sizeof(unsigned long long)));
    }
    if (!enable && ctx->d_phase) {
        (void)hipFree(ctx->d_phase);
        ctx->d_phase = nullptr;
    }
    return CF_OK;
}

int cf_debug_stats(cf_ctx* ctx, int enable, uint64_t* out4) {
    if (!ctx) return CF_EINVAL;
    CF_TRY(set_device(ctx));
    if (enable && !ctx->d_stats) {
        if (hipMalloc(&ctx->d_stats, 8 * sizeof(unsigned long long)) != hipSuccess)
            return cf_set_error(ctx, CF_ENOMEM, "stats allocation");
        CF_HIP_CHECK(ctx, hipMemset(ctx->d_stats, 0, 8 * sizeof(unsigned long long)));
    }
    if (out4 && ctx->d_stats) {
        CF_HIP_CHECK(ctx, hipDeviceSynchronize());
        CF_HIP_CHECK(ctx, hipMemcpy(out4, ctx->d_stats, 8 * sizeof(uint64_t), hipMemcpyDeviceToHost));
        CF_HIP_CHECK(ctx, hipMemset(ctx->d_stats, 0, 8 * sizeof(unsigned long long)));
    }
    if (!enable && ctx->d_stats) {
        (void)hipFree(ctx->d_stats);
        ctx->d_stats = nullptr;
    }
    return CF_OK;
}

const char* cf_last_error(const cf_ctx* ctx) { return ctx ? ctx->last_error.c_str() : "null context"; }

int cf_set_eigen_method(cf_ctx* ctx, int method) {
    if (!ctx || (method != CF_EIGEN_TRIDIAG && method != CF_EIGEN_JACOBI))
        return cf_set_error(ctx, CF_EINVAL, "cf_set_eigen_method: unknown method");
    ctx->eigen_method = method;
    return CF_OK;
}

int cf_set_jacobi(cf_ctx* ctx, float tol_scale, int max_sweeps) {
    if (!ctx || !(tol_scale > 0.0f) || max_sweeps <= 0) return cf_set_error(ctx, CF_EINVAL, "bad jacobi options");
    ctx->tol_scale = tol_scale;
    ctx->max_sweeps = max_sweeps;
    return CF_OK;
}

int cf_set_local_wlim(cf_ctx* ctx, int bisect) {
    if (!ctx) return CF_EINVAL;
    ctx->local_wlim_bisect = bisect != 0;
    return CF_OK;
}

int cf_set_step_masks(cf_ctx* ctx, int enable) {
    if (!ctx) return CF_EINVAL;
    ctx->step_masks = enable != 0;
    if (!ctx->step_masks) ctx->cmask_gen = ~0ull;   // the predictor gathers again from now on
    return CF_OK;
}

int cf_set_eigen_refine(cf_ctx* ctx, int enable, float stop_rel, float delta) {
    if (!ctx || !(stop_rel > 0.0f) || !(delta >= 0.0f)) return cf_set_error(ctx, CF_EINVAL, "bad refine options");
    ctx->eigen_refine = enable != 0;
    ctx->stop_rel = stop_rel;
    ctx->refine_delta = delta;
    return CF_OK;
}

// cf_item_graph_upload / cf_item_graph_upload_dense: cf_graph.hip (dense or CSR layout).

const float* cf_item_graph_device(const cf_ctx* ctx, uint32_t* n_items) {
    if (!ctx) return nullptr;
    if (n_items) *n_items = ctx->n_items;
    return ctx->d_graph;
}

uint64_t cf_evec_slots(uint32_t k) { return (uint64_t)k * std::max<uint32_t>(k, 2u); }

uint64_t cf_evec_offsets(uint32_t n_users, const uint64_t* item_off, uint64_t* evec_off) {
    uint64_t acc = 0;
    for (uint32_t u = 0; u < n_users; ++u) {
        if (evec_off) evec_off[u] = acc;
        acc += cf_evec_slots((uint32_t)(item_off[u + 1] - item_off[u]));
    }
    return acc;
}

int cf_plan_create(cf_ctx* ctx, uint32_t n_users, const uint64_t* item_off, cf_plan** out) {
    // no k cap, as the reference: k > CF_SPILL_MAX_K takes the spill path's HUGE layout
    return cf_plan_create_cap(ctx, n_users, item_off, ~0ull, out);
}

}  // extern "C"

int cf_plan_create_cap(cf_ctx* ctx, uint32_t n_users, const uint64_t* item_off, uint64_t kcap, cf_plan** out) {
    if (!ctx || !out || (!item_off && n_users)) return cf_set_error(ctx, CF_EINVAL, "cf_plan_create: null");
    *out = nullptr;
    CF_TRY(set_device(ctx));
    cf_plan* plan = new (std::nothrow) cf_plan();
    if (!plan) return cf_set_error(ctx, CF_ENOMEM, "plan allocation");
    static std::atomic<uint64_t> next_plan_id{1};
    plan->id = next_plan_id++;
    plan->n_users = n_users;
    plan->h_item_off.assign(item_off, item_off + n_users + 1);
    // Bucket by emax = ceil(k/16); within a bucket, largest k first (cost ~ k^3).
    // by[0]: the spill path (CF_MAX_K < k <= kcap), launched first.
    std::vector<std::vector<uint32_t>> by(13);
    for (uint32_t u = 0; u < n_users; ++u) {
        const uint64_t k = item_off[u + 1] - item_off[u];
        if (k > kcap) {
            delete plan;
            return cf_set_error(ctx, CF_ERANGE,
                                "user " + std::to_string(u) + " has k=" + std::to_string(k) +
                                    " items; the eigen path supports k <= " + std::to_string(kcap));
        }
        by[k == 0 ? 1 : (k > CF_MAX_K ? 0 : (int)((k + 15) / 16))].push_back(u);
        plan->kmax = std::max<uint32_t>(plan->kmax, (uint32_t)k);
    }
    static const int kOrder[13] = {0, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1};
    for (const int e : kOrder) {
        auto& v = by[e];
        if (v.empty()) continue;
        std::stable_sort(v.begin(), v.end(), [&](uint32_t x, uint32_t y) {
            return (item_off[x + 1] - item_off[x]) > (item_off[y + 1] - item_off[y]);
        });
        cf_bucket b;
        b.emax = e == 0 ? kSpillBucket : e;
        b.first = (uint32_t)plan->h_order.size();
        b.count = (uint32_t)v.size();
        b.kmax = (uint32_t)(item_off[v.front() + 1] - item_off[v.front()]);
        plan->buckets.push_back(b);
        plan->h_order.insert(plan->h_order.end(), v.begin(), v.end());
    }
    if (n_users) {
        if (hipMalloc(&plan->d_order, sizeof(uint32_t) * n_users) != hipSuccess) {
            delete plan;
            return cf_set_error(ctx, CF_ENOMEM, "plan order allocation");
        }
        if (hipMemcpy(plan->d_order, plan->h_order.data(), sizeof(uint32_t) * n_users,
                      hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(plan->d_order);
            delete plan;
            return cf_set_error(ctx, CF_EHIP, "plan order copy");
        }
    }
    {
        const int rc = cf_tri_prepare(ctx, plan, item_off);
        if (rc != CF_OK) {
            cf_plan_destroy(plan);
            return rc;
        }
    }
    *out = plan;
    return CF_OK;
}

extern "C" {

void cf_plan_destroy(cf_plan* plan) {
    if (!plan) return;
    if (plan->d_order) (void)hipFree(plan->d_order);
    if (plan->d_tri_roff) (void)hipFree(plan->d_tri_roff);
    if (plan->d_tri_hoff) (void)hipFree(plan->d_tri_hoff);
    cf_plan_destroy(plan->prefix);
    delete plan;
}

int cf_eigen_run(cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off, const uint32_t* d_items,
                 const uint64_t* d_evec_off, int32_t* d_m, float* d_sigs, float* d_evals, float* d_evecs,
                 void* stream) {
    if (!ctx || !plan) return cf_set_error(ctx, CF_EINVAL, "cf_eigen_run: null");
    if (!has_graph(ctx)) return cf_set_error(ctx, CF_ESTATE, "cf_eigen_run: no item graph uploaded");
    CF_TRY(set_device(ctx));
    return cf_launch_eigen(ctx, plan, d_item_off, d_items, d_evec_off, d_m, d_sigs, d_evals, d_evecs,
                           (hipStream_t)stream);
}

}  // extern "C"

namespace {
struct BatchSink {   // cf_eigen_batch: every chunk's records into the caller's flat arrays
    const uint64_t* item_off;
    const uint64_t* evec_off;
    int32_t* m;
    float *sigs, *evals, *evecs;
};
int batch_sink(void* user, const cf_eigen_chunk* c) {
    const BatchSink& B = *static_cast<const BatchSink*>(user);
    const uint64_t e0 = B.item_off[c->first];
    std::memcpy(B.m + c->first, c->m, sizeof(int32_t) * c->count);
    std::memcpy(B.sigs + e0, c->sigs, sizeof(float) * c->item_off[c->count]);
    std::memcpy(B.evals + e0, c->evals, sizeof(float) * c->item_off[c->count]);
    for (uint32_t u = 0; u < c->count; ++u)
        std::memcpy(B.evecs + B.evec_off[c->first + u], c->evecs + c->packed_off[u],
                    sizeof(float) * (c->packed_off[u + 1] - c->packed_off[u]));
    return 0;
}
}  // namespace

extern "C" {

int cf_eigen_batch(cf_ctx* ctx, uint32_t n_users, const uint64_t* item_off, const uint32_t* items,
                   const uint64_t* evec_off, int32_t* m_out, float* sigs, float* evals, float* evecs) {
    if (!ctx || !item_off || !evec_off || !m_out || !sigs || !evals || !evecs)
        return cf_set_error(ctx, CF_EINVAL, "cf_eigen_batch: null argument");
    if (!has_graph(ctx)) return cf_set_error(ctx, CF_ESTATE, "cf_eigen_batch: no item graph uploaded");
    CF_TRY(set_device(ctx));
    // device memory bounded by the stream's chunks; the caller's arrays receive every chunk
    BatchSink B{item_off, evec_off, m_out, sigs, evals, evecs};
    cf_ctx* const ctxs[1] = {ctx};
    return cf_eigen_batch_stream(ctxs, 1, n_users, item_off, items, 0, batch_sink, &B, nullptr);
}

int cf_predict_run_f64(cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off, const uint32_t* d_items,
                       const float* d_ratings, const int32_t* d_m, const double* d_evals,
                       const uint64_t* d_evec_off, const double* d_evecs, const double* d_sigtab, int sig_mode,
                       float* d_mse, int32_t* d_kk, double* d_pred, void* stream) {
    if (!ctx || !plan) return cf_set_error(ctx, CF_EINVAL, "cf_predict_run_f64: null");
    if (!has_graph(ctx)) return cf_set_error(ctx, CF_ESTATE, "cf_predict_run_f64: no item graph uploaded");
    CF_TRY(set_device(ctx));
    return cf_launch_predict<double>(ctx, plan, d_item_off, d_items, d_ratings, d_m, d_evals, d_evec_off,
                                     d_evecs, d_sigtab, sig_mode, d_mse, d_kk, d_pred, nullptr, (hipStream_t)stream);
}

int cf_predict_run_f32(cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off, const uint32_t* d_items,
                       const float* d_ratings, const int32_t* d_m, const float* d_evals,
                       const uint64_t* d_evec_off, const float* d_evecs, const float* d_sigtab, int sig_mode,
                       float* d_mse, int32_t* d_kk, double* d_pred, void* stream) {
    if (!ctx || !plan) return cf_set_error(ctx, CF_EINVAL, "cf_predict_run_f32: null");
    if (!has_graph(ctx)) return cf_set_error(ctx, CF_ESTATE, "cf_predict_run_f32: no item graph uploaded");
    CF_TRY(set_device(ctx));
    return cf_launch_predict<float>(ctx, plan, d_item_off, d_items, d_ratings, d_m, d_evals, d_evec_off,
                                    d_evecs, d_sigtab, sig_mode, d_mse, d_kk, d_pred, nullptr, (hipStream_t)stream);
}

int cf_step_run(cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off, const uint32_t* d_items,
                const float* d_ratings, const uint64_t* d_evec_off, int32_t* d_m, float* d_sigs, float* d_evals,
                float* d_evecs, int sig_mode, float* d_mse, int32_t* d_kk, double* d_pred, void* stream) {
    if (!ctx || !plan) return cf_set_error(ctx, CF_EINVAL, "cf_step_run: null");
    if (sig_mode != CF_SIGS_OWN && sig_mode != CF_SIGS_COMPAT) return cf_set_error(ctx, CF_EINVAL, "cf_step_run: bad sig_mode");
    if (!has_graph(ctx)) return cf_set_error(ctx, CF_ESTATE, "cf_step_run: no item graph uploaded");
    CF_TRY(set_device(ctx));
    return cf_launch_step(ctx, plan, d_item_off, d_items, d_ratings, d_evec_off, d_m, d_sigs, d_evals, d_evecs,
                          sig_mode, d_mse, d_kk, d_pred, (hipStream_t)stream);
}

int cf_step_timing(cf_ctx* ctx, float* eigen_ms, float* total_ms) {
    if (!ctx) return CF_EINVAL;
    if (!ctx->step_time_ev[2]) return cf_set_error(ctx, CF_ESTATE, "cf_step_timing: no cf_step_run yet");
    CF_TRY(set_device(ctx));
    CF_HIP_CHECK(ctx, hipEventSynchronize(ctx->step_time_ev[2]));
    float a = 0.0f, b = 0.0f;
    CF_HIP_CHECK(ctx, hipEventElapsedTime(&a, ctx->step_time_ev[0], ctx->step_time_ev[1]));
    CF_HIP_CHECK(ctx, hipEventElapsedTime(&b, ctx->step_time_ev[0], ctx->step_time_ev[2]));
    if (eigen_ms) *eigen_ms = a;
    if (total_ms) *total_ms = b;
    return CF_OK;
}

int cf_predict_precomp(cf_ctx* ctx, uint32_t n_users, const uint64_t* item_off, const uint32_t* items,
                       const float* ratings, const int32_t* m, const double* evals, const uint64_t* evec_off,
                       const double* evecs, const double* sigtab, uint64_t sigtab_len, int sig_mode,
                       float* mse, int32_t* kk, double* pred) {
    return cf_predict_precomp_sel(ctx, n_users, item_off, items, ratings, m, evals, evec_off, evecs, sigtab,
                                  sigtab_len, sig_mode, nullptr, mse, kk, pred);
}

}  // extern "C"

namespace {
// EV = double (text out_eigen_: decimal values) or float (binary out_eigen_ / device blocks):
// the kernels widen fp32 blocks to fp64 on load, so a float block gives the same predictions
// as the same values passed widened
template <typename EV>
int predict_precomp_impl(cf_ctx* ctx, uint32_t n_users, const uint64_t* item_off, const uint32_t* items,
                         const float* ratings, const int32_t* m, const double* evals, const uint64_t* evec_off,
                         const EV* evecs, const double* sigtab, uint64_t sigtab_len, int sig_mode,
                         const uint8_t* row_sel, float* mse, int32_t* kk, double* pred) {
    if (!ctx || !item_off || !items || !ratings || !m || !evals || !evec_off || !evecs || !sigtab || !mse || !kk)
        return cf_set_error(ctx, CF_EINVAL, "cf_predict_precomp: null argument");
    if (sig_mode != CF_SIGS_OWN && sig_mode != CF_SIGS_COMPAT)
        return cf_set_error(ctx, CF_EINVAL, "cf_predict_precomp: bad sig_mode");
    if (!has_graph(ctx)) return cf_set_error(ctx, CF_ESTATE, "cf_predict_precomp: no item graph uploaded");
    CF_TRY(set_device(ctx));
    const uint64_t n_entries = item_off[n_users];
    uint64_t n_evec = 0;
    for (uint32_t u = 0; u < n_users; ++u) {
        const uint64_t k = item_off[u + 1] - item_off[u];
        if (m[u] < 0 || (uint64_t)m[u] > std::max<uint64_t>(k, 2))
            return cf_set_error(ctx, CF_EINVAL, "cf_predict_precomp: m out of range");
        n_evec = std::max<uint64_t>(n_evec, evec_off[u] + k * (uint64_t)m[u]);
        if (sig_mode == CF_SIGS_COMPAT && k > sigtab_len)
            return cf_set_error(ctx, CF_EINVAL, "cf_predict_precomp: compat sig table shorter than k");
    }
    if (sig_mode == CF_SIGS_OWN && sigtab_len < n_entries)
        return cf_set_error(ctx, CF_EINVAL, "cf_predict_precomp: sig table shorter than item_off[n_users]");
    for (uint64_t e = 0; e < n_entries; ++e)
        if (items[e] >= ctx->n_items) return cf_set_error(ctx, CF_EINVAL, "item index outside the graph");
    cf_plan* plan = nullptr;
    CF_TRY(cf_plan_create(ctx, n_users, item_off, &plan));
    DevBuf doff, ditems, drat, dm, deval, deoff, devec, dsig, dmse, dkk, dpred, dsel, deval32, dsig32;
    int rc = dev_alloc(ctx, doff, sizeof(uint64_t) * (n_users + 1));
    if (rc == CF_OK) rc = dev_alloc(ctx, ditems, sizeof(uint32_t) * n_entries);
    if (rc == CF_OK) rc = dev_alloc(ctx, drat, sizeof(float) * n_entries);
    if (rc == CF_OK) rc = dev_alloc(ctx, dm, sizeof(int32_t) * std::max<uint32_t>(n_users, 1));
    if (rc == CF_OK) rc = dev_alloc(ctx, deval, sizeof(double) * n_entries);
    if (rc == CF_OK) rc = dev_alloc(ctx, deoff, sizeof(uint64_t) * std::max<uint32_t>(n_users, 1));
    if (rc == CF_OK) rc = dev_alloc(ctx, devec, sizeof(EV) * n_evec);
    if (rc == CF_OK) rc = dev_alloc(ctx, dsig, sizeof(double) * sigtab_len);
    if (rc == CF_OK) rc = dev_alloc(ctx, dmse, sizeof(float) * n_entries);
    if (rc == CF_OK) rc = dev_alloc(ctx, dkk, sizeof(int32_t) * n_entries);
    if (rc == CF_OK && pred) rc = dev_alloc(ctx, dpred, sizeof(double) * n_entries);
    if (rc == CF_OK && row_sel) rc = dev_alloc(ctx, dsel, std::max<uint64_t>(n_entries, 1));
    hipError_t e = hipSuccess;
    if (rc == CF_OK) {
        auto h2d = [&](void* d, const void* h, size_t bytes) {
            if (e == hipSuccess && bytes) e = hipMemcpy(d, h, bytes, hipMemcpyHostToDevice);
        };
        h2d(doff.p, item_off, sizeof(uint64_t) * (n_users + 1));
        h2d(ditems.p, items, sizeof(uint32_t) * n_entries);
        h2d(drat.p, ratings, sizeof(float) * n_entries);
        h2d(dm.p, m, sizeof(int32_t) * n_users);
        h2d(deval.p, evals, sizeof(double) * n_entries);
        h2d(deoff.p, evec_off, sizeof(uint64_t) * n_users);
        h2d(devec.p, evecs, sizeof(EV) * n_evec);
        h2d(dsig.p, sigtab, sizeof(double) * sigtab_len);
        if (row_sel) {
            h2d(dsel.p, row_sel, n_entries);
            // rows not selected keep the caller's outputs: seed the device copies with them
            h2d(dmse.p, mse, sizeof(float) * n_entries);
            h2d(dkk.p, kk, sizeof(int32_t) * n_entries);
            if (pred) h2d(dpred.p, pred, sizeof(double) * n_entries);
        }
        if (e != hipSuccess) rc = cf_set_error(ctx, CF_EHIP, std::string("predict H2D: ") + hipGetErrorString(e));
    }
    if (rc == CF_OK) {
        if constexpr (std::is_same<EV, double>::value) {
            rc = cf_launch_predict<double>(ctx, plan, (const uint64_t*)doff.p, (const uint32_t*)ditems.p,
                                           (const float*)drat.p, (const int32_t*)dm.p, (const double*)deval.p,
                                           (const uint64_t*)deoff.p, (const double*)devec.p, (const double*)dsig.p,
                                           sig_mode, (float*)dmse.p, (int32_t*)dkk.p, (double*)dpred.p,
                                           (const uint8_t*)dsel.p, nullptr);
        } else {
            // the fp32 launch takes fp32 evals / sigs: the binary file's values, narrowed back exactly.
            // A value fp32 cannot hold (fp64 text parsed next to fp32 blocks) would move lim / w_lim
            // away from the fp64 path's: rejected rather than silently rounded.
            std::vector<float> ev32(n_entries), sg32(sigtab_len);
            const auto exact = [](double x) { return std::isnan(x) || (double)(float)x == x; };
            for (uint64_t i = 0; i < n_entries && rc == CF_OK; ++i) {
                ev32[i] = (float)evals[i];
                if (!exact(evals[i]))
                    rc = cf_set_error(ctx, CF_EINVAL, "cf_predict_precomp_sel_f32: evals[" + std::to_string(i) +
                                                          "] is not an fp32 value (use the fp64 entry point)");
            }
            for (uint64_t i = 0; i < sigtab_len && rc == CF_OK; ++i) {
                sg32[i] = (float)sigtab[i];
                if (!exact(sigtab[i]))
                    rc = cf_set_error(ctx, CF_EINVAL, "cf_predict_precomp_sel_f32: sigtab[" + std::to_string(i) +
                                                          "] is not an fp32 value (use the fp64 entry point)");
            }
            if (rc == CF_OK) rc = dev_alloc(ctx, deval32, sizeof(float) * std::max<uint64_t>(n_entries, 1));
            if (rc == CF_OK) rc = dev_alloc(ctx, dsig32, sizeof(float) * std::max<uint64_t>(sigtab_len, 1));
            if (rc == CF_OK && n_entries) e = hipMemcpy(deval32.p, ev32.data(), sizeof(float) * n_entries, hipMemcpyHostToDevice);
            if (rc == CF_OK && e == hipSuccess && sigtab_len)
                e = hipMemcpy(dsig32.p, sg32.data(), sizeof(float) * sigtab_len, hipMemcpyHostToDevice);
            if (rc == CF_OK && e != hipSuccess) rc = cf_set_error(ctx, CF_EHIP, std::string("predict H2D: ") + hipGetErrorString(e));
            if (rc == CF_OK)
                rc = cf_launch_predict<float>(ctx, plan, (const uint64_t*)doff.p, (const uint32_t*)ditems.p,
                                              (const float*)drat.p, (const int32_t*)dm.p, (const float*)deval32.p,
                                              (const uint64_t*)deoff.p, (const float*)devec.p, (const float*)dsig32.p,
                                              sig_mode, (float*)dmse.p, (int32_t*)dkk.p, (double*)dpred.p,
                                              (const uint8_t*)dsel.p, nullptr);
        }
    }
    if (rc == CF_OK) {
        e = hipDeviceSynchronize();
        if (e == hipSuccess && n_entries) e = hipMemcpy(mse, dmse.p, sizeof(float) * n_entries, hipMemcpyDeviceToHost);
        if (e == hipSuccess && n_entries) e = hipMemcpy(kk, dkk.p, sizeof(int32_t) * n_entries, hipMemcpyDeviceToHost);
        if (e == hipSuccess && n_entries && pred)
            e = hipMemcpy(pred, dpred.p, sizeof(double) * n_entries, hipMemcpyDeviceToHost);
        if (e != hipSuccess) rc = cf_set_error(ctx, CF_EHIP, std::string("predict run: ") + hipGetErrorString(e));
    }
    cf_plan_destroy(plan);
    return rc;
}
}  // namespace

extern "C" {

int cf_predict_precomp_sel(cf_ctx* ctx, uint32_t n_users, const uint64_t* item_off, const uint32_t* items,
                           const float* ratings, const int32_t* m, const double* evals, const uint64_t* evec_off,
                           const double* evecs, const double* sigtab, uint64_t sigtab_len, int sig_mode,
                           const uint8_t* row_sel, float* mse, int32_t* kk, double* pred) {
    return predict_precomp_impl<double>(ctx, n_users, item_off, items, ratings, m, evals, evec_off, evecs, sigtab,
                                        sigtab_len, sig_mode, row_sel, mse, kk, pred);
}

int cf_predict_precomp_sel_f32(cf_ctx* ctx, uint32_t n_users, const uint64_t* item_off, const uint32_t* items,
                               const float* ratings, const int32_t* m, const double* evals, const uint64_t* evec_off,
                               const float* evecs, const double* sigtab, uint64_t sigtab_len, int sig_mode,
                               const uint8_t* row_sel, float* mse, int32_t* kk, double* pred) {
    return predict_precomp_impl<float>(ctx, n_users, item_off, items, ratings, m, evals, evec_off, evecs, sigtab,
                                       sigtab_len, sig_mode, row_sel, mse, kk, pred);
}

// ---- knn2: weights_calc over transform_edges (knn2.cpp:127-164) ---------------------
static bool integer_small(const float* r, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i)
        if (!(r[i] == std::nearbyint(r[i])) || r[i] < -11.0f || r[i] > 11.0f) return false;
    return true;
}

int cf_item_cosine_run(cf_ctx* ctx, uint32_t n_users, uint32_t n_items, const uint64_t* d_user_off,
                       const uint32_t* d_item, const float* d_rating, int integer_ratings, float w_min,
                       int cnt_min, float* d_w_out, void* stream) {
    if (!ctx || !d_w_out) return cf_set_error(ctx, CF_EINVAL, "cf_item_cosine_run: null");
    CF_TRY(set_device(ctx));
    return cf_launch_knn2(ctx, n_users, n_items, d_user_off, d_item, d_rating, integer_ratings, w_min, cnt_min,
                          d_w_out, (hipStream_t)stream);
}

int cf_knn2_timing(cf_ctx* ctx, float* plane_ms, float* gemm_ms, int* path) {
    if (!ctx) return CF_EINVAL;
    if (!ctx->knn_ev[2]) return cf_set_error(ctx, CF_ESTATE, "cf_knn2_timing: no knn2 launch yet");
    CF_TRY(set_device(ctx));
    CF_HIP_CHECK(ctx, hipEventSynchronize(ctx->knn_ev[2]));
    float a = 0.0f, b = 0.0f;
    CF_HIP_CHECK(ctx, hipEventElapsedTime(&a, ctx->knn_ev[0], ctx->knn_ev[1]));
    CF_HIP_CHECK(ctx, hipEventElapsedTime(&b, ctx->knn_ev[1], ctx->knn_ev[2]));
    if (plane_ms) *plane_ms = a;
    if (gemm_ms) *gemm_ms = b;
    if (path) *path = ctx->knn_path;
    return CF_OK;
}

int cf_set_knn2_chunk(cf_ctx* ctx, uint32_t users_per_chunk) {
    if (!ctx) return CF_EINVAL;
    ctx->knn_chunk_users = users_per_chunk;
    return CF_OK;
}

int cf_knn2_chunks(cf_ctx* ctx, int* n_chunks) {
    if (!ctx || !n_chunks) return CF_EINVAL;
    *n_chunks = ctx->knn_chunks;
    return CF_OK;
}

int cf_knn2_exactness(cf_ctx* ctx, double* max_accumulator, int* exact) {
    if (!ctx) return CF_EINVAL;
    if (!ctx->d_knn_acc || !ctx->knn_ev[2]) return cf_set_error(ctx, CF_ESTATE, "cf_knn2_exactness: no knn2 launch yet");
    CF_TRY(set_device(ctx));
    CF_HIP_CHECK(ctx, hipEventSynchronize(ctx->knn_ev[2]));
    unsigned int bits = 0;
    CF_HIP_CHECK(ctx, hipMemcpy(&bits, ctx->d_knn_acc, sizeof(bits), hipMemcpyDeviceToHost));
    float v;
    std::memcpy(&v, &bits, sizeof(v));
    if (max_accumulator) *max_accumulator = (double)v;
    if (exact) *exact = ctx->knn_path != 3 && (double)v <= 16777216.0;
    return CF_OK;
}

int cf_item_cosine(cf_ctx* ctx, uint32_t n_users, uint32_t n_items, const uint64_t* user_off,
                   const uint32_t* item, const float* rating, float w_min, int cnt_min, int adopt_as_graph,
                   float* w_out) {
    if (!ctx || !user_off || (user_off[n_users] && (!item || !rating)) || (!w_out && !adopt_as_graph))
        return cf_set_error(ctx, CF_EINVAL, "cf_item_cosine: null argument");
    CF_TRY(set_device(ctx));
    const uint64_t n = user_off[n_users];
    for (uint64_t e = 0; e < n; ++e)
        if (item[e] >= n_items) return cf_set_error(ctx, CF_EINVAL, "cf_item_cosine: item index out of range");
    const int integer = integer_small(rating, n);
    DevBuf doff, ditem, drat;
    float* dW = nullptr;
    int rc = dev_alloc(ctx, doff, sizeof(uint64_t) * (n_users + 1));
    if (rc == CF_OK) rc = dev_alloc(ctx, ditem, sizeof(uint32_t) * n);
    if (rc == CF_OK) rc = dev_alloc(ctx, drat, sizeof(float) * n);
    if (rc == CF_OK && hipMalloc(&dW, std::max<size_t>((size_t)n_items * n_items * sizeof(float), 16)) != hipSuccess)
        rc = cf_set_error(ctx, CF_ENOMEM, "cf_item_cosine: weight matrix allocation");
    hipError_t e = hipSuccess;
    if (rc == CF_OK) {
        e = hipMemcpy(doff.p, user_off, sizeof(uint64_t) * (n_users + 1), hipMemcpyHostToDevice);
        if (e == hipSuccess && n) e = hipMemcpy(ditem.p, item, sizeof(uint32_t) * n, hipMemcpyHostToDevice);
        if (e == hipSuccess && n) e = hipMemcpy(drat.p, rating, sizeof(float) * n, hipMemcpyHostToDevice);
        if (e != hipSuccess) rc = cf_set_error(ctx, CF_EHIP, std::string("knn2 H2D: ") + hipGetErrorString(e));
    }
    if (rc == CF_OK)
        rc = cf_launch_knn2(ctx, n_users, n_items, (const uint64_t*)doff.p, (const uint32_t*)ditem.p,
                            (const float*)drat.p, integer, w_min, cnt_min, dW, nullptr);
    if (rc == CF_OK) {
        e = hipDeviceSynchronize();
        if (e == hipSuccess && w_out)
            e = hipMemcpy(w_out, dW, (size_t)n_items * n_items * sizeof(float), hipMemcpyDeviceToHost);
        if (e != hipSuccess) rc = cf_set_error(ctx, CF_EHIP, std::string("knn2 run: ") + hipGetErrorString(e));
    }
    if (rc == CF_OK && adopt_as_graph) {   // in the context's upload layout (cf_graph.hip)
        rc = cf_adopt_dense_graph(ctx, n_items, dW);
        dW = nullptr;
    }
    if (dW) (void)hipFree(dW);
    return rc;
}

// ---- knn3: knn_program + error_vertex_data (knn3.cpp:185-256) ----------------------
int cf_knn_predict(cf_ctx* ctx, uint32_t n_users, const uint64_t* user_off, const uint32_t* items,
                   const float* ratings, double* pred, float* movie_mse, uint32_t* movie_count) {
    if (!ctx || !user_off || !movie_mse || (user_off[n_users] && (!items || !ratings)))
        return cf_set_error(ctx, CF_EINVAL, "cf_knn_predict: null argument");
    if (!has_graph(ctx)) return cf_set_error(ctx, CF_ESTATE, "cf_knn_predict: no item graph uploaded");
    CF_TRY(set_device(ctx));
    const uint64_t n = user_off[n_users];
    for (uint64_t e = 0; e < n; ++e)
        if (items[e] >= ctx->n_items) return cf_set_error(ctx, CF_EINVAL, "cf_knn_predict: item out of range");
    const uint32_t I = ctx->n_items;
    const bool integer = integer_small(ratings, n);
    DevBuf doff, ditem, drat, dpred, dsq, dsqr, dcnt;
    int rc = dev_alloc(ctx, doff, sizeof(uint64_t) * (n_users + 1));
    if (rc == CF_OK) rc = dev_alloc(ctx, ditem, sizeof(uint32_t) * n);
    if (rc == CF_OK) rc = dev_alloc(ctx, drat, sizeof(float) * n);
    if (rc == CF_OK) rc = dev_alloc(ctx, dpred, sizeof(double) * n);
    if (rc == CF_OK) rc = dev_alloc(ctx, dsq, sizeof(unsigned long long) * I);
    if (rc == CF_OK) rc = dev_alloc(ctx, dsqr, sizeof(double) * I);
    if (rc == CF_OK) rc = dev_alloc(ctx, dcnt, sizeof(unsigned int) * I);
    hipError_t e = hipSuccess;
    if (rc == CF_OK) {
        e = hipMemcpy(doff.p, user_off, sizeof(uint64_t) * (n_users + 1), hipMemcpyHostToDevice);
        if (e == hipSuccess && n) e = hipMemcpy(ditem.p, items, sizeof(uint32_t) * n, hipMemcpyHostToDevice);
        if (e == hipSuccess && n) e = hipMemcpy(drat.p, ratings, sizeof(float) * n, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemset(dsq.p, 0, sizeof(unsigned long long) * I);
        if (e == hipSuccess) e = hipMemset(dsqr.p, 0, sizeof(double) * I);
        if (e == hipSuccess) e = hipMemset(dcnt.p, 0, sizeof(unsigned int) * I);
        if (e != hipSuccess) rc = cf_set_error(ctx, CF_EHIP, std::string("knn3 H2D: ") + hipGetErrorString(e));
    }
    if (rc == CF_OK)
        rc = cf_launch_knn3(ctx, n_users, (const uint64_t*)doff.p, (const uint32_t*)ditem.p, (const float*)drat.p,
                            (double*)dpred.p, (unsigned long long*)dsq.p, (double*)dsqr.p, (unsigned int*)dcnt.p,
                            nullptr);
    std::vector<unsigned long long> sq(I);
    std::vector<double> sqr(I);
    std::vector<unsigned int> cnt(I);
    if (rc == CF_OK) {
        e = hipDeviceSynchronize();
        if (e == hipSuccess && pred && n) e = hipMemcpy(pred, dpred.p, sizeof(double) * n, hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(sq.data(), dsq.p, sizeof(unsigned long long) * I, hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(sqr.data(), dsqr.p, sizeof(double) * I, hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(cnt.data(), dcnt.p, sizeof(unsigned int) * I, hipMemcpyDeviceToHost);
        if (e != hipSuccess) rc = cf_set_error(ctx, CF_EHIP, std::string("knn3 run: ") + hipGetErrorString(e));
    }
    if (rc == CF_OK) {
        for (uint32_t i = 0; i < I; ++i) {
            float v = 0.0f;   // vertices without test ratings contribute 0 (:254-255)
            if (cnt[i]) {
                const float err = integer ? (float)sq[i] : (float)sqr[i];
                v = std::isnan(err) ? 0.0f : err / (float)cnt[i];   // (:249-253)
            }
            movie_mse[i] = v;
            if (movie_count) movie_count[i] = cnt[i];
        }
    }
    return rc;
}

}  // extern "C"
