// cf_pack.hip -- the out_eigen_ gather of the multi-GPU path.
//
// The reference writes every user's record into one out_eigen_ file from a thread pool
// (precompute_local_threads.cpp:196-211, 300-314) and every GraphLab rank later reads the
// whole file (local_calc_precomp.cpp:485-486, 509).  Here users are range-split across
// GPUs by cumulative k^3 cost; each GPU packs its variable-size k x m eigenvector blocks
// (stored in k*max(k,2) slots by the eigen kernels) into one contiguous run, and the runs
// are gathered to device 0 over xGMI peer copies, where they form exactly the record
// sequence of the one-device run.
//
//   pack_offsets_kernel : one workgroup scans k_u * m_u over all users (exclusive, u64)
//   pack_copy_kernel    : one workgroup per user copies the k*m floats (16 B per lane)

#include <algorithm>
#include <thread>
#include <vector>

#include "cf_internal.h"

namespace {

constexpr int kScanThreads = 1024;

// packed_off[u] = sum_{v < u} k_v * m_v, packed_off[n_users] = total.  One workgroup: each
// thread owns a contiguous chunk of users, the chunk sums are scanned in LDS.
__global__ void __launch_bounds__(kScanThreads) pack_offsets_kernel(uint32_t n_users, const uint64_t* item_off,
                                                                    const int32_t* m, uint64_t* packed_off) {
    __shared__ uint64_t s_sum[kScanThreads];
    const uint32_t t = threadIdx.x;
    const uint32_t chunk = (n_users + kScanThreads - 1) / kScanThreads;
    const uint32_t u0 = min(n_users, t * chunk), u1 = min(n_users, u0 + chunk);
    uint64_t s = 0;
    for (uint32_t u = u0; u < u1; ++u) s += (item_off[u + 1] - item_off[u]) * (uint64_t)max(m[u], 0);
    s_sum[t] = s;
    __syncthreads();
    for (int d = 1; d < kScanThreads; d <<= 1) {   // Hillis-Steele inclusive scan
        const uint64_t v = t >= (uint32_t)d ? s_sum[t - d] : 0;
        __syncthreads();
        s_sum[t] += v;
        __syncthreads();
    }
    uint64_t run = s_sum[t] - s;
    for (uint32_t u = u0; u < u1; ++u) {
        packed_off[u] = run;
        run += (item_off[u + 1] - item_off[u]) * (uint64_t)max(m[u], 0);
    }
    if (t == kScanThreads - 1) packed_off[n_users] = s_sum[t];
}

// The first k*m floats of user u's slot are its k x m row-major block.
__global__ void __launch_bounds__(256) pack_copy_kernel(uint32_t n_users, const uint64_t* item_off, const int32_t* m,
                                                        const uint64_t* evec_off, const float* evecs,
                                                        const uint64_t* packed_off, float* packed) {
    for (uint32_t u = blockIdx.x; u < n_users; u += gridDim.x) {
        const uint64_t n = (item_off[u + 1] - item_off[u]) * (uint64_t)max(m[u], 0);
        const float* src = evecs + evec_off[u];
        float* dst = packed + packed_off[u];
        // 16-byte lanes where both ends share the alignment (slot and packed offsets are
        // arbitrary multiples of 4 B), scalar head/tail otherwise
        const uint64_t mis_s = ((uintptr_t)src >> 2) & 3, mis_d = ((uintptr_t)dst >> 2) & 3;
        if (mis_s == mis_d) {
            const uint64_t head = min<uint64_t>(n, (4 - mis_s) & 3);
            for (uint64_t i = threadIdx.x; i < head; i += blockDim.x) dst[i] = src[i];
            const uint64_t nv = (n - head) / 4;
            const float4* s4 = reinterpret_cast<const float4*>(src + head);
            float4* d4 = reinterpret_cast<float4*>(dst + head);
            for (uint64_t i = threadIdx.x; i < nv; i += blockDim.x) d4[i] = s4[i];
            for (uint64_t i = head + nv * 4 + threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
        } else {
            for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
        }
    }
}

// Contiguous split points balancing sum(k^3) (the cost of both the eigensolve and the
// per-user predictor basis): split[p] = the first user whose prefix cost reaches p/n_parts
// of the total (the same rule as collaborative_filtering_amd/multi.py:cost_split).
void cost_split(uint32_t n_users, const uint64_t* item_off, int n_parts, uint32_t* split) {
    std::vector<double> cum(n_users + 1, 0.0);
    for (uint32_t u = 0; u < n_users; ++u) {
        const double k = (double)(item_off[u + 1] - item_off[u]);
        cum[u + 1] = cum[u] + k * k * k;
    }
    split[0] = 0;
    for (int p = 1; p < n_parts; ++p) {
        const double target = cum[n_users] * (double)p / (double)n_parts;
        const uint32_t j = (uint32_t)(std::lower_bound(cum.begin(), cum.end(), target) - cum.begin());
        split[p] = std::max(split[p - 1], std::min(j, n_users));
    }
    split[n_parts] = n_users;
}

}  // namespace

namespace {
template <typename EV, typename SEL>
int predict_precomp_multi_impl(SEL sel, cf_ctx* const* ctxs, int n_dev, uint32_t n_users, const uint64_t* item_off,
                               const uint32_t* items, const float* ratings, const int32_t* m, const double* evals,
                               const uint64_t* evec_off, const EV* evecs, const double* sigtab,
                               uint64_t sigtab_len, int sig_mode, const uint8_t* row_sel, float* mse, int32_t* kk,
                               double* pred, uint32_t* split_out) {
    if (!ctxs || n_dev <= 0 || !ctxs[0]) return CF_EINVAL;
    cf_ctx* root = ctxs[0];
    if (!item_off || !items || !ratings || !m || !evals || !evec_off || !evecs || !sigtab || !mse || !kk)
        return cf_set_error(root, CF_EINVAL, "cf_predict_precomp_multi: null argument");
    if (sig_mode != CF_SIGS_OWN && sig_mode != CF_SIGS_COMPAT)
        return cf_set_error(root, CF_EINVAL, "cf_predict_precomp_multi: bad sig_mode");
    if (sig_mode == CF_SIGS_OWN && sigtab_len < item_off[n_users])
        return cf_set_error(root, CF_EINVAL, "cf_predict_precomp_multi: sig table shorter than item_off[n_users]");
    for (int d = 0; d < n_dev; ++d)
        if (!ctxs[d]) return cf_set_error(root, CF_EINVAL, "cf_predict_precomp_multi: null context");
    std::vector<uint32_t> split(n_dev + 1);
    cost_split(n_users, item_off, n_dev, split.data());
    if (split_out) std::copy(split.begin(), split.end(), split_out);
    std::vector<int> rcs(n_dev, CF_OK);
    std::vector<std::thread> pool;
    for (int d = 0; d < n_dev; ++d)
        pool.emplace_back([&, d]() {
            const uint32_t u0 = split[d], nu = split[d + 1] - split[d];
            if (nu == 0) return;
            const uint64_t e0 = item_off[u0], ne = item_off[u0 + nu] - e0;
            // the part's eigenvector blocks start at its smallest offset; offsets re-based on it
            uint64_t lo = UINT64_MAX;
            std::vector<uint64_t> off(nu + 1), eoff(nu);
            for (uint32_t u = 0; u < nu; ++u) lo = std::min(lo, evec_off[u0 + u]);
            for (uint32_t u = 0; u <= nu; ++u) off[u] = item_off[u0 + u] - e0;
            for (uint32_t u = 0; u < nu; ++u) eoff[u] = evec_off[u0 + u] - lo;
            const bool compat = sig_mode == CF_SIGS_COMPAT;
            rcs[d] = sel(ctxs[d], nu, off.data(), items + e0, ratings + e0, m + u0, evals + e0,
                                            eoff.data(), evecs + lo, compat ? sigtab : sigtab + e0,
                                            compat ? sigtab_len : ne, sig_mode, row_sel ? row_sel + e0 : nullptr,
                                            mse + e0, kk + e0, pred ? pred + e0 : nullptr);
        });
    for (auto& t : pool) t.join();
    for (int d = 0; d < n_dev; ++d)
        if (rcs[d] != CF_OK)
            return cf_set_error(root, rcs[d], "device part " + std::to_string(d) + ": " + ctxs[d]->last_error);
    (void)hipSetDevice(root->device);
    return CF_OK;
}

}  // namespace

extern "C" {

int cf_cost_split(uint32_t n_users, const uint64_t* item_off, int n_parts, uint32_t* split) {
    if (!item_off || !split || n_parts <= 0) return CF_EINVAL;
    cost_split(n_users, item_off, n_parts, split);
    return CF_OK;
}

int cf_pack_eigen_run(cf_ctx* ctx, uint32_t n_users, const uint64_t* d_item_off, const int32_t* d_m,
                      const uint64_t* d_evec_off, const float* d_evecs, uint64_t* d_packed_off, float* d_packed,
                      void* stream) {
    if (!ctx || !d_item_off || !d_m || !d_packed_off) return cf_set_error(ctx, CF_EINVAL, "cf_pack_eigen_run: null");
    if (d_packed && (!d_evec_off || !d_evecs)) return cf_set_error(ctx, CF_EINVAL, "cf_pack_eigen_run: null evecs");
    CF_TRY(set_device(ctx));
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(pack_offsets_kernel, dim3(1), dim3(kScanThreads), 0, st, n_users, d_item_off, d_m,
                       d_packed_off);
    CF_HIP_CHECK(ctx, hipGetLastError());
    if (d_packed && n_users) {
        const uint32_t blocks = std::min<uint32_t>(n_users, 65536u);
        hipLaunchKernelGGL(pack_copy_kernel, dim3(blocks), dim3(256), 0, st, n_users, d_item_off, d_m, d_evec_off,
                           d_evecs, (const uint64_t*)d_packed_off, d_packed);
        CF_HIP_CHECK(ctx, hipGetLastError());
    }
    return CF_OK;
}

// One device's share of cf_eigen_batch_multi: its user range on its own context and
// stream, packed on the device.  Buffers stay allocated for the gather.
struct multi_part {
    cf_ctx* ctx = nullptr;
    uint32_t u0 = 0, n = 0;
    uint64_t e0 = 0, ne = 0;     // entry range (item_off) of the part
    uint64_t packed = 0;         // floats in the packed run
    DevBuf off, items, eoff, m, sig, eval, evec, poff, pack;
    hipStream_t stream = nullptr;
    int rc = CF_OK;
};

static int multi_run_part(multi_part& p, const uint64_t* item_off, const uint32_t* items) {
    cf_ctx* ctx = p.ctx;
    CF_TRY(set_device(ctx));
    CF_HIP_CHECK(ctx, hipStreamCreateWithFlags(&p.stream, hipStreamNonBlocking));
    std::vector<uint64_t> off(p.n + 1), eoff(std::max<uint32_t>(p.n, 1));
    for (uint32_t u = 0; u <= p.n; ++u) off[u] = item_off[p.u0 + u] - p.e0;
    const uint64_t n_evec = cf_evec_offsets(p.n, off.data(), eoff.data());
    for (uint64_t e = 0; e < p.ne; ++e)
        if (items[p.e0 + e] >= ctx->n_items) return cf_set_error(ctx, CF_EINVAL, "item index outside the graph");
    cf_plan* plan = nullptr;
    CF_TRY(cf_plan_create(ctx, p.n, off.data(), &plan));
    int rc = dev_alloc(ctx, p.off, sizeof(uint64_t) * (p.n + 1));
    if (rc == CF_OK) rc = dev_alloc(ctx, p.items, sizeof(uint32_t) * p.ne);
    if (rc == CF_OK) rc = dev_alloc(ctx, p.eoff, sizeof(uint64_t) * eoff.size());
    if (rc == CF_OK) rc = dev_alloc(ctx, p.m, sizeof(int32_t) * std::max<uint32_t>(p.n, 1));
    if (rc == CF_OK) rc = dev_alloc(ctx, p.sig, sizeof(float) * p.ne);
    if (rc == CF_OK) rc = dev_alloc(ctx, p.eval, sizeof(float) * p.ne);
    if (rc == CF_OK) rc = dev_alloc(ctx, p.evec, sizeof(float) * n_evec);
    if (rc == CF_OK) rc = dev_alloc(ctx, p.poff, sizeof(uint64_t) * (p.n + 1));
    hipError_t e = hipSuccess;
    if (rc == CF_OK) {
        e = hipMemcpyAsync(p.off.p, off.data(), sizeof(uint64_t) * (p.n + 1), hipMemcpyHostToDevice, p.stream);
        if (e == hipSuccess && p.ne)
            e = hipMemcpyAsync(p.items.p, items + p.e0, sizeof(uint32_t) * p.ne, hipMemcpyHostToDevice, p.stream);
        if (e == hipSuccess && p.n)
            e = hipMemcpyAsync(p.eoff.p, eoff.data(), sizeof(uint64_t) * p.n, hipMemcpyHostToDevice, p.stream);
        if (e == hipSuccess) e = hipMemsetAsync(p.eval.p, 0, sizeof(float) * std::max<uint64_t>(p.ne, 1), p.stream);
        if (e != hipSuccess) rc = cf_set_error(ctx, CF_EHIP, std::string("eigen H2D: ") + hipGetErrorString(e));
    }
    if (rc == CF_OK)
        rc = cf_launch_eigen(ctx, plan, (const uint64_t*)p.off.p, (const uint32_t*)p.items.p,
                             (const uint64_t*)p.eoff.p, (int32_t*)p.m.p, (float*)p.sig.p, (float*)p.eval.p,
                             (float*)p.evec.p, p.stream);
    if (rc == CF_OK)
        rc = cf_pack_eigen_run(ctx, p.n, (const uint64_t*)p.off.p, (const int32_t*)p.m.p, nullptr, nullptr,
                               (uint64_t*)p.poff.p, nullptr, p.stream);
    if (rc == CF_OK) {
        e = hipMemcpyAsync(&p.packed, (const uint64_t*)p.poff.p + p.n, sizeof(uint64_t), hipMemcpyDeviceToHost,
                           p.stream);
        if (e == hipSuccess) e = hipStreamSynchronize(p.stream);
        if (e != hipSuccess) rc = cf_set_error(ctx, CF_EHIP, std::string("eigen run: ") + hipGetErrorString(e));
    }
    if (rc == CF_OK) rc = dev_alloc(ctx, p.pack, sizeof(float) * p.packed);
    if (rc == CF_OK)
        rc = cf_pack_eigen_run(ctx, p.n, (const uint64_t*)p.off.p, (const int32_t*)p.m.p, (const uint64_t*)p.eoff.p,
                               (const float*)p.evec.p, (uint64_t*)p.poff.p, (float*)p.pack.p, p.stream);
    if (rc == CF_OK) {
        e = hipStreamSynchronize(p.stream);
        if (e != hipSuccess) rc = cf_set_error(ctx, CF_EHIP, std::string("eigen pack: ") + hipGetErrorString(e));
    }
    if (p.evec.p) {   // the slots are no longer needed once packed
        (void)hipFree(p.evec.p);
        p.evec.p = nullptr;
    }
    cf_plan_destroy(plan);
    return rc;
}

int cf_eigen_batch_multi(cf_ctx* const* ctxs, int n_dev, uint32_t n_users, const uint64_t* item_off,
                         const uint32_t* items, int32_t* m_out, float* sigs, float* evals, uint64_t* packed_off,
                         float* packed_evecs, uint64_t packed_cap, uint32_t* split_out) {
    if (!ctxs || n_dev <= 0 || !ctxs[0]) return CF_EINVAL;
    cf_ctx* root = ctxs[0];
    if (!item_off || !items || !m_out || !sigs || !evals || !packed_off || !packed_evecs)
        return cf_set_error(root, CF_EINVAL, "cf_eigen_batch_multi: null argument");
    for (int d = 0; d < n_dev; ++d) {
        if (!ctxs[d]) return cf_set_error(root, CF_EINVAL, "cf_eigen_batch_multi: null context");
        if (!has_graph(ctxs[d])) return cf_set_error(root, CF_ESTATE, "cf_eigen_batch_multi: a context has no graph");
    }
    std::vector<uint32_t> split(n_dev + 1);
    cost_split(n_users, item_off, n_dev, split.data());
    if (split_out) std::copy(split.begin(), split.end(), split_out);
    std::vector<multi_part> parts(n_dev);
    for (int d = 0; d < n_dev; ++d) {
        multi_part& p = parts[d];
        p.ctx = ctxs[d];
        p.u0 = split[d];
        p.n = split[d + 1] - split[d];
        p.e0 = item_off[p.u0];
        p.ne = item_off[split[d + 1]] - p.e0;
    }
    // every device computes and packs its range concurrently (one host thread per device,
    // as the reference's thread pool runs compute_eigens per user, :300-314)
    std::vector<std::thread> pool;
    for (int d = 0; d < n_dev; ++d)
        pool.emplace_back([&, d]() { parts[d].rc = multi_run_part(parts[d], item_off, items); });
    for (auto& t : pool) t.join();
    int rc = CF_OK;
    for (int d = 0; d < n_dev && rc == CF_OK; ++d)
        if (parts[d].rc != CF_OK)
            rc = cf_set_error(root, parts[d].rc, "device part " + std::to_string(d) + ": " + parts[d].ctx->last_error);
    uint64_t total = 0;
    for (auto& p : parts) total += p.packed;
    if (rc == CF_OK && total > packed_cap) rc = cf_set_error(root, CF_EINVAL, "cf_eigen_batch_multi: packed_cap");
    // gather to device 0: each part's packed run, m, sigs and evals land at its offsets in
    // device-0 buffers (peer copies over xGMI; a part on device 0 itself is a local copy)
    DevBuf g_m, g_sig, g_eval, g_pack;
    const uint64_t n_entries = item_off[n_users];
    if (rc == CF_OK) rc = set_device(root);
    if (rc == CF_OK) rc = dev_alloc(root, g_m, sizeof(int32_t) * std::max<uint32_t>(n_users, 1));
    if (rc == CF_OK) rc = dev_alloc(root, g_sig, sizeof(float) * n_entries);
    if (rc == CF_OK) rc = dev_alloc(root, g_eval, sizeof(float) * n_entries);
    if (rc == CF_OK) rc = dev_alloc(root, g_pack, sizeof(float) * total);
    if (rc == CF_OK) {
        int can = 0;
        for (int d = 1; d < n_dev; ++d)
            if (ctxs[d]->device != root->device && hipDeviceCanAccessPeer(&can, root->device, ctxs[d]->device) ==
                                                        hipSuccess && can) {
                const hipError_t pe = hipDeviceEnablePeerAccess(ctxs[d]->device, 0);
                if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled)
                    rc = cf_set_error(root, CF_EHIP, std::string("peer access: ") + hipGetErrorString(pe));
                (void)hipGetLastError();
            }
    }
    uint64_t pk = 0;
    for (int d = 0; d < n_dev && rc == CF_OK; ++d) {
        multi_part& p = parts[d];
        const int src = p.ctx->device, dst = root->device;
        hipError_t e = hipSuccess;
        if (p.n) e = hipMemcpyPeerAsync((int32_t*)g_m.p + p.u0, dst, p.m.p, src, sizeof(int32_t) * p.n, p.stream);
        if (e == hipSuccess && p.ne)
            e = hipMemcpyPeerAsync((float*)g_sig.p + p.e0, dst, p.sig.p, src, sizeof(float) * p.ne, p.stream);
        if (e == hipSuccess && p.ne)
            e = hipMemcpyPeerAsync((float*)g_eval.p + p.e0, dst, p.eval.p, src, sizeof(float) * p.ne, p.stream);
        if (e == hipSuccess && p.packed)
            e = hipMemcpyPeerAsync((float*)g_pack.p + pk, dst, p.pack.p, src, sizeof(float) * p.packed, p.stream);
        if (e != hipSuccess) rc = cf_set_error(root, CF_EHIP, std::string("gather: ") + hipGetErrorString(e));
        pk += p.packed;
    }
    for (auto& p : parts)
        if (p.stream) {
            (void)hipSetDevice(p.ctx->device);
            const hipError_t e = hipStreamSynchronize(p.stream);
            if (e != hipSuccess && rc == CF_OK) rc = cf_set_error(root, CF_EHIP, std::string("gather sync: ") +
                                                                                   hipGetErrorString(e));
        }
    // packed offsets on the host (k and m are known there once m is back)
    if (rc == CF_OK) rc = set_device(root);
    if (rc == CF_OK) {
        hipError_t e = hipSuccess;
        if (n_users) e = hipMemcpy(m_out, g_m.p, sizeof(int32_t) * n_users, hipMemcpyDeviceToHost);
        if (e == hipSuccess && n_entries) e = hipMemcpy(sigs, g_sig.p, sizeof(float) * n_entries, hipMemcpyDeviceToHost);
        if (e == hipSuccess && n_entries) e = hipMemcpy(evals, g_eval.p, sizeof(float) * n_entries, hipMemcpyDeviceToHost);
        if (e == hipSuccess && total) e = hipMemcpy(packed_evecs, g_pack.p, sizeof(float) * total, hipMemcpyDeviceToHost);
        if (e != hipSuccess) rc = cf_set_error(root, CF_EHIP, std::string("gather D2H: ") + hipGetErrorString(e));
    }
    if (rc == CF_OK) {
        uint64_t run = 0;
        for (uint32_t u = 0; u < n_users; ++u) {
            packed_off[u] = run;
            run += (item_off[u + 1] - item_off[u]) * (uint64_t)std::max(m_out[u], 0);
        }
        packed_off[n_users] = run;
        if (run != total) rc = cf_set_error(root, CF_EHIP, "cf_eigen_batch_multi: packed size mismatch");
    }
    for (auto& p : parts)
        if (p.stream) {
            (void)hipSetDevice(p.ctx->device);
            (void)hipStreamDestroy(p.stream);
            p.stream = nullptr;
        }
    (void)hipSetDevice(root->device);
    return rc;
}

// neigh_program::apply over ONE user set on n_dev contexts.  The reference loads the whole
// out_eigen_ on every rank and each rank predicts its own movie vertices
// (local_calc_precomp.cpp:485-486, 509, 550-558); here users are range-split by cumulative
// k^3 and every context predicts the rows of its range from its own copy of those records.
// In compat mode every part gets the WHOLE concatenated sig table: w_lim of row r is the r-th
// sig of the file (:414, 437, 440, 271), whatever range the row's user falls in.  Each part's
// rows land at their own offsets of the caller's arrays, so the results equal the one-context
// call's bit for bit.
int cf_predict_precomp_multi(cf_ctx* const* ctxs, int n_dev, uint32_t n_users, const uint64_t* item_off,
                             const uint32_t* items, const float* ratings, const int32_t* m, const double* evals,
                             const uint64_t* evec_off, const double* evecs, const double* sigtab,
                             uint64_t sigtab_len, int sig_mode, const uint8_t* row_sel, float* mse, int32_t* kk,
                             double* pred, uint32_t* split_out) {
    return predict_precomp_multi_impl<double>(cf_predict_precomp_sel, ctxs, n_dev, n_users, item_off, items, ratings, m,
                                              evals, evec_off, evecs, sigtab, sigtab_len, sig_mode, row_sel, mse, kk,
                                              pred, split_out);
}

int cf_predict_precomp_multi_f32(cf_ctx* const* ctxs, int n_dev, uint32_t n_users, const uint64_t* item_off,
                                 const uint32_t* items, const float* ratings, const int32_t* m, const double* evals,
                                 const uint64_t* evec_off, const float* evecs, const double* sigtab,
                                 uint64_t sigtab_len, int sig_mode, const uint8_t* row_sel, float* mse, int32_t* kk,
                                 double* pred, uint32_t* split_out) {
    return predict_precomp_multi_impl<float>(cf_predict_precomp_sel_f32, ctxs, n_dev, n_users, item_off, items, ratings,
                                             m, evals, evec_off, evecs, sigtab, sigtab_len, sig_mode, row_sel, mse, kk,
                                             pred, split_out);
}

}  // extern "C"
