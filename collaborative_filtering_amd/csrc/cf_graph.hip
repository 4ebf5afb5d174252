// cf_graph.hip -- the resident item graph in CSR layout, and knn2's compacted edge list.
//
// The reference holds the item graph as a dense 2000 x 2000 matrix
// (precompute_local_threads.cpp:253-293) or as GraphLab out-edges (local_calc_precomp.cpp:
// 122-136), and knn2 writes it as the edge list "a b w" for w > 0.01 (knn2.cpp:151-164).
// Here the graph is HBM-resident either dense (n^2 fp32, direct indexing: catalogues up to
// ~250k items per GPU) or CSR (u64 row pointers, ascending u32 columns, f32 weights: any
// catalogue whose edges fit), selected by cf_set_graph_layout; every kernel reads it through
// GraphDev::row(a)[b] (cf_internal.h), so both layouts give the same floats.
//
//   row_nnz_kernel      one workgroup per row of a dense matrix: its nonzero count
//   row_compact_kernel  one workgroup per row: the nonzeros in ascending column order
//                       (wave ballots + a per-workgroup running offset), into CSR
#include <algorithm>
#include <cstring>
#include <numeric>
#include <thread>

#include "cf_internal.h"

namespace {

constexpr int kGT = 256;

__global__ __launch_bounds__(kGT) void row_nnz_kernel(uint64_t n, const float* dense, uint64_t* cnt) {
    __shared__ unsigned int s_c[kGT / 64];
    for (uint64_t r = blockIdx.x; r < n; r += gridDim.x) {
        const float* row = dense + r * n;
        unsigned int c = 0;
        for (uint64_t j = threadIdx.x; j < n; j += kGT) c += row[j] != 0.0f;
        for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o);
        if ((threadIdx.x & 63) == 0) s_c[threadIdx.x >> 6] = c;
        __syncthreads();
        if (threadIdx.x == 0) cnt[r] = (uint64_t)s_c[0] + s_c[1] + s_c[2] + s_c[3];
        __syncthreads();
    }
}

// Optional top-K per row (cf_set_knn2_topk): the K largest weights of the row, ties at the
// K-th value broken by ascending column.  One workgroup per row finds the K-th largest key by
// a 4 x 8-bit radix select over order-preserving keys of the float bits (sign bit set for
// positives, all bits flipped for negatives: a w_min < 0 keeps negative cosines, which must
// rank below every positive weight); thr[r] = that key, take[r] = how many of the entries
// equal to it are kept (the first ones in column order), cnt[r] = min(nnz, K).  Rows with at
// most K entries keep them all (thr 0).
__device__ __forceinline__ uint32_t order_key(uint32_t bits) {
    return (bits & 0x80000000u) ? ~bits : (bits | 0x80000000u);
}

__global__ __launch_bounds__(kGT) void row_topk_kernel(uint64_t n, const float* dense, uint32_t K, uint32_t* thr,
                                                       uint32_t* take, uint64_t* cnt) {
    __shared__ unsigned int s_hist[256];
    __shared__ unsigned int s_c[kGT / 64];
    __shared__ unsigned int s_sel[2];
    for (uint64_t r = blockIdx.x; r < n; r += gridDim.x) {
        const uint32_t* row = reinterpret_cast<const uint32_t*>(dense + r * n);
        unsigned int c = 0;
        for (uint64_t j = threadIdx.x; j < n; j += kGT) c += row[j] != 0u && (row[j] << 1) != 0u;
        for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o);
        if ((threadIdx.x & 63) == 0) s_c[threadIdx.x >> 6] = c;
        __syncthreads();
        const unsigned int total = s_c[0] + s_c[1] + s_c[2] + s_c[3];
        __syncthreads();
        if (total <= K) {
            if (threadIdx.x == 0) {
                thr[r] = 0u;
                take[r] = 0xffffffffu;
                cnt[r] = total;
            }
            continue;
        }
        uint32_t prefix = 0, mask = 0, rem = K;   // rem: entries still to take at or below the prefix
        for (int shift = 24; shift >= 0; shift -= 8) {
            s_hist[threadIdx.x] = 0u;   // kGT == 256 bins
            __syncthreads();
            for (uint64_t j = threadIdx.x; j < n; j += kGT) {
                const uint32_t bits = row[j], key = order_key(bits);
                if ((bits << 1) != 0u && (key & mask) == prefix) atomicAdd(&s_hist[(key >> shift) & 255u], 1u);
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                unsigned int above = 0;
                int b = 255;
                for (; b > 0; --b) {
                    if (above + s_hist[b] >= rem) break;
                    above += s_hist[b];
                }
                s_sel[0] = (unsigned int)b;
                s_sel[1] = above;
            }
            __syncthreads();
            prefix |= s_sel[0] << shift;
            mask |= 255u << shift;
            rem -= s_sel[1];
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            thr[r] = prefix;
            take[r] = rem;
            cnt[r] = K;
        }
    }
}

__global__ __launch_bounds__(kGT) void row_compact_kernel(uint64_t n, const float* dense, const uint64_t* rp,
                                                          uint32_t* col, float* w, const uint32_t* thr,
                                                          const uint32_t* take) {
    __shared__ unsigned int s_c[kGT / 64];
    __shared__ unsigned int s_t[kGT / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint64_t r = blockIdx.x; r < n; r += gridDim.x) {
        const float* row = dense + r * n;
        const uint32_t T = thr ? thr[r] : 0u, tk = thr ? take[r] : 0xffffffffu;
        uint64_t pos = rp[r];
        unsigned int ties = 0;   // entries equal to the threshold seen so far (column order)
        for (uint64_t j0 = 0; j0 < n; j0 += kGT) {
            const uint64_t j = j0 + threadIdx.x;
            const float v = j < n ? row[j] : 0.0f;
            const uint32_t key = order_key(__float_as_uint(v));
            const bool nz = v != 0.0f;
            const bool tie = nz && thr && key == T;
            const unsigned long long tb = __ballot(tie);
            if (lane == 0) s_t[wave] = (unsigned int)__popcll(tb);
            __syncthreads();
            unsigned int tbefore = 0, tall = 0;
            for (int x = 0; x < kGT / 64; ++x) {
                tbefore += x < wave ? s_t[x] : 0u;
                tall += s_t[x];
            }
            const unsigned int trank = ties + tbefore + (unsigned int)__popcll(tb & ((1ull << lane) - 1ull));
            const bool keep = nz && (!thr || key > T || (tie && trank < tk));
            const unsigned long long bal = __ballot(keep);
            if (lane == 0) s_c[wave] = (unsigned int)__popcll(bal);
            __syncthreads();
            unsigned int before = 0, all = 0;
            for (int x = 0; x < kGT / 64; ++x) {
                before += x < wave ? s_c[x] : 0u;
                all += s_c[x];
            }
            if (keep) {
                const uint64_t o = pos + before + (unsigned int)__popcll(bal & ((1ull << lane) - 1ull));
                col[o] = (uint32_t)j;
                w[o] = v;
            }
            pos += all;
            ties += tall;
            __syncthreads();
        }
    }
}

void free_graph(cf_ctx* ctx) {
    ++ctx->graph_gen;   // complement masks of earlier eigen runs no longer apply
    if (ctx->d_graph) (void)hipFree(ctx->d_graph);
    if (ctx->d_grp) (void)hipFree(ctx->d_grp);
    if (ctx->d_gcol) (void)hipFree(ctx->d_gcol);
    if (ctx->d_gw) (void)hipFree(ctx->d_gw);
    ctx->d_graph = nullptr;
    ctx->d_grp = nullptr;
    ctx->d_gcol = nullptr;
    ctx->d_gw = nullptr;
    ctx->graph_csr = false;
    ctx->g_nnz = 0;
    ctx->n_items = 0;
}

}  // namespace

// Dense n x n device matrix -> CSR in new device buffers (row pointers through the host: n + 1
// words).  Synchronous on `stream`.
int cf_dense_to_csr(cf_ctx* ctx, uint32_t n, const float* d_dense, uint64_t** d_rp, uint32_t** d_col, float** d_w,
                    uint64_t* nnz, hipStream_t stream, uint32_t topk) {
    *d_rp = nullptr;
    *d_col = nullptr;
    *d_w = nullptr;
    std::vector<uint64_t> rp((size_t)n + 1, 0);
    CF_HIP_CHECK(ctx, hipMalloc(d_rp, sizeof(uint64_t) * ((size_t)n + 1)));
    DevBuf dthr, dtake;
    if (topk) {
        CF_TRY(dev_alloc(ctx, dthr, sizeof(uint32_t) * std::max<uint32_t>(n, 1)));
        CF_TRY(dev_alloc(ctx, dtake, sizeof(uint32_t) * std::max<uint32_t>(n, 1)));
    }
    const unsigned grid = (unsigned)std::max<uint32_t>(1, std::min<uint32_t>(n, 65536u));
    if (n) {
        if (topk)
            hipLaunchKernelGGL(row_topk_kernel, dim3(grid), dim3(kGT), 0, stream, (uint64_t)n, d_dense, topk,
                               (uint32_t*)dthr.p, (uint32_t*)dtake.p, *d_rp + 1);
        else
            hipLaunchKernelGGL(row_nnz_kernel, dim3(grid), dim3(kGT), 0, stream, (uint64_t)n, d_dense, *d_rp + 1);
        CF_HIP_CHECK(ctx, hipGetLastError());
        CF_HIP_CHECK(ctx, hipMemcpyAsync(rp.data() + 1, *d_rp + 1, sizeof(uint64_t) * n, hipMemcpyDeviceToHost, stream));
        CF_HIP_CHECK(ctx, hipStreamSynchronize(stream));
    }
    for (uint32_t i = 0; i < n; ++i) rp[i + 1] += rp[i];
    *nnz = rp[n];
    CF_HIP_CHECK(ctx, hipMemcpyAsync(*d_rp, rp.data(), sizeof(uint64_t) * ((size_t)n + 1), hipMemcpyHostToDevice,
                                     stream));
    if (hipMalloc(d_col, sizeof(uint32_t) * std::max<uint64_t>(*nnz, 1)) != hipSuccess ||
        hipMalloc(d_w, sizeof(float) * std::max<uint64_t>(*nnz, 1)) != hipSuccess)
        return cf_set_error(ctx, CF_ENOMEM, "CSR graph allocation");
    if (n) {
        hipLaunchKernelGGL(row_compact_kernel, dim3(grid), dim3(kGT), 0, stream, (uint64_t)n, d_dense,
                           (const uint64_t*)*d_rp, *d_col, *d_w, topk ? (const uint32_t*)dthr.p : nullptr,
                           topk ? (const uint32_t*)dtake.p : nullptr);
        CF_HIP_CHECK(ctx, hipGetLastError());
    }
    CF_HIP_CHECK(ctx, hipStreamSynchronize(stream));
    return CF_OK;
}

// Install a device dense matrix as the context's graph in its upload layout (adopting the
// buffer when dense; compacting it and freeing it when CSR).
int cf_adopt_dense_graph(cf_ctx* ctx, uint32_t n, float* d_dense) {
    free_graph(ctx);
    if (ctx->graph_layout == CF_GRAPH_DENSE) {
        ctx->d_graph = d_dense;
        ctx->n_items = n;
        return CF_OK;
    }
    uint64_t *rp = nullptr, nnz = 0;
    uint32_t* col = nullptr;
    float* w = nullptr;
    const int rc = cf_dense_to_csr(ctx, n, d_dense, &rp, &col, &w, &nnz, nullptr, 0);
    (void)hipFree(d_dense);
    if (rc != CF_OK) {
        if (rp) (void)hipFree(rp);
        if (col) (void)hipFree(col);
        if (w) (void)hipFree(w);
        return rc;
    }
    ctx->d_grp = rp;
    ctx->d_gcol = col;
    ctx->d_gw = w;
    ctx->g_nnz = nnz;
    ctx->graph_csr = true;
    ctx->n_items = n;
    return CF_OK;
}

extern "C" {

int cf_set_graph_layout(cf_ctx* ctx, int layout) {
    if (!ctx || (layout != CF_GRAPH_DENSE && layout != CF_GRAPH_CSR))
        return cf_set_error(ctx, CF_EINVAL, "cf_set_graph_layout: unknown layout");
    ctx->graph_layout = layout;
    return CF_OK;
}

int cf_graph_info(const cf_ctx* ctx, int* layout, uint32_t* n_items, uint64_t* nnz) {
    if (!ctx) return CF_EINVAL;
    if (layout) *layout = ctx->graph_csr ? CF_GRAPH_CSR : CF_GRAPH_DENSE;
    if (n_items) *n_items = ctx->n_items;
    if (nnz) *nnz = ctx->graph_csr ? ctx->g_nnz : 0;
    return CF_OK;
}

int cf_item_graph_upload(cf_ctx* ctx, uint32_t n_items, const uint64_t* row_ptr, const uint32_t* col,
                         const float* w) {
    if (!ctx || !row_ptr || (row_ptr[n_items] > 0 && (!col || !w)))
        return cf_set_error(ctx, CF_EINVAL, "cf_item_graph_upload: null argument");
    CF_TRY(set_device(ctx));
    // row_ptr must start at 0 and never decrease: every row range below (the dense scatter's,
    // the CSR sort's idx.resize(e - b) on a worker thread) trusts it
    if (row_ptr[0] != 0) return cf_set_error(ctx, CF_EINVAL, "cf_item_graph_upload: row_ptr[0] != 0");
    for (uint32_t r = 0; r < n_items; ++r)
        if (row_ptr[r + 1] < row_ptr[r])
            return cf_set_error(ctx, CF_EINVAL, "cf_item_graph_upload: row_ptr decreases at row " + std::to_string(r));
    const uint64_t nnz = row_ptr[n_items];
    for (uint64_t e = 0; e < nnz; ++e)
        if (col[e] >= n_items) return cf_set_error(ctx, CF_EINVAL, "cf_item_graph_upload: column out of range");
    if (ctx->graph_layout == CF_GRAPH_DENSE) {
        // dense: the rows scattered on the device, the last duplicate of a pair winning
        // (repeated `weights(m1,m2) = w` assignments, precompute_local_threads.cpp:284)
        free_graph(ctx);
        const size_t dense_bytes = (size_t)n_items * n_items * sizeof(float);
        float* dense = nullptr;
        if (hipMalloc(&dense, std::max<size_t>(dense_bytes, 16)) != hipSuccess)
            return cf_set_error(ctx, CF_ENOMEM, "cf_item_graph_upload: dense graph allocation failed");
        DevBuf drp, dcol, dw;
        int rc = dev_alloc(ctx, drp, sizeof(uint64_t) * (n_items + 1));
        if (rc == CF_OK) rc = dev_alloc(ctx, dcol, sizeof(uint32_t) * nnz);
        if (rc == CF_OK) rc = dev_alloc(ctx, dw, sizeof(float) * nnz);
        hipError_t e = rc == CF_OK ? hipMemset(dense, 0, dense_bytes) : hipSuccess;
        if (rc == CF_OK && e == hipSuccess)
            e = hipMemcpy(drp.p, row_ptr, sizeof(uint64_t) * (n_items + 1), hipMemcpyHostToDevice);
        if (rc == CF_OK && e == hipSuccess && nnz) e = hipMemcpy(dcol.p, col, sizeof(uint32_t) * nnz, hipMemcpyHostToDevice);
        if (rc == CF_OK && e == hipSuccess && nnz) e = hipMemcpy(dw.p, w, sizeof(float) * nnz, hipMemcpyHostToDevice);
        if (rc == CF_OK && e != hipSuccess) rc = cf_set_error(ctx, CF_EHIP, std::string("graph upload: ") + hipGetErrorString(e));
        if (rc == CF_OK)
            rc = cf_launch_dense_scatter(ctx, n_items, (const uint64_t*)drp.p, (const uint32_t*)dcol.p,
                                         (const float*)dw.p, dense, nullptr);
        if (rc == CF_OK && hipDeviceSynchronize() != hipSuccess) rc = cf_set_error(ctx, CF_EHIP, "graph scatter failed");
        if (rc != CF_OK) {
            (void)hipFree(dense);
            return rc;
        }
        ctx->d_graph = dense;
        ctx->n_items = n_items;
        return CF_OK;
    }
    // CSR: every row sorted by column, the LAST duplicate of a column kept (the dense scatter's
    // rule), zero weights dropped (a zero and a missing edge read the same); rows on threads
    std::vector<uint64_t> rp((size_t)n_items + 1, 0);
    std::vector<uint32_t> cols(nnz);
    std::vector<float> ws(nnz);
    std::vector<uint64_t> kept(n_items, 0);
    const unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    {
        std::vector<std::thread> pool;
        for (unsigned t = 0; t < T; ++t)
            pool.emplace_back([&, t]() {
                std::vector<uint64_t> idx;
                for (uint32_t r = (uint32_t)((uint64_t)n_items * t / T); r < (uint32_t)((uint64_t)n_items * (t + 1) / T);
                     ++r) {
                    const uint64_t b = row_ptr[r], e = row_ptr[r + 1];
                    idx.resize(e - b);
                    std::iota(idx.begin(), idx.end(), b);
                    std::stable_sort(idx.begin(), idx.end(), [&](uint64_t x, uint64_t y) { return col[x] < col[y]; });
                    uint64_t o = b;
                    for (size_t q = 0; q < idx.size(); ++q) {
                        if (q + 1 < idx.size() && col[idx[q + 1]] == col[idx[q]]) continue;   // a later one wins
                        if (w[idx[q]] == 0.0f) continue;
                        cols[o] = col[idx[q]];
                        ws[o] = w[idx[q]];
                        ++o;
                    }
                    kept[r] = o - b;
                }
            });
        for (auto& th : pool) th.join();
    }
    for (uint32_t r = 0; r < n_items; ++r) rp[r + 1] = rp[r] + kept[r];
    for (uint32_t r = 0; r < n_items; ++r)   // close the gaps left by dropped entries
        if (rp[r] != row_ptr[r]) {
            std::memmove(cols.data() + rp[r], cols.data() + row_ptr[r], sizeof(uint32_t) * kept[r]);
            std::memmove(ws.data() + rp[r], ws.data() + row_ptr[r], sizeof(float) * kept[r]);
        }
    free_graph(ctx);
    const uint64_t n2 = rp[n_items];
    if (hipMalloc(&ctx->d_grp, sizeof(uint64_t) * ((size_t)n_items + 1)) != hipSuccess ||
        hipMalloc(&ctx->d_gcol, sizeof(uint32_t) * std::max<uint64_t>(n2, 1)) != hipSuccess ||
        hipMalloc(&ctx->d_gw, sizeof(float) * std::max<uint64_t>(n2, 1)) != hipSuccess) {
        free_graph(ctx);
        return cf_set_error(ctx, CF_ENOMEM, "cf_item_graph_upload: CSR graph allocation failed");
    }
    hipError_t e = hipMemcpy(ctx->d_grp, rp.data(), sizeof(uint64_t) * ((size_t)n_items + 1), hipMemcpyHostToDevice);
    if (e == hipSuccess && n2) e = hipMemcpy(ctx->d_gcol, cols.data(), sizeof(uint32_t) * n2, hipMemcpyHostToDevice);
    if (e == hipSuccess && n2) e = hipMemcpy(ctx->d_gw, ws.data(), sizeof(float) * n2, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        free_graph(ctx);
        return cf_set_error(ctx, CF_EHIP, std::string("CSR graph upload: ") + hipGetErrorString(e));
    }
    ctx->graph_csr = true;
    ctx->g_nnz = n2;
    ctx->n_items = n_items;
    return CF_OK;
}

int cf_item_graph_upload_dense(cf_ctx* ctx, uint32_t n_items, const float* w_dense, int on_device) {
    if (!ctx || (!w_dense && n_items)) return cf_set_error(ctx, CF_EINVAL, "cf_item_graph_upload_dense: null");
    CF_TRY(set_device(ctx));
    const size_t bytes = (size_t)n_items * n_items * sizeof(float);
    float* dense = nullptr;
    if (hipMalloc(&dense, std::max<size_t>(bytes, 16)) != hipSuccess)
        return cf_set_error(ctx, CF_ENOMEM, "dense graph allocation failed");
    hipError_t e = hipMemcpy(dense, w_dense, bytes, on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(dense);
        return cf_set_error(ctx, CF_EHIP, std::string("dense graph copy: ") + hipGetErrorString(e));
    }
    return cf_adopt_dense_graph(ctx, n_items, dense);
}

// knn2 (knn2.cpp:127-164) returning the compacted edge list the reference writes: per source
// item a (compact id), its targets b ascending with w(a, b) > w_min (and cnt > cnt_min), as
// CSR edge_off[n_items + 1] / edge_col / edge_w.  The dense similarity matrix stays on the
// device (compacted there); only the edges cross PCIe.  edge_cap too small: CF_ERANGE with
// *n_edges = the size needed (edge_off complete).  adopt_as_graph != 0 installs the result
// as the context's graph in its upload layout (cf_set_graph_layout).
int cf_item_cosine_edges(cf_ctx* ctx, uint32_t n_users, uint32_t n_items, const uint64_t* user_off,
                         const uint32_t* item, const float* rating, float w_min, int cnt_min, int adopt_as_graph,
                         uint64_t* edge_off, uint32_t* edge_col, float* edge_w, uint64_t edge_cap, uint64_t* n_edges) {
    if (!ctx || !user_off || (user_off[n_users] && (!item || !rating)) || !edge_off || !n_edges)
        return cf_set_error(ctx, CF_EINVAL, "cf_item_cosine_edges: null argument");
    CF_TRY(set_device(ctx));
    const uint64_t n = user_off[n_users];
    for (uint64_t e = 0; e < n; ++e)
        if (item[e] >= n_items) return cf_set_error(ctx, CF_EINVAL, "cf_item_cosine_edges: item index out of range");
    bool integer = true;
    for (uint64_t i = 0; i < n && integer; ++i)
        integer = rating[i] == std::nearbyint(rating[i]) && rating[i] >= -11.0f && rating[i] <= 11.0f;
    DevBuf doff, ditem, drat;
    float* dW = nullptr;
    int rc = dev_alloc(ctx, doff, sizeof(uint64_t) * (n_users + 1));
    if (rc == CF_OK) rc = dev_alloc(ctx, ditem, sizeof(uint32_t) * n);
    if (rc == CF_OK) rc = dev_alloc(ctx, drat, sizeof(float) * n);
    if (rc == CF_OK && hipMalloc(&dW, std::max<size_t>((size_t)n_items * n_items * sizeof(float), 16)) != hipSuccess)
        rc = cf_set_error(ctx, CF_ENOMEM, "cf_item_cosine_edges: weight matrix allocation");
    hipError_t e = hipSuccess;
    if (rc == CF_OK) {
        e = hipMemcpy(doff.p, user_off, sizeof(uint64_t) * (n_users + 1), hipMemcpyHostToDevice);
        if (e == hipSuccess && n) e = hipMemcpy(ditem.p, item, sizeof(uint32_t) * n, hipMemcpyHostToDevice);
        if (e == hipSuccess && n) e = hipMemcpy(drat.p, rating, sizeof(float) * n, hipMemcpyHostToDevice);
        if (e != hipSuccess) rc = cf_set_error(ctx, CF_EHIP, std::string("knn2 H2D: ") + hipGetErrorString(e));
    }
    if (rc == CF_OK)
        rc = cf_launch_knn2(ctx, n_users, n_items, (const uint64_t*)doff.p, (const uint32_t*)ditem.p,
                            (const float*)drat.p, integer ? 1 : 0, w_min, cnt_min, dW, nullptr);
    uint64_t *rp = nullptr, nnz = 0;
    uint32_t* col = nullptr;
    float* wv = nullptr;
    if (rc == CF_OK) rc = cf_dense_to_csr(ctx, n_items, dW, &rp, &col, &wv, &nnz, nullptr, ctx->knn2_topk);
    if (rc == CF_OK) {
        *n_edges = nnz;
        e = hipMemcpy(edge_off, rp, sizeof(uint64_t) * ((size_t)n_items + 1), hipMemcpyDeviceToHost);
        if (e == hipSuccess && nnz <= edge_cap && nnz) {
            if (!edge_col || !edge_w) rc = cf_set_error(ctx, CF_EINVAL, "cf_item_cosine_edges: null edge arrays");
            else e = hipMemcpy(edge_col, col, sizeof(uint32_t) * nnz, hipMemcpyDeviceToHost);
            if (rc == CF_OK && e == hipSuccess) e = hipMemcpy(edge_w, wv, sizeof(float) * nnz, hipMemcpyDeviceToHost);
        }
        if (rc == CF_OK && e != hipSuccess) rc = cf_set_error(ctx, CF_EHIP, std::string("edges D2H: ") + hipGetErrorString(e));
        if (rc == CF_OK && nnz > edge_cap) rc = cf_set_error(ctx, CF_ERANGE, "cf_item_cosine_edges: edge_cap too small");
    }
    if (rc == CF_OK && adopt_as_graph) {
        free_graph(ctx);
        if (ctx->graph_layout == CF_GRAPH_CSR) {   // the compacted list IS the CSR graph
            ctx->d_grp = rp;
            ctx->d_gcol = col;
            ctx->d_gw = wv;
            ctx->g_nnz = nnz;
            ctx->graph_csr = true;
            rp = nullptr;
            col = nullptr;
            wv = nullptr;
        } else {
            if (ctx->knn2_topk) {   // the dense graph holds the top-K list only
                e = hipMemset(dW, 0, (size_t)n_items * n_items * sizeof(float));
                if (e == hipSuccess)
                    rc = cf_launch_dense_scatter(ctx, n_items, rp, col, wv, dW, nullptr);
                else
                    rc = cf_set_error(ctx, CF_EHIP, "top-k dense graph reset");
                if (rc == CF_OK && hipDeviceSynchronize() != hipSuccess) rc = cf_set_error(ctx, CF_EHIP, "top-k scatter");
            }
            if (rc == CF_OK) {   // a failed reset / scatter leaves the context with no graph (dW freed below)
                ctx->d_graph = dW;
                dW = nullptr;
            }
        }
        if (rc == CF_OK) ctx->n_items = n_items;
    }
    if (rp) (void)hipFree(rp);
    if (col) (void)hipFree(col);
    if (wv) (void)hipFree(wv);
    if (dW) (void)hipFree(dW);
    return rc;
}

int cf_set_knn2_topk(cf_ctx* ctx, uint32_t topk) {
    if (!ctx) return CF_EINVAL;
    ctx->knn2_topk = topk;
    return CF_OK;
}

}  // extern "C"
